#!/bin/bash
# scripts/profile.sh <tag> -- rocprofv3 kernel statistics of the default bench
# and separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the same workload, then
# per-kernel HBM traffic (scripts/traffic.py).  Outputs under gpurun_out/prof_<tag>/.
set -u
tag=${1:-r01}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p "$out"
run() {
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$out/$name.log"
  [ $rc -eq 0 ] || { echo "stopping after $name"; exit $rc; }
}
ARGS="--no-cpu-baseline ${BENCH_ARGS:-}"
run bench_plain 600 python3 bench.py ${BENCH_ARGS:-}
run stats 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run -- \
    python3 bench.py $ARGS
run pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/pmc_fetch" -o run -- \
    python3 bench.py $ARGS --steps 3 --warmup 1 --verify 0
run pmc_write 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/pmc_write" -o run -- \
    python3 bench.py $ARGS --steps 3 --warmup 1 --verify 0
python3 -c "
import json; d=json.loads(open('$out/bench_plain.log').read().strip().splitlines()[-1])
json.dump(d['config'], open('$out/config.json','w'))"
python3 scripts/traffic.py "$out" "$out/traffic.json"
