#!/bin/bash
# scripts/profile.sh <tag> -- rocprofv3 kernel stats of the default bench and
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) on K1 alone.  Outputs under
# gpurun_out/prof_<tag>/.  Each GPU step has its own time limit.
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
  echo "== $name rc=$rc"; tail -n 5 "$out/$name.log"
  [ $rc -eq 0 ] || { echo "stopping after $name"; exit $rc; }
}
run bench_plain 600 python3 bench.py ${BENCH_ARGS:-}
run stats 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run -- \
    python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-}
run pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/pmc_fetch" -o run -- \
    python3 bench.py --mode dct --steps 3 --warmup 1 --no-cpu-baseline --verify 0
run pmc_write 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/pmc_write" -o run -- \
    python3 bench.py --mode dct --steps 3 --warmup 1 --no-cpu-baseline --verify 0
find "$out" -name "*.csv" | head -20
