#!/bin/bash
# scripts/kstats.sh <tag> [bench args] -- rocprofv3 kernel statistics of a short
# bench run; prints per-kernel average duration.  Output: gpurun_out/kstats_<tag>/
set -u
tag=${1:-x}; shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/kstats_$tag
mkdir -p "$out"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --verify 0 "$@" > "$out/bench.log" 2>&1 || { tail -5 "$out/bench.log"; exit 1; }
python3 - "$out" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:60]:60s} calls={r['Calls']:>5s} avg_ms={float(r['AverageNs'])/1e6:8.4f} pct={float(r['Percentage']):6.2f}")
PY
