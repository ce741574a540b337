#!/bin/bash
# scripts/single_prof.sh -- kernel durations of one 1920x1280 frame per step
# (config 2's shape): rocprofv3 kernel trace + stats over 200 steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/single_prof; rm -rf $out; mkdir -p $out
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 bench.py --frames 1 --width 1920 --height 1280 --steps 200 --warmup 20 --no-cpu-baseline --coef-launches 0 --verify 0 > $out/bench.log 2>&1 || { echo "rocprofv3 failed"; tail -5 $out/bench.log; exit 1; }
f=$(find $out -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>6s} avg {float(r["AverageNs"])/1000:8.2f} us')
PY
