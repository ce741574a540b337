#!/bin/bash
# scripts/c4_prof.sh -- kernel durations of the config-4 band path at N=1
# (8 frames of 7680x4320 per step, root or band emission: EMIT=root|bands):
# rocprofv3 kernel trace + stats over 100 steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/c4_prof_${EMIT:-root}; rm -rf $out; mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 bench.py --workload config4 --band-emit ${EMIT:-root} --steps 100 --warmup 10 --no-cpu-baseline --verify 0 > $out/bench.log 2>&1 || { echo "rocprofv3 failed"; tail -5 $out/bench.log; exit 1; }
f=$(find $out -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>6s} avg {float(r["AverageNs"])/1000:8.2f} us')
PY
