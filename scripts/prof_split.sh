#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/prof_split; mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --verify 0 > $out/stats.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $out/pmc -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --verify 0 > $out/pmc.log 2>&1 || exit 1
python3 - <<'PY'
import csv, collections
for r in csv.DictReader(open('gpurun_out/prof_split/stats/run_kernel_stats.csv')):
    print(f"{r['Name'][:60]:60s} calls={r['Calls']:>4s} avg_ms={float(r['AverageNs'])/1e6:8.3f}")
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open('gpurun_out/prof_split/pmc/run_counter_collection.csv')):
    acc[r['Kernel_Name'][:50]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in acc.items():
    if 'mcu' in k:
        print(k, {c: f"{sum(v)/len(v):.3g}" for c, v in d.items()})
PY
