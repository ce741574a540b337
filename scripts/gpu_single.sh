#!/bin/bash
# single-frame latency (config 2's shape) and small batches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for fr in 1 1 4; do
  timeout -k 10 120 python3 bench.py --frames $fr --width 1920 --height 1280 --steps 200 --warmup 20 --no-cpu-baseline --coef-launches 0 > gpurun_out/single.log 2>&1 || { tail -3 gpurun_out/single.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/single.log').read().strip().splitlines()[-1]);print('frames', sys.argv[1], 'ms', d['ms_per_step'], d['stages_ms'], d['verified_frames'])" $fr
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/single_prof -o s -- python3 bench.py --frames 1 --width 1920 --height 1280 --steps 50 --warmup 5 --no-cpu-baseline --coef-launches 0 > gpurun_out/single_prof.log 2>&1 || { tail -3 gpurun_out/single_prof.log; exit 1; }
f=$(find gpurun_out/single_prof -name "s_kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:44]) for r in rows)
k1 = [i for i, k in enumerate(ks) if 'k_mcu_dct' in k[2]]
i0, i1 = k1[-3], k1[-2]
t0 = ks[i0][0]; pe = t0
for s, e, n in ks[i0 - 3:i1]:
    print(f"{(s - t0) / 1e3:8.1f} dur {(e - s) / 1e3:6.1f} gap {(s - pe) / 1e3:6.1f} {n}")
    pe = max(pe, e)
PY
