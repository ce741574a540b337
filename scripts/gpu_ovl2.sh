#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="ab/libmijpeg_w12.so ab/libmijpeg_w10.so" OVS="1 2 4" bash scripts/gpu_ovl.sh || exit 1
MIJ_LIB=$PWD/ab/libmijpeg_w10.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ovlprof -o ov -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --coef-launches 0 --overlap 2 --verify 0 > gpurun_out/ovlprof.log 2>&1 || { tail -5 gpurun_out/ovlprof.log; exit 1; }
f=$(find gpurun_out/ovlprof -name "ov_kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in rows)
k1 = [i for i, k in enumerate(ks) if 'k_mcu_dct' in k[2]]
i0 = k1[-4]
t0 = ks[i0][0]
for s, e, n in ks[i0:]:
    if e - s > 3000: print(f"{(s - t0) / 1e3:9.1f} -> {(e - t0) / 1e3:9.1f} ({(e - s) / 1e3:7.1f}) {n}")
PY
