#!/bin/bash
# K1 wave count x overlap sub-batches on config 3 (A/B)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in ${LIBS:-ab/libmijpeg_w12.so ab/libmijpeg_w10.so ab/libmijpeg_w9.so}; do
  for ov in ${OVS:-1 2 4 8}; do
    MIJ_LIB=$PWD/$lib timeout -k 10 150 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --coef-launches 0 --overlap $ov > gpurun_out/ovl.log 2>&1 || { tail -3 gpurun_out/ovl.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/ovl.log').read().strip().splitlines()[-1]);print(sys.argv[1], 'ov', sys.argv[2], d['ms_per_step'], {k: v for k, v in d['stages_ms'].items() if v > 0.01}, d['verified_frames'])" $lib $ov
  done
done
