#!/bin/bash
# k_pack_lb group size A/B on config 3 (Q=50 and 90)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for q in 50 90; do
for lib in ${LIBS:-ab/libmijpeg_base.so ab/libmijpeg_s128o3.so ab/libmijpeg_s128o2.so ab/libmijpeg_base.so ab/libmijpeg_s128o3.so ab/libmijpeg_s128o2.so}; do
  MIJ_LIB=$PWD/$lib timeout -k 10 150 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --coef-launches 0 --quality $q > gpurun_out/pk.log 2>&1 || { tail -3 gpurun_out/pk.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/pk.log').read().strip().splitlines()[-1]);s=d['stages_ms'];print('Q', sys.argv[2], sys.argv[1], d['ms_per_step'], 'pack', s['pack'], d['verified_frames'])" $lib $q
done
done
