#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in ab/libmijpeg_pw6144.so ab/libmijpeg_pw7168.so ab/libmijpeg_pw8192.so ab/libmijpeg_pw6144.so ab/libmijpeg_pw7168.so ab/libmijpeg_pw8192.so; do
  MIJ_LIB=$PWD/$lib timeout -k 10 150 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --coef-launches 0 --quality 90 > gpurun_out/q.log 2>&1 || { tail -3 gpurun_out/q.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/q.log').read().strip().splitlines()[-1]);s=d['stages_ms'];print(sys.argv[1], d['ms_per_step'], 'pack', s['pack'], d['verified_frames'])" $lib
done
