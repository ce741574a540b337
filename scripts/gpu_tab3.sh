#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MIJ_TAB_TIME=1
for lib in ${LIBS:-ab/libmijpeg_u8.so ab/libmijpeg_u16.so ab/libmijpeg_u32.so ab/libmijpeg_bf8.so}; do
  MIJ_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --frames 1 --width 1920 --height 1280 --steps 2 --warmup 1 --no-cpu-baseline --coef-launches 0 --verify 0 > gpurun_out/tab1.log 2>&1 || { tail -5 gpurun_out/tab1.log; exit 1; }
  echo "== $lib"; grep k_tables gpurun_out/tab1.log | tail -3
  MIJ_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --coef-launches 0 --verify 0 > gpurun_out/tab256.log 2>&1 || { tail -5 gpurun_out/tab256.log; exit 1; }
  grep k_tables gpurun_out/tab256.log | tail -3
done
