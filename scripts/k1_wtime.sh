#!/bin/bash
# scripts/k1_wtime.sh -- per-wave lifetimes and phase clocks of K1 (diag
# build, MIJ_K1_WTIME) for one 1920x1280 frame and for config 3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for args in "--frames 1 --width 1920 --height 1280" "--frames 16"; do
  echo "== $args"
  MIJ_LIB=$PWD/jpeg-encoder-decoder_amd/libmijpeg_diag.so MIJ_K1_WTIME=1 timeout -k 10 120 python3 bench.py $args --steps 2 --warmup 1 --no-cpu-baseline --coef-launches 0 --verify 0 > gpurun_out/wtime.log 2>&1 || { tail -5 gpurun_out/wtime.log; exit 1; }
  grep "^K1" gpurun_out/wtime.log | tail -2
done
