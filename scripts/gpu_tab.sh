#!/bin/bash
# k_tables phase clocks (diag build, MIJ_TAB_TIME) on a single 1920x1280
# frame and on the config-3 batch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MIJ_LIB=$PWD/jpeg-encoder-decoder_amd/libmijpeg_diag.so MIJ_TAB_TIME=1
timeout -k 10 120 python3 bench.py --frames 1 --width 1920 --height 1280 --steps 2 --warmup 1 --no-cpu-baseline --coef-launches 0 --verify 0 > gpurun_out/tab1.log 2>&1 || { tail -5 gpurun_out/tab1.log; exit 1; }
grep k_tables gpurun_out/tab1.log | tail -7
timeout -k 10 120 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --coef-launches 0 --verify 0 > gpurun_out/tab256.log 2>&1 || { tail -5 gpurun_out/tab256.log; exit 1; }
grep k_tables gpurun_out/tab256.log | tail -3
