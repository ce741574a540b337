#!/bin/bash
# K1 per-phase wall clocks (diag build, MIJ_K1_WTIME): coefficient and token variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for mode in dct encode; do
  MIJ_K1_WTIME=1 MIJ_LIB=$PWD/jpeg-encoder-decoder_amd/libmijpeg_diag.so timeout -k 10 200 python3 bench.py --mode $mode --steps 2 --warmup 1 --no-cpu-baseline --verify 0 --coef-launches 0 ${ARGS:-} > gpurun_out/phases_$mode.log 2>&1 || { tail -3 gpurun_out/phases_$mode.log; exit 1; }
  echo "== $mode"; grep "K1 " gpurun_out/phases_$mode.log | tail -2
done
