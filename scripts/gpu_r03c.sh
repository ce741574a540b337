#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./build/valu_rate3 > gpurun_out/valu_rate3.txt 2>&1 || { tail -5 gpurun_out/valu_rate3.txt; exit 1; }
cat gpurun_out/valu_rate3.txt
timeout -k 10 300 ./build/tile_stream 256 > gpurun_out/tile_stream2.txt 2>&1 || { tail -5 gpurun_out/tile_stream2.txt; exit 1; }
cat gpurun_out/tile_stream2.txt
bash scripts/gpu_phases.sh
