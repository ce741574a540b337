#!/bin/bash
# round-3 probe: new state tests, the tiling's memory floor, K1 attribution
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_api_state.py "tests/test_gpu_parity.py::test_pack_window_paths_in_one_scan" > gpurun_out/state_tests.log 2>&1; rc=$?
tail -3 gpurun_out/state_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/state_tests.log | head -20; exit $rc; }
timeout -k 10 300 ./build/tile_stream 256 > gpurun_out/tile_stream.txt 2>&1 || { tail -5 gpurun_out/tile_stream.txt; exit 1; }
cat gpurun_out/tile_stream.txt
MODE=dct FLAGS="0 4 36 100 8 12 16 20 1" bash scripts/k1_attrib.sh 2>&1 | tee gpurun_out/attrib_dct.txt
