#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['stages_ms'], d['roofline_k1_coefficient_variant']['ms_per_launch'])"
MIJ_PACK_TIME=1 MIJ_LIB=$PWD/jpeg-encoder-decoder_amd/libmijpeg_diag.so timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --verify 0 --coef-launches 0 > gpurun_out/packtime.log 2>&1 || { tail -3 gpurun_out/packtime.log; exit 1; }
grep "pack groups" gpurun_out/packtime.log | tail -2
