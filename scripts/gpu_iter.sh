#!/bin/bash
# scripts/gpu_iter.sh -- one iteration on the GPU box: parity tests (-x),
# default bench (no CPU baseline), optional K1 wave-lifetime diagnostics.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['stages_ms'], d.get('fp64_fixups_per_frame'))"
if [ -n "${WTIME:-}" ]; then
  MIJ_K1_WTIME=1 MIJ_LIB=$PWD/jpeg-encoder-decoder_amd/libmijpeg_diag.so timeout -k 10 200 python3 bench.py --mode dct --steps 3 --warmup 1 --no-cpu-baseline --verify 0 > gpurun_out/wt.log 2>&1 || { tail -3 gpurun_out/wt.log; exit 1; }
  grep "K1 waves" gpurun_out/wt.log
fi
