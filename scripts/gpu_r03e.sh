#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="ab/libmijpeg_base.so ab/libmijpeg_share16.so ab/libmijpeg_share12.so" ROUNDS=2 bash scripts/gpu_ab.sh || exit 1
timeout -k 10 600 python3 bench.py --workload stream --steps 3 --warmup 1 --cpu-seconds 8 > gpurun_out/bench_stream.log 2>&1 || { tail -5 gpurun_out/bench_stream.log; exit 1; }
tail -1 gpurun_out/bench_stream.log
