#!/bin/bash
# scripts/gpu_iter2.sh -- parity tests (-x), then the default bench N times
# (default 2; every slot verified), printing the stage times of each run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -2 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
fi
for i in $(seq 1 ${RUNS:-2}); do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench$i.log 2>&1 || { tail -3 gpurun_out/bench$i.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/bench$i.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['stages_ms'], d.get('verified_frames'))"
done
