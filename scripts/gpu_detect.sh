#!/bin/bash
# scripts/gpu_detect.sh -- change detector on the GPU: parity tests, the
# detect bench workload, and its rocprofv3 kernel-trace summary.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/detect
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/detect/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 12 "gpurun_out/detect/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_detect 600 python -u -m pytest tests/test_detect.py -m gpu -x -q --timeout 120 --timeout-method thread
step bench_detect 300 python bench.py --workload detect --region-frame 3840x2160 --steps 20 --warmup 3 --cpu-seconds 10
step bench_detect_1080 300 python bench.py --workload detect --region-frame 1920x1080 --steps 50 --warmup 3 --no-cpu-baseline
step prof_detect 300 rocprofv3 --kernel-trace --stats -d gpurun_out/detect/prof -o run -- python bench.py --workload detect --region-frame 3840x2160 --steps 20 --warmup 3 --no-cpu-baseline
find gpurun_out/detect/prof -name '*kernel_stats.csv' | head -3
