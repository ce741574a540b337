#!/bin/bash
# scripts/gpu_decode.sh -- round-trip verifier on the GPU: tests, bench, rocprof stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/decode
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/decode/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 12 "gpurun_out/decode/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_decode 600 python -u -m pytest tests/test_decode.py -m gpu -x -q --timeout 120 --timeout-method thread
step bench_decode 300 python bench.py --workload decode --steps 3 --warmup 1
step prof_decode 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/decode/prof -o run -- python bench.py --workload decode --steps 3 --warmup 1
find gpurun_out/decode/prof -name '*kernel_stats.csv' -exec cat {} \;
