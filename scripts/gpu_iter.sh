#!/bin/bash
# scripts/gpu_iter.sh -- one development iteration on the GPU: the GPU suite
# on the in-tree library, then A/B timings of the libraries in $LIBS
# (scripts/ab.sh) at each quality in $QS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -2 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
fi
for q in ${QS:-50}; do
  echo "Q=$q"
  ARGS="--quality $q --coef-launches 0 ${ARGS:-}" ROUNDS=${ROUNDS:-3} bash scripts/ab.sh || exit 1
done
