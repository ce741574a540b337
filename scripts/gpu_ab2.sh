#!/bin/bash
# scripts/gpu_ab2.sh -- the GPU suite on the in-tree library, then A/B rounds
# of $LIBS at Q=50 (with the coefficient K1) and at $QS_EXTRA (token K1 only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -2 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
fi
echo "Q=50"
ARGS="--quality 50 ${ARGS:-}" ROUNDS=${ROUNDS:-3} VERIFY=${VERIFY:-0} bash scripts/ab.sh || exit 1
for q in ${QS_EXTRA:-}; do
  echo "Q=$q"
  ARGS="--quality $q --coef-launches 0 ${ARGS:-}" ROUNDS=${ROUNDS_EXTRA:-2} bash scripts/ab.sh || exit 1
done
