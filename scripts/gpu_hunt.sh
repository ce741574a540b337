#!/bin/bash
# scripts/gpu_hunt.sh -- a few GPU tests per library in $LIBS (MIJ_LIB), each
# library's run under its own short time limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in $LIBS; do
  n=$(basename $lib .so)
  MIJ_LIB=$PWD/$lib timeout -k 10 ${SECS:-120} python -u -m pytest tests -m gpu -x -q --timeout 60 --timeout-method thread ${TESTS:-tests/test_api_state.py} > gpurun_out/hunt_$n.log 2>&1
  rc=$?
  echo "$n rc=$rc $(tail -1 gpurun_out/hunt_$n.log)"
  [ $rc -eq 0 ] || exit $rc
done
