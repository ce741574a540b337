#!/bin/bash
# scripts/gpu_check.sh -- one GPU session: smoke, parity tests, a short bench.
# Every GPU step has its own time limit; a crash/abort/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>; ok for exit 0/1 (test failures)
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-}
if [ "${BENCH:-1}" = 1 ]; then
  step bench 600 python bench.py ${BENCH_ARGS:---steps 5 --warmup 2}
fi
