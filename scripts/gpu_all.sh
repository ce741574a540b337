#!/bin/bash
# the whole GPU suite, then the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/t_all.log 2>&1 || { grep -E "^E |FAILED|Timeout|Error" gpurun_out/t_all.log | head -20; tail -5 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-600
