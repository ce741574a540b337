#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MIJ_LIB=$PWD/ab/libmijpeg_s64.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tables.py > gpurun_out/t_tab.log 2>&1; echo "s64 rc=$?"; grep -E "^E  |passed|failed" gpurun_out/t_tab.log | head -5
