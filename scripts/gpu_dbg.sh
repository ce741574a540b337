#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python3 -u scripts/debug_band.py 1 2 3 4 > gpurun_out/dbg.log 2>&1 || { tail -20 gpurun_out/dbg.log; exit 1; }; grep -v amdgpu.ids gpurun_out/dbg.log | grep -v "True$"
