#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 90 python3 -u scripts/debug_dev.py none > gpurun_out/dbg_none.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/dbg_none.log | tail -30
timeout -k 10 90 python3 -u scripts/debug_dev.py nccl > gpurun_out/dbg_nccl.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/dbg_nccl.log | tail -30
exit $rc
