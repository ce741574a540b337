#!/bin/bash
# round-3 closing run on the final tree: GPU suite + smoke, the bench set
# (scripts/gpu_final_r03.sh -> gpurun_out/final_r03/) and the profiles
# (scripts/gpu_prof_r03.sh -> gpurun_out/prof_r03/, gpurun_out/util_r03/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/final_pytest.log 2>&1 || { grep -E "^E |FAILED|Timeout|Error" gpurun_out/final_pytest.log | head -20; tail -5 gpurun_out/final_pytest.log; exit 1; }
echo "suite: $(tail -1 gpurun_out/final_pytest.log)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -5 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
bash scripts/gpu_final_r03.sh || exit 1
bash scripts/gpu_prof_r03.sh || exit 1
