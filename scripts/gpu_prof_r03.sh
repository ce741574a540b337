#!/bin/bash
# round-3 profiles of the default bench: kernel stats + PMC traffic passes
# (scripts/profile.sh) and the utilisation passes (scripts/pmc_util.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/profile.sh r03 > gpurun_out/prof_r03.txt 2>&1 || { tail -20 gpurun_out/prof_r03.txt; exit 1; }
tail -12 gpurun_out/prof_r03.txt
bash scripts/pmc_util.sh r03 > gpurun_out/util_r03.txt 2>&1 || { tail -20 gpurun_out/util_r03.txt; exit 1; }
tail -5 gpurun_out/util_r03.txt
