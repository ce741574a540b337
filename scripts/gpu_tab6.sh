#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 5 60 ./build/fetch_check | grep -c "bad 0" && timeout -k 5 60 ./build/sort32_check | tail -1 && bash scripts/gpu_tab4.sh
