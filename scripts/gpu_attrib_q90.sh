#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_EXTRA="--quality 90" FLAGS="0 2 4096 8192" bash scripts/k1_attrib.sh
