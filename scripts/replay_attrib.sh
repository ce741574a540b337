#!/bin/bash
# scripts/replay_attrib.sh -- the token K1's FP64 replay pass split (diag
# build): all, none, the pass without its FP64 rounds, and the pass count.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for q in ${QS:-90 50}; do
  echo "== Q=$q"
  FLAGS="${FLAGS:-0 2 32768 65536}" BENCH_EXTRA="--quality $q" bash scripts/k1_attrib.sh || exit 1
done
