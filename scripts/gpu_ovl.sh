#!/bin/bash
# scripts/gpu_ovl.sh -- sub-batch overlap of the entropy stages with the next
# K1 (bench --overlap N) for the libraries in $LIBS, at each N in $NS
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in ${NS:-1 2 3}; do
  echo "overlap=$n"
  ARGS="--overlap $n ${ARGS:-}" ROUNDS=${ROUNDS:-2} bash scripts/ab.sh || exit 1
done
