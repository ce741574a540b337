#!/bin/bash
# scripts/gpu_coefstore.sh -- GPU parity suite, the coefficient-K1 store A/B
# (ab/libmijpeg_old.so vs ab/libmijpeg_new.so) and the split pipeline's
# WRITE_SIZE / FETCH_SIZE passes on the current library; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/coefstore; mkdir -p $out
NO_BENCH=1 bash scripts/gpu_check.sh || exit 1
LIBS="ab/libmijpeg_old.so ab/libmijpeg_new.so" ROUNDS=2 bash scripts/ab_coef.sh | tee $out/ab.txt || exit 1
for c in WRITE_SIZE FETCH_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $out/pmc_$c -o run -- \
    python3 bench.py --split --steps 3 --warmup 1 --verify 0 --no-cpu-baseline > $out/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $out/pmc_$c.log; exit 1; }
done
echo done
