#!/bin/bash
# scripts/ab_coef.sh -- A/B of the coefficient K1 (k_mcu_dct<COEF_OUT>) across
# library builds: the bench's three extra coefficient launches, timed with
# HIP events.  Usage: LIBS="ab/A.so ab/B.so" [ROUNDS=2] bash scripts/ab_coef.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-2}); do
  for lib in $LIBS; do
    MIJ_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --verify 0 --coef-launches 5 ${ARGS:-} > gpurun_out/ab_coef.log 2>&1 || { echo "$lib failed"; tail -5 gpurun_out/ab_coef.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab_coef.log').read().strip().splitlines()[-1]);c=d['roofline_k1_coefficient_variant'];print(sys.argv[1], 'step', round(d['ms_per_step'],3), 'coefK1', c['ms_per_launch'], 'frac', c['frac'])" $lib
  done
done
