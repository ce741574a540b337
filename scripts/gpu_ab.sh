#!/bin/bash
# A/B of library builds (ab/*.so) on one box: full step and the coefficient K1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-2}); do
  for lib in $LIBS; do
    MIJ_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --verify ${VERIFY:-0} --coef-launches 5 ${ARGS:-} > gpurun_out/ab.log 2>&1 || { echo "$lib failed"; tail -5 gpurun_out/ab.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]);s=d['stages_ms'];c=d.get('roofline_k1_coefficient_variant',{});print(sys.argv[1], 'step', round(d['ms_per_step'],3), 'tokK1', s['k1_colour_dct_quant'], 'coefK1', c.get('ms_per_launch'), 'pack', s.get('pack'), 'emit', s.get('emit'), 'verified', d['verified_frames'])" $lib
  done
done
