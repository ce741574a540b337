#!/bin/bash
# scripts/ab.sh -- A/B timing of library builds in one GPU session.
# Usage: LIBS="ab/A.so ab/B.so" [ARGS="--mode dct"] [ROUNDS=3] bash scripts/ab.sh
# Prints per run: ms/step, the token K1, the coefficient K1 (3 launches after
# the timed region), pack, emit, tables.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
# (ENVS="A=0 A=1" instead of LIBS: the in-tree library under each setting)
for r in $(seq ${ROUNDS:-3}); do
  for lib in ${ENVS:-$LIBS}; do
    if [ -n "${ENVS:-}" ]; then setting=$lib; else setting=MIJ_LIB=$PWD/$lib; fi
    env $setting timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --verify ${VERIFY:-0} ${ARGS:-} > gpurun_out/ab.log 2>&1 || { echo "$lib failed"; tail -5 gpurun_out/ab.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]);s=d['stages_ms'];r=d.get('roofline_k1_coefficient_variant',{});c=r.get('ms_per_launch');print(sys.argv[1], round(d['ms_per_step'],3), 'k1', s['k1_colour_dct_quant'], 'k1coef', c, 'floor', r.get('pattern_floor_ms'), 'pack', s.get('pack'), 'emit', s.get('emit'), 'stats', s.get('stats'), 'tables', s.get('tables'), 'verified', d.get('verified_frames'))" $lib
  done
done
