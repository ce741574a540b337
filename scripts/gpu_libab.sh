#!/bin/bash
# library-variant A/B on config 3 (bytes verified): LIBS, QS (default "50 90"), ROUNDS
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-2}); do
for q in ${QS:-50 90}; do
for lib in $LIBS; do
  MIJ_LIB=$PWD/$lib timeout -k 10 150 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --coef-launches 0 --quality $q > gpurun_out/lab.log 2>&1 || { tail -3 gpurun_out/lab.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/lab.log').read().strip().splitlines()[-1]);s=d['stages_ms'];print('Q', sys.argv[2], sys.argv[1], d['ms_per_step'], 'pack', s['pack'], 'emit', s['emit'], d['verified_frames'])" $lib $q
done
done
done
