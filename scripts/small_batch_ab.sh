#!/bin/bash
# scripts/small_batch_ab.sh -- small batches of 1920x1280 frames (config 2's
# shape): with ENVS, the in-tree library under each environment setting in
# turn (e.g. ENVS="MIJ_X=0 MIJ_X=1"); with LIBS, the library builds
# alternating (MIJ_LIB); otherwise the in-tree library with and without
# option $OPT (default segdc_fused=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OPT=${OPT:-segdc_fused=1}
run() {  # <label> <env-or-empty> <extra args>
  env $2 timeout -k 10 120 python3 bench.py --frames $n --width 1920 --height 1280 --steps 200 --warmup 20 --no-cpu-baseline --coef-launches 0 --verify 0 $3 > gpurun_out/sb.log 2>&1 || { echo "failed: n=$n $1"; tail -5 gpurun_out/sb.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/sb.log').read().strip().splitlines()[-1]);s=d['stages_ms'];print('n', sys.argv[1], sys.argv[2], round(d['ms_per_step'],4), {k: s[k] for k in s})" $n "$1"
}
for n in ${NS:-1 4 16}; do
  for r in $(seq ${ROUNDS:-2}); do
    if [ -n "${ENVS:-}" ]; then
      for e in $ENVS; do run "$e" "$e" "" || exit 1; done
    elif [ -n "${LIBS:-}" ]; then
      for lib in $LIBS; do run "$lib" "MIJ_LIB=$PWD/$lib" "" || exit 1; done
    else
      run "default" "" "" || exit 1
      run "$OPT" "" "--opt $OPT" || exit 1
    fi
  done
done
