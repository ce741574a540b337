#!/bin/bash
# scripts/ab_env.sh "LIB:ENV=V ..." ... -- A/B timing of (library, environment)
# pairs in one GPU session (ab/libmijpeg_LIB.so, or LIB=cur for the in-tree build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-2}); do
for v in "$@"; do
  lib=${v%%:*}; ev=${v#*:}
  so=$PWD/ab/libmijpeg_$lib.so; [ "$lib" = cur ] && so=$PWD/jpeg-encoder-decoder_amd/libmijpeg.so
  [ "$lib" = diag ] && so=$PWD/jpeg-encoder-decoder_amd/libmijpeg_diag.so
  env $ev MIJ_LIB=$so timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --verify 0 ${ARGS:-} > gpurun_out/ab.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]);s=d['stages_ms'];print(sys.argv[1], round(d['ms_per_step'],3), {k: s[k] for k in s if k not in ('fix','tokenize','total')})" "$v"
done; done
