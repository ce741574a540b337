#!/bin/bash
# emit workgroups dealt over a frame's three scans: GPU suite, then chunk
# size x workgroups-per-frame sweep at Q=50 and Q=90 (bytes verified)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/t_all.log 2>&1 || { grep -E "^E |FAILED|Timeout|Error" gpurun_out/t_all.log | head -20; tail -5 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
for q in 50 90; do
for lib in ab/libmijpeg_bal4096.so ab/libmijpeg_bal8192.so; do
for sl in 0 24 96 384; do
  MIJ_EMIT_SLOTS=$sl MIJ_LIB=$PWD/$lib timeout -k 10 150 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --coef-launches 0 --quality $q > gpurun_out/lab.log 2>&1 || { tail -3 gpurun_out/lab.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/lab.log').read().strip().splitlines()[-1]);s=d['stages_ms'];print('Q', sys.argv[2], sys.argv[1], 'slots', sys.argv[3], d['ms_per_step'], 'emit', s['emit'], d['verified_frames'])" $lib $q $sl
done
done
done
