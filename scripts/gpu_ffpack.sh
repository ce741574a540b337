#!/bin/bash
# 0xFF counting in k_pack_lb / k_seam_fix (ff_pack): GPU suite, then A/B
# against k_emit_count (MIJ_FF_PACK=0) on config 3 at Q=50 and Q=90
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/t_ffpack.log 2>&1 || { grep -E "^E |FAILED|Timeout|Error" gpurun_out/t_ffpack.log | head -20; tail -5 gpurun_out/t_ffpack.log; exit 1; }
echo "suite: $(tail -1 gpurun_out/t_ffpack.log)"
run() {  # q ffpack
  MIJ_FF_PACK=$2 timeout -k 10 150 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --coef-launches 0 --quality $1 > gpurun_out/ff.log 2>&1 || { tail -3 gpurun_out/ff.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ff.log').read().strip().splitlines()[-1]);s=d['stages_ms'];print('Q', sys.argv[1], 'ff_pack', sys.argv[2], d['ms_per_step'], 'pack', s['pack'], 'emit', s['emit'], d['verified_frames'])" $1 $2
}
for q in 50 90; do run $q 0; run $q 1; run $q 0; run $q 1; done
