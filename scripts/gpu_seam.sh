#!/bin/bash
# seam mode (k_pack_lb whole-word stores + k_seam_fix, no zeroing in k_emit_write):
# GPU suite in both modes, then A/B on config 3 at Q=50 and Q=90
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in 1 0; do
MIJ_SEAM=$m timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/t_s$m.log 2>&1 || { grep -E "^E |FAILED|Timeout|Error" gpurun_out/t_s$m.log | head -20; tail -5 gpurun_out/t_s$m.log; exit 1; }
echo "seam $m: $(tail -1 gpurun_out/t_s$m.log)"
done
run() {  # q seam
  MIJ_SEAM=$2 timeout -k 10 150 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --coef-launches 0 --quality $1 > gpurun_out/sm.log 2>&1 || { tail -3 gpurun_out/sm.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/sm.log').read().strip().splitlines()[-1]);s=d['stages_ms'];print('Q', sys.argv[1], 'seam', sys.argv[2], d['ms_per_step'], 'pack', s['pack'], 'emit', s['emit'], d['verified_frames'])" $1 $2
}
for q in 50 90; do run $q 0; run $q 1; run $q 0; run $q 1; done
