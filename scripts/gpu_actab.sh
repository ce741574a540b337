#!/bin/bash
# AC tables beside the segment DCs (k_segdc_actab + DC-only k_tables_1w):
# GPU suite, then A/B against k_seg_dc + k_tables_1w (MIJ_ACTAB=0): config 3
# at Q=50 and Q=90, and one 1920x1280 frame
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/t_actab.log 2>&1 || { grep -E "^E |FAILED|Timeout|Error" gpurun_out/t_actab.log | head -20; tail -5 gpurun_out/t_actab.log; exit 1; }
echo "suite: $(tail -1 gpurun_out/t_actab.log)"
run() {  # name actab args...
  local n=$1 v=$2; shift 2
  MIJ_ACTAB=$v timeout -k 10 150 python3 bench.py --no-cpu-baseline --coef-launches 0 "$@" > gpurun_out/at.log 2>&1 || { tail -3 gpurun_out/at.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/at.log').read().strip().splitlines()[-1]);s=d['stages_ms'];print(sys.argv[1], 'actab', sys.argv[2], d['ms_per_step'], 'stats', s['stats'], 'tables', s['tables'], 'pack', s['pack'], d['verified_frames'])" $n $v
}
for r in 1 2; do
  run q50 0 --steps 10 --warmup 3; run q50 1 --steps 10 --warmup 3
  run q90 0 --steps 10 --warmup 3 --quality 90; run q90 1 --steps 10 --warmup 3 --quality 90
  run single 0 --frames 1 --width 1920 --height 1280 --steps 200 --warmup 20; run single 1 --frames 1 --width 1920 --height 1280 --steps 200 --warmup 20
done
