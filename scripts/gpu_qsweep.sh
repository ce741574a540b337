#!/bin/bash
# scripts/gpu_qsweep.sh -- config 5's quality sweep (Q = 50/75/90) on config-3
# frames and config 2's single 1920x1280 frame, each oracle-verified; lines
# under gpurun_out/qsweep/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/qsweep
for q in 50 75 90; do
  timeout -k 10 300 python3 bench.py --quality $q --no-cpu-baseline > gpurun_out/qsweep/q$q.log 2>&1 || { tail -5 gpurun_out/qsweep/q$q.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/qsweep/q$q.log').read().strip().splitlines()[-1]);print('Q$q', d['value'], d['ms_per_step'], d['stages_ms'], d['verified_frames'])"
done
timeout -k 10 300 python3 bench.py --frames 1 --width 1920 --height 1280 --distinct 1 --steps 50 --warmup 5 --no-cpu-baseline --coef-launches 0 > gpurun_out/qsweep/single_1920x1280.log 2>&1 || { tail -5 gpurun_out/qsweep/single_1920x1280.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/qsweep/single_1920x1280.log').read().strip().splitlines()[-1]);print('1920x1280 x1', d['value'], d['ms_per_step'], d['stages_ms'], d['verified_frames'])"
