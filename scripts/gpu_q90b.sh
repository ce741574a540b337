#!/bin/bash
# Q=90 / 75 config-3 steps with the pack window 4096 / 8192 words (A/B), after the parity suite
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_parity.py tests/test_api_state.py > gpurun_out/t_q.log 2>&1 || { grep -E "^E |FAILED|Timeout|rror" gpurun_out/t_q.log | head; tail -3 gpurun_out/t_q.log; exit 1; }
tail -1 gpurun_out/t_q.log
for q in 90 75; do
  for w in 0 1 0 1; do
    MIJ_PACK_WIDE=$w timeout -k 10 150 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --coef-launches 0 --quality $q > gpurun_out/q.log 2>&1 || { tail -3 gpurun_out/q.log; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/q.log').read().strip().splitlines()[-1]);s=d['stages_ms'];print('Q', sys.argv[2], 'wide', sys.argv[1], d['ms_per_step'], 'K1', s['k1_colour_dct_quant'], 'pack', s['pack'], 'emit', s['emit'], d['verified_frames'])" $w $q
  done
done
