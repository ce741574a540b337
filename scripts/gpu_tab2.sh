#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tables.py tests/test_gpu_parity.py > gpurun_out/t_tables.log 2>&1 || { grep -E "Error|assert|FAILED|Timeout" gpurun_out/t_tables.log | head -20; tail -5 gpurun_out/t_tables.log; exit 1; }
tail -1 gpurun_out/t_tables.log
for lib in ab/libmijpeg_tabq1.so ab/libmijpeg_base.so ab/libmijpeg_tabq1.so ab/libmijpeg_base.so; do
  MIJ_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --frames 1 --width 1920 --height 1280 --steps 50 --warmup 5 --no-cpu-baseline --coef-launches 0 > gpurun_out/single.log 2>&1 || { tail -3 gpurun_out/single.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/single.log').read().strip().splitlines()[-1]);print(sys.argv[1], 'single 1920x1280 ms', d['ms_per_step'], d['stages_ms'])" $lib
done
bash scripts/gpu_tab.sh
