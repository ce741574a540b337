#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rc=0; [ -n "$SKIP_T" ] || { timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tables.py tests/test_gpu_parity.py > gpurun_out/t_tables.log 2>&1; rc=$?; }
[ -n "$SKIP_T" ] || tail -2 gpurun_out/t_tables.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t_tables.log | head -20; exit $rc; }
[ -n "$SKIP_T" ] || { LIBS="ab/libmijpeg_tabq0.so ab/libmijpeg_base.so" ROUNDS=2 bash scripts/gpu_ab.sh || exit 1; }
for lib in $SINGLE_LIBS; do
  MIJ_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --frames 1 --width 1920 --height 1280 --steps 50 --warmup 5 --no-cpu-baseline --coef-launches 0 > gpurun_out/single.log 2>&1 || { tail -3 gpurun_out/single.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/single.log').read().strip().splitlines()[-1]);print(sys.argv[1], 'single 1920x1280 ms', d['ms_per_step'], d['stages_ms'])" $lib
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bands.py tests/test_api_state.py > gpurun_out/t_bands.log 2>&1 || { tail -30 gpurun_out/t_bands.log; exit 1; }
tail -2 gpurun_out/t_bands.log
timeout -k 10 200 python3 bench.py --workload config4 --steps 20 --warmup 3 > gpurun_out/c4.log 2>&1 || { tail -20 gpurun_out/c4.log; exit 1; }
tail -1 gpurun_out/c4.log
if [ -n "$C4PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4prof -o c4 -- python3 bench.py --workload config4 --steps 10 --warmup 2 > gpurun_out/c4prof.log 2>&1 || { tail -20 gpurun_out/c4prof.log; exit 1; }
  f=$(find gpurun_out/c4prof -name "c4_kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-4 "$f" | head -20; python3 scripts/trace_gaps.py "${f%_kernel_stats.csv}_kernel_trace.csv" 30
fi
