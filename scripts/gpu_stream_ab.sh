#!/bin/bash
# scripts/gpu_stream_ab.sh -- the stream tests on the in-tree library, then
# A/B rounds of the host-fed stream bench over the libraries in $LIBS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_stream.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/pytest_stream.log 2>&1 || { tail -20 gpurun_out/pytest_stream.log; exit 1; }
tail -1 gpurun_out/pytest_stream.log
for r in $(seq ${ROUNDS:-2}); do
  for lib in $LIBS; do
    MIJ_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --workload stream --steps 8 --warmup 2 --no-cpu-baseline ${ARGS:-} > gpurun_out/stream_ab.log 2>&1 || { echo "$lib failed"; tail -5 gpurun_out/stream_ab.log; exit 1; }
    python3 -c "import json,sys;d=json.loads([l for l in open('gpurun_out/stream_ab.log').read().splitlines() if l.startswith('{')][-1]);print(sys.argv[1], d['ms_per_step'], d['value'], d['stage_s_per_step'], d.get('verified_files'))" $lib
  done
done
