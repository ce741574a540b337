#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_bands.py -k "device_resident or config4_shape" > gpurun_out/t_b.log 2>&1 || { grep -E "^E |FAILED|Timeout" gpurun_out/t_b.log | head; tail -3 gpurun_out/t_b.log; exit 1; }
tail -1 gpurun_out/t_b.log
for sl in 256 512 1024 256; do
  MIJ_EMIT_SLOTS=$sl timeout -k 10 200 python3 bench.py --workload config4 --steps 20 --warmup 3 --verify 2 > gpurun_out/c4.log 2>&1 || { tail -5 gpurun_out/c4.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/c4.log').read().strip().splitlines()[-1]);print('slots', sys.argv[1], d['ms_per_step'], d['verified_against_reference_sha'], d.get('phases_ms'))" $sl
done
