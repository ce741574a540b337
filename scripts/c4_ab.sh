#!/bin/bash
# scripts/c4_ab.sh -- A/B of config-4 settings in one GPU session.
# Usage: ENVS="MIJ_HOST_READ=default MIJ_HOST_READ=batch" [EMITS="root bands"] [ROUNDS=3] bash scripts/c4_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-3}); do
  for emit in ${EMITS:-root bands}; do
    for e in $ENVS; do
      env $e timeout -k 10 300 python3 bench.py --workload config4 --band-emit $emit --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/c4_ab.log 2>&1 || { echo "$e $emit failed"; tail -5 gpurun_out/c4_ab.log; exit 1; }
      python3 -c "import json,sys;d=json.loads(open('gpurun_out/c4_ab.log').read().strip().splitlines()[-1]);print(sys.argv[1], sys.argv[2], d['ms_per_step'], d.get('phases_ms'), 'verified', d.get('verified_frames'))" $e $emit
    done
  done
done
