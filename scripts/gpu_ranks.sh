#!/bin/bash
# scripts/gpu_ranks.sh -- bench.py's own rank launcher on one GPU: two ranks
# over gloo sharing GPU 0 (config 3 at 16 frames, every slot verified; config
# 4 in two bands, every frame verified).  The 8-GPU curve is the driver's run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
MIJ_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --frames 16 --steps 5 --warmup 2 --no-cpu-baseline --coef-launches 0 > gpurun_out/ranks2.log 2>&1 || { tail -5 gpurun_out/ranks2.log; exit 1; }
grep '^{' gpurun_out/ranks2.log | tail -1
MIJ_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --workload config4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ranks2_c4.log 2>&1 || { tail -5 gpurun_out/ranks2_c4.log; exit 1; }
grep '^{' gpurun_out/ranks2_c4.log | tail -1
