#!/bin/bash
# scripts/gpu_dist.sh -- config-4 bench at N=1 and a 2-rank rehearsal on one GPU
# (gloo collectives, both ranks on GPU 0) of the config-3 and config-4 paths.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --workload config4 --steps 5 --warmup 2 > gpurun_out/c4_n1.log 2>&1 || { tail -5 gpurun_out/c4_n1.log; exit 1; }
tail -1 gpurun_out/c4_n1.log
MIJ_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --workload config4 --steps 3 --warmup 1 \
  > gpurun_out/c4_n2_gloo.log 2>&1 || { tail -20 gpurun_out/c4_n2_gloo.log; exit 1; }
grep metric gpurun_out/c4_n2_gloo.log
MIJ_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --steps 3 --warmup 1 --frames 64 \
  > gpurun_out/c3_n2_gloo.log 2>&1 || { tail -20 gpurun_out/c3_n2_gloo.log; exit 1; }
grep metric gpurun_out/c3_n2_gloo.log
# the nccl (RCCL) device branch of the config-4 exchange on one GPU: a
# one-rank process group
MIJ_DIST_FORCE=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29521 bench.py --workload config4 --steps 5 --warmup 2 \
  > gpurun_out/c4_n1_nccl.log 2>&1 || { tail -20 gpurun_out/c4_n1_nccl.log; exit 1; }
grep metric gpurun_out/c4_n1_nccl.log
