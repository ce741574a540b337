#!/bin/bash
# config 4: the device-resident band protocol on one GPU and
# over a one-rank nccl group (per-phase times), a 2-rank gloo rehearsal on
# one GPU against the reference shas, and the band tests (incl. the
# full-size two-process gloo encode)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/dist; mkdir -p $out
export TMPDIR=/tmp
[ -n "$SKIP_T" ] || { timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_bands.py > $out/t_bands.log 2>&1 || { grep -E "^E |FAILED|Timeout" $out/t_bands.log | head; tail -3 $out/t_bands.log; exit 1; }; }
[ -n "$SKIP_T" ] || tail -1 $out/t_bands.log
timeout -k 10 200 python3 bench.py --workload config4 --steps 20 --warmup 3 --verify 2 > $out/c4_n1.log 2>&1 || { tail -5 $out/c4_n1.log; exit 1; }
tail -1 $out/c4_n1.log > $out/c4_n1.json
MIJ_DIST_FORCE=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29641 timeout -k 10 200 python3 bench.py --workload config4 --steps 20 --warmup 3 --verify 2 > $out/c4_nccl1.log 2>&1 || { tail -5 $out/c4_nccl1.log; exit 1; }
tail -1 $out/c4_nccl1.log > $out/c4_nccl1.json
MIJ_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29651 bench.py --workload config4 --steps 5 --warmup 2 --verify 2 > $out/c4_gloo2.log 2>&1 || { tail -8 $out/c4_gloo2.log; exit 1; }
grep '^{' $out/c4_gloo2.log | tail -1 > $out/c4_gloo2.json
for f in c4_n1 c4_nccl1 c4_gloo2; do python3 -c "import json,sys;d=json.load(open('$out/'+sys.argv[1]+'.json'));print(sys.argv[1], d['ms_per_step'], d['value'], d['config']['backend'], d['verified_frames'], d['verified_against_reference_sha'], d.get('phases_ms'))" $f; done
