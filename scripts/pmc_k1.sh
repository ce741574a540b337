#!/bin/bash
# scripts/pmc_k1.sh -- SQ/SQC counter passes on K1 (dct mode), one pass per group.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/pmc_k1${TAG:-}; mkdir -p $out
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  [ -n "${QUICK:-}" ] && [ $i -gt 1 ] && break
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "${KRE:-mcu}" --output-format csv -d $out/p$i -o run -- \
      python3 bench.py --mode ${MODE:-dct} --steps 2 --warmup 1 --no-cpu-baseline --verify 0 > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $out/p$i.log; exit 1; }
done <<'G'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU
SQ_IFETCH SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH
SQC_ICACHE_MISSES SQC_ICACHE_REQ SQC_ICACHE_HITS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS
G
OUT=$out python3 - <<'PY'
import csv, glob, collections, os
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.environ['OUT'] + '/p*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        acc[r['Kernel_Name'][:40]][r['Counter_Name']].append(float(r['Counter_Value']))
names = sorted({c for d in acc.values() for c in d})
ks = sorted(acc)
print(f"{'counter':28s}" + "".join(f"{k[:18]:>20s}" for k in ks))
for c in names:
    print(f"{c:28s}" + "".join(f"{(sum(acc[k][c])/len(acc[k][c]) if acc[k][c] else float('nan')):20.4g}" for k in ks))
PY
