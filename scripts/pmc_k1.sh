#!/bin/bash
# scripts/pmc_k1.sh -- SQ counters on K1 (separate passes; no tracing domains)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/pmc_k1; mkdir -p $out
rocprofv3 -L > $out/counters_list.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $out/p$i -o run -- \
     python3 bench.py --mode dct --steps 2 --warmup 1 --no-cpu-baseline --verify 0 > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $out/p$i.log; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob('gpurun_out/pmc_k1/p*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        if 'k_mcu_dct' in r['Kernel_Name']:
            acc[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(acc.items()):
    print(f"{k:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
