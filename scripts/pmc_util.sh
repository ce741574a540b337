#!/bin/bash
# scripts/pmc_util.sh <tag> -- VALU / MFMA / LDS utilisation counters of the
# default bench workload (config 3, fused pipeline, plus the coefficient K1's
# extra launches), one rocprofv3 --pmc pass per counter group (<= 8 SQ + 2 GRBM
# counters per pass, MI355X_MICROARCH.md "rocprofv3 PMC slots"), each pass its
# own time-limited run with the program directly after `--`.  Then
# scripts/util.py folds the passes into gpurun_out/util_<tag>/util.json.
set -u
tag=${1:-r02}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/util_$tag
mkdir -p "$out"
ARGS="--steps 2 --warmup 1 --verify 0 --no-cpu-baseline --coef-launches 2 ${BENCH_ARGS:-}"
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i + 1))
  echo "== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o run -- \
      python3 bench.py $ARGS > "$out/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$out/p$i.log"; exit 1; }
done <<'G'
GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES
G
# the bench line (rocprofv3 writes its own lines after it): the workload
# the counters belong to, so bench.py attaches them only to a matching run
python3 -c "
import json; d=json.loads([l for l in open('$out/p1.log').read().splitlines() if l.startswith('{')][-1])
json.dump(d['config'], open('$out/config.json','w'))" || { echo "no bench line in pass 1"; exit 1; }
python3 scripts/util.py "$out" "$out/util.json"
