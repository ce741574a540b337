#!/bin/bash
# scripts/pmc_ab.sh -- the utilisation PMC passes of scripts/pmc_util.sh for
# each library in $LIBS (MIJ_LIB), folded per library by scripts/util.py into
# gpurun_out/pmcab_<name>/util.json; prints the kernels matching $KPAT.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --verify 0 --no-cpu-baseline --coef-launches 0 ${BENCH_ARGS:-}"
for lib in $LIBS; do
  name=$(basename $lib .so); out=gpurun_out/pmcab_$name; mkdir -p $out
  i=0
  while read -r grp; do
    [ -z "$grp" ] && continue
    i=$((i + 1))
    MIJ_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o run -- \
        python3 bench.py $ARGS > "$out/p$i.log" 2>&1 || { echo "$name pass $i failed"; tail -5 "$out/p$i.log"; exit 1; }
  done <<'G'
GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES
G
  python3 scripts/util.py $out $out/util.json > /dev/null
  python3 - $out/util.json "${KPAT:-pack|mcu_dct<2>}" $name <<'P'
import json, re, sys
d = json.load(open(sys.argv[1]))["kernels"]
for k, e in d.items():
    if re.search(sys.argv[2], k):
        print(sys.argv[3], k[:40], {x: e.get(x) for x in ("launch_us", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "valu_busy", "lds_conflict_frac", "wave_wait", "wave_waitinst", "wave_active")})
P
done
