#!/bin/bash
# scripts/k1_lds_pmc.sh -- one PMC pass over the token K1 (default encode):
# LDS instructions, bank-conflict cycles, LDS-issue stalls per tile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/k1lds${TAG:-}; rm -rf $out; mkdir -p $out
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-include-regex "${KRE:-mcu_dct<2>}" --output-format csv -d $out -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --verify 0 --coef-launches 0 > $out/log 2>&1 || { tail -3 $out/log; exit 1; }
python3 - $out <<'PY'
import csv, glob, sys, collections
pc = collections.defaultdict(dict)
for r in csv.DictReader(open(glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)[0])):
    pc[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    pc[r["Dispatch_Id"]]["ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
tiles = 256 * 4050
for k, v in sorted(pc.items(), key=lambda kv: int(kv[0]))[-1:]:
    cyc = v["GRBM_GUI_ACTIVE"] / 8
    print(f"dispatch {k}: {v['ns']/1e6:.3f} ms; per tile: VALU {v['SQ_INSTS_VALU']/tiles:.0f} LDS {v['SQ_INSTS_LDS']/tiles:.1f} "
          f"conflict cycles {v['SQ_LDS_BANK_CONFLICT']/tiles:.0f} LDS active cycles {v['SQ_LDS_IDX_ACTIVE']/tiles:.0f}; "
          f"per CU: conflict {v['SQ_LDS_BANK_CONFLICT']/256/cyc:.2f} active {v['SQ_LDS_IDX_ACTIVE']/256/cyc:.2f} of kernel cycles; "
          f"wave: waitinst_lds {v['SQ_WAIT_INST_LDS']/v['SQ_WAVE_CYCLES']:.2f} waitinst {v['SQ_WAIT_INST_ANY']/v['SQ_WAVE_CYCLES']:.2f} wait {v['SQ_WAIT_ANY']/v['SQ_WAVE_CYCLES']:.2f}")
PY
