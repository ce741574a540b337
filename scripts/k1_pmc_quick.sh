#!/bin/bash
# scripts/k1_pmc_quick.sh -- one PMC pass over K1 (dct mode): VALU/SALU
# instruction counts, VALU busy, wave cycles, effective clock; per-tile figures.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/k1pmc${TAG:-}; rm -rf $out; mkdir -p $out
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS --kernel-include-regex "${KRE:-mcu_dct<1>}" --output-format csv -d $out -o run -- \
  python3 bench.py --mode ${MODE:-dct} --steps 2 --warmup 1 --no-cpu-baseline --verify 0 > $out/log 2>&1 || { tail -3 $out/log; exit 1; }
python3 - $out <<'PY'
import csv, glob, sys, collections
pc = collections.defaultdict(dict)
for r in csv.DictReader(open(glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)[0])):
    pc[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    pc[r["Dispatch_Id"]]["ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
tiles = 256 * 4050
for k, v in sorted(pc.items(), key=lambda kv: int(kv[0]))[-1:]:
    clk = v["GRBM_GUI_ACTIVE"] / 8 / v["ns"]
    print(f"dispatch {k}: {v['ns']/1e6:.3f} ms, clock {clk:.2f} GHz, per tile: VALU {v['SQ_INSTS_VALU']/tiles:.0f} SALU {v['SQ_INSTS_SALU']/tiles:.0f} LDS {v['SQ_INSTS_LDS']/tiles:.0f}; "
          f"VALU busy {v['SQ_ACTIVE_INST_VALU']*4/1024/(v['GRBM_GUI_ACTIVE']/8):.2f} of kernel cycles; wave: active {1-(v['SQ_WAIT_INST_ANY']+v['SQ_WAIT_ANY'])/v['SQ_WAVE_CYCLES']:.2f} waitinst {v['SQ_WAIT_INST_ANY']/v['SQ_WAVE_CYCLES']:.2f} wait {v['SQ_WAIT_ANY']/v['SQ_WAVE_CYCLES']:.2f}")
PY
