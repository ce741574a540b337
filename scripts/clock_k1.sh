#!/bin/bash
# scripts/clock_k1.sh -- effective shader clock during K1: GRBM_GUI_ACTIVE
# cycles per launch divided by the launch's duration (one PMC pass with the
# kernel trace).  Output: gpurun_out/clock_k1/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/clock_k1${TAG:-}; mkdir -p $out
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace --kernel-include-regex "${KRE:-mcu_dct<1>}" --output-format csv -d $out -o run -- \
  python3 bench.py --mode dct --steps 3 --warmup 1 --no-cpu-baseline --verify 0 > $out/run.log 2>&1 || { tail -3 $out/run.log; exit 1; }
python3 - $out <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
pc = collections.defaultdict(dict)
for r in csv.DictReader(open(glob.glob(d + "/**/run_counter_collection.csv", recursive=True)[0])):
    pc[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    pc[r["Dispatch_Id"]]["ns"] = float(r.get("End_Timestamp", 0) or 0) - float(r.get("Start_Timestamp", 0) or 0)
for k, v in sorted(pc.items()):
    ns = v.get("ns", 0)
    print(k, {c: f"{x:.4g}" for c, x in v.items()}, f"GUI_ACTIVE/ns = {v.get('GRBM_GUI_ACTIVE', 0) / ns:.3f} GHz" if ns else "")
PY
