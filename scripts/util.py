#!/usr/bin/env python3
"""scripts/util.py <dir> <out.json> -- per-kernel utilisation from the
rocprofv3 PMC passes of scripts/pmc_util.sh.

Per launch (counters averaged over a kernel's launches):
  cycles      = GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs)
  mfma_util   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles): fraction of
                the chip's matrix-pipe cycles busy (the dense i8 peak runs the
                pipe every cycle; MI355X_MICROARCH.md counts BUSY_CYCLES in
                cycles, e.g. 16 per v_mfma_i32_16x16x64_i8)
  valu_util   = (SQ_INSTS_VALU - SQ_INSTS_MFMA) x 2 / (1024 x cycles): fraction
                of the VALU issue slots used (a wave64 VALU instruction issues
                over 2 cycles of a SIMD-32, so 1 per 2 cycles per SIMD is peak)
  valu_busy   = SQ_ACTIVE_INST_VALU x 4 / (1024 x cycles) (quad-cycle counter)
  lds_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  wave_active/wait/waitinst = SQ_ACTIVE_INST_ANY, SQ_WAIT_ANY,
                SQ_WAIT_INST_ANY over SQ_WAVE_CYCLES
"""
import collections
import csv
import glob
import json
import os
import sys

SIMDS = 1024

d, out = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
ns = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        per[(k, r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        per[(k, r["Dispatch_Id"])]["_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    for (k, _), v in per.items():
        for c, x in v.items():
            if c == "_ns":
                ns[k].append(x)
            else:
                acc[k][c].append(x)

res = {}
for k, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
    if cyc <= 0:
        continue
    e = {"launch_us": round(sum(ns[k]) / len(ns[k]) / 1e3, 2), "cycles": round(cyc),
         "clock_GHz": round(cyc / (sum(ns[k]) / len(ns[k])), 3)}
    for c in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_LDS",
              "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
        if c in m:
            e[c] = round(m[c])
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        e["mfma_util"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc), 4)
    if "SQ_INSTS_VALU" in m:
        e["valu_util"] = round((m["SQ_INSTS_VALU"] - m.get("SQ_INSTS_MFMA", 0)) * 2 / (SIMDS * cyc), 4)
    if "SQ_ACTIVE_INST_VALU" in m:
        e["valu_busy"] = round(m["SQ_ACTIVE_INST_VALU"] * 4 / (SIMDS * cyc), 4)
    if m.get("SQ_LDS_IDX_ACTIVE"):
        e["lds_conflict_frac"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"], 4)
    if m.get("SQ_WAVE_CYCLES"):
        wc = m["SQ_WAVE_CYCLES"]
        for c, name in (("SQ_ACTIVE_INST_ANY", "wave_active"), ("SQ_WAIT_ANY", "wave_wait"),
                        ("SQ_WAIT_INST_ANY", "wave_waitinst")):
            if c in m:
                e[name] = round(m[c] / wc, 4)
    res[k] = e

# the profiled bench run's workload (scripts/pmc_util.sh writes it from the
# first pass's bench line): bench.py attaches these numbers only to a run of
# the same workload
meta = {}
mf = os.path.join(d, "config.json")
if os.path.exists(mf):
    meta = json.load(open(mf))
json.dump({"config": meta, "method": __doc__.strip(), "kernels": res}, open(out, "w"), indent=1)
for k, e in sorted(res.items(), key=lambda kv: -kv[1]["launch_us"])[:10]:
    print(f"{k[:44]:44s} {e['launch_us']:9.1f} us  mfma {e.get('mfma_util', float('nan')):.3f}  "
          f"valu {e.get('valu_util', float('nan')):.3f}  busy {e.get('valu_busy', float('nan')):.3f}  "
          f"ldsconf {e.get('lds_conflict_frac', float('nan')):.3f}")
