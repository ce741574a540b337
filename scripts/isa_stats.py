#!/usr/bin/env python3
"""scripts/isa_stats.py [kernel-substring ...] -- static ISA statistics of the
gfx950 kernels in mij_kernels.hip: registers, LDS, and instruction counts by
class (VALU / MFMA / SALU / LDS / VMEM).  Compiles to assembly in /tmp."""
import os, re, subprocess, sys
HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(HERE, "..", "jpeg-encoder-decoder_amd")
out = "/tmp/mij_kernels.s"
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                       "-ffp-contract=off", "-I../include", "-Icsrc", "--cuda-device-only", "-S",
                       "csrc/mij_kernels.hip", "-o", out],
                      cwd=PKG, stderr=subprocess.DEVNULL)
asm = open(out).read()
pat = sys.argv[1] if len(sys.argv) > 1 else "k_mcu_dct"
for m in re.finditer(r"^(_Z\S+):[^\n]*\n(.*?)^\.Lfunc_end", asm, re.S | re.M):
    name, body = m.group(1), m.group(2)
    if pat not in name:
        continue
    ops = [l.split()[0] for l in body.splitlines() if l.startswith("\t") and not l.strip().startswith((".", ";"))]
    cnt = lambda f: sum(1 for o in ops if f(o))
    md = next((b for b in asm.split("\n  - ") if re.search(r"\.name:\s+" + re.escape(name) + r"\n", b)), "")
    g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", md) or [None, "?"])[1]
    print(f"{name}: vgpr={g('vgpr_count')} sgpr={g('sgpr_count')} spill={g('vgpr_spill_count')}/{g('sgpr_spill_count')} "
          f"lds={g('group_segment_fixed_size')} | valu={cnt(lambda o: o.startswith('v_') and not o.startswith('v_mfma'))} "
          f"mfma={cnt(lambda o: o.startswith('v_mfma'))} salu={cnt(lambda o: o.startswith('s_'))} "
          f"lds_ops={cnt(lambda o: o.startswith('ds_'))} vmem={cnt(lambda o: o.startswith(('global_', 'buffer_')))} "
          f"branches={cnt(lambda o: 'branch' in o)}")
