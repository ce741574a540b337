#!/usr/bin/env python3
"""scripts/phase_stats.py [kernel-substring] [--lines a-b:name,...] -- static
per-phase VALU budget of a K1 instantiation.

Compiles mij_kernels.hip to gfx950 assembly with line tables (-g changes no
code generation, only adds .loc directives), attributes every instruction of
the kernel to the source line it came from (after inlining: the callee's
line), maps lines to K1's phases and prices each VALU instruction with the
issue costs measured on the box (wave-cycles per wave64 instruction at 3
waves per SIMD, profiles/r03/probe/valu_rate3.txt, valu_rate4.txt,
profiles/r04/probe/valu_rate5.txt):

  fast class ~2.4: fp32 add/sub/mul/fma/fmac/fmamk, add/sub_u32 (clamp too),
                   and/or/xor, bitop3, lshrrev/ashrrev, mov_b32 with VGPR,
                   inline-constant or literal sources (an SGPR source, an
                   SDWA or a DPP form makes them slow,
                   profiles/r05/probe/valu_rate6.txt)
  slow class ~4.3: every other VALU (conversions, left shifts, min/max,
                   compares, cndmask, perm, packed ops, bfe, ffbh, bcnt, ...)
  permlane*_swap 8.3, transcendentals 8, an MFMA 16x16 blocks VALU issue 8.

The K1 tile loop is straight-line apart from its rare paths and the AC-token
loop, so the hot-phase totals are close to the per-tile dynamic counts; rare
phases are listed separately and the AC loop per iteration."""
import os, re, subprocess, sys
from collections import defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(HERE, "..", "jpeg-encoder-decoder_amd")
SRC = "csrc/mij_kernels.hip"

FAST = {"v_add_f32", "v_sub_f32", "v_subrev_f32", "v_mul_f32", "v_fma_f32", "v_fmac_f32", "v_fmamk_f32",
        "v_fmaak_f32", "v_add_u32", "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32", "v_xor_b32",
        "v_bitop3_b32", "v_lshrrev_b32", "v_ashrrev_i32", "v_mov_b32", "v_not_b32", "v_readfirstlane_b32",
        "v_add_co_u32", "v_sub_co_u32"}
TRANS = {"v_exp_f32", "v_log_f32", "v_rcp_f32", "v_rsq_f32", "v_sqrt_f32", "v_sin_f32", "v_cos_f32",
         "v_rcp_f64", "v_rcp_iflag_f32"}


def cost(op, args):
    base = re.sub(r"_e(32|64)$", "", op)
    if base.startswith("v_mfma"):
        return 8.0
    if "permlane" in base:
        return 8.3
    if base in TRANS:
        return 8.0
    if base in FAST and "sdwa" not in op and "dpp" not in args and "row_" not in args and "quad_perm" not in args \
            and "op_sel" not in args and "sel:" not in args and not sgpr_src(args):
        return 2.4
    return 4.3


def sgpr_src(args):
    """an SGPR source operand (v_xor_b32 v, s, v issues at 4.4 wave-cycles
    where the all-VGPR or literal form issues at 2.4:
    profiles/r05/probe/valu_rate6.txt)"""
    ops = [o.strip() for o in args.split(",")]
    return any(re.match(r"^-?\|?s(\d+|\[)", o) for o in ops[1:])


def compile_asm(extra):
    out = "/tmp/mij_kernels_g.s"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                           "-I../include", "-Icsrc", "--cuda-device-only", "-S", "-g", SRC, "-o", out] + extra,
                          cwd=PKG, stderr=subprocess.DEVNULL)
    return open(out).read()


# K1 phases by source line of mij_kernels.hip (see the kernel's comments)
def default_phases(src_lines):
    """Locate the phase boundaries by anchors in the source, so the table
    survives edits."""
    def find(pat, start=0):
        for i in range(start, len(src_lines)):
            if re.search(pat, src_lines[i]):
                return i + 1
        raise SystemExit(f"anchor not found: {pat}")
    ph = []
    add = lambda a, b, n: ph.append((a, b, n))
    add(find(r"^__device__ __forceinline__ TilePos tile_pos\("), find(r"^typedef __attribute__\(\(address_space\(3\)\)\)"), "tile position")
    add(find(r"^struct DmaOff"), find(r"^__device__ __forceinline__ void dma_wait_behind_stores"), "DMA issue/wait")
    add(find(r"^template <int N>\s*$", find(r"byte N of w as float")), find(r"^typedef float f2v"), "colour")
    add(find(r"^__device__ __forceinline__ uint32_t pack_i16x2"), find(r"^__device__ __forceinline__ uint32_t pack_i16x2") + 3, "pack int16")
    add(find(r"^constexpr float CH_BIAS"), find(r"^// Rare path: the Y corrections"), "colour")
    add(find(r"^// Rare path: the Y corrections"), find(r"^__device__ __forceinline__ uint32_t pack_y"), "colour rare (exceptions)")
    add(find(r"^__device__ __forceinline__ uint32_t pack_y"), find(r"if \(!use_lut\) continue;"), "colour")
    add(find(r"if \(!use_lut\) continue;") + 1, find(r"^// Token of the per-segment streams"), "colour rare (exceptions)")
    e0 = find(r"^__device__ __forceinline__ void emit_tokens")
    ac = find(r"if \(!acz && valid && !\(kflags & K1F_NO_ACLOOP\)\)", e0)
    add(e0, ac, "tokens: masks, scan, DC/EOB, hist")
    add(ac, find(r"^// K1 modes"), "tokens: AC loop (per iteration x lanes' max)")
    k = find(r"^__global__ __launch_bounds__\(64 \* k1_waves")
    add(k, find(r"const bool do_dct = !\(kflags & K1F_NO_DCT\);", k), "kernel setup / tile loop")
    d0 = find(r"auto dct_digit = \[&\]", k)
    add(d0, find(r"auto dct_ntile = \[&\]", k), "DCT: MFMA chain + digit shifts")
    add(find(r"auto dct_ntile = \[&\]", k), find(r"// coefficient input: this tile's planes were loaded", k), "DCT: B operand + L1 bound")
    f0 = find(r"auto block_at = \[&\]", k)
    add(find(r"// coefficient input: this tile's planes were loaded", k), f0, "kernel setup / tile loop")
    add(f0, find(r"if \(\(MODE & K1M_COEF_OUT\) && !\(kflags & K1F_NO_STORE\)\)", k), "finish: block/segment index")
    add(find(r"if \(\(MODE & K1M_COEF_OUT\) && !\(kflags & K1F_NO_STORE\)\)", k), find(r"if \(PIX && valid && g == 0\) a.dc", k), "coef store")
    add(find(r"if \(PIX && valid && g == 0\) a.dc", k), find(r"if \(PIX && do_dct\) \{", k), "finish: raw DC + emit call")
    q0 = find(r"if \(PIX && do_dct\) \{", k)
    add(q0, find(r"if constexpr \(!AUDIT\) \{", q0), "N-tile loop")
    add(find(r"if constexpr \(!AUDIT\) \{", q0), find(r"// trunc\(t - tau\) is the output", q0), "chroma all-AC-zero test")
    add(find(r"// trunc\(t - tau\) is the output", q0), find(r"auto straddle_mask = \[&\]", q0), "quantise + straddle sums")
    add(find(r"auto straddle_mask = \[&\]", q0), find(r"if constexpr \(AUDIT\) \{", q0), "replay (rare)")
    add(find(r"if constexpr \(AUDIT\) \{", q0), find(r"\{  // z = 0: exact from the pixel sum", q0), "audit")
    add(find(r"\{  // z = 0: exact from the pixel sum", q0), find(r"if constexpr \(DEFER\) \{", q0), "DC")
    add(find(r"if constexpr \(DEFER\) \{", q0), find(r"if \(!DEFER && __ballot\(hz != 0\)", q0), "replay listing (DEFER)")
    add(find(r"if \(!DEFER && __ballot\(hz != 0\)", q0), find(r"// token variants: the next tile's DMA has landed", q0), "replay (rare)")
    add(find(r"// token variants: the next tile's DMA has landed", q0), find(r"// k_fix_blocks: the blocks K1 listed", q0), "kernel setup / tile loop")
    add(find(r"^__device__ __forceinline__ int dc_exact"), find(r"^// DC at a tie"), "DC")
    add(find(r"^// DC at a tie"), find(r"^// ==========", find(r"^// DC at a tie")), "replay (rare)")
    add(find(r"^__device__ __forceinline__ int mag_class"), find(r"^// Colour-exception bitmaps"), "tokens: masks, scan, DC/EOB, hist")
    add(find(r"^template <int N>\s*$"), find(r"^// inclusive prefix sum over the wave") + 6, "tokens: masks, scan, DC/EOB, hist")
    return ph


def main():
    pat = sys.argv[1] if len(sys.argv) > 1 else "k_mcu_dctILi1E"
    extra = [a for a in sys.argv[2:] if a.startswith("-D")]
    asm = compile_asm(extra)
    src = open(os.path.join(PKG, SRC)).read().splitlines()
    phases = default_phases(src)

    def phase_of(fileno, line):
        if fileno != 0:
            return "other (headers)"
        best = None
        for a, b, n in phases:
            if a <= line < b and (best is None or b - a < best[1] - best[0]):
                best = (a, b, n)
        return best[2] if best else f"other (line {line})"

    for m in re.finditer(r"^(_Z\S+):[^\n]*\n(.*?)^\.Lfunc_end", asm, re.S | re.M):
        name, body = m.group(1), m.group(2)
        if pat not in name:
            continue
        cur = (0, 0)
        cnt = defaultdict(lambda: [0, 0.0, 0, 0])  # valu, cycles, mfma, lds
        ops = defaultdict(lambda: defaultdict(int))
        lines = defaultdict(lambda: defaultdict(int))
        for l in body.splitlines():
            s = l.strip()
            mm = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
            if mm:
                cur = (int(mm.group(1)), int(mm.group(2)))
                continue
            if not l.startswith("\t") or s.startswith((".", ";")) or not s:
                continue
            parts = s.split(None, 1)
            op, args = parts[0], (parts[1] if len(parts) > 1 else "")
            ph = phase_of(*cur)
            if op.startswith("v_"):
                c = cost(op, args)
                if op.startswith("v_mfma"):
                    cnt[ph][2] += 1
                else:
                    cnt[ph][0] += 1
                cnt[ph][1] += c
                ops[ph][re.sub(r"_e(32|64)$", "", op)] += 1
                if not op.startswith("v_mfma"):
                    lines[ph][cur[1]] += 1
            elif op.startswith("ds_"):
                cnt[ph][3] += 1
        print(name)
        print(f"{'phase':48s} {'VALU':>6s} {'cycles':>8s} {'MFMA':>5s} {'LDS':>5s}")
        tot = [0, 0.0, 0, 0]
        for ph, v in sorted(cnt.items(), key=lambda kv: -kv[1][1]):
            print(f"{ph:48s} {v[0]:6d} {v[1]:8.0f} {v[2]:5d} {v[3]:5d}")
            for i in range(4):
                tot[i] += v[i]
        print(f"{'total (static)':48s} {tot[0]:6d} {tot[1]:8.0f} {tot[2]:5d} {tot[3]:5d}")
        for a in sys.argv:
            if a.startswith("--phase="):
                want = a.split("=", 1)[1]
                for ph in ops:
                    if want in ph:
                        print(f"  {ph}: " + ", ".join(f"{o[2:]}x{n}" for o, n in
                                                     sorted(ops[ph].items(), key=lambda kv: -kv[1])))
                        print("    lines: " + ", ".join(f"{l}:{n}" for l, n in sorted(lines[ph].items())))
        if "-v" in sys.argv:
            for ph in sorted(ops):
                top = sorted(ops[ph].items(), key=lambda kv: -kv[1])[:14]
                print(f"  {ph}: " + ", ".join(f"{o[2:]}×{n}" for o, n in top))


if __name__ == "__main__":
    main()
