"""CPU test: exhaustive machine check of K1's fp32 colour rules (DESIGN.md
§5.1) over all 2^24 colours -- tests/colour_check.c restates convert4
(csrc/mij_kernels.hip) bit for bit and compares with the exact values of the
reference's colour conversion (/root/reference/main/encoder.c:133-135):
floor(Y) and the integer-Y flag from the magic form fl(Y + 12288) (round 5),
floor(Cb) / floor(Cr) from the biased magic forms."""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_colour_rules_exhaustive(tmp_path):
    exe = str(tmp_path / "colour_check")
    # -mfma: fmaf is the fused instruction (the same IEEE operation as
    # v_fma_f32 / each half of v_pk_fma_f32); nothing else contracted
    subprocess.check_call(["gcc", "-O3", "-mfma", "-ffp-contract=off", "-o", exe,
                           os.path.join(HERE, "colour_check.c"), "-lm"])
    r = subprocess.run([exe], capture_output=True, text=True)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0, out
    assert out["colours"] == 1 << 24
    assert out["bad_y"] == out["bad_y_flag"] == out["bad_cb"] == out["bad_cr"] == 0, out
    # integer points: S = 299R + 587G + 114B = 0 (mod 1000) for Y; for Cb
    # R == G with B - G even (and Cr likewise): 256 x 128 colours
    assert out["y_integer_points"] > 0
    assert out["cb_integer_points"] == out["cr_integer_points"] == 256 * 128
