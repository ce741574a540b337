"""CPU test: machine check of K1's fast-path quantisation rules (DESIGN.md §5.2,
verdict r01 item 7, integer-domain luma rule since round 5).

tests/tau_check.c restates bit for bit what k_mcu_dct does per AC coefficient
-- the exact three-digit integer DCT N' of fill_tables' int8 matrix, whose
rows carry the luma prescale 2^s_g / q_z of the batch's quality; then the
luma integer rule (hi = |N'| + E + 1, lo = max(|N'| - E, 0), a hazard when
they differ above bit k = 21 + s_g, else a shift) and the chroma fp32 rule
(t -+ tau with tau = fac (0.72 L1 + 80) + 1e-6 on the luma-scaled N') -- and
asserts that every value the kernel keeps equals the reference's (int)(F /
q) (encoder.c:81-109, F from the oracle's FP64 restatement), for every
quality 1..100 (original.c:504-509) and both tables.  Blocks: random, flat,
checkerboards, ramps, near-flat noise, 0/255 extremes, DCT basis patterns
and blocks synthesised onto quantisation boundaries.

Default size 2 x 10^5 blocks x 100 qualities x 126 decisions (~2.5e9);
MIJ_TAU_BLOCKS raises it.  tests/golden/tau_check_int_1e7.json records a 10^7
block run of the same program."""
import json
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


@pytest.fixture(scope="module")
def tau_check(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("tau") / "tau_check")
    lib = os.path.join(REPO, "oracle")
    if not os.path.exists(os.path.join(lib, "libcref.so")):
        subprocess.check_call(["make", "-s", "-C", lib, "libcref.so"])
    # -mfma: fmaf compiles to the fused instruction (the same IEEE operation
    # as v_fma_f32); no contraction of anything else
    subprocess.check_call(["gcc", "-O3", "-mfma", "-ffp-contract=off", "-o", exe,
                           os.path.join(HERE, "tau_check.c"), "-L" + lib, "-lcref", "-lm", "-lpthread",
                           "-Wl,-rpath," + lib])
    return exe


def run(exe, blocks, seed):
    threads = min(16, os.cpu_count() or 1)
    r = subprocess.run([exe, str(blocks), str(seed), str(threads)], capture_output=True, text=True)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    return r.returncode, out


def test_tau_rule_never_keeps_a_wrong_value(tau_check):
    n = int(os.environ.get("MIJ_TAU_BLOCKS", "200000"))
    rc, out = run(tau_check, n, 11)
    assert out["misses"] == 0 and rc == 0, out
    assert out["blocks"] == n and out["qualities"] == 100
    # the integer DCT's error stays inside the bound the luma rule assumes
    # (|N' - 2^k F / q| <= L1/2, the rule's E = floor(L1 / 2) + 1)
    assert out["worst_err_over_bound"] <= 1.0, out
    # the rule is not vacuous: it keeps nearly everything and flags a few
    assert out["kept"] > 0.999 * out["checks"] and out["hazards"] > 0


def test_recorded_1e7_run():
    with open(os.path.join(HERE, "golden", "tau_check_int_1e7.json")) as f:
        rec = json.load(f)
    assert rec["blocks"] >= 10_000_000 and rec["misses"] == 0
    assert rec["qualities"] == 100 and rec["worst_err_over_bound"] <= 1.0
