"""GPU: K1's own keep/replay decisions against the machine-checked model
(verdict r02 "tie the tau proof to the kernel").

tests/tau_check.c restates K1's fast-path rule and proves on
the CPU (test_tau_bound.py) that every value it keeps equals the
reference's (int)(F / q) (/root/reference/main/encoder.c:104-109; the Q
scaling of /root/reference/utils/original.c:504-509).  This test closes the
loop on the device: tau_check's adversarial block generators make >= 10^5
luma blocks per quality, each becomes a luma block of a frame (every Y value
v is written as a B, G, R triple whose reference Y is exactly v), and the
coefficient K1's audit variant (mij_batch_audit) exports its per-coefficient
straddle decisions.  They must equal tau_check's decisions bit for bit, and
the encoded bytes must equal the oracle's."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import mijpeg
import oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
BW, BH = 256, 392          # blocks per row / rows: 2048 x 3136 px, 100,352 blocks


@pytest.fixture(scope="module")
def tau_check(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("tauk") / "tau_check")
    lib = os.path.join(REPO, "oracle")
    if not os.path.exists(os.path.join(lib, "libcref.so")):
        subprocess.check_call(["make", "-s", "-C", lib, "libcref.so"])
    subprocess.check_call(["gcc", "-O3", "-mfma", "-ffp-contract=off", "-o", exe,
                           os.path.join(HERE, "tau_check.c"), "-L" + lib, "-lcref", "-lm", "-lpthread",
                           "-Wl,-rpath," + lib])
    return exe


def bgr_for_y():
    """[256, 3] B, G, R triples whose reference luma (encoder.c:133, FP64,
    truncated; evaluated by the oracle's cref_pixel_ycc) is exactly v."""
    lib = O.cref()
    out = np.zeros(3, np.uint8)
    tab = np.zeros((256, 3), np.uint8)
    for v in range(256):
        for d in [(0, 0, 0)] + [(db, 0, dr) for db in range(-2, 3) for dr in range(-2, 3)]:
            b, g, r = v + d[0], v + d[1], v + d[2]
            if not (0 <= b <= 255 and 0 <= r <= 255):
                continue
            lib.cref_pixel_ycc(ctypes.c_uint8(b), ctypes.c_uint8(g), ctypes.c_uint8(r), out.ctypes.data)
            if out[0] == v:
                tab[v] = (b, g, r)
                break
        else:
            raise AssertionError(f"no B, G, R triple with Y = {v}")
    return tab


@pytest.mark.parametrize("q", [1, 10, 50, 75, 90, 100])
def test_kernel_decisions_equal_tau_check(tau_check, tmp_path, q):
    n = BW * BH
    out = str(tmp_path / f"blk_q{q}")
    subprocess.check_call([tau_check, "dump", str(n), str(1000 + q), str(q), out])
    px = np.fromfile(out + ".px", np.uint8).reshape(BH, BW, 8, 8)
    want = np.fromfile(out + ".mask", np.uint64)
    assert want.size == n
    Y = px.transpose(0, 2, 1, 3).reshape(BH * 8, BW * 8)       # blocks in raster order
    frame = np.ascontiguousarray(bgr_for_y()[Y])                # H x W x 3, B, G, R
    H, W = frame.shape[:2]
    b = mijpeg.Batch(W, H, 1, q)
    b.upload(frame)
    got = b.audit(1)[0][:n]                                     # the luma blocks come first
    diff = np.nonzero(got != want)[0]
    assert diff.size == 0, (f"Q={q}: {diff.size} blocks differ, first {int(diff[0])}: "
                            f"kernel {int(got[diff[0]]):#x} model {int(want[diff[0]]):#x}")
    hazards = int(sum(bin(int(m)).count("1") for m in want[want != 0]))
    assert hazards > 0, "the generators must reach the replay path"
    # and the bytes (the replays included) are the oracle's
    b.encode(1)
    assert b.output(0) == O.cref_encode(frame, q)
    b.close()
