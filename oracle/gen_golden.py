#!/usr/bin/env python3
"""oracle/gen_golden.py -- TEST INFRASTRUCTURE ONLY.

Regenerates tests/golden/ from the reference itself, compiled here from its
own sources (oracle/_ref, see oracle/Makefile).  Run in the build container
(where /root/reference exists):  python oracle/gen_golden.py

Every expected output in the manifest comes from the REFERENCE build
(main/encoder.c for Q=50, utils/original.c + set_quality for the Q sweep);
the plain-C restatement (libcref.so) is checked against each one on the way,
so a fixture is written only if both agree byte for byte.

Outputs (data only, no reference source):
  sample_64x64.ppm, sample_640x640.ppm.gz, sample_640x640_diffs.ppm.gz
                    the reference's own image fixtures (images/*.ppm)
  manifest.json     per case: recipe, region, quality, jpg sha256 + length,
                    coefficient-plane sha256s (Q=50 cases)
  sample_64x64.{jpg,coefs.npz,tables.json}, sample_640x640.jpg
                    full expected outputs for the small cases
  cos_table.json    the 64 int64 cosine bit patterns of encoder.c:8-16
  colour_exceptions.npz
                    every RGB triple whose FP64 colour conversion truncates
                    one below the exact integer (restatement, exhaustive)
"""
from __future__ import annotations

import gzip
import hashlib
import json
import os
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "tests"))

import oracle as O  # noqa: E402
import ppm  # noqa: E402
import recipes  # noqa: E402

REF_IMAGES = "/root/reference/images"
GOLDEN = os.path.join(REPO, "tests", "golden")


def sha(b) -> str:
    if isinstance(b, np.ndarray):
        b = np.ascontiguousarray(b).tobytes()
    return hashlib.sha256(b).hexdigest()


def huff_dict(h) -> dict:
    return {f: list(getattr(h, f)) for f, _ in h._fields_}


def case_q50(name: str, bgr: np.ndarray, region=None, keep=False) -> dict:
    a = O.ref_stages(bgr, region)
    b = O.cref_stages(bgr, 50, region)
    assert a[4] == b[4], f"{name}: restatement != reference bytes"
    for x, y in zip(a[:3], b[:3]):
        assert (x == y).all(), f"{name}: coefficient mismatch"
    for x, y in zip(a[3], b[3]):
        assert bytes(x) == bytes(y), f"{name}: table struct mismatch"
    H, W = bgr.shape[:2]
    ent = {
        "quality": 50,
        "frame": [W, H],
        "region": list(region) if region else [0, 0, W, H],
        "jpg_sha256": sha(a[4]),
        "jpg_len": len(a[4]),
        "coef_sha256": [sha(a[0]), sha(a[1]), sha(a[2])],
        "source": "reference main/encoder.c (oracle/_ref)",
    }
    if keep:
        with open(os.path.join(GOLDEN, name + ".jpg"), "wb") as f:
            f.write(a[4])
    print(f"  {name}: {len(a[4])} B {ent['jpg_sha256'][:16]}")
    return ent


def main() -> None:
    O.build()
    assert O.ref_available(), "oracle/_ref not built (needs /root/reference)"
    os.makedirs(GOLDEN, exist_ok=True)

    # the reference's own image fixtures (data files)
    shutil.copyfile(os.path.join(REF_IMAGES, "sample_64x64.ppm"),
                    os.path.join(GOLDEN, "sample_64x64.ppm"))
    for n in ("sample_640x640", "sample_640x640_diffs"):
        with open(os.path.join(REF_IMAGES, n + ".ppm"), "rb") as f:
            data = f.read()
        with open(os.path.join(GOLDEN, n + ".ppm.gz"), "wb") as f:
            f.write(gzip.compress(data, 9, mtime=0))

    man: dict = {"cases": {}}
    C = man["cases"]
    print("reference images")
    for n in ("sample_64x64", "sample_640x640", "sample_640x640_diffs"):
        bgr = ppm.rgb_to_bgr(recipes.sample(n))
        C[n] = case_q50(n, bgr, keep=n != "sample_640x640_diffs")
        C[n]["input"] = n
    print("stand-in 1920x1280 (tile 640x640 3x2)")
    C["standin_1920x1280"] = case_q50("standin_1920x1280",
                                      ppm.rgb_to_bgr(recipes.standin_1920x1280_rgb()))
    C["standin_1920x1280"]["input"] = "standin_1920x1280"

    print("drop-in regions on a 320-stride frame (main.c:144 caller shape)")
    frame = ppm.rgb_to_bgr(np.tile(recipes.sample("sample_640x640"), (1, 1, 1))[:240, :320])
    for i, reg in enumerate([(0, 0, 320, 240), (16, 32, 128, 96), (3, 5, 64, 48),
                             (304, 224, 16, 16), (7, 0, 304, 240)]):
        k = f"region_{i}"
        C[k] = case_q50(k, frame, reg)
        C[k]["input"] = "sample_640x640[:240,:320]"

    print("adversarial suite")
    for n, fn in recipes.ADVERSARIAL.items():
        C[n] = case_q50(n, np.ascontiguousarray(fn()))
        C[n]["input"] = f"recipes.{n}()"

    print("config 3 frames (3840x2160)")
    for f in (0, 1):
        k = f"config3_frame{f}"
        C[k] = case_q50(k, recipes.config3_frame(f))
        C[k]["input"] = f"recipes.config3_frame({f})"
    C["config3_uniform0"] = case_q50("config3_uniform0", recipes.config3_uniform(0))
    C["config3_uniform0"]["input"] = "recipes.config3_uniform(0)"
    # the rest of bench.py's 16 distinct config-3 contents (rank 0): every
    # slot of the timed 256-frame batch is checked against these
    for f in range(2, 16):
        k = f"config3_frame{f}"
        C[k] = case_q50(k, recipes.config3_frame(f))
        C[k]["input"] = f"recipes.config3_frame({f})"

    print("config 4 frames (7680x4320)")
    for f in (0, 1):
        k = f"config4_frame{f}"
        C[k] = case_q50(k, recipes.config4_frame(f))
        C[k]["input"] = f"recipes.config4_frame({f})"

    print("quality sweep via original.c set_quality")
    with tempfile.TemporaryDirectory() as d:
        for n in ("sample_640x640", "sample_64x64"):
            rgb = recipes.sample(n)
            p = os.path.join(d, "in.ppm")
            with open(p, "wb") as f:
                f.write(ppm.ppm_bytes(rgb))
            for q in (10, 50, 75, 90, 100):
                r = O.ref_quality_encode(p, q, d)
                c = O.cref_encode(ppm.rgb_to_bgr(rgb), q)
                assert r == c, f"Q={q} restatement mismatch"
                k = f"{n}_q{q}"
                C[k] = {"quality": q, "input": n, "frame": list(rgb.shape[1::-1]),
                        "region": [0, 0, rgb.shape[1], rgb.shape[0]],
                        "jpg_sha256": sha(r), "jpg_len": len(r),
                        "source": "reference utils/original.c + set_quality (oracle/_ref)"}
                print(f"  {k}: {len(r)} B")
        # config 5 at frame size: a config-3 frame at Q=75 and one at Q=90
        # (bench.py --quality 75 / 90 encodes exactly these contents)
        for f, q in ((0, 75), (1, 90)):
            rgb = recipes.config3_frame(f)[:, :, ::-1]  # the recipe is B, G, R
            p = os.path.join(d, "in.ppm")
            with open(p, "wb") as fh:
                fh.write(ppm.ppm_bytes(np.ascontiguousarray(rgb)))
            r = O.ref_quality_encode(p, q, d)
            c = O.cref_encode(recipes.config3_frame(f), q)
            assert r == c, f"config3_frame{f} Q={q} restatement mismatch"
            k = f"config3_frame{f}_q{q}"
            C[k] = {"quality": q, "input": f"recipes.config3_frame({f})", "frame": [3840, 2160],
                    "region": [0, 0, 3840, 2160], "jpg_sha256": sha(r), "jpg_len": len(r),
                    "source": "reference utils/original.c + set_quality (oracle/_ref)"}
            print(f"  {k}: {len(r)} B")

    # full intermediates for the 64x64 plumbing case
    bgr = ppm.rgb_to_bgr(recipes.sample("sample_64x64"))
    Y, Cb, Cr, tabs, jpg = O.ref_stages(bgr)
    np.savez_compressed(os.path.join(GOLDEN, "sample_64x64.coefs.npz"), Y=Y, Cb=Cb, Cr=Cr)
    with open(os.path.join(GOLDEN, "sample_64x64.tables.json"), "w") as f:
        json.dump([huff_dict(t) for t in tabs], f)
    with open(os.path.join(GOLDEN, "cos_table.json"), "w") as f:
        json.dump([int(v) for v in O.cos_bits_ref()], f)
    assert (O.cos_bits_ref() == O.cos_bits_cref()).all()

    # colour exceptions: exhaustive over 2^24 with the restatement
    print("colour exception sets (exhaustive)")
    import ctypes
    out = np.zeros(3, np.uint8)
    lib = O.cref()
    # vectorised exact-integer candidates, then FP64 check through the C code
    r, g, b = np.meshgrid(np.arange(256), np.arange(256), np.arange(256), indexing="ij")
    r = r.ravel().astype(np.int64); g = g.ravel().astype(np.int64); b = b.ravel().astype(np.int64)
    cand = {
        0: (299 * r + 587 * g + 114 * b) % 1000 == 0,
        1: (128_000_000 - 168736 * r - 331264 * g + 500000 * b) % 1_000_000 == 0,
        2: (128_000_000 + 500000 * r - 418688 * g - 81312 * b) % 1_000_000 == 0,
    }
    exact = {
        0: (299 * r + 587 * g + 114 * b) // 1000,
        1: (128_000_000 - 168736 * r - 331264 * g + 500000 * b) // 1_000_000,
        2: (128_000_000 + 500000 * r - 418688 * g - 81312 * b) // 1_000_000,
    }
    exc = {}
    for ch in range(3):
        idx = np.nonzero(cand[ch])[0]
        lst = []
        for i in idx:
            lib.cref_pixel_ycc(ctypes.c_uint8(b[i]), ctypes.c_uint8(g[i]), ctypes.c_uint8(r[i]),
                               out.ctypes.data)
            if out[ch] != exact[ch][i]:
                assert out[ch] == exact[ch][i] - 1
                lst.append((r[i], g[i], b[i]))
        exc[ch] = np.array(lst, np.uint8).reshape(-1, 3)
        print(f"  channel {ch}: {len(idx)} exact-integer triples, {len(lst)} exceptions")
    np.savez_compressed(os.path.join(GOLDEN, "colour_exceptions.npz"),
                        Y=exc[0], Cb=exc[1], Cr=exc[2])
    with open(os.path.join(GOLDEN, "manifest.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)
    print("wrote", GOLDEN)


if __name__ == "__main__":
    main()
