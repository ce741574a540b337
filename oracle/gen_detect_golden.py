"""oracle/gen_detect_golden.py -- TEST INFRASTRUCTURE ONLY.

Writes tests/golden/detect.json: for every recipes.DETECT_CASES scene and
for the reference's own image pair (images/sample_640x640{,_diffs}.ppm,
committed under tests/golden/), the outputs of the UNMODIFIED reference
main/brain.c (oracle/_ref/libref_brain.so): sha256 of subsample() of both
frames, and compare()'s count and areas.  The C restatement (libcref.so) is
checked against the same values before anything is written.

Run here (where /root/reference exists):  python oracle/gen_detect_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(HERE, "..", "tests")]

import oracle as O  # noqa: E402
import ppm  # noqa: E402
import recipes  # noqa: E402


def case(stored_bgr, cur_bgr) -> dict:
    H, W = cur_bgr.shape[:2]
    s0, s1 = O.ref_subsample(stored_bgr), O.ref_subsample(cur_bgr)
    n, areas = O.ref_compare(s1, s0, W, H)
    assert (O.cref_subsample(stored_bgr) == s0).all() and (O.cref_subsample(cur_bgr) == s1).all()
    assert O.cref_compare(s1, s0, W, H) == (n, areas), "restatement disagrees with the reference"
    return {"w": W, "h": H, "sub_stored_sha256": hashlib.sha256(s0.tobytes()).hexdigest(),
            "sub_current_sha256": hashlib.sha256(s1.tobytes()).hexdigest(),
            "count": n, "areas": [list(a) for a in areas]}


def main() -> None:
    O.build()
    out = {"source": "reference main/brain.c via oracle/_ref/libref_brain.so", "cases": []}
    for seed, w, h, kind in recipes.DETECT_CASES:
        stored, cur = recipes.detect_scene(seed, w, h, kind)
        c = case(stored, cur)
        c["recipe"] = [seed, w, h, kind]
        out["cases"].append(c)
        print(seed, w, h, kind, c["count"])
    a = ppm.rgb_to_bgr(recipes.sample("sample_640x640"))
    b = ppm.rgb_to_bgr(recipes.sample("sample_640x640_diffs"))
    for name, (s, c_) in {"sample_640x640->diffs": (a, b), "diffs->sample_640x640": (b, a)}.items():
        c = case(s, c_)
        c["images"] = name
        out["cases"].append(c)
        print(name, c["count"], c["areas"])
    with open(os.path.join(HERE, "..", "tests", "golden", "detect.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
