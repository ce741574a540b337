"""bench.py's reporting helpers (CPU): utilisation counters are attached
only from a profiled run of the same workload, and everything they report
(counts and time) comes from that one run."""
import importlib.util
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_util_counters_require_matching_workload(tmp_path, monkeypatch):
    b = _bench()
    cfg = {"width": 3840, "height": 2160, "frames_per_gpu": 256, "quality": 50, "mode": "encode",
           "pipeline": "fused"}
    d = tmp_path / "profiles" / "r99"
    d.mkdir(parents=True)
    k = {"void mij::k_mcu_dct<2>(mij::K1Args)": {"launch_us": 1000.0, "SQ_INSTS_MFMA": 1000000,
                                                 "mfma_util": 0.1, "valu_util": 0.4}}
    (d / "util.json").write_text(json.dumps({"config": cfg, "kernels": k}))
    monkeypatch.setattr(b, "REPO", str(tmp_path))
    u, src = b.util_counters("k_mcu_dct<2>", dict(cfg))
    assert u is not None and src.endswith("util.json")
    f = b.util_fields(u, src)
    # 1e6 MFMA x 32768 ops in the profiled run's own 1 ms
    assert f["mfma_i8_TOPs"] == round(1e6 * 32768 / 1e-3 / 1e12, 1)
    for key, val in (("quality", 90), ("frames_per_gpu", 64), ("pipeline", "split"), ("width", 1920)):
        other = dict(cfg, **{key: val})
        assert b.util_counters("k_mcu_dct<2>", other) == (None, None), key
    # a util.json without a recorded workload is never attached
    (d / "util.json").write_text(json.dumps({"kernels": k}))
    assert b.util_counters("k_mcu_dct<2>", dict(cfg)) == (None, None)


def test_committed_profiles_attach_to_the_default_bench():
    """The newest committed util.json and traffic.json record the workload
    they were measured on, and it is the default bench's (config 3), so the
    driver's bench line carries mfma_util / valu_util and PMC traffic."""
    b = _bench()
    cfg = {"width": 3840, "height": 2160, "frames_per_gpu": 256, "quality": 50, "mode": "encode",
           "pipeline": "fused"}
    u, src = b.util_counters("k_mcu_dct<2>", dict(cfg))
    assert u is not None, "no committed util.json matches the default workload"
    assert 0 < u["mfma_util"] < 1 and 0 < u["valu_util"] < 1
    assert b.pmc_traffic("k_mcu_dct<2>", dict(cfg))[0] is not None
