"""bench.py's rank launcher (CPU, gloo): `bench.py --gpus N` run without a
launcher starts N rank processes itself, and a --gpus that disagrees with a
launcher's WORLD_SIZE is an error, never a one-GPU line labelled N GPUs
(BASELINE.json metric: Mpixels/s at 1/2/4/8 GPUs)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(MIJ_DIST_BACKEND="gloo", **kw)
    return env


def _bench(args, env, timeout=180):
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=timeout, cwd=REPO)


def test_gpus_two_starts_two_ranks():
    r = _bench(["--gpus", "2", "--workload", "ranks"], _env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 alone prints
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["ranks"] == [0, 1] and res["backend"] == "gloo"
    assert len(set(res["pids"])) == 2          # two processes, not one


def test_gpus_four_starts_four_ranks():
    r = _bench(["--gpus", "4", "--workload", "ranks"], _env())
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert res["n_gpus"] == 4 and res["ranks"] == [0, 1, 2, 3]


def test_gpus_disagreeing_with_world_size_fails():
    env = _env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT="29999")
    r = _bench(["--gpus", "1", "--workload", "ranks"], env)
    assert r.returncode != 0 and "disagrees with WORLD_SIZE" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    env["WORLD_SIZE"] = "1"
    r = _bench(["--gpus", "2", "--workload", "ranks"], env)
    assert r.returncode != 0 and "disagrees with WORLD_SIZE" in r.stderr


def test_one_gpu_needs_no_process_group():
    r = _bench(["--gpus", "1", "--workload", "ranks"], _env())
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert res["n_gpus"] == 1 and res["backend"] == "none" and res["ranks"] == [0]


def test_failing_rank_fails_the_launch():
    # ranks that reject their arguments end the launch with a non-zero
    # code, and the parent prints no line of its own
    r = _bench(["--gpus", "2", "--workload", "ranks", "--quality", "0"], _env())
    assert r.returncode != 0 and "outside 1..100" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
