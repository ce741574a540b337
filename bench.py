#!/usr/bin/env python3
"""bench.py -- Mpixels/s encoded on MI355X (BASELINE.json metric).

One step = the whole encode path (colour -> DCT -> quant -> zigzag ->
histograms -> optimized Huffman tables -> bit pack -> JFIF with stuffing) over
one batch of synthetic frames already resident in HBM.  Default workload is
SURVEY §8(d) config 3: 256 frames of 3840x2160 per GPU (weak scaling: each
rank encodes its own 256 frames; frames are independent, so there is no
data-path collective -- DESIGN.md §Multi-GPU).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--frames F]
      (N > 1: the script starts N rank processes itself, one per GPU)
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)
--gpus must equal WORLD_SIZE when a launcher sets it; otherwise bench.py exits
non-zero instead of reporting a one-GPU number as an N-GPU one.

Rank 0 prints one JSON line (metric, value, roofline, cpu_baseline, ...).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(REPO, "jpeg-encoder-decoder_amd"), os.path.join(REPO, "tests"),
          os.path.join(REPO, "oracle")):
    sys.path.insert(0, p)

import mijpeg  # noqa: E402
import sharding  # noqa: E402
import recipes  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--quality", type=int, default=50)
    ap.add_argument("--distinct", type=int, default=16,
                    help="distinct synthetic frames cycled through the batch")
    ap.add_argument("--mode", choices=["encode", "dct"], default="encode",
                    help="dct = K1 only (used for rocprof roofline runs)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="bound on the CPU-baseline sample (rank 0, N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-workers", type=int, default=min(16, os.cpu_count() or 1),
                    help="processes for the frame-parallel CPU baseline (the GPU box's CPU "
                         "share is 16 cores per GPU); 1 disables it")
    ap.add_argument("--overlap", type=int, default=int(os.environ.get("MIJ_OVERLAP", "1")),
                    help="fused pipeline in this many sub-batches, the entropy stages of one "
                         "on a second stream beside K1 of the next (1: off)")
    ap.add_argument("--split", action="store_true",
                    help="split pipeline: K1 writes coefficient planes and a second pass "
                         "tokenizes them (default: fused, K1 emits the symbol tokens itself)")
    ap.add_argument("--coef-launches", type=int, default=5,
                    help="extra launches of the coefficient-output K1 variant after the timed "
                         "region, for its own 6 B/px roofline line (0 disables)")
    ap.add_argument("--workload", choices=["config3", "config4", "regions", "detect", "decode", "stream",
                                               "ranks"],
                    default="config3",
                    help="config4: a stream of 7680x4320 frames, each split into MCU-row bands "
                         "over the ranks with the RCCL exchange steps (strong scaling)")
    ap.add_argument("--detect-frames", type=int, default=8, help="detect: distinct frames cycled")
    ap.add_argument("--stream-files", type=int, default=64,
                    help="stream: PPM files per step (config-3 recipe contents, 16 distinct)")
    ap.add_argument("--stream-chunk", type=int, default=16, help="stream: frames per device batch")
    ap.add_argument("--frames4", type=int, default=8, help="config4 frames per step")
    ap.add_argument("--band-emit", choices=["auto", "root", "bands"], default="auto",
                    help="config4: JFIF byte emission on the root alone, or distributed over the bands "
                         "(each band stuffs its own bytes; auto: bands when there is more than one rank)")
    ap.add_argument("--regions", type=int, default=100,
                    help="regions workload: rectangles per frame (main.c's diffDims holds up to 100)")
    ap.add_argument("--region-frame", default="1920x1080",
                    help="regions workload: the frame the rectangles are cut from")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=V",
                    help="entropy-stage variant for A/B timing (mij_batch_set_option, "
                         "include/mijpeg.h MIJ_OPT_*; same bytes), repeatable")
    ap.add_argument("--verify", type=int, default=-1,
                    help="frames re-checked against the oracle after timing (-1: every frame "
                         "of the batch; config3 checks each distinct content with the oracle and "
                         "the reference-build sha256 of tests/golden, then every slot's bytes)")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """`bench.py --gpus N` with no WORLD_SIZE in the environment: start N
    child processes of this same script, one rank per GPU (RANK = LOCAL_RANK
    = r, WORLD_SIZE = N, MASTER_ADDR 127.0.0.1 and a free port), wait for all
    of them and return the worst exit code.  The parent touches no GPU: it
    never initialises HIP (torch.cuda.device_count() does not on this image)
    and starts the ranks as children instead of exec'ing itself.  Rank 0
    prints the one JSON line.  A rank that fails ends the others."""
    import signal
    import subprocess
    backend = os.environ.get("MIJ_DIST_BACKEND", "nccl")
    if backend == "nccl" and args.workload != "ranks":
        import torch
        have = torch.cuda.device_count()
        if have < args.gpus:
            print(f"bench.py: --gpus {args.gpus} but only {have} GPU(s) visible", file=sys.stderr)
            return 2
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        # same process group as this parent: a `timeout` around the launch
        # reaches every rank
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))

    def _forward(sig, _frame):
        for q in procs:
            if q.poll() is None:
                q.send_signal(sig)
        raise SystemExit(128 + sig)
    signal.signal(signal.SIGTERM, _forward)
    signal.signal(signal.SIGINT, _forward)
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0:
                rc = rc or (code if code > 0 else 128 - code)
                for q in live:      # the exact children this parent started
                    q.terminate()
        if live:
            time.sleep(0.05)
    return rc


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        # a mis-launched scaling run must not print a valid-looking line
        raise SystemExit(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={world} "
                         f"(launch with --gpus N alone, or torchrun --nproc-per-node N ... --gpus N)")
    # MIJ_DIST_FORCE=1: a process group even for one rank (runs the device
    # branch of the nccl exchanges on a single GPU)
    if world > 1 or os.environ.get("MIJ_DIST_FORCE"):
        import torch
        import torch.distributed as dist
        # nccl (= RCCL) between GPUs; MIJ_DIST_BACKEND=gloo rehearses several
        # ranks on one GPU (collectives then go through host memory)
        backend = os.environ.get("MIJ_DIST_BACKEND", "nccl")
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend, init_method="env://")
        return world, rank, local, dist, torch
    return 1, 0, 0, None, None


def dist_device(dist, local):
    return f"cuda:{local}" if dist is not None and dist.get_backend() == "nccl" else "cpu"


def run_config4(args, world, rank, local, dist):
    """each step encodes --frames4 frames of 7680x4320;
    every frame is split into world MCU-row bands, one per rank, joined by the
    exchanges of sharding.encode_banded (last DCs, histograms, bit counts,
    packed words to rank 0 -- RCCL when the backend is nccl)."""
    W, H, n = 7680, 4320, args.frames4
    backend = dist.get_backend() if dist is not None else "none"
    gpu = 0 if backend == "gloo" else local
    # device-resident protocol (mij_band_*_async, sharding.encode_banded_dev):
    # collectives on device tensors -- RCCL, or one rank; with gloo (several
    # ranks sharing one GPU) the same protocol with every collective staged
    # through host memory (sharding.StagedExchange), unless
    # MIJ_BAND_PROTOCOL=host asks for the host-array protocol (encode_banded)
    on_dev = not (backend == "gloo" and os.environ.get("MIJ_BAND_PROTOCOL") == "host")
    if on_dev and backend != "nccl":  # torch's HIP runtime first (dist_setup did it for nccl)
        import torch
        torch.cuda.set_device(gpu)
    r0, rows = sharding.band_rows(H, world, rank)
    band = mijpeg.Batch(W, rows, n, args.quality, device=gpu)
    distinct = min(n, args.distinct)
    frames = [recipes.config4_frame(f) for f in range(distinct)]
    for f in range(n):
        band.upload(np.ascontiguousarray(frames[f % distinct][r0:r0 + rows]), first=f)
    # the root assembles on an assembler batch: tables, scan buffers and
    # outputs only (no whole-frame input, coefficient or token buffers)
    full = mijpeg.Batch(W, H, n, args.quality, device=gpu, assembler=True) if rank == 0 else None
    for k, v in (o.split("=", 1) for o in args.opt):  # (A/B variants; the assembler's emission slots)
        band.set_option(k, int(v))
        if full is not None and k == "emit_slots":
            full.set_option(k, int(v))
    if not on_dev:
        xch = sharding.TorchExchange(dist, dist_device(dist, local))
    elif backend == "gloo":
        xch = sharding.StagedExchange(dist, f"cuda:{gpu}")
    else:
        xch = sharding.DeviceExchange(dist, f"cuda:{gpu}")

    emit = args.band_emit if args.band_emit != "auto" else ("bands" if world > 1 else "root")

    def step(events=None):
        if on_dev:
            sharding.encode_banded_dev(band, n, xch, full, events=events, emit=emit)
        else:
            sharding.encode_banded(band, n, xch, full)

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    if full is not None:
        full.sync()
    band.sync()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if full is not None:
        full.sync()
    band.sync()
    el = time.perf_counter() - t0
    barrier()
    # per-phase times of one more step (device protocol: events on the band
    # stream between the phases)
    phases = None
    if on_dev:
        import torch
        ev = []
        step(ev)
        torch.cuda.synchronize()
        phases = {ev[i][0]: round(ev[i - 1][1].elapsed_time(ev[i][1]), 4) for i in range(1, len(ev))}
    el, _ = sharding.reduce_timing(el, 0, dist, dist_device(dist, local))
    verified = golden = 0
    if rank == 0 and args.verify:
        import hashlib
        import oracle as O
        # config4_frame0/1 also against the reference build's sha256
        # (tests/golden/manifest.json, oracle/gen_golden.py)
        man = {}
        mpath = os.path.join(REPO, "tests", "golden", "manifest.json")
        if args.quality == 50 and os.path.exists(mpath):
            with open(mpath) as fh:
                man = json.load(fh)["cases"]
        for f in range(n if args.verify < 0 else min(args.verify, n)):
            out = full.output(f)
            want = man.get(f"config4_frame{f % distinct}")
            if want is not None:
                if (len(out), hashlib.sha256(out).hexdigest()) != (want["jpg_len"], want["jpg_sha256"]):
                    raise SystemExit(f"bench config4: frame {f} differs from the reference's sha256")
                golden += 1
            elif out != O.cref_encode(frames[f % distinct], args.quality):
                raise SystemExit(f"bench config4: frame {f} differs from the oracle")
            verified += 1
    px = W * H * n * args.steps
    res = {
        "metric": "Mpixels/s encoded (device-resident BGR888 -> JFIF bytes)",
        "value": round(px / el / 1e6, 1), "unit": "Mpixels/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "int8-MFMA exact + fp64 replay (bit-exact)",
        "data": f"synthetic: SURVEY §8(d) config-4 recipe, {distinct} distinct frames",
        "config": {"workload": f"config 4: {n} frames of {W}x{H} per step, each split into {world} "
                               f"MCU-row bands (one per rank) with DC/histogram/bit-offset "
                               f"exchanges and a packed-word gather to rank 0",
                   "frames_per_step": n, "width": W, "height": H, "quality": args.quality,
                   "parallelism": f"band-parallel x{world}",
                   "backend": backend,
                   "emit": emit if on_dev else "root",
                   "protocol": ("host arrays (gloo)" if not on_dev else
                                "device-resident (mij_band_*_async)" +
                                (", collectives staged through host memory (gloo)" if backend == "gloo" else ""))},
        "verified_frames": verified,
        "verified_against_reference_sha": golden,
    }
    if phases:
        res["phases_ms"] = phases
    if rank == 0:
        print(json.dumps(res), flush=True)
    band.close()
    if full is not None:
        full.close()
    if dist is not None:
        dist.destroy_process_group()


def region_set(W, H, n, seed=7):
    """n rectangles (x, y, w, h) with w, h multiples of 16 (brain.c:244-261
    enlargeAdjust makes them so), 16..512 px per side, inside a W x H frame."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        w = 16 * int(rng.integers(1, min(32, W // 16) + 1))
        h = 16 * int(rng.integers(1, min(32, H // 16) + 1))
        out.append((int(rng.integers(0, W - w + 1)), int(rng.integers(0, H - h + 1)), w, h))
    return out


def run_regions(args, world, rank, local, dist):
    """SURVEY §8(f) rank 2, the reference's own workload shape (main.c:142-155):
    every step encodes --regions rectangles of one device-resident frame, each
    to its own JFIF, through one region batch (one gather launch + one encode
    launch sequence).  Frame-parallel over ranks (each rank its own frame)."""
    import torch
    W, H = map(int, args.region_frame.split("x"))
    gpu = 0 if dist is not None and dist.get_backend() != "nccl" else local
    torch.cuda.set_device(gpu)
    frame = np.ascontiguousarray(recipes.config3_frame(rank, H, W) if W <= 3840 and H <= 2160
                                 else recipes.config4_frame(rank, H, W))
    regions = region_set(W, H, args.regions, 7 + rank)
    cw, ch = max(r[2] for r in regions), max(r[3] for r in regions)
    batch = mijpeg.Batch(cw, ch, len(regions), args.quality, device=gpu)
    dframe = torch.from_numpy(frame).to(f"cuda:{gpu}")
    torch.cuda.synchronize()

    def step():
        batch.gather_regions(dframe.data_ptr(), W * 3, W, H, regions)
        batch.encode(len(regions))

    for _ in range(args.warmup):
        step()
    batch.sync()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    batch.sync()
    el = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    px = sum(r[2] * r[3] for r in regions)
    el, px_all = sharding.reduce_timing(el, px * args.steps, dist, dist_device(dist, local))
    verified = 0
    if args.verify:
        import oracle as O
        for i in range(len(regions) if args.verify < 0 else min(len(regions), 4 * args.verify)):
            if batch.output(i) != O.cref_encode(frame, args.quality, regions[i]):
                raise SystemExit(f"bench regions: region {i} differs from the oracle")
            verified += 1
    res = {
        "metric": "Mpixels/s encoded (device-resident BGR888 -> JFIF bytes)",
        "value": round(px_all / el / 1e6, 1), "unit": "Mpixels/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int8-MFMA exact + fp64 replay (bit-exact)",
        "data": "synthetic: config-3 recipe frame, seeded rectangles",
        "config": {"workload": f"regions: {len(regions)} rectangles (16..512 px a side, "
                               f"{px / 1e6:.2f} Mpixels) of one {W}x{H} frame per step, each its own JFIF "
                               f"(main.c:142-155), one region batch",
                   "regions": len(regions), "frame": f"{W}x{H}", "region_pixels": px,
                   "quality": args.quality, "parallelism": f"frame-parallel x{world}"},
        "regions_per_s": round(len(regions) * args.steps * world / el, 1),
        "verified_regions": verified,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle as O
        use_ref = O.ref_available()
        n, npx, t0 = 0, 0, time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_seconds or n < len(regions):
            r = regions[n % len(regions)]
            (O.ref_stages(frame, r) if use_ref else O.cref_encode(frame, args.quality, r))
            n += 1
            npx += r[2] * r[3]
        el_c = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(npx / el_c / 1e6, 3), "unit": "Mpixels/s", "cores": 1,
                               "kind": "reference" if use_ref else "port",
                               "sample": f"{n} region encodes of the same rectangles, {el_c:.1f} s, "
                                         f"1 thread, main.c's per-region call sequence"}
    if rank == 0:
        print(json.dumps(res), flush=True)
    batch.close()
    if dist is not None:
        dist.destroy_process_group()


def run_detect(args, world, rank, local, dist):
    """the reference's whole per-frame loop (main.c:136-163)
    on a device-resident stream of --detect-frames distinct frames of
    --region-frame size: one detector kernel (4x4 subsample + weighted colour
    distance vs the stored frame, brain.c:16-45/:184-195) + the host area
    joining (brain.c:104-233), then every detected area encoded to its own
    JFIF through one region batch, then store.  Frame-parallel over ranks."""
    import torch
    W, H = map(int, args.region_frame.split("x"))
    gpu = 0 if dist is not None and dist.get_backend() != "nccl" else local
    torch.cuda.set_device(gpu)
    nf = args.detect_frames
    frames = [np.ascontiguousarray(recipes.detect_scene(500 + 97 * rank + i, W, H, "objects")[1])
              for i in range(nf)]
    dframes = [torch.from_numpy(f).to(f"cuda:{gpu}") for f in frames]
    det = mijpeg.Detector(W, H, device=gpu)
    torch.cuda.synchronize()
    # one pass to size the region batch (detection is deterministic)
    plan = []
    det.subsample(dframes[-1].data_ptr())
    det.store()
    for f in dframes:
        plan.append(det.step(f.data_ptr())[1])
        det.store()
    cw = max([a[2] for areas in plan for a in areas] + [16])
    ch = max([a[3] for areas in plan for a in areas] + [16])
    batch = mijpeg.Batch(cw, ch, max(max(len(a) for a in plan), 1), args.quality, device=gpu)

    def step(i):
        f = dframes[i % nf]
        n, areas = det.step(f.data_ptr())
        if n:
            batch.gather_regions(f.data_ptr(), 3 * W, W, H, areas)
            batch.encode(n)
        det.store()
        return areas

    for i in range(args.warmup):
        step(i)
    batch.sync()
    if dist is not None:
        dist.barrier()
    nreg = 0
    t0 = time.perf_counter()
    for i in range(args.steps):
        nreg += len(step(args.warmup + i))
    batch.sync()
    el = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    el, px_all = sharding.reduce_timing(el, W * H * args.steps, dist, dist_device(dist, local))
    # the detector kernel alone, HIP events on the detector's own stream
    ds = torch.cuda.ExternalStream(det.stream())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    e0.record(ds)
    for i in range(reps):
        det.launch(dframes[i % nf].data_ptr())
    e1.record(ds)
    e1.synchronize()
    k_ms = e0.elapsed_time(e1) / reps
    sw, sh = W // 4, H // 4
    k_bytes = 3 * W * H + 2 * 4 * sw * sh + 8 * ((sw + 63) // 64) * sh
    # verification: the last step's areas and a few JFIFs against the oracle
    import oracle as O
    last = (args.warmup + args.steps - 1) % nf
    prev = O.cref_subsample(frames[(last - 1) % nf])
    want = O.cref_compare(O.cref_subsample(frames[last]), prev, W, H)
    got_areas = plan[last]
    if (len(got_areas), got_areas) != (want[0], want[1]):
        raise SystemExit("bench detect: areas differ from the oracle")
    verified = 0
    if args.verify and want[0]:
        n, areas = want
        for i in range(n if args.verify < 0 else min(n, 4 * args.verify)):
            if batch.output(i) != O.cref_encode(frames[last], args.quality, areas[i]):
                raise SystemExit(f"bench detect: area {i} differs from the oracle")
            verified += 1
    res = {
        "metric": "Mpixels/s encoded (device-resident BGR888 -> JFIF bytes)",
        "value": round(px_all / el / 1e6, 1), "unit": "Mpixels/s (frame pixels through detect+encode)",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: tests/recipes.detect_scene moving-object frames",
        "config": {"workload": f"detect: main.c:136-163 loop on {W}x{H} frames -- detector kernel, "
                               f"host area joining, every area its own JFIF (one region batch), store",
                   "frame": f"{W}x{H}", "distinct_frames": nf, "quality": args.quality,
                   "parallelism": f"frame-parallel x{world}"},
        "frames_per_s": round(args.steps * world / el, 1),
        "areas_per_frame": round(nreg / args.steps, 2),
        "roofline": {"bound": "hbm", "kernel": "k_detect<true> (4x4 subsample + compare + ballot mask)",
                     "achieved": round(k_bytes / k_ms / 1e6, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(k_bytes / k_ms / 1e6 / HBM_PEAK_GBS, 4), "traffic": None,
                     "ms_per_launch": round(k_ms, 4), "algorithmic_bytes_per_launch": k_bytes},
        "verified_areas": verified,
    }
    # PMC-measured HBM bytes of the same kernel on the same workload
    # (scripts/profile.sh detect -> profiles/rNN/detect/traffic.json)
    import glob
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "detect", "traffic.json")), reverse=True):
        d = json.load(open(path))
        if d.get("config", {}).get("frame") != f"{W}x{H}":
            continue
        for name, v in d.get("kernels", {}).items():
            if "k_detect<true>" in name:
                res["roofline"]["traffic"] = v["hbm_bytes"]
                res["roofline"]["traffic_source"] = (f"{os.path.relpath(path, REPO)} (rocprofv3 PMC "
                                                     f"FETCH_SIZE x2 + WRITE_SIZE, same workload)")
        break
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        use_ref = O.ref_brain_available() and O.ref_available()
        sub_fn = O.ref_subsample if use_ref else O.cref_subsample
        cmp_fn = O.ref_compare if use_ref else O.cref_compare
        n, t0 = 0, time.perf_counter()
        saved = sub_fn(frames[-1])
        while time.perf_counter() - t0 < args.cpu_seconds or n < 1:
            f = frames[n % nf]
            sub = sub_fn(f)
            cnt, areas = cmp_fn(sub, saved, W, H)
            for a in areas[:cnt]:
                (O.ref_stages(f, a) if use_ref else O.cref_encode(f, args.quality, a))
            saved = sub
            n += 1
        el_c = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(n * W * H / el_c / 1e6, 3), "unit": "Mpixels/s", "cores": 1,
                               "kind": "reference" if use_ref else "port",
                               "sample": f"{n} frames through brain.c subsample/compare + encoder.c per "
                                         f"area, {el_c:.1f} s, 1 thread"}
    if rank == 0:
        print(json.dumps(res), flush=True)
    batch.close()
    det.close()
    if dist is not None:
        dist.destroy_process_group()


def run_decode(args, world, rank, local, dist):
    """SURVEY §8(f) rank 4, the round-trip verifier: --frames JFIF streams of
    the config-3 frames (encoded by this library) decoded back to coefficient
    planes per step (host parse + H2D of the streams + the GPU entropy decode,
    one lane per scan).  Verified against the encoder's kept coefficients."""
    import torch
    gpu = 0 if dist is not None and dist.get_backend() != "nccl" else local
    torch.cuda.set_device(gpu)
    W, H, F = args.width, args.height, args.frames
    frames = make_frames(args, rank)
    enc = mijpeg.Batch(W, H, F, args.quality, device=gpu, keep_coefs=True)
    host = np.stack([frames[i % len(frames)] for i in range(F)])
    enc.upload(host)
    enc.encode(F)
    streams = [enc.output(i) for i in range(F)]
    dec = mijpeg.Decoder(W, H, F, device=gpu)

    for _ in range(args.warmup):
        dec.decode(streams)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dec.decode(streams)
    el = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    el, px_all = sharding.reduce_timing(el, W * H * F * args.steps, dist, dist_device(dist, local))
    verified = 0
    for i in range(F if args.verify < 0 else min(F, args.verify)):
        for g, w in zip(dec.coefs(i), enc.coefs(i, diffed=True)):
            if not (g == w).all():
                raise SystemExit(f"bench decode: frame {i} coefficients differ from the encoder's")
        verified += 1
    res = {
        "metric": "Mpixels/s decoded (JFIF -> coefficient planes, round-trip verifier)",
        "value": round(px_all / el / 1e6, 1), "unit": "Mpixels/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int16",
        "data": "synthetic: config-3 frames encoded by this library",
        "config": {"workload": f"decode: {F} x {W}x{H} JFIF streams per step (host parse + "
                               f"unstuffing + H2D + GPU chunk-parallel entropy decode)", "frames": F, "width": W, "height": H,
                   "stream_MB": round(sum(len(s) for s in streams) / 1e6, 2),
                   "parallelism": f"frame-parallel x{world}"},
        "verified_frames": verified,
        "sync_passes": dec.passes(),
    }
    if rank == 0:
        print(json.dumps(res), flush=True)
    dec.close()
    enc.close()
    if dist is not None:
        dist.destroy_process_group()


def run_stream(args, world, rank, local, dist):
    """SURVEY §8(f) rank 1, host-fed: PPM files on the host file system ->
    .jpg files, through mij_stream (PPM parsing by original.c:294-365's rules
    on host threads into pinned memory, H2D, encode, D2H and file writes of
    one chunk overlapped with the GPU work of the other; two device batches in
    ping-pong).  The timed region covers everything from the first file read
    to the last .jpg written -- value is host-to-host Mpixels/s, PCIe and file
    I/O included.  Frame-parallel over ranks (each rank its own files)."""
    import hashlib
    import shutil
    import tempfile
    import ppm
    W, H, n = args.width, args.height, args.stream_files
    gpu = 0 if dist is not None and dist.get_backend() != "nccl" else local
    import torch  # its HIP runtime before the library's (the PCIe probe below uses it)
    torch.cuda.set_device(gpu)
    tmp = tempfile.mkdtemp(prefix=f"mij_stream_r{rank}_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        distinct = min(n, args.distinct)
        contents = [rank * args.distinct + i for i in range(distinct)]
        ins, outs = [], []
        for i in range(n):
            c = contents[i % distinct]
            p = os.path.join(tmp, f"in_{i:04d}.ppm")
            if i < distinct:
                with open(p, "wb") as f:  # PPM is R, G, B; the recipe is B, G, R
                    f.write(ppm.ppm_bytes(np.ascontiguousarray(recipes.config3_frame(c, H, W)[:, :, ::-1])))
            else:
                shutil.copyfile(ins[i % distinct], p)
            ins.append(p)
            outs.append(os.path.join(tmp, f"out_{i:04d}.jpg"))
        st = mijpeg.Stream(W, H, args.stream_chunk, args.quality, device=gpu)
        for _ in range(args.warmup):
            st.encode_files(ins, outs)
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        agg = {k: 0.0 for k in mijpeg.Stream.STATS}
        for _ in range(args.steps):
            st.encode_files(ins, outs)
            for k, v in st.stats().items():
                agg[k] += v
        el = time.perf_counter() - t0
        if dist is not None:
            dist.barrier()
        el, px_all = sharding.reduce_timing(el, W * H * n * args.steps, dist, dist_device(dist, local))
        st.close()
        # every output file against the reference's bytes: the manifest's
        # sha256 (reference build) where it holds the content, the oracle else
        verified = pinned = 0
        if args.verify:
            gold = json.load(open(os.path.join(REPO, "tests", "golden", "manifest.json")))["cases"]
            want = {}
            for i in range(n):
                c = contents[i % distinct]
                if c not in want:
                    g = gold.get(f"config3_frame{c}")
                    if g and g["quality"] == args.quality and [W, H] == [3840, 2160]:
                        want[c] = g["jpg_sha256"]
                        pinned += 1
                    else:
                        import oracle as O
                        want[c] = hashlib.sha256(O.cref_encode(recipes.config3_frame(c, H, W),
                                                               args.quality)).hexdigest()
                with open(outs[i], "rb") as f:
                    if hashlib.sha256(f.read()).hexdigest() != want[c]:
                        raise SystemExit(f"bench stream: {outs[i]} differs from the reference bytes")
                verified += 1
        res = {
            "metric": "Mpixels/s encoded host-to-host (PPM files -> .jpg files, PCIe and file I/O included)",
            "value": round(px_all / el / 1e6, 1), "unit": "Mpixels/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int8-MFMA exact + fp64 replay (bit-exact)",
            "data": f"synthetic: {n} PPM files of the config-3 recipe ({distinct} distinct contents) "
                    f"written to {os.path.dirname(tmp)} before timing",
            "config": {"workload": f"stream: {n} x {W}x{H} PPM files -> .jpg files per step through "
                                   f"mij_stream ({args.stream_chunk}-frame chunks, 2 batches in ping-pong)",
                       "files": n, "width": W, "height": H, "quality": args.quality,
                       "chunk": args.stream_chunk, "parallelism": f"frame-parallel x{world}"},
            "files_per_s": round(n * args.steps * world / el, 1),
            # per step, summed over the chunks (host read/parse, GPU encode
            # between its events, D2H + file writes): they overlap, so their sum
            # exceeds the step
            "stage_s_per_step": {k: round(agg[k] / args.steps, 4) for k in ("read_s", "gpu_s", "write_s")},
            "input_GB_per_s": round(agg["bytes_in"] / el / 1e9, 2),
            "verified_files": verified, "verified_contents_pinned_to_reference_sha": pinned,
        }
        # the PCIe ceiling of a host-fed stream: pinned host -> HBM copies of
        # one chunk's bytes (torch on this GPU, after the stream is closed)
        try:
            nb = W * H * 3 * args.stream_chunk
            src = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
            dst = torch.empty(nb, dtype=torch.uint8, device=f"cuda:{gpu}")
            dst.copy_(src, non_blocking=True)
            torch.cuda.synchronize(gpu)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                dst.copy_(src, non_blocking=True)
            e1.record()
            torch.cuda.synchronize(gpu)
            h2d = 3 * nb / (e0.elapsed_time(e1) * 1e-3) / 1e9
            res["pcie_h2d_GB_per_s"] = round(h2d, 1)
            res["pcie_ceiling_Mpix_s"] = round(h2d * 1e9 / 3 / 1e6, 1)
            del src, dst
        except Exception as e:  # noqa: BLE001 (a report field, not the measurement)
            res["pcie_h2d_GB_per_s"] = f"unmeasured: {e}"
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"], par = stream_cpu_baseline(ins[:distinct], outs, W, H, args)
            if par is not None:
                res["cpu_baseline_parallel"] = par
        if rank == 0:
            print(json.dumps(res), flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    if dist is not None:
        dist.destroy_process_group()


def _stream_cpu_worker(job):
    """One process of the stream's CPU baseline: files -> .jpg files for
    `seconds` (the reference's globals make it single-threaded per process)."""
    ins, out_dir, seconds, quality, use_ref = job
    import oracle as O
    n, t0 = 0, time.perf_counter()
    while True:
        src = ins[n % len(ins)]
        dst = os.path.join(out_dir, f"cpu_{os.getpid()}.jpg")
        if use_ref:
            if not O.ref_encode_file(src, dst):
                raise SystemExit(f"bench stream: the reference failed on {src}")
        else:
            import ppm
            with open(src, "rb") as f:
                rgb = ppm.parse_ppm(f.read())
            with open(dst, "wb") as f:
                f.write(O.cref_encode(np.ascontiguousarray(rgb[:, :, ::-1]), quality))
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds and n >= 2:
            return n, el


def stream_cpu_baseline(ins, outs, W, H, args):
    """The reference on the same files, the way its caller runs it (main.c:
    131-155 with the camera replaced by the PPM file): PPM read, the three
    encoder.c entry points, write_jpg writing the .jpg file itself
    (oracle/_ref ref_encode_file, compiled from the reference sources).  One
    core, and frame-parallel over --cpu-workers processes.  encoder.c has no
    quality knob, so at Q != 50 the C restatement (cpu_ref, file -> file)
    stands in.  Returns (1-core entry, parallel entry or None)."""
    import multiprocessing as mp
    import oracle as O
    use_ref = O.ref_available() and args.quality == 50
    out_dir = os.path.dirname(outs[0])
    what = ("reference main/encoder.c via oracle/_ref ref_encode_file (PPM read, rgb_to_dct, "
            "init_huffman, write_jpg -> file)" if use_ref else "oracle/cpu_ref.c, PPM file -> .jpg file")
    kind = "reference" if use_ref else "port"
    n, el = _stream_cpu_worker((ins, out_dir, args.cpu_seconds, args.quality, use_ref))
    one = {"value": round(n * W * H / el / 1e6, 3), "unit": "Mpixels/s", "cores": 1, "kind": kind,
           "sample": f"{n} files of {W}x{H} in {el:.1f} s, {what}"}
    par = None
    if args.cpu_workers > 1:
        ctx = mp.get_context("spawn")
        jobs = [(ins[i % len(ins):] + ins[:i % len(ins)], out_dir, args.cpu_seconds, args.quality, use_ref)
                for i in range(args.cpu_workers)]
        with ctx.Pool(args.cpu_workers) as pool:
            parts = pool.map(_stream_cpu_worker, jobs)
        files = sum(p for p, _ in parts)
        busy = max(e for _, e in parts)
        par = {"value": round(files * W * H / busy / 1e6, 3), "unit": "Mpixels/s", "cores": args.cpu_workers,
               "kind": kind, "sample": f"{args.cpu_workers} processes x >= {args.cpu_seconds:.0f} s, "
                                       f"{files} files in all, {what}"}
    return one, par


def make_frames(args, rank):
    """Distinct config-3 frames (recipe in tests/recipes.py), rank-offset so
    ranks encode different content."""
    out = []
    for i in range(args.distinct):
        f = rank * args.distinct + i
        if (args.width, args.height) == (3840, 2160):
            out.append(recipes.config3_frame(f))
        else:
            out.append(recipes.config3_frame(f, args.height, args.width)
                       if args.width <= 3840 and args.height <= 2160
                       else recipes.config4_frame(f, args.height, args.width))
    return out


def verify_batch(batch, frames, F, args, rank):
    """(slots verified, distinct contents pinned to the reference sha256)."""
    import hashlib
    import oracle as O
    gold = {}
    path = os.path.join(REPO, "tests", "golden", "manifest.json")
    if os.path.exists(path):
        gold = json.load(open(path))["cases"]
    n = F if args.verify < 0 else min(args.verify, F)
    want, pinned = {}, 0
    for c in range(min(len(frames), n)):
        want[c] = O.cref_encode(frames[c], args.quality)
        key = f"config3_frame{rank * args.distinct + c}"
        g = gold.get(key)
        if (g and g["quality"] == args.quality and (args.width, args.height) == (3840, 2160)
                and g["frame"] == [args.width, args.height]):
            if hashlib.sha256(want[c]).hexdigest() != g["jpg_sha256"]:
                raise SystemExit(f"bench: oracle bytes of {key} differ from the reference golden")
            pinned += 1
    bad = [i for i in range(n) if batch.output(i) != want[i % len(frames)]]
    if bad:
        raise SystemExit(f"bench: {len(bad)} frames differ from the oracle: {bad[:16]}")
    return n, pinned


UTIL_KEYS = ("width", "height", "frames_per_gpu", "quality", "mode", "pipeline")


def util_counters(kernel_sym, config):
    """VALU / MFMA utilisation of `kernel_sym` from the newest profiles/rNN/util.json
    (scripts/pmc_util.sh + scripts/util.py: rocprofv3 PMC passes of a bench
    run) whose recorded workload matches `config` (size, frames, quality,
    mode, pipeline); (None, None) when none does.  mfma_util = matrix-pipe
    busy cycles / (1024 SIMDs x cycles) -- 1.0 is the dense i8 peak at the
    clock held; valu_util = VALU issue slots used (2 cycles per wave64
    instruction) / available.  Everything attached comes from that one
    profiled run (its counters and its own launch time)."""
    import glob
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "util.json")), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if any(d.get("config", {}).get(k) != config.get(k) for k in UTIL_KEYS):
            continue
        for name, v in d.get("kernels", {}).items():
            if kernel_sym in name:
                return v, os.path.relpath(path, REPO)
    return None, None


def util_fields(u, src):
    """The roofline fields of one util.json kernel entry (util_counters)."""
    r = {"mfma_util": u.get("mfma_util"), "valu_util": u.get("valu_util"),
         "util_source": f"{src} (rocprofv3 PMC: SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU, "
                        f"GRBM_GUI_ACTIVE; same workload)"}
    if u.get("SQ_INSTS_MFMA") and u.get("launch_us"):
        # v_mfma_i32_16x16x64_i8: 16*16*64 MACs = 32768 int8 ops each; dense
        # i8 peak 5 POP/s (MI355X_MICROARCH.md, 2x bf16's 2.5 PF); counts and
        # time both from the profiled run
        tops = u["SQ_INSTS_MFMA"] * 32768 / (u["launch_us"] * 1e-6) / 1e12
        r["mfma_i8_TOPs"] = round(tops, 1)
        r["mfma_frac_of_i8_peak"] = round(tops / 5000.0, 4)
    return r


# rocprofv3 symbol of each K1 variant (for the PMC traffic lookup)
K1_SYMBOL = {"k_mcu_dct<COEF_OUT>": "k_mcu_dct<1>", "k_mcu_dct<TOK_OUT>": "k_mcu_dct<2>",
             "k_mcu_dct<COEF_IN|TOK_OUT>": "k_mcu_dct<6>"}


def pmc_traffic(kernel, config):
    """HBM bytes per launch of `kernel` measured by rocprofv3 PMC passes
    (FETCH_SIZE x2 + WRITE_SIZE, scripts/profile.sh + scripts/traffic.py) on
    the same workload, from the newest profiles/rNN/traffic.json whose
    recorded configuration matches; None if there is none."""
    import glob
    keys = ("width", "height", "frames_per_gpu", "quality", "mode", "pipeline")
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "traffic.json")), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if any(d.get("config", {}).get(k) != config.get(k) for k in keys):
            continue
        for name, v in d.get("kernels", {}).items():
            if K1_SYMBOL.get(kernel, kernel) in name:
                return v["hbm_bytes"], os.path.relpath(path, REPO)
    return None, None


def cpu_baseline(frames, seconds):
    """The reference encoder.c itself (oracle/_ref, compiled from the
    reference sources) when present, else the C restatement; 1 thread."""
    import oracle as O
    use_ref = O.ref_available()
    enc = (lambda f: O.ref_stages(f)[4]) if use_ref else (lambda f: O.cref_encode(f))
    n_px, n, t0 = 0, 0, time.perf_counter()
    while True:
        f = frames[n % len(frames)]
        enc(f)
        n += 1
        n_px += f.shape[0] * f.shape[1]
        el = time.perf_counter() - t0
        if el >= seconds and n >= 2:
            break
    import platform
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    h, w = frames[0].shape[:2]
    return {"value": round(n_px / el / 1e6, 3), "unit": "Mpixels/s", "cores": 1,
            "kind": "reference" if use_ref else "port",
            "sample": f"{n} frames of {w}x{h} (config-3 recipe), {el:.1f} s, 1 thread, "
                      f"{'reference main/encoder.c via oracle/_ref' if use_ref else 'oracle/cpu_ref.c'}"
                      f", output to memory, on {cpu}"}


def _cpu_worker(job):
    """One process of the frame-parallel CPU baseline: the reference keeps
    its bit-writer state in globals (encoder.c:383-384), so frames are spread
    over processes, not threads.  Returns (pixels, seconds)."""
    seed, h, w, seconds = job
    import oracle as O
    use_ref = O.ref_available()
    frame = recipes.config3_frame(seed) if (w, h) == (3840, 2160) else recipes.config3_frame(seed, h, w)
    enc = (lambda f: O.ref_stages(f)[4]) if use_ref else (lambda f: O.cref_encode(f))
    n, t0 = 0, time.perf_counter()
    while True:
        enc(frame)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds and n >= 1:
            return n * h * w, el


def cpu_baseline_parallel(h, w, seconds, workers):
    """Frame-parallel reference encoder over `workers` host cores (BASELINE.md
    CPU-baseline plan (ii)): aggregate pixels / wall time."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        parts = pool.map(_cpu_worker, [(i, h, w, seconds) for i in range(workers)])
    wall = time.perf_counter() - t0
    px = sum(p for p, _ in parts)
    busy = max(e for _, e in parts)
    import oracle as O
    return {"value": round(px / busy / 1e6, 3), "unit": "Mpixels/s", "cores": workers,
            "kind": "reference" if O.ref_available() else "port",
            "sample": f"{workers} processes x >= {seconds:.0f} s each, one {w}x{h} config-3 frame "
                      f"per process, aggregate over the slowest process ({wall:.1f} s wall incl. start-up)"}


def run_ranks(args, world, rank, local, dist):
    """--workload ranks: the launcher's own check, no encode.  Every rank
    joins the process group, meets the others at a barrier and reports its
    rank; rank 0 prints who came.  (tests/test_bench_launch.py runs it over
    gloo on the CPU.)"""
    el = 0.0
    t0 = time.perf_counter()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    ranks = sharding.gather_ints([rank, os.getpid()], dist, dist_device(dist, local))
    el, _ = sharding.reduce_timing(el, 0, dist, dist_device(dist, local))
    if rank == 0:
        print(json.dumps({"workload": "ranks", "n_gpus": world,
                          "backend": dist.get_backend() if dist is not None else "none",
                          "ranks": [r[0] for r in ranks], "pids": [r[1] for r in ranks],
                          "barrier_s": round(el, 6)}), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if not 1 <= args.quality <= 100:
        raise SystemExit(f"bench.py: --quality {args.quality} outside 1..100")
    world, rank, local, dist, torch = dist_setup(args)
    if args.workload == "ranks":
        return run_ranks(args, world, rank, local, dist)
    if args.workload == "config4":
        return run_config4(args, world, rank, local, dist)
    if args.workload == "regions":
        return run_regions(args, world, rank, local, dist)
    if args.workload == "detect":
        return run_detect(args, world, rank, local, dist)
    if args.workload == "decode":
        return run_decode(args, world, rank, local, dist)
    if args.workload == "stream":
        return run_stream(args, world, rank, local, dist)
    W, H, F = args.width, args.height, args.frames
    frames = make_frames(args, rank)
    gpu = 0 if dist is not None and dist.get_backend() != "nccl" else local
    batch = mijpeg.Batch(W, H, F, args.quality, device=gpu)
    batch.set_split(args.split)
    opts = dict(o.split("=", 1) for o in args.opt)
    for k, v in opts.items():
        batch.set_option(k, int(v))
    if args.overlap > 1:
        batch.set_overlap(args.overlap)
    for i in range(F):
        batch.upload(frames[i % len(frames)], first=i)
    run = batch.encode if args.mode == "encode" else batch.dct

    for _ in range(args.warmup):
        run(F)
    batch.sync()

    def barrier():
        if dist is not None:
            dist.barrier()

    # the timed steps run without the per-stage events (on a one-frame step
    # their records are a fifth of the time); the stage breakdown comes from
    # as many steps again with them, after the timed region
    batch.set_timing(False)
    barrier()
    batch.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run(F)
    batch.sync()
    el = time.perf_counter() - t0
    barrier()
    # max time over ranks, pixels over all ranks (sharding.py; no data-path collective)
    el, px_all = sharding.reduce_timing(el, W * H * F * args.steps, dist, dist_device(dist, local))

    batch.set_timing(True)
    for _ in range(args.steps):
        run(F)
    batch.sync()
    hist = batch.stage_history(args.steps)
    stage_avg = {k: round(float(np.mean([h[k] for h in hist])), 4) for k in mijpeg.Batch.STAGES}
    k1_ms, tok_ms = stage_avg["k1_colour_dct_quant"], stage_avg["tokenize"]
    if args.mode == "dct":
        stage_avg = {"k1_colour_dct_quant": k1_ms}

    # The coefficient-output K1 variant (BASELINE.json north_star's "fused
    # DCT+quant kernel" at 6 B/px) is not on the default (fused) path: a few
    # launches of it right after the timed region -- the GPU still at the
    # clocks of the timed steps, like the dominant kernel it stands beside
    # (launched after the seconds-long CPU verification instead, its first
    # launches run ~20% slower while the clocks come back: 2.96-3.01 ms
    # against 2.45-2.52 warm, profiles/r05) -- HIP events on the batch
    # stream, one untimed launch first.  Then the same number of launches of
    # its access pattern without the arithmetic (mij_batch_pattern_floor):
    # K1's time beside the floor of its own memory traffic on this GPU.
    replays = batch.replays()
    coef_ms = floor_ms = None
    if args.coef_launches > 0 and args.mode == "encode" and not args.split:
        batch.set_timing(True)
        batch.dct(F)
        for _ in range(args.coef_launches):
            batch.dct(F)
        coef_ms = float(np.mean([h["k1_colour_dct_quant"]
                                 for h in batch.stage_history(args.coef_launches)]))
        batch.pattern_floor(F)
        for _ in range(args.coef_launches):
            batch.pattern_floor(F)
        floor_ms = float(np.mean([h["k1_colour_dct_quant"]
                                  for h in batch.stage_history(args.coef_launches)]))

    # correctness after timing (not timed): every distinct content against
    # the oracle and, where tests/golden holds it, the reference build's
    # sha256; then every slot of the batch against its content's bytes
    verified, pinned = 0, 0
    if args.verify and args.mode == "encode" and not os.environ.get("MIJ_K1_FLAGS"):
        verified, pinned = verify_batch(batch, frames, F, args, rank)

    # per-rank verification counts (every rank checks its own batch)
    ver_ranks = sharding.gather_ints([verified, pinned], dist, dist_device(dist, local))
    px_step = W * H * F
    value = px_all / el / 1e6
    geo = batch.geometry()
    # algorithmic HBM bytes per launch (DESIGN.md "Roofline accounting"):
    # BGR in 3 B/px; coefficient planes 2 B x 64 per block (= 3 B/px at 4:2:0);
    # one raw DC (2 B) per block; tokens 4 B each + one count (4 B) per segment
    coef_bytes = F * geo["nblk"] * 64 * 2
    dc_bytes = F * geo["nblk"] * 2
    tok_bytes = batch.token_count(F) * 4 + F * geo["nseg"] * 4 if args.mode == "encode" else 0
    kernels = {}
    if args.mode == "encode" and not args.split:
        kernels["k_mcu_dct<TOK_OUT>"] = (px_step * 3 + tok_bytes + dc_bytes, k1_ms,
                                         "K1 fused: colour+DCT+quant+zigzag+symbol tokens")
    else:
        kernels["k_mcu_dct<COEF_OUT>"] = (px_step * 3 + coef_bytes + dc_bytes, k1_ms,
                                          "K1: colour+DCT+quant+zigzag -> int16 planes")
        if args.mode == "encode":
            kernels["k_mcu_dct<COEF_IN|TOK_OUT>"] = (coef_bytes + tok_bytes, tok_ms,
                                                     "tokenize: planes -> symbol tokens + histograms")
    dom = max(kernels, key=lambda k: kernels[k][1])
    k1_bytes, dom_ms, dom_desc = kernels[dom]
    k1_gbs = k1_bytes / (dom_ms * 1e-3) / 1e9
    res = {
        "metric": "Mpixels/s encoded (device-resident BGR888 -> JFIF bytes)",
        "value": round(value, 1),
        "unit": "Mpixels/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int8-MFMA exact + fp64 replay (bit-exact)",
        "data": f"synthetic: SURVEY §8(d) config-3 recipe, {args.distinct} distinct frames "
                f"cycled over the batch",
        "config": {"workload": f"config 3: {F} x {W}x{H} BGR888 frames per GPU, 4:2:0, "
                               f"Q={args.quality}, one independent JFIF per frame",
                   "frames_per_gpu": F, "width": W, "height": H, "quality": args.quality,
                   "mode": args.mode, "pipeline": "split" if args.split else "fused",
                   "parallelism": f"frame-parallel x{world}",
                   **({"options": {k: int(v) for k, v in opts.items()}} if opts else {})},
        "roofline": {"bound": "hbm", "kernel": f"{dom} ({dom_desc})",
                     "achieved": round(k1_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(k1_gbs / HBM_PEAK_GBS, 4), "traffic": None,
                     "ms_per_launch": round(dom_ms, 4),
                     "algorithmic_bytes_per_launch": int(k1_bytes),
                     # SURVEY §8(d)'s unit: 6 B per image pixel (3 B BGR in +
                     # 3 B int16 coefficients out), whatever the kernel moves
                     "frac_8d_6Bpx": round(6 * px_step / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
        "kernels": {k: {"ms": round(v[1], 4), "algorithmic_GB": round(v[0] / 1e9, 3),
                        "GB_per_s": round(v[0] / (v[1] * 1e-3) / 1e9, 1)}
                    for k, v in kernels.items()},
        "stages_ms": stage_avg,
        "verified_frames": verified,
        "verified_contents_pinned_to_reference_sha": pinned,
        "verified_frames_per_rank": [v[0] for v in ver_ranks],
        # ranks in the RCCL (nccl backend) process group; 0 for one process or gloo
        "rccl_world": world if dist is not None and dist.get_backend() == "nccl" else 0,
        # blocks re-encoded in FP64 by k_fix_blocks (split pipeline) or coefficients
        # replayed in place (fused pipeline), per frame
        "fp64_fixups_per_frame": round(replays / (F * (args.warmup + 2 * args.steps)), 2),  # timed + events pass
    }
    if coef_ms is not None:
        cb = px_step * 3 + coef_bytes + dc_bytes
        res["roofline_k1_coefficient_variant"] = {
            "bound": "hbm", "kernel": "k_mcu_dct<COEF_OUT> (K1: colour+DCT+quant+zigzag -> int16 planes, "
                                      "the split pipeline's first kernel; not in the timed region)",
            "achieved": round(cb / (coef_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(cb / (coef_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "ms_per_launch": round(coef_ms, 4), "algorithmic_bytes_per_launch": int(cb),
            "launches": args.coef_launches,
            # the same traffic with no arithmetic, same GPU, same call
            "pattern_floor_ms": round(floor_ms, 4),
            "pattern_floor_frac_of_peak": round(cb / (floor_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "frac_of_pattern_floor": round(floor_ms / coef_ms, 4)}
        u1, usrc1 = util_counters("k_mcu_dct<1>", res["config"])
        if u1 is not None:
            res["roofline_k1_coefficient_variant"].update(util_fields(u1, usrc1))
    u, usrc = util_counters(K1_SYMBOL.get(dom, dom), res["config"])
    if u is not None:
        res["roofline"].update(util_fields(u, usrc))
    traffic, src = pmc_traffic(dom, res["config"])
    if traffic is not None:
        res["roofline"]["traffic"] = traffic
        res["roofline"]["traffic_source"] = f"{src} (rocprofv3 PMC FETCH_SIZE x2 + WRITE_SIZE, same workload)"
    if os.environ.get("MIJ_K1_FLAGS"):
        res["diagnostic_k1_flags"] = int(os.environ["MIJ_K1_FLAGS"])
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(frames[:4], args.cpu_seconds)
        if args.cpu_workers > 1:
            res["cpu_baseline_parallel"] = cpu_baseline_parallel(H, W, args.cpu_seconds,
                                                                 args.cpu_workers)
    if rank == 0:
        print(json.dumps(res), flush=True)
    batch.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
