"""debug: encode_banded_dev over a one-rank group (nccl, or none with
argv[1] == "none"), Python stacks dumped if it stalls."""
import faulthandler, os, sys
R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(R, "jpeg-encoder-decoder_amd"), os.path.join(R, "tests"), os.path.join(R, "oracle")]
faulthandler.dump_traceback_later(40, exit=True)
import numpy as np
import torch
import torch.distributed as dist
torch.cuda.set_device(0)
import mijpeg, sharding, recipes
import oracle as O
frames = np.stack([recipes.config3_frame(5, 320, 480), recipes.noise(320, 480, 9), recipes.config3_frame(6, 320, 480)])
n, H, W = frames.shape[:3]
want = [O.cref_encode(f) for f in frames]
mode = sys.argv[1] if len(sys.argv) > 1 else "nccl"
if mode == "nccl":
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533")
    dist.init_process_group("nccl", rank=0, world_size=1)
band = mijpeg.Batch(W, H, n)
band.upload(frames)
full = mijpeg.Batch(W, H, n, assembler=True)
xch = sharding.DeviceExchange(dist if mode == "nccl" else None, "cuda:0")
for it in range(2):
    ev = []
    print("step", it, flush=True)
    sharding.encode_banded_dev(band, n, xch, full, events=ev)
    print("issued", flush=True)
    full.sync()
    print("ok", [full.output(f) == w for f, w in enumerate(want)], flush=True)
band.close()
full.close()
print("closed", flush=True)
if mode == "nccl":
    dist.destroy_process_group()
print("done", flush=True)
