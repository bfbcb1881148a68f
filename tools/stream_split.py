"""Per-rank compute at small frame counts is launch/latency bound: does running the two CFG
halves of the UNet on two streams (parallel graph branches) beat one batch-2 forward?

    python tools/stream_split.py [frames]
(a) one graph: forward of both CFG halves as one batch (what DenoiseLoop does);
(b) one graph: the cond and uncond halves as two forwards on two forked streams;
(c) one graph: the two half forwards back to back on one stream.
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402
from vdiff.models.unet_motion import CIN_PAD  # noqa: E402
from vdiff.weights import materialize_synthetic  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 2
unet = materialize_synthetic("full", device="cuda", seed=0)
unet.prepare()
H = W = 64
lat = torch.randn((1, 4, F, H, W), generator=torch.Generator().manual_seed(42)).cuda()
ehs = torch.randn((2, 77, 768), generator=torch.Generator().manual_seed(1)).cuda().to(torch.bfloat16)
ts = torch.tensor([500.0], device="cuda")
x2 = ops.pack_latents(lat, dup=2, cpad=CIN_PAD)
x1 = x2[:F * H * W]
caches = [{}, {}, {}]


def fwd(x, e, bsz, cache):
    te = ops.timestep_embed(ts, unet.time_proj.num_channels, batch=bsz)
    ctx = unet.make_ctx(te, e.reshape(bsz * 77, -1), bsz, F, 77, kv_cache=cache)
    return unet.forward_rows(x, H, W, ctx)


def run_a():
    return fwd(x2, ehs, 2, caches[0])


def run_c():
    return fwd(x1, ehs[:1], 1, caches[1]), fwd(x1, ehs[1:], 1, caches[2])


side = torch.cuda.Stream()


def run_b():
    main = torch.cuda.current_stream()
    side.wait_stream(main)
    e0 = fwd(x1, ehs[:1], 1, caches[1])
    with torch.cuda.stream(side):
        e1 = fwd(x1, ehs[1:], 1, caches[2])
    main.wait_stream(side)
    return e0, e1


only = sys.argv[2] if len(sys.argv) > 2 else "abc"
res = {}
for name, fn in (("a batch-2 forward", run_a), ("b two streams", run_b), ("c two forwards, one stream", run_c)):
    if name[0] not in only:
        continue
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts_ = []
    for _ in range(5):
        ev[0].record()
        for _ in range(5):
            g.replay()
        ev[1].record()
        ev[1].synchronize()
        ts_.append(ev[0].elapsed_time(ev[1]) / 5)
    ts_.sort()
    print(f"frames {F}: {name:28s} {ts_[2]:7.2f} ms per UNet forward pair (median of 5 x 5 replays)", flush=True)
