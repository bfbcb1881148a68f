"""GroupNorm paths at the UNet's image-norm shapes: two-launch (per-group records, finalize in
the apply prologue) vs partial/finalize/apply.  python tools/gn_bench.py"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402

for n_inst, pix, C in [(32, 4096, 320), (32, 1024, 640), (32, 256, 1280), (32, 64, 1280), (32, 64, 2560),
                       (4, 4096, 320), (4, 1024, 640), (4, 256, 1280), (4, 64, 2560)]:
    x = torch.randn(n_inst * pix, C, device="cuda").to(torch.bfloat16)
    g, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
    res = []
    for tp in (True, False):
        f = lambda: ops.group_norm(x, n_inst, pix, 32, 1e-5, g, b, silu=True, two_pass=tp)  # noqa: E731
        for _ in range(3):
            f()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(20):
                f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        graph.replay()
        e0.record()
        graph.replay()
        e1.record()
        e1.synchronize()
        res.append(e0.elapsed_time(e1) / 20 * 1e3)
    print(f"inst={n_inst:3d} pix={pix:5d} C={C:5d}  two-launch {res[0]:7.1f} us   four-launch {res[1]:7.1f} us", flush=True)
