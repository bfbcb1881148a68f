"""LayerNorm kernels at the UNet's shapes (16 frames x CFG): multi-row vs one-row-per-wave, in a graph."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402
from vdiff._lib import lib  # noqa: E402

imgs = int(sys.argv[1]) if len(sys.argv) > 1 else 32
for hw, C in [(4096, 320), (1024, 640), (256, 1280), (64, 1280)]:
    x = torch.randn(imgs * hw, C, device="cuda").to(torch.bfloat16)
    g, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
    res = []
    for mr in (1, 0):
        lib().vd_layernorm_select(mr)
        for _ in range(3):
            ops.layer_norm(x, g, b)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(20):
                ops.layer_norm(x, g, b)
        graph.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        graph.replay()
        e1.record()
        e1.synchronize()
        res.append(e0.elapsed_time(e1) / 20 * 1e3)
    lib().vd_layernorm_select(1)
    gbs = 2 * x.numel() * 2 / (res[0] * 1e-6) / 1e9
    print(f"rows={imgs * hw:7d} C={C:5d}  multi-row {res[0]:7.1f} us ({gbs:6.0f} GB/s)   one-row {res[1]:7.1f} us", flush=True)
