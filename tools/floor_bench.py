"""Per-launch floor in a captured graph: tiny GEMMs on each path vs a tiny LayerNorm."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402
from vdiff._lib import lib  # noqa: E402


def graph_us(fn, reps=50):
    for _ in range(3):
        fn()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


x = torch.randn(256, 1280, device="cuda").to(torch.bfloat16)
gm, bt = torch.ones(1280, device="cuda"), torch.zeros(1280, device="cuda")
print(f"layernorm 256x1280: {graph_us(lambda: ops.layer_norm(x, gm, bt)):.1f} us")
for M, N, K in [(256, 64, 64), (256, 64, 320), (256, 64, 1280), (256, 1280, 1280), (4096, 640, 640)]:
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    row = []
    for path, code in (("auto", 0), ("v1", 1), ("v2", 2), ("v6", 8)):
        ops._PLAN.path = code  # per-call vd_gemm_desc.path
        row.append(f"{path} {graph_us(lambda: ops.gemm(a, w, out=out)):6.1f}")
    ops._PLAN.path = 0  # per-call vd_gemm_desc.path
    print(f"gemm M={M:5d} N={N:5d} K={K:5d}: " + "  ".join(row) + " us", flush=True)
