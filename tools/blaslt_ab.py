"""Dense GEMM + residual epilogue: our vd_gemm (auto plan) vs hipBLASLt through torch.addmm
(beta = 1 residual, the library's fused form) on the UNet's K >= 640 shapes.

    python tools/blaslt_ab.py
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(0)


def rnd(*s, std=1.0):
    return (torch.randn(*s, device="cuda", generator=g) * std).to(torch.bfloat16)


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps * 1e3)
    return best


for imgs in (32, 4):
    for name, hw, N, K, res in [("L1 ff2", 4096, 320, 1280, 1), ("L2 proj", 1024, 640, 640, 1),
                                ("L2 ff2", 1024, 640, 2560, 1), ("L3 proj", 256, 1280, 1280, 1),
                                ("L3 ff2", 256, 1280, 5120, 1), ("L3 qkv", 256, 3840, 1280, 0),
                                ("L4 proj", 64, 1280, 1280, 1), ("L4 ff2", 64, 1280, 5120, 1),
                                ("L4 qkv", 64, 3840, 1280, 0), ("L2 qkv", 1024, 1920, 640, 0)]:
        M = imgs * hw
        a, w = rnd(M, K), rnd(N, K, std=K ** -0.5)
        b = torch.randn(N, device="cuda")
        r = rnd(M, N) if res else None
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ours = timeit(lambda: ops.gemm(a, w, bias=b, res=r, out=out))
        bb = b.to(torch.bfloat16)
        if res:
            lt = timeit(lambda: torch.addmm(r, a, w.t(), out=out))
        else:
            lt = timeit(lambda: torch.nn.functional.linear(a, w, bb))
        print(f"{imgs:2d} img {name:8s} M={M:6d} N={N:5d} K={K:5d} {'+res' if res else '    '}  ours {ours:7.1f} us  "
              f"hipBLASLt {lt:7.1f} us  ({ours / lt:4.2f}x)", flush=True)
