"""gemm3 (256x256 8-phase) efficiency vs K at fixed M x N: how much of a short-K launch is the
per-tile pipeline fill/drain and epilogue (the non-persistent kernel refills per tile).

    python tools/v3_k_sweep.py
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402
from vdiff._lib import lib  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(0)


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


for M, N in ((32768, 2560), (8192, 3840)):
    for K in (320, 640, 1280, 2560, 5120):
        a = (torch.randn(M, K, device="cuda", generator=g)).to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        res = []
        for path, code in (("v3", 3), ("v2", 2)):
            lib().vd_gemm_select_path(code)
            us = timeit(lambda: ops.gemm(a, w, out=out))
            res.append(f"{path} {us:7.1f} us {2.0 * M * N * K / us / 1e6:6.0f} TF/s")
        lib().vd_gemm_select_path(0)
        us = timeit(lambda: torch.nn.functional.linear(a, w))
        res.append(f"hipBLASLt {us:7.1f} us {2.0 * M * N * K / us / 1e6:6.0f} TF/s")
        print(f"M={M} N={N} K={K:5d} | " + " | ".join(res), flush=True)
