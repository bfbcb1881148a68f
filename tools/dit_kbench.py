"""GEMM path sweep over the DiT's (BASELINE config 5) projection shapes, 1x MI355X.

python tools/dit_kbench.py  -> per shape and path (vd_gemm_desc.path): us, TFLOP/s
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402
from vdiff._lib import lib  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
M = 2 * 32 * 2304
D = 1152
SHAPES = [("qkv", D, 3 * D, None), ("out/cross", D, D, None), ("out+res", D, D, "res"),
          ("fc1 gelu", D, 4 * D, "gelu"), ("fc2", 4 * D, D, None)]


def timeit(fn, reps=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for name, K, N, epi in SHAPES:
    a = (torch.randn(M, K, device=dev, generator=g)).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=g) * 0.03).to(torch.bfloat16)
    bias = torch.randn(N, device=dev, generator=g) * 0.1
    res = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16) if epi == "res" else None
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    act = ops.ACT_GELU if epi == "gelu" else ops.ACT_NONE
    line = f"{name:10s} M={M} N={N} K={K}"
    ref = None
    for path in (0, 2, 3, 5, 6):
        ops._PLAN.path = path  # per-call vd_gemm_desc.path
        try:
            fn = lambda: ops.gemm(a, w, bias=bias, res=res, act=act, out=out)  # noqa: E731
            us = timeit(fn)
            o = out.float()
            if ref is None:
                ref = o.clone()
            ok = (o - ref).abs().max().item() < 0.1
            line += f" | p{path} {us:8.1f} us {2 * M * N * K / us / 1e6:6.0f} TF/s{'' if ok else ' MISMATCH'}"
        except Exception as e:  # noqa: BLE001
            line += f" | p{path} err {str(e)[:30]}"
    ops._PLAN.path = 0  # per-call vd_gemm_desc.path
    print(line, flush=True)
    del a, w, res, out
