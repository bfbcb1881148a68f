"""Where the GEMM time could go: our paths vs hipBLASLt (torch F.linear, no epilogue) on the
UNet's dominant shapes and their conv-equivalent dense GEMMs (implicit-GEMM conv K = 9*Cin).

    python tools/gemm_ceiling.py
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


def rnd(*s, std=1.0):
    return (torch.randn(*s, device=dev, generator=g) * std).to(torch.bfloat16)


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


SHAPES = [  # (name, M, N, K, act)
    ("conv L1 as dense", 131072, 320, 2880, 0), ("conv L1 up as dense", 131072, 320, 5760, 0),
    ("conv L2 as dense", 32768, 640, 5760, 0), ("conv L3 as dense", 8192, 1280, 11520, 0),
    ("conv L4 as dense", 2048, 1280, 11520, 0),
    ("L1 proj K320", 131072, 320, 320, 0), ("L1 qkv", 131072, 960, 320, 0), ("L1 geglu", 131072, 2560, 320, 2),
    ("L1 ff2", 131072, 320, 1280, 0), ("L2 proj", 32768, 640, 640, 0), ("L2 qkv", 32768, 1920, 640, 0),
    ("L2 geglu", 32768, 5120, 640, 2), ("L2 ff2", 32768, 640, 2560, 0), ("L3 qkv", 8192, 3840, 1280, 0),
    ("L3 geglu", 8192, 10240, 1280, 2), ("8192^3", 8192, 8192, 8192, 0),
]
for name, M, N, K, act in SHAPES:
    a, w = rnd(M, K), rnd(N, K, std=K ** -0.5)
    b = torch.zeros(N, device=dev)
    nout = N // 2 if act == 2 else N
    out = torch.empty(M, nout, device=dev, dtype=torch.bfloat16)
    res = []
    for path, code in (("auto", 0), ("v2", 2), ("v3", 3)):
        ops._PLAN.path = code  # per-call vd_gemm_desc.path
        us = timeit(lambda: ops.gemm(a, w, bias=b, act=act, out=out))
        res.append(f"{path} {us:7.1f}us {2.0 * M * N * K / us / 1e6:6.0f}TF")
    ops._PLAN.path = 0  # per-call vd_gemm_desc.path
    us = timeit(lambda: torch.nn.functional.linear(a, w))
    res.append(f"hipblaslt {us:7.1f}us {2.0 * M * N * K / us / 1e6:6.0f}TF")
    print(f"{name:22s} M={M:6d} N={N:5d} K={K:5d} | " + " | ".join(res), flush=True)
