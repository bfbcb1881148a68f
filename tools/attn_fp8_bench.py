"""fp8 vs bf16 spatial self-attention at the DiT's shape (S = 2304, d = 64, 64 images x 18
heads), timed with HIP events; used under rocprofv3 --pmc for the kernel's counters.

    python tools/attn_fp8_bench.py [--reps 10] [--images 64]
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402
from vdiff._lib import lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--images", type=int, default=64)
ap.add_argument("--seq", type=int, default=2304)
a = ap.parse_args()
n, heads, S, d = a.images, 18, a.seq, 64
D = heads * d
qkv = torch.randn(n * S, 3 * D, device="cuda").to(torch.bfloat16)
q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
o = torch.empty(n * S, D, device="cuda", dtype=torch.bfloat16)
ws = ops.attention_fp8_quant(q, k, v, n, heads, S, S, d, q_scale=d ** -0.5 * ops.LOG2E)  # ops.attention_fp8's fold
ws1 = ops.attention_fp8_quant(q, k, v, n, heads, S, S, d)                                # unfolded operands


def fp8():
    ops.attention_fp8_run(ws, o)


def fp8_unfolded():  # the kernel's per-score-multiply form (scale not folded into q8)
    ops.attention_fp8_run(ws1, o)


def bf16():
    ops.attention(q, k, v, n, heads, S, S, d, out=o)


flop = 4.0 * n * heads * S * S * d


for name, fn in (("warm-up", fp8), ("fp8", fp8), ("fp8 unfolded", fp8_unfolded), ("bf16", bf16), ("fp8", fp8),
                 ("fp8 unfolded", fp8_unfolded), ("bf16", bf16)):  # the first case pays the clock ramp
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        fn()
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    print(f"{name}: {ms:.4f} ms  {flop / ms / 1e9:.1f} TFLOP/s", flush=True)
