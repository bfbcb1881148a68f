"""A/B of flash40 schedule variants in one process (interleaved rounds), L1 shape (S 4096,
8 heads, 32 images, d 40), the model's inputs (softmax scale * log2 e folded into q):
    python tools/attn_variant_ab.py [rounds] [--pairs=25:26] [--imgs=32] [--S=4096] [--d=40]
each pair "a:b" = vd_attention_select(a) vs vd_attention_select(b) on top of the automatic d = 40
choice (flash40); results must be bitwise equal (the variants only move work between phases).
"""
import math
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402
from vdiff._lib import lib  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 7
pairs = next((a.split("=")[1] for a in sys.argv if a.startswith("--pairs=")), "25:26")
sels = sorted({int(x) for p in pairs.split(",") for x in p.split(":")})
n_img = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--imgs=")), "32"))
S = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--S=")), "4096"))
d = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--d=")), "40"))
heads = 8
C = heads * d
g = torch.Generator(device="cuda").manual_seed(7)
qkv = (torch.randn(n_img * S, 3 * C, device="cuda", generator=g) * 1.5)
qkv[:, :C] *= d ** -0.5 * math.log2(math.e)
qkv = qkv.to(torch.bfloat16)
q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
scale = 1.0 / math.log2(math.e)
flop = 4.0 * S * S * d * heads * n_img
res, outs = {s: [] for s in sels}, {}
for s in sels:
    lib().vd_attention_select(s)
    outs[s] = ops.attention(q, k, v, n_img, heads, S, S, d, scale=scale)
torch.cuda.synchronize()
out = torch.empty_like(outs[sels[0]])
for _ in range(rounds):
    for s in sels:
        lib().vd_attention_select(s)
        for _ in range(2):
            ops.attention(q, k, v, n_img, heads, S, S, d, scale=scale, out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            ops.attention(q, k, v, n_img, heads, S, S, d, scale=scale, out=out)
        e1.record()
        e1.synchronize()
        res[s].append(e0.elapsed_time(e1) / 10)
for s in sels:
    ms = sorted(res[s])
    med = ms[len(ms) // 2]
    print(f"select({s:2d}) median {med * 1e3:7.1f} us  min {ms[0] * 1e3:7.1f} us  {flop / med / 1e9:7.1f} TF/s "
          f"({flop / med / 1e9 / 2500:.3f} of peak)  bitwise == select({sels[0]}): {torch.equal(outs[s], outs[sels[0]])}")
