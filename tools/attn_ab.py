"""A/B of the d = 40 spatial self-attention kernels in one process (MI355X_MICROARCH rule 24:
interleaved rounds): flash40 (round 3) vs flash32 (4 waves) vs the 16x16x32 kernel (--sels=7,8,1 default),
at the level-1 shape (S = 4096, 8 heads, 32 images = 16 frames x CFG 2), random data.

    python tools/attn_ab.py [rounds]
"""
import math
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402
from vdiff._lib import lib  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 5
n_img, S, heads, d = 32, 4096, 8, 40
C = heads * d
g = torch.Generator(device="cuda").manual_seed(7)
qkv = (torch.randn(n_img * S, 3 * C, device="cuda", generator=g) * 1.5).to(torch.bfloat16)
q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
scale = 1.0 / math.log2(math.e)
flop = 4.0 * S * S * d * heads * n_img
SELS = tuple(int(x) for x in next((a.split('=')[1] for a in sys.argv if a.startswith('--sels=')), '7,8,1').split(','))
outs, res = {}, {sel: [] for sel in SELS}
names = {1: "flash_attn 16x16x32", 2: "flash32 (4 waves)", 3: "flash32pp (pipelined stagger)",
         4: "flash32 interleaved", 5: "flash32, 1 WG per CU", 6: "flash32, 1 q-block/wave (3/SIMD)",
         7: "flash40 (ping-pong, LDS-DMA ring)", 8: "flash32 (4 waves)"}
if "--model-scale" in sys.argv:  # bench.py's roofline inputs: softmax scale folded into q
    qkv[:, :C] = (qkv[:, :C].float() * (d ** -0.5 * math.log2(math.e))).to(torch.bfloat16)
for sel in SELS:
    lib().vd_attention_select(sel)
    outs[sel] = ops.attention(q, k, v, n_img, heads, S, S, d, scale=scale)
torch.cuda.synchronize()
for _ in range(rounds):
    for sel in SELS:
        lib().vd_attention_select(sel)
        out = torch.empty_like(outs[sel])
        for _ in range(2):
            ops.attention(q, k, v, n_img, heads, S, S, d, scale=scale, out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            ops.attention(q, k, v, n_img, heads, S, S, d, scale=scale, out=out)
        e1.record()
        e1.synchronize()
        res[sel].append(e0.elapsed_time(e1) / 10)
lib().vd_attention_select(0)
for sel in SELS:
    ms = sorted(res[sel])
    print(f"{names[sel]:30s} median {ms[len(ms) // 2] * 1e3:7.1f} us  min {ms[0] * 1e3:7.1f} us  "
          f"{flop / ms[len(ms) // 2] / 1e9:7.1f} TF/s  ({flop / ms[len(ms) // 2] / 1e9 / 2500:.3f} of peak)")
if 7 in outs and 8 in outs:
    print("flash40 == flash32 bitwise:", torch.equal(outs[7], outs[8]))
