"""flash512 (d = 512 VAE attention) DMA A/B: vd_attention_select(20 / 21 / 22) = K two tiles
ahead in a 3-slot ring, V one ahead / K and V one tile ahead (2 + 2 slots, the default) / no DMA
after tile 0 (the ablation: wrong results, timing only), 16 frames x S 4096, interleaved rounds."""
import math
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402
from vdiff._lib import lib  # noqa: E402

n, S, C = 16, 4096, 512
g = torch.Generator(device="cuda").manual_seed(1)
qkv = torch.randn(n * S, 3 * C, device="cuda", generator=g)
qkv[:, :C] *= C ** -0.5 * math.log2(math.e) * 0.5
qkv = qkv.to(torch.bfloat16)
q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
flop = 4.0 * S * S * C * n
res, outs = {pd: [] for pd in (0, 1, 2)}, {}
for pd in res:
    lib().vd_attention_select(20 + pd)
    outs[pd] = ops.attention(q, k, v, n, 1, S, S, C, scale=1.0 / math.log2(math.e))
torch.cuda.synchronize()
for _ in range(7):
    for pd in res:
        lib().vd_attention_select(20 + pd)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            ops.attention(q, k, v, n, 1, S, S, C, scale=1.0 / math.log2(math.e))
        e1.record()
        e1.synchronize()
        res[pd].append(e0.elapsed_time(e1) / 5)
lib().vd_attention_select(21)
for pd, ms in res.items():
    ms = sorted(ms)
    med = ms[len(ms) // 2]
    print(f"flash512 DV={pd}: median {med * 1e3:7.1f} us  {flop / med / 1e9:7.1f} TF/s ({flop / med / 1e9 / 2500:.3f})  "
          f"bitwise == DV 0: {torch.equal(outs[pd], outs[0])}")
