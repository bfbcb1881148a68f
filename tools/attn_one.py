"""Run ONE d = 40 spatial self-attention kernel variant (for PMC passes): the level-1 shape
(S 4096, 8 heads, 32 images), `reps` launches.

    python tools/attn_one.py <select: 1 16x16 | 2 flash32 | 3 flash32pp> [reps]
"""
import math
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402
from vdiff._lib import lib  # noqa: E402

sel = int(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n_img, S, heads, d = 32, 4096, 8, 40
C = heads * d
g = torch.Generator(device="cuda").manual_seed(7)
qkv = (torch.randn(n_img * S, 3 * C, device="cuda", generator=g) * 1.5).to(torch.bfloat16)
out = torch.empty(n_img * S, C, device="cuda", dtype=torch.bfloat16)
lib().vd_attention_select(sel)
for _ in range(reps):
    ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], n_img, heads, S, S, d, scale=1.0 / math.log2(math.e),
                  out=out)
torch.cuda.synchronize()
print("ok")
