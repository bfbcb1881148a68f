"""Barrier timeline of flash40 (vd_attention_select(9), the stamped diagnostic build): for
workgroup 0's 8 waves, per phase, the work time (barrier release -> arrival at the next one) and
the barrier wait (arrival -> release), split by group and by phase kind (V = softmax, M =
PV + QK^T).  s_memtime ticks = shader clock cycles.  Model-scale inputs, L1 shape.

    python tools/flash40_stamps.py
"""
import math
import statistics as st
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402
from vdiff._lib import check, lib  # noqa: E402

n_img, S, heads, d = 32, 4096, 8, 40
C = heads * d
g = torch.Generator(device="cuda").manual_seed(7)
qkv = torch.randn(n_img * S, 3 * C, device="cuda", generator=g) * 1.5
qkv[:, :C] *= d ** -0.5 * math.log2(math.e)
qkv = qkv.to(torch.bfloat16)
q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
lib().vd_attention_select(9)
for _ in range(5):
    o = ops.attention(q, k, v, n_img, heads, S, S, d, scale=1.0 / math.log2(math.e))
buf = torch.zeros(8 * 512, dtype=torch.int64, device="cuda")
check(lib().vd_attention_stamps(buf.data_ptr(), buf.numel(), torch.cuda.current_stream().cuda_stream), "stamps")
lib().vd_attention_select(0)
torch.cuda.synchronize()
t = buf.cpu().view(8, 512).tolist()
T = S // 64
nb = 2 * (2 * T + 3)  # stamps per wave: before/after each of 2T+3 barriers
for w in range(8):
    ts = t[w][:nb]
    work = [ts[2 * i] - ts[2 * i - 1] for i in range(1, nb // 2)]      # release i-1 -> arrival i
    wait = [ts[2 * i + 1] - ts[2 * i] for i in range(nb // 2)]          # arrival i -> release i
    # group 0: barrier 0 = prologue, 1 = phase 0 end, then (V, M) pairs; group 1 has the stagger first
    off = 2 if w < 4 else 3
    V = work[off - 1::2][:T - 2]
    M = work[off::2][:T - 2]
    print(f"wave {w} (group {w // 4}): V work median {st.median(V):6.0f}  M work median {st.median(M):6.0f}  "
          f"barrier wait median {st.median(wait[3:-3]):6.0f}  total {ts[nb - 1] - ts[0]} cycles, "
          f"per tile {(ts[nb - 1] - ts[0]) / T:.0f}")
