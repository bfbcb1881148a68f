"""Phase timeline of flash40 (vd_attention_select(9), the stamped diagnostic build): workgroup
0's 8 waves record tagged s_memtime stamps (shader-clock cycles; tag in bits 56+):
1 barrier arrival, 2 release, 3 exps done, 4 V reads issued, 5 DMA issued, 6 PV(db 0) issued,
7 PV(db 1) issued, 8 QK^T issued, 9 decisions done.  Per group and phase kind (V = softmax, M =
PV + QK^T), the median cycles of each interval between consecutive stamps.  Model-scale inputs,
L1 shape (32 images x 8 heads x 4096 x 4096).

    python tools/flash40_stamps.py
"""
import collections
import math
import statistics as st
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402
from vdiff._lib import check, lib  # noqa: E402

NAMES = {1: "arrive", 2: "release", 3: "exps", 4: "Vreads", 5: "DMA", 6: "PV0", 7: "PV1", 8: "QK", 9: "decide"}
n_img, S, heads, d = 32, 4096, 8, 40
C = heads * d
g = torch.Generator(device="cuda").manual_seed(7)
qkv = torch.randn(n_img * S, 3 * C, device="cuda", generator=g) * 1.5
qkv[:, :C] *= d ** -0.5 * math.log2(math.e)
qkv = qkv.to(torch.bfloat16)
q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
lib().vd_attention_select(9)
for _ in range(5):
    ops.attention(q, k, v, n_img, heads, S, S, d, scale=1.0 / math.log2(math.e))
NST = 1024
buf = torch.zeros(8 * NST, dtype=torch.int64, device="cuda")
check(lib().vd_attention_stamps(buf.data_ptr(), buf.numel(), torch.cuda.current_stream().cuda_stream), "stamps")
lib().vd_attention_select(0)
torch.cuda.synchronize()
raw = buf.cpu().view(8, NST).tolist()
for grp in (0, 1):
    acc = collections.defaultdict(list)
    tot = []
    for w in range(4 * grp, 4 * grp + 4):
        ev = [((x >> 56) & 0xFF, x & ((1 << 56) - 1)) for x in raw[w] if x]
        tot.append((ev[-1][1] - ev[0][1]) / (S // 64))
        phase = []
        for tag, t in ev:
            phase.append((tag, t))
            if tag == 2:  # a phase = from the previous release to this release
                tags = [p[0] for p in phase]
                kind = "M" if 6 in tags else ("V" if 3 in tags else None)
                if kind and len(phase) > 2:
                    for (a, ta), (b, tb) in zip(phase, phase[1:]):
                        acc[(kind, f"{NAMES[a]}->{NAMES[b]}")].append(tb - ta)
                    acc[(kind, "total")].append(phase[-1][1] - phase[0][1])
                phase = [(tag, t)]
    print(f"group {grp}: {st.median(tot):.0f} cycles per tile per wave")
    for key in sorted(acc):
        vals = acc[key][2:-2] or acc[key]
        print(f"  {key[0]} {key[1]:18s} median {st.median(vals):6.0f}  (n={len(vals)})")
