"""Level-1 motion-module attention: Q/K/V projection fused into the temporal attention
(vd_motion_qkv_attention) vs the QKV GEMM + vd_temporal_attention, one GPU.

python tools/motion_qkv_bench.py [batch] [positions] -> us per call of each form (default M = 2 x 16 x 4096
rows; 2 512 = a 2-frame rank of the 8-way frame-sharded step, whose motion blocks run position-sharded)."""
import math
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402

B, F, P, C, heads, d = int(sys.argv[1]) if len(sys.argv) > 1 else 2, 16, int(sys.argv[2]) if len(sys.argv) > 2 else 4096, 320, 8, 40
g = torch.Generator(device="cuda").manual_seed(0)
x = (torch.randn(B * F * P, C, device="cuda", generator=g)).to(torch.bfloat16)
w = (torch.randn(3 * C, C, device="cuda", generator=g) * C ** -0.5).to(torch.bfloat16)
sc = 1.0 / math.log2(math.e)
out = torch.empty(B * F * P, C, device="cuda", dtype=torch.bfloat16)


def timeit(fn, reps=20):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def unfused():
    qkv = ops.gemm(x, w)
    ops.temporal_attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], B, F, P, heads, d, scale=sc, out=out)


from vdiff._lib import lib  # noqa: E402

lib().vd_attention_select(33)  # the fused kernels at any grid size (the A/B below)

flop = 2.0 * B * F * P * 3 * C * C
# forms: round 2's kernel (31), round 3's with one position per wave (32 + 40), two per wave (32 + 41)
forms = {"v1": (31, 42), "v2 pw1": (32, 40), "v2 pw2": (32, 41)}


def use(f):
    for sel in forms[f]:
        lib().vd_attention_select(sel)


outs = {}
for f in forms:
    use(f)
    outs[f] = ops.motion_qkv_attention(x, w, B, F, P, heads, d, scale=sc).clone()
res = {f: [] for f in forms}
for _ in range(5):
    for f in forms:
        use(f)
        res[f].append(timeit(lambda: ops.motion_qkv_attention(x, w, B, F, P, heads, d, scale=sc, out=out)))
lib().vd_attention_select(32)
lib().vd_attention_select(42)
lib().vd_attention_select(34)
t_u = timeit(unfused)
for f in forms:
    t_f = sorted(res[f])[2]
    print(f"rows {B * F * P}: fused {f} {t_f:.1f} us ({flop / t_f / 1e6:.0f} TF/s on the projection)", flush=True)
same = all(torch.equal(outs["v1"], outs[f]) for f in forms)
print(f"gemm + temporal attention {t_u:.1f} us; all fused forms bitwise equal: {same}", flush=True)
