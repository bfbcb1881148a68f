"""VAE mid-block attention (d = 512, one head, S = 4096 per frame, 16 frames): round 2's
materialised path (per frame: S = q.k^T GEMM into 64 MB of fp32 -> vd_softmax_rows -> P.V GEMM)
against round 3's flash512_kernel (vd_attention d = 512), same inputs, interleaved rounds.

    python tools/vae_attn_ab.py [rounds]
"""
import math
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
n, S, C = 16, 4096, 512
g = torch.Generator(device="cuda").manual_seed(1)
qkv = torch.randn(n * S, 3 * C, device="cuda", generator=g)
qkv[:, :C] *= C ** -0.5 * math.log2(math.e) * 0.5
qkv = qkv.to(torch.bfloat16)
q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
vt = v.t().contiguous()  # round 2 produced V^T directly from GEMM(W_v, rows)
o_old = torch.empty(n * S, C, device="cuda", dtype=torch.bfloat16)
s = torch.empty(S, S, device="cuda", dtype=torch.float32)
flop = 4.0 * S * S * C * n


def old():
    for i in range(n):
        r = slice(i * S, (i + 1) * S)
        ops.gemm(q[r], k[r], out=s, out_f32=True)
        p = ops.softmax_rows(s)
        ops.gemm(p, vt[:, r], out=o_old[r])
    return o_old


def new():
    return ops.attention(q, k, v, n, 1, S, S, C, scale=1.0 / math.log2(math.e))


res = {"materialised (GEMM, softmax_rows, GEMM per frame)": [], "flash512_kernel": []}
fns = list(zip(res, (old, new)))
for _ in range(2):
    for _, f in fns:
        f()
torch.cuda.synchronize()
for _ in range(rounds):
    for name, f in fns:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            f()
        e1.record()
        e1.synchronize()
        res[name].append(e0.elapsed_time(e1) / 3)
for name, ms in res.items():
    ms = sorted(ms)
    med = ms[len(ms) // 2]
    print(f"{name:52s} median {med * 1e3:8.1f} us  {flop / med / 1e9:7.1f} TF/s ({flop / med / 1e9 / 2500:.3f} of peak)")
a, b = old().float(), new().float()
print(f"rel-L2 materialised vs flash: {((a - b).norm() / a.norm()).item():.2e}")
