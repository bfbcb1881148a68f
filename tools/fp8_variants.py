"""fp8 spatial attention (d = 64) variants, accuracy and time: vd_attention_select(34 + v) for
v = 1 (round 1's kernel), 2 (round 3: LDS-DMA ring, lazy offset, row sum on the MFMA), 3 (eager
offset), 4 (row sum on the VALU: the default), 5 (both).  Accuracy: rel-L2 against exact fp32 SDPA on
N(0, 1.5^2) inputs (tests/test_gpu_dit.py's data); time: the DiT shape (64 images x 18 heads,
S = 2304)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd"), str(ROOT / "tests")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402
from vdiff._lib import lib  # noqa: E402

VERS = (1, 2, 3, 4, 5)
for S in (256, 2304):
    g = torch.Generator().manual_seed(S)
    B, heads, d = 2, 3, 64
    D = heads * d
    qkv = (torch.randn(B * S, 3 * D, generator=g) * 1.5).to(torch.bfloat16)
    c = qkv.cuda()
    t = qkv.float().reshape(B, S, 3, heads, d).permute(2, 0, 3, 1, 4)
    want = torch.nn.functional.scaled_dot_product_attention(t[0], t[1], t[2]).permute(0, 2, 1, 3).reshape(B * S, D)
    line = []
    for v in VERS:
        lib().vd_attention_select(34 + v)
        got = ops.attention_fp8(c[:, :D], c[:, D:2 * D], c[:, 2 * D:], B, heads, S, S, d).float().cpu()
        line.append(f"v{v} {((got - want).norm() / want.norm()).item():.4f}")
    print(f"S={S} rel-L2 vs fp32 SDPA: " + "  ".join(line), flush=True)
n, heads, S, d = 64, 18, 2304, 64
D = heads * d
qkv = torch.randn(n * S, 3 * D, device="cuda").to(torch.bfloat16)
q, k, v_ = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
o = torch.empty(n * S, D, device="cuda", dtype=torch.bfloat16)
ws = ops.attention_fp8_quant(q, k, v_, n, heads, S, S, d)
st = torch.cuda.current_stream().cuda_stream
flop = 4.0 * n * heads * S * S * d
res = {v: [] for v in VERS}
for rep in range(4):
    for v in VERS:
        lib().vd_attention_select(34 + v)
        args = (ws["q8"].data_ptr(), ws["k8"].data_ptr(), ws["ld8"], ws["qs"].data_ptr(), ws["ks"].data_ptr(),
                ws["vt8"].data_ptr(), ws["vs"].data_ptr(), o.data_ptr(), o.stride(0), n, heads, S, S, d, d ** -0.5, st)
        lib().vd_attention_fp8(*args)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            lib().vd_attention_fp8(*args)
        e1.record()
        e1.synchronize()
        res[v].append(e0.elapsed_time(e1) / 5)
lib().vd_attention_select(38)
for v in VERS:
    ms = sorted(res[v])[1]
    print(f"v{v}: {ms:.4f} ms  {flop / ms / 1e9:.1f} TF/s ({flop / ms / 1e9 / 5000:.3f} of the fp8 dense peak)", flush=True)
