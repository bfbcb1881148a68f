"""Same-process A/B of the attention kernels that vd_attention_ex selects per call (kernel ids:
1 the 16x16x32 flash kernel, 2 flash32, 3 flash40 at d = 40 / flash80 at d = 80; 4 = flash48 on
branch flash48-pv16-experiment, profiles/r06_flash48_refuted.txt), on the level-1 shape (32 images
x 8 heads, S = 4096, d = 40) or with --d 80 --S 1024 the level-2 one, the model's unit scale, arms
interleaved, each launch incl. the exact fix-up launch that follows flash40.  Also prints the arms'
output differences (fp32 outputs).

    python tools/attn_kernel_ab.py [--arms 3,2] [--d 40 --S 4096] [--rounds 15]      # GPU box
"""
from __future__ import annotations

import argparse
import math
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-diffusion-experiments_amd"))

NAMES = {0: "auto", 1: "v1", 2: "flash32", 3: "flash40", 4: "flash48"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", default="3,2")
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--imgs", type=int, default=32)
    ap.add_argument("--d", type=int, default=40)
    ap.add_argument("--S", type=int, default=4096)
    ap.add_argument("--skv", type=int, default=0, help="keys (default S: self-attention)")
    ap.add_argument("--kvdiv", type=int, default=1, help="query batches per K/V batch (cross-attention: frames)")
    args = ap.parse_args()
    import torch
    from vdiff import ops

    arms = [int(a) for a in args.arms.split(",")]
    imgs, heads, S, d = args.imgs, 8, args.S, args.d
    C = heads * d
    g = torch.Generator(device="cuda").manual_seed(0)
    skv, kvd = (args.skv or S), args.kvdiv
    q = (torch.randn(imgs * S, C, device="cuda", generator=g) * 1.5 * d ** -0.5 * math.log2(math.e)).to(torch.bfloat16)
    k = (torch.randn(imgs // kvd * skv, C, device="cuda", generator=g) * 1.5).to(torch.bfloat16)
    v = (torch.randn(imgs // kvd * skv, C, device="cuda", generator=g) * 1.5).to(torch.bfloat16)
    sc = 1.0 / math.log2(math.e)
    out = torch.empty(imgs * S, C, device="cuda", dtype=torch.bfloat16)

    def call(a, o=out, f32=False):
        ops.attention(q, k, v, imgs, heads, S, skv, d, kv_div=kvd, scale=sc, out=o, out_f32=f32, kernel=NAMES[a])

    ref = {}
    for a in arms:
        o32 = torch.empty(imgs * S, C, device="cuda", dtype=torch.float32)
        call(a, o32, True)
        call(a)
        torch.cuda.synchronize()
        ref[a] = (o32, out.clone())
    a0 = arms[0]
    for a in arms[1:]:
        d32 = (ref[a][0] - ref[a0][0]).abs()
        rel = (d32 / ref[a0][0].abs().clamp_min(1e-3)).max().item()
        nbf = (ref[a][1] != ref[a0][1]).float().mean().item()
        print(f"{NAMES[a]} vs {NAMES[a0]}: fp32 out max |diff| {d32.max().item():.3e} (max rel {rel:.3e}); "
              f"bf16 out elements that differ {nbf:.2e}", flush=True)
    fl = 4.0 * S * skv * d * heads * imgs
    res = {a: [] for a in arms}
    for r in range(args.rounds + 1):
        for a in arms:
            for _ in range(3):
                call(a)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                call(a)
            e1.record()
            torch.cuda.synchronize()
            if r:
                res[a].append(e0.elapsed_time(e1) * 100.0)
    base = sorted(res[a0])[len(res[a0]) // 2]
    for a, t in res.items():
        t = sorted(t)
        med = t[len(t) // 2]
        print(f"{NAMES[a] if d == 40 or a != 3 else 'flash80':8s} median {med:7.1f} us ({med / base - 1:+6.1%})  min {t[0]:.1f} max {t[-1]:.1f}  "
              f"{fl / med / 1e6:7.1f} TF/s = {fl / med / 1e6 / 2500:.4f} of 2.5 PF", flush=True)


if __name__ == "__main__":
    main()
