"""The motion-module GroupNorm (instance = a whole video: 2 x 16 frames x 4096 positions at level 1)
as partial / finalize / apply (the current path) vs the two-launch path with per-group records
(F x spf splits per video). python tools/gn_motion_bench.py"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402


def timeit(f, reps=20):
    for _ in range(3):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps * 1e3)
    return best


for B, F, hw, C in [(2, 16, 4096, 320), (2, 16, 1024, 640), (2, 16, 256, 1280), (2, 16, 64, 1280), (2, 2, 4096, 320)]:
    x = torch.randn(B * F * hw, C, device="cuda").to(torch.bfloat16)
    g, b = 1 + 0.1 * torch.randn(C, device="cuda"), 0.1 * torch.randn(C, device="cuda")
    ref = ops.group_norm(x, B, F * hw, 32, 1e-6, g, b, two_pass=False, n_split=F * ops.gn_splits_per_frame(hw))
    line = [f"B={B} F={F} hw={hw} C={C}: 4-pass {timeit(lambda: ops.group_norm(x, B, F * hw, 32, 1e-6, g, b, two_pass=False, n_split=F * ops.gn_splits_per_frame(hw))):6.1f} us"]
    for spf in (1, 2, 4, 8):
        ns = F * min(spf, max(1, hw // 16))
        got = ops.group_norm_2pass(x, B, F * hw, 32, 1e-6, g, b, n_split=ns)
        err = ((got.float() - ref.float()).abs().max()).item()
        line.append(f"2-pass spf={spf} {timeit(lambda: ops.group_norm_2pass(x, B, F * hw, 32, 1e-6, g, b, n_split=ns)):6.1f} us (max|d| {err:.1e})")
    print("  ".join(line), flush=True)
