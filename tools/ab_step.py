"""A/B of a host-side policy on the full denoising step, in one process on one box (box-to-box
variance is ~3 %): python tools/ab_step.py gn [frames]  — alternates the GroupNorm policy
(two-launch image norms vs partial/finalize/apply everywhere) over captured-graph steps."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import DDIMScheduler, DenoiseLoop, ops  # noqa: E402
from vdiff.weights import materialize_synthetic  # noqa: E402

frames = int(sys.argv[2]) if len(sys.argv) > 2 else 16
unet = materialize_synthetic("full", device="cuda", seed=0)
unet.prepare()
lat = torch.randn((1, 4, frames, 64, 64), generator=torch.Generator().manual_seed(42)).cuda()
ehs = torch.randn((2, 77, 768), generator=torch.Generator().manual_seed(1)).cuda()
sched = DDIMScheduler(beta_schedule="linear", steps_offset=1, clip_sample=False)
sched.set_timesteps(50)
orig = ops.group_norm


def four_pass(*a, **k):
    k["two_pass"] = False
    return orig(*a, **k)


loops = {}
for name, fn in (("two-launch", orig), ("four-launch", four_pass)):
    ops.group_norm = fn
    import vdiff.models.blocks as B  # noqa: E402  (modules hold `ops`, so patching ops is enough)
    loops[name] = DenoiseLoop(unet, sched, lat, ehs, 7.5).prime()
ops.group_norm = orig
res = {k: [] for k in loops}
for rep in range(4):
    for name, lp in loops.items():
        lp.reset(lat.to(lp.lat.device))  # 13 steps per round: restart the 50-step schedule
        lp.run(3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lp.run(10)
        torch.cuda.synchronize()
        res[name].append((time.perf_counter() - t0) / 10 * 1e3)
for k, v in res.items():
    print(f"{k:12s} frames={frames} ms/step: " + " ".join(f"{x:.2f}" for x in v) + f"  min {min(v):.2f}", flush=True)
