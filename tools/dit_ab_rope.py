"""In-process A/B of the RoPE fusions on the full DiT config (BASELINE config 5 shapes):
the same model and inputs, graph-captured CFG+DDIM loop, fuse_rope False/True alternated so
box-to-box variance cancels.  Usage: python tools/dit_ab_rope.py [--fp8] [--rounds 2]."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "video-diffusion-experiments_amd"))
from vdiff.sched.ddim import DDIMScheduler  # noqa: E402
from vdiff.models.dit import DIT_FULL, DiT3DModel, DiTDenoiseLoop, init_dit_state_dict  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    cfg = dict(DIT_FULL)
    model = DiT3DModel(cfg, init_dit_state_dict(cfg, seed=0, device="cuda"), device="cuda", attn_fp8=args.fp8)
    F, H = cfg["num_frames"], cfg["sample_size"]
    lat = torch.randn((1, 4, F, H, H), generator=torch.Generator().manual_seed(42)).cuda()
    ehs = torch.randn((2, 77, cfg["text_dim"]), generator=torch.Generator().manual_seed(1)).cuda()
    res = {False: [], True: []}
    for _ in range(args.rounds):
        for fuse in (False, True):
            model.fuse_rope = fuse
            s = DDIMScheduler(beta_schedule="linear", steps_offset=1, clip_sample=False)
            s.set_timesteps(50)
            loop = DiTDenoiseLoop(model, s, lat, ehs, 7.5).prime()
            loop.run(2)
            torch.cuda.synchronize()
            t = time.perf_counter()
            loop.run(args.steps)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t) / args.steps * 1e3
            res[fuse].append(ms)
            print(f"[ab] fp8={args.fp8} fuse_rope={fuse}: {ms:.2f} ms/step", flush=True)
            del loop
            torch.cuda.empty_cache()
    print(f"[ab] fp8={args.fp8} best unfused {min(res[False]):.2f} ms, fused {min(res[True]):.2f} ms, "
          f"saved {min(res[False]) - min(res[True]):.2f} ms/step", flush=True)


if __name__ == "__main__":
    main()
