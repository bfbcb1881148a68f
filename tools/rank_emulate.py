"""Per-rank step time of an N-way frame-sharded run, emulated on ONE GPU.

    python tools/rank_emulate.py --world 8 --chunks 1 2 4 [--comm copy|none]

Rank 0 of the "frame" layout: 16/N frames of both CFG halves, the motion modules'
re-shards exactly as FrameShard issues them (same transposes, same chunking, same
side stream), but every collective replaced by a device copy of the same size
(`--comm copy`: the local share of the traffic) or by nothing (`--comm none`).
The numerics are not a video's (the copies do not exchange frames); the launches,
shapes and stream structure are rank 0's.  This isolates what chunking costs in
compute (smaller GEMMs, more launches) from what it can hide (the all-to-all time,
DESIGN.md §6's communication budget)."""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]

import torch  # noqa: E402

from vdiff import DDIMScheduler, DenoiseLoop  # noqa: E402
from vdiff.dist import FrameShard  # noqa: E402
from vdiff.weights import materialize_synthetic  # noqa: E402


class EmulatedShard(FrameShard):
    def __init__(self, world, chunks, comm, window="a2a"):
        self.group, self.world, self.rank, self.chunks, self.window = None, world, 0, chunks, window
        self._side = {}
        self.comm = comm

    def _a2a(self, x, out=None):
        out = torch.empty_like(x) if out is None else out
        if self.comm == "copy":
            out.copy_(x)
        return out

    def _all_gather(self, x):
        out = torch.empty((self.world * x.shape[0],) + tuple(x.shape[1:]), device=x.device, dtype=x.dtype)
        if self.comm == "copy":
            out.view(self.world, *x.shape).copy_(x.unsqueeze(0).expand(self.world, *x.shape))
        return out

    def gather_gn_partials(self, ws):
        return ws.repeat_interleave(self.world, dim=1) if self.world > 1 else ws

    def gather_gn_records(self, ws):  # the all-gather's output write, as _all_gather
        out = torch.empty((self.world,) + tuple(ws.shape), device=ws.device, dtype=ws.dtype)
        if self.comm == "copy":
            out.copy_(ws.unsqueeze(0).expand(self.world, *ws.shape))
        return out

    def all_gather_frames(self, x):
        return x


def ab_fused(args):
    """Both arms captured once on one model, then replayed in alternating rounds (one box, one
    process: the guide's rule 24)."""
    unet = materialize_synthetic("full", device="cuda", seed=0)
    fl = args.frames // args.world
    lat = torch.randn(1, 4, fl, 64, 64, device="cuda")
    ehs = torch.randn(2, 77, unet.config["cross_attention_dim"], device="cuda")
    s = DDIMScheduler(beta_schedule="linear", steps_offset=1, clip_sample=False)
    s.set_timesteps(50)
    ts = s.timesteps.repeat(40)
    loops = {}
    for arm in ("fused", "transposes"):
        sh = EmulatedShard(args.world, 1, args.comm, args.window)
        sh.fused = arm == "fused"
        unet.dist = sh
        unet.prepare()
        loops[arm] = DenoiseLoop(unet, s, lat.clone(), ehs, 7.5, timesteps=ts, use_graph=True).prime()
        assert loops[arm].graph is not None, loops[arm].graph_error
        loops[arm].run(3)
    res = {a: [] for a in loops}
    for _ in range(args.ab_fused):
        for arm, lp in loops.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            lp.run(args.steps)
            torch.cuda.synchronize()
            res[arm].append(1e3 * (time.perf_counter() - t0) / args.steps)
    for arm, v in res.items():
        v = sorted(v)
        print(f"world {args.world} {arm}: median {v[len(v) // 2]:.3f} ms/step, min {v[0]:.3f} (rounds {len(v)})")
    print(json.dumps({"world": args.world, "ab": {a: sorted(v) for a, v in res.items()}}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--chunks", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--comm", default="copy", choices=["copy", "none"])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--window", default="a2a", choices=["a2a", "kv-gather"])
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--mq", default="on", choices=["on", "off", "both"],
                    help="motion-module Q/K/V projection fused into the temporal attention (A/B with both)")
    ap.add_argument("--ab-fused", type=int, default=0,
                    help="same-process A/B of FrameShard.fused (the round-5 re-shard without transposes) "
                         "against the transposes: N alternating rounds of --steps steps per arm")
    args = ap.parse_args()
    if args.ab_fused:
        return ab_fused(args)
    unet = materialize_synthetic("full", device="cuda", seed=0)
    fl = args.frames // args.world
    lat = torch.randn(1, 4, fl, 64, 64, device="cuda")
    ehs = torch.randn(2, 77, unet.config["cross_attention_dim"], device="cuda")
    s = DDIMScheduler(beta_schedule="linear", steps_offset=1, clip_sample=False)
    s.set_timesteps(50)
    ts = s.timesteps.repeat(2)
    res = {}
    from vdiff.models.blocks import BasicTransformerBlock
    blocks = [m for m in unet.modules() if isinstance(m, BasicTransformerBlock)]
    runs = [(c, mq) for c in args.chunks for mq in ({"on": [True], "off": [False], "both": [True, False]}[args.mq])]
    for c, mq in runs:
        for m in blocks:
            m.fuse_qkv_attention = mq
        unet.dist = EmulatedShard(args.world, c, args.comm, args.window) if args.world > 1 else None
        unet.prepare()
        loop = DenoiseLoop(unet, s, lat, ehs, 7.5, timesteps=ts, use_graph=True).prime()
        assert loop.graph is not None, loop.graph_error
        loop.run(3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        loop.run(args.steps)
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / args.steps
        res[f"{c}{'' if mq else ' (mq off)'}"] = round(ms, 3)
        print(f"world {args.world} frames/rank {fl} window {args.window} chunks {c} comm {args.comm}"
              f"{'' if mq else ' qkv-attn unfused'}: {ms:.3f} ms/step", flush=True)
        del loop
    print(json.dumps({"world": args.world, "frames_local": fl, "window": args.window, "comm": args.comm,
                      "ms_per_step": res}))


if __name__ == "__main__":
    main()
