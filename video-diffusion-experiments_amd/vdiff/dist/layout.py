"""Placement of the CFG batch and the frames of one video on the GPUs of a node.

SURVEY.md §8e lists two ways to split the denoising step of one 16-frame CFG video:

* frame sharding (``frame``): every rank holds F/N frames of BOTH CFG halves; the 21
  motion modules re-shard with two all-to-alls each (vdiff.dist.FrameShard);
* CFG-parallel x frame-parallel (``cfg-frame``, §8e (ii)): the uncond half runs on ranks
  0..N/2-1, the cond half on N/2..N-1, each half frame-sharded over its N/2 ranks.  The
  two halves are independent videos for every op of the UNet (the motion GroupNorm's
  instance is one (video, group)), so the only new exchange is the CFG combine: after
  the UNet each rank swaps its eps rows with the rank holding the same frames of the other
  half (one all-gather of F/(N/2)·H·W·4 fp32 per step, 256 KB at N = 8), and both ranks
  then apply the same CFG + scheduler update to their replicated latents.

Per-rank compute is identical (2F/N images either way); the difference is the motion
modules' all-to-all.  Its bytes per rank per xGMI link are (local activation)/N_frame_group
spread over N_frame_group-1 peers, so halving the frame group doubles the bytes per link:
``cfg-frame`` only wins where it removes the all-to-all altogether, i.e. at N = 2 (each
rank runs one whole CFG half, no motion-module collective at all).  ``auto`` picks
``cfg-frame`` at N = 2 and ``frame`` otherwise.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .frame_shard import FrameShard


class CfgShard:
    """The CFG pair of a rank: group of 2 ranks holding the same frames of the uncond
    (group rank 0) and cond (group rank 1) halves."""

    def __init__(self, group=None):
        self.group = group
        if dist.get_world_size(group) != 2:
            raise ValueError("a CFG pair has exactly 2 ranks")
        self.index = dist.get_rank(group)  # 0 = uncond, 1 = cond (diffusers' cat order)

    def gather_eps(self, eps: torch.Tensor) -> torch.Tensor:
        """eps rows [R, w] of this rank's half -> [2R, w], uncond rows first, on both ranks
        (the layout the fused CFG+scheduler kernel reads with ncfg = 2)."""
        out = torch.empty((2 * eps.shape[0],) + tuple(eps.shape[1:]), device=eps.device, dtype=eps.dtype)
        dist.all_gather_into_tensor(out, eps.contiguous(), group=self.group)
        return out


class NodeLayout:
    """Group construction for a layout; every rank must build it (new_group is collective)."""

    def __init__(self, layout: str = "auto", frames: int = 16, cfg: bool = True, world=None, rank=None,
                 backend=None, overlap_chunks: int = 1, window: str = "a2a"):
        """overlap_chunks > 1: the motion modules' all-to-alls are chunked over positions and
        overlapped with the transformer blocks on a second stream (FrameShard).  window:
        "a2a" (default) or "kv-gather" (FrameShard: the north star's K/V all-gather)."""
        self.world = dist.get_world_size() if world is None else world
        self.rank = dist.get_rank() if rank is None else rank
        self.layout = layout = self.resolve(layout, self.world, cfg)
        self.cfg_ranks = 2 if layout == "cfg-frame" else 1
        self.frame_ranks = self.world // self.cfg_ranks
        if frames % self.frame_ranks:
            raise ValueError(f"{frames} frames do not shard over {self.frame_ranks} ranks")
        self.half = self.rank // self.frame_ranks          # CFG half this rank runs (cfg-frame)
        self.frame_index = self.rank % self.frame_ranks    # which frame slice
        self.frames_local = frames // self.frame_ranks
        self.frame_shard = None
        self.cfg_shard = None
        if self.world == 1:
            return
        if layout == "frame":
            self.frame_shard = FrameShard(overlap_chunks=overlap_chunks, window=window)
            return
        # every rank creates every group, in the same order
        kw = {} if backend is None else {"backend": backend}
        fgroups = [dist.new_group(list(range(h * self.frame_ranks, (h + 1) * self.frame_ranks)), **kw)
                   for h in range(2)]
        pairs = [dist.new_group([j, self.frame_ranks + j], **kw) for j in range(self.frame_ranks)]
        if self.frame_ranks > 1:
            self.frame_shard = FrameShard(fgroups[self.half], overlap_chunks=overlap_chunks, window=window)
        self.cfg_shard = CfgShard(pairs[self.frame_index])

    @staticmethod
    def resolve(layout: str, world: int, cfg: bool = True) -> str:
        if layout == "auto":
            layout = "cfg-frame" if (cfg and world == 2) else "frame"
        if layout not in ("frame", "cfg-frame"):
            raise ValueError(f"unknown layout {layout!r}")
        if layout == "cfg-frame" and (not cfg or world % 2):
            raise ValueError("cfg-frame needs CFG and an even number of ranks")
        return layout

    def frame_slice(self):
        f0 = self.frame_index * self.frames_local
        return slice(f0, f0 + self.frames_local)

    def describe(self) -> str:
        if self.world == 1:
            return "single-GPU"
        win = ""
        if self.frame_shard is not None:
            win = f" ({self.frame_shard.window}" + (f", overlap {self.frame_shard.chunks}" if self.frame_shard.chunks > 1 else "") + ")"
        if self.layout == "frame":
            return f"frame-shard x{self.world}{win}"
        return f"cfg x2, frame-shard x{self.frame_ranks}{win}"
