"""UNetMotionModel — drop-in for diffusers:UNetMotionModel (SD-1.5 +
animatediff-motion-adapter) on MI355X.

Call surface kept from the reference's use (experiments/03_trace_forward_pass.py:
86-115): `unet(sample[B,C,F,H,W], timestep, encoder_hidden_states=
[B,L,D]).sample`, `.config`, `.dtype`, `.device`, and the diffusers module tree
(`down_blocks[i].{resnets,attentions,motion_modules,downsamplers}`, `mid_block`,
`up_blocks`, class `Attention` with `.heads`/`.to_q.in_features`).

Compute: every op runs in libvdiff_hip.so (bf16 activations, fp32
accumulation/statistics, fp32 output).  Call `prepare()` once after moving the
model to the GPU (done lazily by forward).
"""
from __future__ import annotations

from collections import namedtuple
from typing import Optional

import torch
import torch.nn as nn

from .. import ops
from ..config import down_block_plan, get_config, up_block_plan
from .blocks import (CrossAttnDownBlockMotion, CrossAttnUpBlockMotion, Ctx, DownBlockMotion,
                     ResnetBlock2D, UNetMidBlockCrossAttnMotion, UpBlockMotion)
from .layers import Act, Conv2d, GroupNorm, SiLU, TimestepEmbedding, Timesteps, bf, f32, fmap_rows, token_rows


class FrozenDict(dict):
    """diffusers-style config: dict + attribute access."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


UNetMotionOutput = namedtuple("UNetMotionOutput", ["sample"])


def fmap_rows_f32(x):
    """fp32 channels-last (N, C, H, W) -> its NHWC rows (conv_out's output)."""
    return x.permute(0, 2, 3, 1).reshape(-1, x.shape[1])

CIN_PAD = 8  # conv_in input channels padded 4 -> 8 (16-byte NHWC rows)


class UNetMotionModel(nn.Module):
    def __init__(self, config="full"):
        super().__init__()
        cfg = get_config(config)
        self.config = FrozenDict(cfg)
        boc = cfg["block_out_channels"]
        g, eps = cfg["norm_num_groups"], cfg["norm_eps"]
        heads, mheads = cfg["num_attention_heads"], cfg["motion_num_attention_heads"]
        cross, mlen = cfg["cross_attention_dim"], cfg["motion_max_seq_length"]
        tdim = boc[0] * 4
        self.conv_in = Conv2d(cfg["in_channels"], boc[0], 3, padding=1)
        self.time_proj = Timesteps(boc[0])
        self.time_embedding = TimestepEmbedding(boc[0], tdim)
        self.down_blocks = nn.ModuleList()
        for (out_ch, ins, has_attn, down) in down_block_plan(cfg):
            if has_attn:
                blk = CrossAttnDownBlockMotion(ins[0], out_ch, tdim, len(ins), heads, cross, mheads, down,
                                               g, eps, mlen)
            else:
                blk = DownBlockMotion(ins[0], out_ch, tdim, len(ins), mheads, down, g, eps, mlen)
            self.down_blocks.append(blk)
        self.up_blocks = nn.ModuleList()
        for (out_ch, ins, has_attn, up) in up_block_plan(cfg):
            if has_attn:
                blk = CrossAttnUpBlockMotion(ins, out_ch, tdim, heads, cross, mheads, up, g, eps, mlen)
            else:
                blk = UpBlockMotion(ins, out_ch, tdim, mheads, up, g, eps, mlen)
            self.up_blocks.append(blk)
        self.mid_block = UNetMidBlockCrossAttnMotion(boc[-1], tdim, heads, cross, mheads, g, eps, mlen,
                                                     use_motion=cfg.get("use_motion_mid_block", True))
        self.conv_norm_out = GroupNorm(g, boc[0], eps=eps)
        self.conv_act = SiLU()
        self.conv_out = Conv2d(boc[0], cfg["out_channels"], 3, padding=1)
        self.conv_out.out_f32 = True  # eps leaves the UNet in fp32
        self._prepared = False
        self.dist = None  # vdiff.dist.FrameShard when frames are sharded across ranks

    # ------------------------------------------------------------------ utils
    @property
    def dtype(self):
        return next(self.parameters()).dtype

    @property
    def device(self):
        return next(self.parameters()).device

    def resnets_in_order(self):
        return [m for m in self.modules() if isinstance(m, ResnetBlock2D)]

    @torch.no_grad()
    def prepare(self):
        """Pack device operands for the HIP kernels (idempotent; re-run after a weight load)."""
        if not next(self.parameters()).is_cuda:
            raise RuntimeError("UNetMotionModel.prepare(): move the model to the GPU first (no CPU path)")
        for m in self.modules():
            if m is not self and hasattr(m, "prepare"):
                m.prepare()  # every module packs only its own operands
        assert self.conv_in._cin_pad == CIN_PAD
        res = self.resnets_in_order()
        off = 0
        for r in res:
            r.temb_offset = off
            off += r.out_channels
        self._w_temb = bf(torch.cat([r.time_emb_proj.weight for r in res], 0))
        self._b_temb = f32(torch.cat([r.time_emb_proj.bias for r in res], 0))
        self._prepared = True
        return self

    # ------------------------------------------------------------------ core
    def make_ctx(self, t_emb_bf16, ehs_rows, batch, frames, ctx_len, kv_cache=None):
        temb_silu = self.time_embedding.forward_silu(t_emb_bf16)
        temb_all = ops.gemm(temb_silu, self._w_temb, bias=self._b_temb, out_f32=True)
        return Ctx(batch, frames, temb_all, ehs_rows, ctx_len, dist=self.dist, kv_cache=kv_cache)

    def forward_rows(self, x_rows, h, w, ctx: Ctx):
        """Packed NHWC input rows [batch*frames*h*w, 8] -> eps rows fp32 [..., out_channels]."""
        g = self.config["norm_num_groups"]
        n_img = ctx.batch * ctx.frames
        blocks = list(self.down_blocks)
        res0 = None
        if ctx.cfg_dup and ctx.batch % 2 == 0:
            # CFG dedup: both halves of x_rows are the same latents and the same timestep, so
            # conv_in, down_blocks[0].resnets[0] and attentions[0] up to its cross-attention
            # (nothing reads the text embeddings before it) run on one half; their outputs are
            # copied to the other
            # (planned as the whole batch, ops.plan_scaled: the same kernels, the same bits)
            half = x_rows.shape[0] // 2
            t = torch.empty(x_rows.shape[0], self.conv_in.out_channels, device=x_rows.device, dtype=torch.bfloat16)
            with ops.plan_scaled(2):
                ops.conv3x3(x_rows[:half], n_img // 2, h, w, self.conv_in._w, bias=self.conv_in._b, out=t[:half])
                r1 = blocks[0].resnets[0].run(Act(t[:half], n_img // 2, h, w), ctx)
            t[half:].copy_(t[:half])
            res0 = (Act(None, n_img, h, w), r1)  # the full batch is never materialised
        else:
            t, _, _ = ops.conv3x3(x_rows, n_img, h, w, self.conv_in._w, bias=self.conv_in._b)
        x = Act(t, n_img, h, w)
        skips = [x]
        for i, blk in enumerate(blocks):
            x, outs = blk.run(x, ctx, res0=res0) if i == 0 else blk.run(x, ctx)
            skips.extend(outs)
        x = self.mid_block.run(x, ctx)
        for blk in self.up_blocks:
            x = blk.run(x, ctx, skips)
        no = self.conv_norm_out
        hn = ops.group_norm(x.t, x.n, x.h * x.w, g, self.config["norm_eps"], no._g, no._b, silu=True)
        eps, _, _ = ops.conv3x3(hn, x.n, x.h, x.w, self.conv_out._w, bias=self.conv_out._b, out_f32=True)
        return eps

    def has_hooks(self) -> bool:
        """Forward (pre-)hooks registered on any module of the tree, or globally."""
        from torch.nn.modules import module as _m
        if _m._global_forward_hooks or _m._global_forward_pre_hooks:
            return True
        return any(m._forward_hooks or m._forward_pre_hooks for m in self.modules() if m is not self)

    def forward_modules(self, sample, t, ehs):
        """diffusers UNetMotionModel.forward module by module: every block
        and leaf through __call__ with diffusers-layout tensors, all on the HIP kernels — the
        path a forward-hook trace (experiments/03_trace_forward_pass.py:105-113) observes.
        Unsharded only: its motion modules attend over the frames they are given, so under a
        FrameShard they would see the rank's local frames alone."""
        if getattr(self, "dist", None) is not None:
            raise NotImplementedError("forward hooks are not supported under frame sharding "
                                      "(UNetMotionModel.dist is set): the module path has no "
                                      "cross-rank temporal window; detach the hooks or the FrameShard")
        B, Cc, Fr, H, W = sample.shape
        L = ehs.shape[1]
        emb = self.time_embedding(self.time_proj(t))                       # (B, 1280)
        emb = ops.rows_add(None, emb, y_div=Fr, out=torch.empty(B * Fr, emb.shape[1], device=emb.device,
                                                                dtype=torch.bfloat16))  # repeat_interleave(F)
        ehs_rows = token_rows(ehs)
        ehs_rep = torch.empty(B * Fr * L, ehs.shape[2], device=ehs.device, dtype=torch.bfloat16)
        for b in range(B):  # ehs.repeat_interleave(F, 0)
            ops.rows_add(None, ehs_rows[b * L:(b + 1) * L], out=ehs_rep[b * Fr * L:(b + 1) * Fr * L])
        ehs_rep = ehs_rep.view(B * Fr, L, -1)
        x = sample.permute(0, 2, 1, 3, 4).reshape(B * Fr, Cc, H, W)
        h = self.conv_in(x)
        skips = (h,)
        for blk in self.down_blocks:
            if isinstance(blk, DownBlockMotion):
                h, res = blk(h, emb, num_frames=Fr)
            else:
                h, res = blk(h, emb, encoder_hidden_states=ehs_rep, num_frames=Fr)
            skips = skips + res
        h = self.mid_block(h, emb, encoder_hidden_states=ehs_rep, num_frames=Fr)
        for blk in self.up_blocks:
            n = len(blk.resnets)
            res, skips = skips[-n:], skips[:-n]
            if isinstance(blk, UpBlockMotion):
                h = blk(h, res, emb, num_frames=Fr)
            else:
                h = blk(h, res, emb, encoder_hidden_states=ehs_rep, num_frames=Fr)
        h = self.conv_out(self.conv_act(self.conv_norm_out(h)))            # fp32 (B*F, C, H, W)
        return ops.unpack_nhwc(fmap_rows_f32(h), B, h.shape[1], Fr, H, W)

    def forward(self, sample, timestep, encoder_hidden_states, timestep_cond=None, attention_mask=None,
                cross_attention_kwargs=None, added_cond_kwargs=None,
                down_block_additional_residuals=None, mid_block_additional_residual=None,
                return_dict: bool = True, num_frames: Optional[int] = None):
        if not self._prepared:
            self.prepare()
        for unsupported, name in ((timestep_cond, "timestep_cond"), (attention_mask, "attention_mask"),
                                  (down_block_additional_residuals, "down_block_additional_residuals"),
                                  (mid_block_additional_residual, "mid_block_additional_residual")):
            if unsupported is not None:
                raise NotImplementedError(f"{name} is not used by the reference's pipeline")
        dev = self.device
        B, Cc, Fr, H, W = sample.shape
        t = torch.as_tensor(timestep, device=dev)
        if t.ndim == 0:
            t = t[None]
        t = t.to(torch.float32).expand(B).contiguous()
        ehs = encoder_hidden_states.to(device=dev, dtype=torch.bfloat16).contiguous()
        L = ehs.shape[1]
        if self.has_hooks():
            out = self.forward_modules(sample.to(dev, torch.float32), t, ehs)
        else:
            te = ops.timestep_embed(t, self.time_proj.num_channels)
            ctx = self.make_ctx(te, ehs.reshape(B * L, -1), B, Fr, L)
            x_rows = ops.pack_latents(sample.to(dev), dup=1, cpad=CIN_PAD)
            eps_rows = self.forward_rows(x_rows, H, W, ctx)
            out = ops.unpack_nhwc(eps_rows, B, self.config["out_channels"], Fr, H, W)
        out = out.to(sample.dtype) if sample.dtype.is_floating_point else out
        return UNetMotionOutput(out) if return_dict else (out,)
