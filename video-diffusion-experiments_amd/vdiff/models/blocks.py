"""ResnetBlock2D, Transformer2DModel, AnimateDiffTransformer3D and the
down/mid/up blocks of diffusers' UNetMotionModel,
re-expressed over NHWC row activations and the HIP kernels of vdiff.ops.

Fusions relative to the diffusers op sequence (same math):
  * GroupNorm + SiLU in one apply pass; statistics in a split/finalize pair;
  * the time-embedding broadcast add, the conv bias and the residual add are
    GEMM epilogues of the convolution that produces them;
  * up-block skip concatenation is read from both sources by GN and the conv
    loaders (never materialised);
  * Attention q/k/v are one fused GEMM; GEGLU is a GEMM epilogue; every
    residual add (attention out, FF out, proj_out) is a GEMM epilogue;
  * motion modules attend over frames directly on the NHWC rows (no permute).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from .. import ops
from .layers import (Act, Attention, Downsample2D, FeedForward, SinusoidalPositionalEmbedding,
                     Upsample2D, bf, f32, pack_conv3x3)


class Ctx:
    """Per-forward state shared by every block."""

    def __init__(self, batch, frames, temb_all, ehs_rows, ctx_len, dist=None, kv_cache=None):
        self.batch = batch            # videos in this forward (2 with CFG)
        self.frames = frames          # frames held by THIS rank
        self.temb_all = temb_all      # fp32 [batch, sum(resnet Cout)] = time_emb_proj(silu(temb))
        self.ehs_rows = ehs_rows      # bf16 [batch*ctx_len, D]
        self.ctx_len = ctx_len
        self.dist = dist              # vdiff.dist.FrameShard or None
        self.kv_cache = kv_cache      # {id(attn): kv rows} or None


class ResnetBlock2D(nn.Module):
    def __init__(self, in_channels, out_channels, temb_channels, groups=32, eps=1e-5):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.groups, self.eps = groups, eps
        self.norm1 = nn.GroupNorm(groups, in_channels, eps=eps, affine=True)
        self.conv1 = nn.Conv2d(in_channels, out_channels, 3, padding=1)
        self.time_emb_proj = nn.Linear(temb_channels, out_channels)
        self.norm2 = nn.GroupNorm(groups, out_channels, eps=eps, affine=True)
        self.dropout = nn.Dropout(0.0)
        self.conv2 = nn.Conv2d(out_channels, out_channels, 3, padding=1)
        self.nonlinearity = nn.SiLU()
        self.conv_shortcut = (nn.Conv2d(in_channels, out_channels, 1) if in_channels != out_channels
                              else None)
        self.temb_offset = 0  # column offset into Ctx.temb_all, set by UNetMotionModel.prepare

    def prepare(self):
        self._g1, self._b1 = f32(self.norm1.weight), f32(self.norm1.bias)
        self._g2, self._b2 = f32(self.norm2.weight), f32(self.norm2.bias)
        self._w1, self._c1 = pack_conv3x3(self.conv1.weight), f32(self.conv1.bias)
        self._w2, self._c2 = pack_conv3x3(self.conv2.weight), f32(self.conv2.bias)
        if self.conv_shortcut is not None:
            self._ws = bf(self.conv_shortcut.weight.reshape(self.out_channels, self.in_channels))
            self._bs = f32(self.conv_shortcut.bias)

    def forward(self, x: Act, ctx: Ctx, skip: Optional[Act] = None) -> Act:
        hw = x.h * x.w
        x1 = skip.t if skip is not None else None
        h = ops.group_norm(x.t, x.n, hw, self.groups, self.eps, self._g1, self._b1, silu=True, x1=x1)
        rb = ctx.temb_all[:, self.temb_offset:self.temb_offset + self.out_channels]
        h, _, _ = ops.conv3x3(h, x.n, x.h, x.w, self._w1, bias=self._c1, rowbias=rb,
                              rb_div=ctx.frames * hw)
        h = ops.group_norm(h, x.n, hw, self.groups, self.eps, self._g2, self._b2, silu=True)
        if self.conv_shortcut is not None:
            sc = ops.gemm(x.t, self._ws, a1=x1, bias=self._bs)
        else:
            sc = x.t
        out, _, _ = ops.conv3x3(h, x.n, x.h, x.w, self._w2, bias=self._c2, res=sc)
        return Act(out, x.n, x.h, x.w)


class BasicTransformerBlock(nn.Module):
    """diffusers:BasicTransformerBlock, norm_type='layer_norm'."""

    def __init__(self, dim, heads, dim_head, cross_attention_dim=None, double_self_attention=False,
                 positional_embeddings=None, num_positional_embeddings=None):
        super().__init__()
        self.heads, self.dim_head = heads, dim_head
        self.norm1 = nn.LayerNorm(dim, eps=1e-5)
        self.attn1 = Attention(dim, heads, dim_head)
        self.norm2 = nn.LayerNorm(dim, eps=1e-5)
        self.attn2 = Attention(dim, heads, dim_head,
                               cross_attention_dim=None if double_self_attention else cross_attention_dim)
        self.norm3 = nn.LayerNorm(dim, eps=1e-5)
        self.ff = FeedForward(dim)
        self.pos_embed = (SinusoidalPositionalEmbedding(dim, num_positional_embeddings)
                          if positional_embeddings == "sinusoidal" else None)

    def prepare(self):
        for n in ("norm1", "norm2", "norm3"):
            m = getattr(self, n)
            setattr(self, "_" + n, (f32(m.weight), f32(m.bias)))
        self._pe = f32(self.pos_embed.pe[0]) if self.pos_embed is not None else None

    # spatial: tokens are (image, pixel) rows
    def forward_spatial(self, h, n_img, hw, ctx: Ctx):
        C = h.shape[1]
        d = self.dim_head
        n = ops.layer_norm(h, *self._norm1)
        qkv = ops.gemm(n, self.attn1._wqkv)
        a = ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], n_img, self.heads, hw, hw, d,
                          scale=self.attn1.attn_scale)
        h = ops.gemm(a, self.attn1._wo, bias=self.attn1._bo, res=h)
        n = ops.layer_norm(h, *self._norm2)
        q = ops.gemm(n, self.attn2._wq)
        kv = None if ctx.kv_cache is None else ctx.kv_cache.get(id(self.attn2))
        if kv is None:
            kv = self.attn2.project_kv(ctx.ehs_rows)
            if ctx.kv_cache is not None:
                ctx.kv_cache[id(self.attn2)] = kv
        a = ops.attention(q, kv[:, :C], kv[:, C:], n_img, self.heads, hw, ctx.ctx_len, d,
                          kv_div=ctx.frames, scale=self.attn2.attn_scale)
        h = ops.gemm(a, self.attn2._wo, bias=self.attn2._bo, res=h)
        n = ops.layer_norm(h, *self._norm3)
        return self.ff.forward_rows(n, h)

    # temporal: tokens are (video, frame, position) rows; attention over frames
    def forward_temporal(self, h, batch, frames, positions):
        C = h.shape[1]
        d = self.dim_head
        for attn, nrm in ((self.attn1, self._norm1), (self.attn2, self._norm2)):
            n = ops.layer_norm(h, *nrm, pe=self._pe, pe_div=positions, pe_period=frames)
            qkv = ops.gemm(n, attn._wqkv)
            a = ops.temporal_attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], batch, frames,
                                       positions, self.heads, d, scale=attn.attn_scale)
            h = ops.gemm(a, attn._wo, bias=attn._bo, res=h)
        n = ops.layer_norm(h, *self._norm3)
        return self.ff.forward_rows(n, h)


class Transformer2DModel(nn.Module):
    """Legacy SD-1.5 Transformer2DModel (use_linear_projection=False)."""

    def __init__(self, heads, dim_head, in_channels, cross_attention_dim, groups=32):
        super().__init__()
        inner = heads * dim_head
        self.groups = groups
        self.norm = nn.GroupNorm(groups, in_channels, eps=1e-6, affine=True)
        self.proj_in = nn.Conv2d(in_channels, inner, 1)
        self.transformer_blocks = nn.ModuleList(
            [BasicTransformerBlock(inner, heads, dim_head, cross_attention_dim=cross_attention_dim)])
        self.proj_out = nn.Conv2d(inner, in_channels, 1)

    def prepare(self):
        self._g, self._b = f32(self.norm.weight), f32(self.norm.bias)
        self._wi, self._bi = bf(self.proj_in.weight.flatten(1)), f32(self.proj_in.bias)
        self._wo, self._bo = bf(self.proj_out.weight.flatten(1)), f32(self.proj_out.bias)

    def forward(self, x: Act, ctx: Ctx) -> Act:
        hw = x.h * x.w
        hn = ops.group_norm(x.t, x.n, hw, self.groups, 1e-6, self._g, self._b)
        h = ops.gemm(hn, self._wi, bias=self._bi)
        h = self.transformer_blocks[0].forward_spatial(h, x.n, hw, ctx)
        out = ops.gemm(h, self._wo, bias=self._bo, res=x.t)
        return Act(out, x.n, x.h, x.w)


class AnimateDiffTransformer3D(nn.Module):
    """diffusers:AnimateDiffTransformer3D (motion module).  GroupNorm statistics
    span all F frames of a video; attention runs over frames per position."""

    def __init__(self, heads, dim_head, in_channels, groups=32, max_seq_length=32):
        super().__init__()
        inner = heads * dim_head
        self.groups = groups
        self.norm = nn.GroupNorm(groups, in_channels, eps=1e-6, affine=True)
        self.proj_in = nn.Linear(in_channels, inner)
        self.transformer_blocks = nn.ModuleList([BasicTransformerBlock(
            inner, heads, dim_head, double_self_attention=True, positional_embeddings="sinusoidal",
            num_positional_embeddings=max_seq_length)])
        self.proj_out = nn.Linear(inner, in_channels)

    def prepare(self):
        self._g, self._b = f32(self.norm.weight), f32(self.norm.bias)
        self._wi, self._bi = bf(self.proj_in.weight), f32(self.proj_in.bias)
        self._wo, self._bo = bf(self.proj_out.weight), f32(self.proj_out.bias)

    def forward(self, x: Act, ctx: Ctx) -> Act:
        hw = x.h * x.w
        B, Fl = ctx.batch, ctx.frames
        dist = ctx.dist
        gather = dist.gather_gn_partials if dist is not None else None
        hn = ops.group_norm(x.t, B, Fl * hw, self.groups, 1e-6, self._g, self._b, gather=gather, two_pass=False)
        h = ops.gemm(hn, self._wi, bias=self._bi)
        blk = self.transformer_blocks[0]
        if dist is None:
            h = blk.forward_temporal(h, B, Fl, hw)
        else:
            hp = dist.to_position_shards(h, B, Fl, hw, ops.block_transpose)
            hp = blk.forward_temporal(hp, B, Fl * dist.world, hw // dist.world)
            h = dist.to_frame_shards(hp, B, Fl, hw, ops.block_transpose)
        out = ops.gemm(h, self._wo, bias=self._bo, res=x.t)
        return Act(out, x.n, x.h, x.w)


class _MotionBlockBase(nn.Module):
    def _run_layers(self, x, ctx, skips_in=None):
        outs = []
        attns = getattr(self, "attentions", None)
        for i, res in enumerate(self.resnets):
            skip = skips_in.pop() if skips_in is not None else None
            x = res(x, ctx, skip=skip)
            if attns is not None:
                x = attns[i](x, ctx)
            x = self.motion_modules[i](x, ctx)
            outs.append(x)
        return x, outs


class CrossAttnDownBlockMotion(_MotionBlockBase):
    def __init__(self, in_channels, out_channels, temb_channels, num_layers, heads, cross_dim,
                 motion_heads, add_downsample, groups, eps, max_seq_length):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(in_channels if i == 0 else out_channels, out_channels,
                                                    temb_channels, groups, eps) for i in range(num_layers)])
        self.attentions = nn.ModuleList([Transformer2DModel(heads, out_channels // heads, out_channels,
                                                            cross_dim, groups) for _ in range(num_layers)])
        self.motion_modules = nn.ModuleList([AnimateDiffTransformer3D(
            motion_heads, out_channels // motion_heads, out_channels, groups, max_seq_length)
            for _ in range(num_layers)])
        self.downsamplers = (nn.ModuleList([Downsample2D(out_channels, out_channels)])
                             if add_downsample else None)

    def forward(self, x, ctx):
        x, outs = self._run_layers(x, ctx)
        if self.downsamplers is not None:
            x = self.downsamplers[0](x)
            outs.append(x)
        return x, outs


class DownBlockMotion(CrossAttnDownBlockMotion):
    def __init__(self, in_channels, out_channels, temb_channels, num_layers, motion_heads,
                 add_downsample, groups, eps, max_seq_length):
        nn.Module.__init__(self)
        self.resnets = nn.ModuleList([ResnetBlock2D(in_channels if i == 0 else out_channels, out_channels,
                                                    temb_channels, groups, eps) for i in range(num_layers)])
        self.motion_modules = nn.ModuleList([AnimateDiffTransformer3D(
            motion_heads, out_channels // motion_heads, out_channels, groups, max_seq_length)
            for _ in range(num_layers)])
        self.downsamplers = (nn.ModuleList([Downsample2D(out_channels, out_channels)])
                             if add_downsample else None)


class CrossAttnUpBlockMotion(_MotionBlockBase):
    def __init__(self, resnet_in, out_channels, temb_channels, heads, cross_dim, motion_heads,
                 add_upsample, groups, eps, max_seq_length, with_attn=True):
        super().__init__()
        n = len(resnet_in)
        self.resnets = nn.ModuleList([ResnetBlock2D(ci, out_channels, temb_channels, groups, eps)
                                      for ci in resnet_in])
        if with_attn:
            self.attentions = nn.ModuleList([Transformer2DModel(heads, out_channels // heads, out_channels,
                                                                cross_dim, groups) for _ in range(n)])
        self.motion_modules = nn.ModuleList([AnimateDiffTransformer3D(
            motion_heads, out_channels // motion_heads, out_channels, groups, max_seq_length)
            for _ in range(n)])
        self.upsamplers = (nn.ModuleList([Upsample2D(out_channels, out_channels)])
                           if add_upsample else None)

    def forward(self, x, ctx, skips):
        x, _ = self._run_layers(x, ctx, skips_in=skips)
        if self.upsamplers is not None:
            x = self.upsamplers[0](x)
        return x


class UpBlockMotion(CrossAttnUpBlockMotion):
    def __init__(self, resnet_in, out_channels, temb_channels, motion_heads, add_upsample, groups,
                 eps, max_seq_length):
        super().__init__(resnet_in, out_channels, temb_channels, None, None, motion_heads, add_upsample,
                         groups, eps, max_seq_length, with_attn=False)


class UNetMidBlockCrossAttnMotion(nn.Module):
    def __init__(self, channels, temb_channels, heads, cross_dim, motion_heads, groups, eps,
                 max_seq_length, use_motion=True):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(channels, channels, temb_channels, groups, eps)
                                      for _ in range(2)])
        self.attentions = nn.ModuleList([Transformer2DModel(heads, channels // heads, channels, cross_dim,
                                                            groups)])
        self.motion_modules = (nn.ModuleList([AnimateDiffTransformer3D(
            motion_heads, channels // motion_heads, channels, groups, max_seq_length)])
            if use_motion else None)

    def forward(self, x, ctx):
        x = self.resnets[0](x, ctx)
        x = self.attentions[0](x, ctx)
        if self.motion_modules is not None:
            x = self.motion_modules[0](x, ctx)
        return self.resnets[1](x, ctx)
