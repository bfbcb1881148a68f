"""Leaf modules of the UNetMotionModel tree, named and shaped exactly like
diffusers' so the reference's inspection tooling (experiments/02_architecture_
inspection.py:51-60, experiments/03_trace_forward_pass.py:134-139) and
diffusers-keyed state dicts work unchanged.

Parameters live in the standard torch containers (nn.Linear, nn.Conv2d, ...);
`prepare()` derives the packed device operands the HIP kernels consume
(conv weights [Cout][3][3][Cin], fused QKV, GEGLU row interleave, fp32
biases/affines).  The forward passes run over NHWC row activations (see
`Act`) and call vdiff.ops only.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn as nn

from .. import ops


@dataclass
class Act:
    """An activation as NHWC rows: t[(n*h + y)*w + x, c], n = video*F + frame."""

    t: torch.Tensor
    n: int
    h: int
    w: int

    @property
    def c(self):
        return self.t.shape[1]


def f32(p):
    return None if p is None else p.detach().float().contiguous()


def bf(p):
    return p.detach().to(torch.bfloat16).contiguous()


def prepare_tree(module: nn.Module) -> nn.Module:
    """Run prepare() on every submodule that defines one (children first)."""
    for m in reversed(list(module.modules())):
        if m is not module and hasattr(m, "prepare") and not hasattr(m, "_prepared"):
            m.prepare()
    if hasattr(module, "prepare"):
        module.prepare()
    return module


def pack_conv3x3(wt: torch.Tensor, cin_pad: Optional[int] = None) -> torch.Tensor:
    """[Cout, Cin, 3, 3] -> [Cout, 9*Cin'] with K = tap*Cin' + ci (tap = 3*dy + dx)."""
    co, ci = wt.shape[:2]
    w = wt.detach().permute(0, 2, 3, 1)
    if cin_pad and cin_pad > ci:
        w = torch.nn.functional.pad(w, (0, cin_pad - ci))
    return w.reshape(co, -1).to(torch.bfloat16).contiguous()


def pack_geglu(w: torch.Tensor) -> torch.Tensor:
    """Interleave the hidden/gate halves of GEGLU.proj in 16-row blocks
    (hidden block i, gate block i, ...) so both halves of an output column land
    in one GEMM lane (csrc/gemm.hip VD_ACT_GEGLU)."""
    n = w.shape[0] // 2
    h, g = w[:n], w[n:]
    shp = (n // 16, 16) + tuple(w.shape[1:])
    return torch.stack([h.reshape(shp), g.reshape(shp)], 1).reshape(w.shape).contiguous()


class Timesteps(nn.Module):
    """diffusers:Timesteps(num_channels, flip_sin_to_cos=True, downscale_freq_shift=0)."""

    def __init__(self, num_channels: int):
        super().__init__()
        self.num_channels = num_channels


class TimestepEmbedding(nn.Module):
    def __init__(self, in_channels: int, time_embed_dim: int):
        super().__init__()
        self.linear_1 = nn.Linear(in_channels, time_embed_dim)
        self.act = nn.SiLU()
        self.linear_2 = nn.Linear(time_embed_dim, time_embed_dim)

    def prepare(self):
        self._w1, self._b1 = bf(self.linear_1.weight), f32(self.linear_1.bias)
        self._w2, self._b2 = bf(self.linear_2.weight), f32(self.linear_2.bias)

    def forward_silu(self, t_emb):
        """silu(linear_2(silu(linear_1(t_emb)))) — ResnetBlock2D consumes only silu(temb)."""
        h = ops.gemm(t_emb, self._w1, bias=self._b1, act=ops.ACT_SILU)
        return ops.gemm(h, self._w2, bias=self._b2, act=ops.ACT_SILU)


class SinusoidalPositionalEmbedding(nn.Module):
    """diffusers:SinusoidalPositionalEmbedding — buffer `pe` [1, max_seq_length, dim]."""

    def __init__(self, embed_dim: int, max_seq_length: int = 32):
        super().__init__()
        self.register_buffer("pe", self.table(embed_dim, max_seq_length))

    @staticmethod
    def table(embed_dim: int, max_seq_length: int) -> torch.Tensor:
        pos = torch.arange(max_seq_length, dtype=torch.float32, device="cpu").unsqueeze(1)
        div = torch.exp(torch.arange(0, embed_dim, 2, dtype=torch.float32, device="cpu")
                        * (-math.log(10000.0) / embed_dim))
        pe = torch.zeros(1, max_seq_length, embed_dim, device="cpu")
        pe[0, :, 0::2] = torch.sin(pos * div)
        pe[0, :, 1::2] = torch.cos(pos * div)
        return pe

    def reset_buffers(self):
        self.pe = self.table(self.pe.shape[2], self.pe.shape[1]).to(self.pe.device)


class Attention(nn.Module):
    """diffusers:Attention (AttnProcessor2_0 semantics): to_q/k/v without bias,
    to_out = [Linear(bias), Dropout]."""

    def __init__(self, query_dim: int, heads: int, dim_head: int, cross_attention_dim: Optional[int] = None):
        super().__init__()
        inner = heads * dim_head
        kv_dim = cross_attention_dim or query_dim
        self.heads = heads
        self.dim_head = dim_head
        self.is_cross = cross_attention_dim is not None
        self.to_q = nn.Linear(query_dim, inner, bias=False)
        self.to_k = nn.Linear(kv_dim, inner, bias=False)
        self.to_v = nn.Linear(kv_dim, inner, bias=False)
        self.to_out = nn.ModuleList([nn.Linear(inner, query_dim), nn.Dropout(0.0)])

    # The softmax scale dim_head^-0.5 (and the log2(e) of the kernels' exp2) is
    # folded into the packed to_q rows: the projection GEMM rounds c*q to bf16 ONCE
    # and the attention kernels run with c = scale*log2(e) == 1 exactly (their
    # exp-only path).  `attn_scale` is the scale to hand them.
    attn_scale = 1.0 / math.log2(math.e)

    def prepare(self):
        c = self.dim_head ** -0.5 * math.log2(math.e)
        wq = self.to_q.weight.float() * c
        if self.is_cross:
            self._wq = bf(wq)
            self._wkv = bf(torch.cat([self.to_k.weight, self.to_v.weight], 0))
        else:
            self._wqkv = bf(torch.cat([wq, self.to_k.weight.float(), self.to_v.weight.float()], 0))
        self._wo, self._bo = bf(self.to_out[0].weight), f32(self.to_out[0].bias)

    def project_kv(self, ctx_rows):
        return ops.gemm(ctx_rows, self._wkv)


class GEGLU(nn.Module):
    def __init__(self, dim_in: int, dim_out: int):
        super().__init__()
        self.proj = nn.Linear(dim_in, dim_out * 2)


class FeedForward(nn.Module):
    """diffusers:FeedForward(activation_fn='geglu'): net = [GEGLU, Dropout, Linear]."""

    def __init__(self, dim: int, mult: int = 4):
        super().__init__()
        inner = dim * mult
        self.net = nn.ModuleList([GEGLU(dim, inner), nn.Dropout(0.0), nn.Linear(inner, dim)])

    def prepare(self):
        p = self.net[0].proj
        self._w1 = pack_geglu(bf(p.weight))
        self._b1 = pack_geglu(f32(p.bias))
        self._w2, self._b2 = bf(self.net[2].weight), f32(self.net[2].bias)

    def forward_rows(self, n, res):
        g = ops.gemm(n, self._w1, bias=self._b1, act=ops.ACT_GEGLU)
        return ops.gemm(g, self._w2, bias=self._b2, res=res)


class Downsample2D(nn.Module):
    def __init__(self, channels: int, out_channels: int):
        super().__init__()
        self.conv = nn.Conv2d(channels, out_channels, 3, stride=2, padding=1)

    def prepare(self):
        self._w, self._b = pack_conv3x3(self.conv.weight), f32(self.conv.bias)

    def forward(self, x: Act) -> Act:
        t, h, w = ops.conv3x3(x.t, x.n, x.h, x.w, self._w, stride=2, bias=self._b)
        return Act(t, x.n, h, w)


class Upsample2D(nn.Module):
    def __init__(self, channels: int, out_channels: int):
        super().__init__()
        self.conv = nn.Conv2d(channels, out_channels, 3, padding=1)

    def prepare(self):
        self._w, self._b = pack_conv3x3(self.conv.weight), f32(self.conv.bias)

    def forward(self, x: Act) -> Act:
        t, h, w = ops.conv3x3(x.t, x.n, x.h, x.w, self._w, upsample=True, bias=self._b)
        return Act(t, x.n, h, w)
