"""Leaf modules of the UNetMotionModel tree, named and shaped exactly like
diffusers' so the reference's inspection tooling (experiments/02_architecture_
inspection.py:51-60, experiments/03_trace_forward_pass.py:134-139) and
diffusers-keyed state dicts work unchanged.

Two ways through every module, one set of kernels:

* the fused fast path (`run` methods, NHWC row activations `Act`, epilogue fusions) —
  what the denoising loop and `UNetMotionModel.forward` use;
* the module path (`forward` / `__call__`, diffusers' signatures and tensor layouts:
  (B*F, C, H, W) feature maps as channels-last views of the same rows, (N, S, C) token
  tensors) — what runs when a caller drives modules one by one: a direct
  `motion_modules[i](x, num_frames=F)` (03:182) or a forward-hook trace of the whole
  UNet (utils/forward_tracer.py:177-206), whose hooks then see the diffusers shapes.

The leaf classes below subclass torch's (same class names, same parameters) and only
replace `forward` with the HIP kernels of vdiff.ops; `prepare()` derives the packed
device operands (conv weights [Cout][3][3][Cin], fused QKV, GEGLU row interleave, fp32
biases/affines) that both paths share.
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


def pack_conv3d(wt: torch.Tensor) -> torch.Tensor:
    """[Cout, Cin, kt, ks, ks] -> [Cout, kt*ks*ks*Cin] with K = (dt*ks*ks + tap)*Cin + ci."""
    co = wt.shape[0]
    return wt.detach().permute(0, 2, 3, 4, 1).reshape(co, -1).to(torch.bfloat16).contiguous()


def pack_geglu(w: torch.Tensor) -> torch.Tensor:
    """Interleave the hidden/gate halves of GEGLU.proj in 16-row blocks
    (hidden block i, gate block i, ...) so both halves of an output column land
    in one GEMM lane (csrc/gemm.hip VD_ACT_GEGLU)."""
    n = w.shape[0] // 2
    h, g = w[:n], w[n:]
    shp = (n // 16, 16) + tuple(w.shape[1:])
    return torch.stack([h.reshape(shp), g.reshape(shp)], 1).reshape(w.shape).contiguous()


class LnFold:
    """Linear(LayerNorm(x)) as ONE GEMM over the un-normalised rows (vd_gemm_desc.ln_fold_s):
        W·(gamma∘(x − mean)·rstd + beta) + b = rstd·(W'x − mean·s) + b',
    W' = W∘gamma (column k scaled by gamma[k], rounded to bf16 once), s[n] = Σ_k W'[n][k] (fp32,
    of the bf16 W' so the mean term cancels against the MFMA's own products), b' = b + W·beta.
    The kernel takes mean / rstd of each row from the A fragments it already holds, so the
    normalised rows are never written.  `pack` reorders output rows (GEGLU's interleave) after
    folding; `w` is the Linear's weight in fp32 as the unfolded path would round it (the q rows
    already carry the softmax scale).
    pe ([frames][K], the motion block's sinusoidal table, added after the norm): folded as the row
    bias W·pe[frame] (fp32 [frames][N], `pe_b`), frame = (row / pe_div) % frames as
    vd_layernorm's; only the v6 plan takes a row bias with the fold."""

    def __init__(self, norm: nn.LayerNorm, w: torch.Tensor, b: Optional[torch.Tensor] = None, pack=None,
                 pe: Optional[torch.Tensor] = None):
        g = norm.weight.detach().double()
        be = norm.bias.detach().double()
        wd = w.detach().double()
        wf = wd * g[None, :]
        bp = wd @ be
        if b is not None:
            bp = bp + b.detach().double()
        if pack is not None:
            wf, bp = pack(wf), pack(bp)
        self.w = wf.to(torch.bfloat16).contiguous()
        self.s = self.w.double().sum(1).float().contiguous()
        self.b = bp.float().contiguous()
        self.eps = float(norm.eps)
        self.pe_b = None
        if pe is not None:
            assert pack is None
            self.pe_b = (pe.detach().double().to(wd.device) @ wd.T).float().contiguous()
        self._rb = {}

    def runs(self, M: int, act: int = 0) -> bool:
        return ops.ln_fold_runs(M, self.w, self.s, act=act, rowbias=self.pe_b is not None)

    def slice(self, lo: int, hi: int) -> "LnFold":
        """The same fold for output rows lo .. hi of the Linear (e.g. the Q or the K/V part of a
        fused QKV projection): per output column the arithmetic is unchanged."""
        f = object.__new__(LnFold)
        f.w, f.s, f.b, f.eps = self.w[lo:hi], self.s[lo:hi], self.b[lo:hi], self.eps
        f.pe_b = None if self.pe_b is None else self.pe_b[:, lo:hi].contiguous()
        f._rb = {}
        return f

    def _rowbias(self, M, pe_div, pe_period, pe_off=0):
        """fp32 [ceil(M / pe_div)][N]: row r = W·pe[pe_off + r % pe_period] (cached per shape)."""
        key = ((M + pe_div - 1) // pe_div, pe_period, pe_off)
        t = self._rb.get(key)
        if t is None:
            idx = pe_off + torch.arange(key[0], device=self.pe_b.device) % pe_period
            t = self._rb[key] = self.pe_b[idx].contiguous()
        return t

    def gemm(self, x, act: int = 0, pe_div: int = 1, pe_period: int = 1, pe_off: int = 0):
        if self.pe_b is None:
            return ops.gemm(x, self.w, bias=self.b, act=act, ln_fold=(self.s, self.eps))
        return ops.gemm(x, self.w, bias=self.b, act=act,
                        rowbias=self._rowbias(x.shape[0], pe_div, pe_period, pe_off), rb_div=pe_div,
                        ln_fold=(self.s, self.eps))


class MotionLnFold:
    """The motion block's norm1 / norm2 (+ the sinusoidal PE by frame) folded into the fused
    temporal QKV attention (vd_motion_qkv_attention's ln_fold_tab): W' = W_qkv∘gamma in bf16 and
    the [8 heads][2048] fp32 table — per head the 120 row sums of W' (q | k | v rows of the head)
    and, per frame f < 16, W·(beta + pe[f]) of the same rows."""

    FRAMES = 16

    def __init__(self, norm: nn.LayerNorm, w: torch.Tensor, pe: torch.Tensor, heads: int, d: int):
        C = heads * d
        g = norm.weight.detach().double()
        wd = w.detach().double()
        self.w = (wd * g[None, :]).to(torch.bfloat16).contiguous()
        s = self.w.double().sum(1)
        p = (norm.bias.detach().double()[None, :] + pe[:self.FRAMES].detach().double().to(wd.device)) @ wd.T  # [16][3C]
        tab = torch.zeros(heads, 2048, dtype=torch.float64, device=wd.device)
        cols = torch.arange(3 * d, device=wd.device)
        for h in range(heads):
            n = (cols // d) * C + h * d + cols % d
            tab[h, :3 * d] = s[n]
            tab[h, 3 * d:3 * d * (1 + self.FRAMES)] = p[:, n].reshape(-1)
        self.tab = tab.float().contiguous()
        self.eps = float(norm.eps)


# ------------------------------------------------------------------ layout helpers
def to_bf16_cuda(x: torch.Tensor) -> torch.Tensor:
    if not x.is_cuda:
        raise ValueError("vdiff modules run on the GPU only (got a CPU tensor); no CPU fallback")
    return x if x.dtype == torch.bfloat16 else x.to(torch.bfloat16)


def fmap_rows(x: torch.Tensor):
    """(N, C, H, W) or (B, C, F, H, W) feature map -> its NHWC rows [(..., y, x), C] (a view
    when x is channels-last, e.g. every map the module path produces)."""
    x = to_bf16_cuda(x)
    perm = (0, 2, 3, 1) if x.dim() == 4 else (0, 2, 3, 4, 1)
    xp = x.permute(*perm)
    if not xp.is_contiguous():
        xp = xp.contiguous()
    return xp.reshape(-1, x.shape[1])


def rows_fmap(rows: torch.Tensor, shape) -> torch.Tensor:
    """NHWC rows -> a channels-last view of shape (N, C, H, W) or (B, C, F, H, W)."""
    C = shape[1]
    if len(shape) == 4:
        n, _, h, w = shape
        return rows.view(n, h, w, C).permute(0, 3, 1, 2)
    b, _, f, h, w = shape
    return rows.view(b, f, h, w, C).permute(0, 4, 1, 2, 3)


def token_rows(x: torch.Tensor) -> torch.Tensor:
    """(..., C) token tensor -> contiguous 2-D rows (a view when already contiguous)."""
    x = to_bf16_cuda(x)
    return (x if x.is_contiguous() else x.contiguous()).reshape(-1, x.shape[-1])


def any_rows(x: torch.Tensor):
    """Rows and an inverse for the layouts the module path passes around: token tensors
    (..., C) and channels-last feature maps (N, C, H, W) / (B, C, F, H, W)."""
    if x.dim() in (4, 5):
        return fmap_rows(x), (lambda r, s=tuple(x.shape): rows_fmap(r, s))
    return token_rows(x), (lambda r, s=tuple(x.shape): r.view(s))


def add(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a + b of two equally shaped module-path tensors (the residual adds of diffusers' forwards)."""
    ra, back = any_rows(a)
    rb, _ = any_rows(b)
    return back(ops.rows_add(ra, rb))


# ------------------------------------------------------------------ torch leaves on HIP kernels
class Linear(nn.Linear):
    """torch.nn.Linear (same name and parameters); forward = the HIP GEMM, bias fused."""

    def prepare(self):
        self._w, self._b = bf(self.weight), f32(self.bias)

    def forward(self, x):
        out = ops.gemm(token_rows(x), self._w, bias=self._b)
        return out.view(*x.shape[:-1], self.out_features)


class Conv2d(nn.Conv2d):
    """torch.nn.Conv2d (3x3 pad 1 stride 1/2, or 1x1) on the implicit-GEMM MFMA kernel."""

    out_f32 = False  # conv_out: fp32 eps, as the fused path

    def prepare(self):
        k = self.kernel_size
        if k == (3, 3):
            self._cin_pad = (self.in_channels + 7) // 8 * 8
            self._w = pack_conv3x3(self.weight, cin_pad=self._cin_pad)
        elif k == (1, 1):
            self._cin_pad = self.in_channels
            self._w = bf(self.weight.reshape(self.out_channels, self.in_channels))
        else:
            raise NotImplementedError(f"kernel {k}")
        self._b = f32(self.bias)

    def forward(self, x):
        if x.dim() != 4:
            raise ValueError(f"Conv2d expects (N, C, H, W), got {tuple(x.shape)}")
        n, c, h, w = x.shape
        if c != self._cin_pad:  # conv_in: 4 channels -> 16-byte rows (zero channels 4..7)
            rows = ops.pack_latents(x.float()[:, :, None], dup=1, cpad=self._cin_pad)
        else:
            rows = fmap_rows(x)
        if self.kernel_size == (1, 1):
            out = ops.gemm(rows, self._w, bias=self._b, out_f32=self.out_f32)
            return rows_fmap(out, (n, self.out_channels, h, w))
        out, ho, wo = ops.conv3x3(rows, n, h, w, self._w, stride=self.stride[0], bias=self._b,
                                  out_f32=self.out_f32)
        return rows_fmap(out, (n, self.out_channels, ho, wo))


class Conv3d(nn.Conv3d):
    """torch.nn.Conv3d over (B, C, T, H, W) videos, kernel (kt, ks, ks) with kt in {1, 3},
    ks in {1, 3}, padding (kt//2, ks//2, ks//2), stride (1, s, s) — the north star's 3-D /
    (2+1)D conv (kernel (3,3,3), or (1,3,3) then (3,1,1)) on the implicit-GEMM MFMA kernel
    with temporal taps; (1,3,3) is the reference's per-frame conv."""

    def prepare(self):
        kt, ks, ks2 = self.kernel_size
        if kt not in (1, 3) or ks != ks2 or ks not in (1, 3) or self.padding != (kt // 2, ks // 2, ks // 2) \
                or self.stride[0] != 1 or self.stride[1] != self.stride[2] or self.in_channels % 8:
            raise NotImplementedError(f"Conv3d kernel {self.kernel_size} pad {self.padding} stride {self.stride}")
        self._w, self._b = pack_conv3d(self.weight), f32(self.bias)

    def forward(self, x):
        if x.dim() != 5:
            raise ValueError(f"Conv3d expects (B, C, T, H, W), got {tuple(x.shape)}")
        b, c, t, h, w = x.shape
        kt, ks, _ = self.kernel_size
        out, ho, wo = ops.conv3d(fmap_rows(x), b, t, h, w, self._w, kt=kt, ks=ks, stride=self.stride[1],
                                 bias=self._b)
        return rows_fmap(out, (b, self.out_channels, t, ho, wo))


class GroupNorm(nn.GroupNorm):
    """torch.nn.GroupNorm over (N, C, H, W) images or (B, C, F, H, W) videos (the motion
    module's norm: statistics over C/G channels x F x H x W) on the HIP norm kernels."""

    def prepare(self):
        self._g, self._b = f32(self.weight), f32(self.bias)

    def forward(self, x):
        rows = fmap_rows(x)
        pix = math.prod(x.shape[2:])
        video = x.dim() == 5  # the motion norm: frame-aligned splits, as the fused path's
        out = ops.group_norm(rows, x.shape[0], pix, self.num_groups, self.eps, self._g, self._b, two_pass=not video,
                             n_split=x.shape[2] * ops.gn_splits_per_frame(x.shape[3] * x.shape[4]) if video else None)
        return rows_fmap(out, tuple(x.shape))


class LayerNorm(nn.LayerNorm):
    """torch.nn.LayerNorm over the last dim on the HIP row kernel."""

    def prepare(self):
        self._g, self._b = f32(self.weight), f32(self.bias)

    def forward(self, x):
        return ops.layer_norm(token_rows(x), self._g, self._b, eps=self.eps).view(x.shape)


class SiLU(nn.SiLU):
    def forward(self, x):
        rows, back = any_rows(x)
        return back(ops.silu_rows(rows))


class Dropout(nn.Dropout):
    """p = 0 everywhere in the reference's models (inference): the identity."""

    def forward(self, x):
        if self.p != 0.0 and self.training:
            raise NotImplementedError("dropout with p > 0")
        return x


# ------------------------------------------------------------------ diffusers leaves
class Timesteps(nn.Module):
    """diffusers:Timesteps(num_channels, flip_sin_to_cos=True, downscale_freq_shift=0)."""

    def __init__(self, num_channels: int):
        super().__init__()
        self.num_channels = num_channels

    def forward(self, timesteps):
        return ops.timestep_embed(timesteps.to(torch.float32).contiguous(), self.num_channels)


class TimestepEmbedding(nn.Module):
    def __init__(self, in_channels: int, time_embed_dim: int):
        super().__init__()
        self.linear_1 = Linear(in_channels, time_embed_dim)
        self.act = SiLU()
        self.linear_2 = Linear(time_embed_dim, time_embed_dim)

    def prepare(self):
        self._w1, self._b1 = bf(self.linear_1.weight), f32(self.linear_1.bias)
        self._w2, self._b2 = bf(self.linear_2.weight), f32(self.linear_2.bias)

    def forward_silu(self, t_emb):
        """silu(linear_2(silu(linear_1(t_emb)))) — ResnetBlock2D consumes only silu(temb)."""
        h = ops.gemm(t_emb, self._w1, bias=self._b1, act=ops.ACT_SILU)
        return ops.gemm(h, self._w2, bias=self._b2, act=ops.ACT_SILU)

    def forward(self, sample, condition=None):
        if condition is not None:
            raise NotImplementedError("timestep_cond is not used by the reference's pipeline")
        return self.linear_2(self.act(self.linear_1(sample)))


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

    def prepare(self):
        self._pe = f32(self.pe[0])

    def forward(self, x):
        """x (N, S, C) + pe[:, :S]."""
        return ops.rows_add(token_rows(x), self._pe, y_period=x.shape[1]).view(x.shape)


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
        self.to_q = Linear(query_dim, inner, bias=False)
        self.to_k = Linear(kv_dim, inner, bias=False)
        self.to_v = Linear(kv_dim, inner, bias=False)
        self.to_out = nn.ModuleList([Linear(inner, query_dim), Dropout(0.0)])

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

    def forward(self, hidden_states, encoder_hidden_states=None, attention_mask=None, **cross_attention_kwargs):
        """AttnProcessor2_0 over (N, S, C) tokens: to_q/to_k/to_v modules, softmax(q k^T /
        sqrt(d)) v per head on the flash kernel (the frame-attention kernel when the
        sequence is a motion module's <= 32 frames), to_out modules."""
        if attention_mask is not None:
            raise NotImplementedError("attention_mask is not used by the reference's pipeline")
        x = to_bf16_cuda(hidden_states)
        ctx = x if encoder_hidden_states is None else to_bf16_cuda(encoder_hidden_states)
        N, S, _ = x.shape
        L = ctx.shape[1]
        q, k, v = self.to_q(x), self.to_k(ctx), self.to_v(ctx)
        h, d = self.heads, self.dim_head
        qr, kr, vr = token_rows(q), token_rows(k), token_rows(v)
        scale = d ** -0.5
        if encoder_hidden_states is None and S <= 32:
            o = ops.temporal_attention(qr, kr, vr, N, S, 1, h, d, scale=scale)
        else:
            o = ops.attention(qr, kr, vr, N, h, S, L, d, kv_div=N // ctx.shape[0], scale=scale)
        out = self.to_out[0](o.view(N, S, h * d))
        return self.to_out[1](out)


class GEGLU(nn.Module):
    def __init__(self, dim_in: int, dim_out: int):
        super().__init__()
        self.proj = Linear(dim_in, dim_out * 2)

    def prepare(self):
        self._w = pack_geglu(bf(self.proj.weight))
        self._b = pack_geglu(f32(self.proj.bias))

    def forward(self, hidden_states):
        """h, g = proj(x).chunk(2); h * gelu(g) — one GEMM with the GEGLU epilogue."""
        out = ops.gemm(token_rows(hidden_states), self._w, bias=self._b, act=ops.ACT_GEGLU)
        return out.view(*hidden_states.shape[:-1], self._w.shape[0] // 2)


class FeedForward(nn.Module):
    """diffusers:FeedForward(activation_fn='geglu'): net = [GEGLU, Dropout, Linear]."""

    def __init__(self, dim: int, mult: int = 4):
        super().__init__()
        inner = dim * mult
        self.net = nn.ModuleList([GEGLU(dim, inner), Dropout(0.0), Linear(inner, dim)])

    def prepare(self):
        self._w2, self._b2 = bf(self.net[2].weight), f32(self.net[2].bias)

    def forward_rows(self, n, res, fold: Optional[LnFold] = None):
        """ff(n) + res; with `fold` (the block's norm3 folded into the GEGLU GEMM) n is the
        un-normalised residual stream itself."""
        if fold is not None:
            g = fold.gemm(n, act=ops.ACT_GEGLU)
        else:
            g = ops.gemm(n, self.net[0]._w, bias=self.net[0]._b, act=ops.ACT_GEGLU)
        return ops.gemm(g, self._w2, bias=self._b2, res=res)

    def forward(self, hidden_states):
        for m in self.net:
            hidden_states = m(hidden_states)
        return hidden_states


class Downsample2D(nn.Module):
    def __init__(self, channels: int, out_channels: int):
        super().__init__()
        self.conv = Conv2d(channels, out_channels, 3, stride=2, padding=1)

    def run(self, x: Act) -> Act:
        t, h, w = ops.conv3x3(x.t, x.n, x.h, x.w, self.conv._w, stride=2, bias=self.conv._b)
        return Act(t, x.n, h, w)

    def forward(self, hidden_states, *args, **kwargs):
        return self.conv(hidden_states)


class Upsample2D(nn.Module):
    def __init__(self, channels: int, out_channels: int):
        super().__init__()
        self.conv = Conv2d(channels, out_channels, 3, padding=1)

    def run(self, x: Act) -> Act:
        t, h, w = ops.conv3x3(x.t, x.n, x.h, x.w, self.conv._w, upsample=True, bias=self.conv._b)
        return Act(t, x.n, h, w)

    def forward(self, hidden_states, output_size=None, *args, **kwargs):
        """F.interpolate(x, scale_factor=2.0, mode="nearest") then conv (the fast path folds
        the upsample into the conv's loader instead)."""
        if output_size is not None:
            raise NotImplementedError("output_size")
        n, c, h, w = hidden_states.shape
        up = ops.upsample2x_rows(fmap_rows(hidden_states), n, h, w)
        return self.conv(rows_fmap(up, (n, c, 2 * h, 2 * w)))
