"""ResnetBlock2D, Transformer2DModel, AnimateDiffTransformer3D and the
down/mid/up blocks of diffusers' UNetMotionModel,
re-expressed over NHWC row activations and the HIP kernels of vdiff.ops.

Every block has two entry points over the same kernels (see layers.py):
  * `run(...)` — the fused fast path on `Act` rows.  Fusions relative to the diffusers
    op sequence (same math): GroupNorm + SiLU in one apply pass; the time-embedding
    broadcast add, the conv bias and the residual add are GEMM epilogues; up-block skip
    concatenation is read from both sources by GN and the conv loaders (never
    materialised); Attention q/k/v are one fused GEMM with the softmax scale folded into
    q; GEGLU is a GEMM epilogue; every residual add (attention out, FF out, proj_out) is
    a GEMM epilogue; motion modules attend over frames directly on the NHWC rows.
  * `forward(...)` — diffusers' signature and control flow, module by module through
    `__call__` (so forward hooks fire with the diffusers tensor shapes: spatial tokens
    (B*F, H*W, C), temporal tokens (B*H*W, F, C) — experiments/03_trace_forward_pass.py:
    160-169), each leaf on its HIP kernel.
"""
from __future__ import annotations

import contextlib
import math
from collections import namedtuple
from typing import Optional

import torch
import torch.nn as nn

from .. import ops
from .layers import (Act, Attention, Conv2d, Downsample2D, Dropout, FeedForward, GroupNorm, LayerNorm, LnFold,
                     Linear, MotionLnFold, pack_geglu, SiLU, SinusoidalPositionalEmbedding, Upsample2D, add, bf, f32, fmap_rows,
                     rows_fmap, token_rows)

Transformer2DModelOutput = namedtuple("Transformer2DModelOutput", ["sample"])


class Ctx:
    """Per-forward state shared by every block (fast path)."""

    def __init__(self, batch, frames, temb_all, ehs_rows, ctx_len, dist=None, kv_cache=None):
        self.batch = batch            # videos in this forward (2 with CFG)
        self.frames = frames          # frames held by THIS rank
        self.temb_all = temb_all      # fp32 [batch, sum(resnet Cout)] = time_emb_proj(silu(temb))
        self.ehs_rows = ehs_rows      # bf16 [batch*ctx_len, D]
        self.ctx_len = ctx_len
        self.dist = dist              # vdiff.dist.FrameShard or None
        self.kv_cache = kv_cache      # {id(attn): kv rows} or None
        # the two CFG halves of the input are the same latents (DenoiseLoop): everything before
        # the first cross-attention — conv_in and down_blocks[0].resnets[0] — runs on one half
        self.cfg_dup = False


def concat_channels(a, b):
    """torch.cat([a, b], dim=1) of two channels-last feature maps (module path)."""
    n, ca, h, w = a.shape
    cb = b.shape[1]
    out = torch.empty(n * h * w, ca + cb, device=a.device, dtype=torch.bfloat16)
    ops.rows_add(None, fmap_rows(a), out=out[:, :ca])
    ops.rows_add(None, fmap_rows(b), out=out[:, ca:])
    return rows_fmap(out, (n, ca + cb, h, w))


class ResnetBlock2D(nn.Module):
    def __init__(self, in_channels, out_channels, temb_channels, groups=32, eps=1e-5):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.groups, self.eps = groups, eps
        self.norm1 = GroupNorm(groups, in_channels, eps=eps, affine=True)
        self.conv1 = Conv2d(in_channels, out_channels, 3, padding=1)
        self.time_emb_proj = Linear(temb_channels, out_channels)
        self.norm2 = GroupNorm(groups, out_channels, eps=eps, affine=True)
        self.dropout = Dropout(0.0)
        self.conv2 = Conv2d(out_channels, out_channels, 3, padding=1)
        self.nonlinearity = SiLU()
        self.conv_shortcut = (Conv2d(in_channels, out_channels, 1) if in_channels != out_channels
                              else None)
        self.temb_offset = 0  # column offset into Ctx.temb_all, set by UNetMotionModel.prepare

    def run(self, x: Act, ctx: Ctx, skip: Optional[Act] = None) -> Act:
        hw = x.h * x.w
        x1 = skip.t if skip is not None else None
        n1, n2 = self.norm1, self.norm2
        h = ops.group_norm(x.t, x.n, hw, self.groups, self.eps, n1._g, n1._b, silu=True, x1=x1)
        rb = ctx.temb_all[:, self.temb_offset:self.temb_offset + self.out_channels]
        h, _, _ = ops.conv3x3(h, x.n, x.h, x.w, self.conv1._w, bias=self.conv1._b, rowbias=rb,
                              rb_div=ctx.frames * hw)
        h = ops.group_norm(h, x.n, hw, self.groups, self.eps, n2._g, n2._b, silu=True)
        if self.conv_shortcut is not None:
            sc = ops.gemm(x.t, self.conv_shortcut._w, a1=x1, bias=self.conv_shortcut._b)
        else:
            sc = x.t
        out, _, _ = ops.conv3x3(h, x.n, x.h, x.w, self.conv2._w, bias=self.conv2._b, res=sc)
        return Act(out, x.n, x.h, x.w)

    def forward(self, input_tensor, temb, *args, **kwargs):
        """diffusers ResnetBlock2D.forward (output_scale_factor 1, pre-norm, time_embedding_norm
        "default"): temb (B*F, temb_channels) is broadcast over each image's pixels."""
        h = self.nonlinearity(self.norm1(input_tensor))
        h = self.conv1(h)
        t = self.time_emb_proj(self.nonlinearity(temb))               # (B*F, Cout)
        n, c, hh, ww = h.shape
        h = rows_fmap(ops.rows_add(fmap_rows(h), token_rows(t), y_div=hh * ww), tuple(h.shape))
        h = self.dropout(self.nonlinearity(self.norm2(h)))
        h = self.conv2(h)
        sc = self.conv_shortcut(input_tensor) if self.conv_shortcut is not None else input_tensor
        return add(sc, h)


class BasicTransformerBlock(nn.Module):
    """diffusers:BasicTransformerBlock, norm_type='layer_norm'."""

    def __init__(self, dim, heads, dim_head, cross_attention_dim=None, double_self_attention=False,
                 positional_embeddings=None, num_positional_embeddings=None):
        super().__init__()
        self.heads, self.dim_head = heads, dim_head
        self.norm1 = LayerNorm(dim, eps=1e-5)
        self.attn1 = Attention(dim, heads, dim_head)
        self.norm2 = LayerNorm(dim, eps=1e-5)
        self.attn2 = Attention(dim, heads, dim_head,
                               cross_attention_dim=None if double_self_attention else cross_attention_dim)
        self.norm3 = LayerNorm(dim, eps=1e-5)
        self.ff = FeedForward(dim)
        self.pos_embed = (SinusoidalPositionalEmbedding(dim, num_positional_embeddings)
                          if positional_embeddings == "sinusoidal" else None)
        self.fuse_qkv_attention = True  # run_temporal: ops.motion_qkv_attention where it applies

    def _nrm(self, i):
        m = getattr(self, f"norm{i}")
        return m._g, m._b

    def prepare(self):
        """LayerNorms folded into the GEMM that consumes them (LnFold, vd_gemm_desc.ln_fold_s)
        wherever the library's plan takes the shape (the weight-stationary K = 320 GEMM): the
        spatial block's norm1 -> fused QKV, norm2 -> to_q, norm3 -> GEGLU; the motion block's
        norm3 -> GEGLU (its norm1 / norm2 add the positional encoding after the norm and feed
        the fused temporal QKV kernel)."""
        self._fold = {}
        proj = self.ff.net[0].proj
        cand = {3: (self.norm3, proj.weight.float(), proj.bias, pack_geglu, ops.ACT_GEGLU)}
        if self.attn2.is_cross:
            c = self.attn1.dim_head ** -0.5 * math.log2(math.e)  # Attention.prepare's q scale
            a1 = self.attn1
            cand[1] = (self.norm1, torch.cat([a1.to_q.weight.float() * c, a1.to_k.weight.float(),
                                              a1.to_v.weight.float()], 0), None, None, ops.ACT_NONE)
            cand[2] = (self.norm2, self.attn2.to_q.weight.float() * c, None, None, ops.ACT_NONE)
        for i, (nrm, w, b, pack, act) in cand.items():
            if ops.ln_fold_shape_ok(w.shape[0], w.shape[1], act=act):
                self._fold[i] = (LnFold(nrm, w, b, pack=pack), act)
        # the motion block's norm1 / norm2 + PE folded into the fused temporal QKV attention
        # (level 1: 8 heads of d = 40, 16 frames)
        self._mfold = {}
        if self.pos_embed is not None and self.heads * self.dim_head == 320 and self.dim_head == 40:
            c = self.attn1.dim_head ** -0.5 * math.log2(math.e)
            for i, (nrm, attn) in ((1, (self.norm1, self.attn1)), (2, (self.norm2, self.attn2))):
                w = torch.cat([attn.to_q.weight.float() * c, attn.to_k.weight.float(), attn.to_v.weight.float()], 0)
                self._mfold[i] = MotionLnFold(nrm, w, self.pos_embed.pe[0], self.heads, self.dim_head)
        # elsewhere (levels 2-4: d = 80 / 160, no fused QKV attention) norm1 / norm2 + PE fold into
        # the QKV GEMM, the PE as the row bias W·pe[frame] (LnFold(pe=...), the v6 plan)
        self._pfold = {}
        self._pfold_split = {}  # the kv-gather window's Q and K/V slices of a _pfold (run_temporal_gathered)
        if self.pos_embed is not None:
            c = self.attn1.dim_head ** -0.5 * math.log2(math.e)
            for i, (nrm, attn) in ((1, (self.norm1, self.attn1)), (2, (self.norm2, self.attn2))):
                w = torch.cat([attn.to_q.weight.float() * c, attn.to_k.weight.float(), attn.to_v.weight.float()], 0)
                if ops.ln_fold_shape_ok(w.shape[0], w.shape[1], rowbias=True):
                    self._pfold[i] = LnFold(nrm, w, pe=self.pos_embed.pe[0])

    def temporal_fold(self, i, batch, frames, positions):
        """How norm i (+ PE) of a temporal block over (batch, frames, positions) rows folds: ("m", f)
        into the fused QKV attention, ("p", f) into the QKV GEMM with the PE as a row bias, or None
        (the norm is written) — one decision for the producer (_out_norm, the motion module's
        proj_in) and the consumer (run_temporal)."""
        mf = self.mfold(i, batch, frames, positions)
        if mf is not None:
            return "m", mf
        if self.fuse_qkv_attention and ops.motion_qkv_takes(batch, frames, positions, self.heads, self.dim_head):
            return None  # the fused attention runs on normalised rows
        f = getattr(self, "_pfold", {}).get(i)
        return ("p", f) if f is not None and f.runs(batch * frames * positions) else None

    def mfold(self, i, batch, frames, positions):
        """norm i's MotionLnFold when the fused temporal QKV attention takes this shape, else None."""
        f = getattr(self, "_mfold", {}).get(i)
        if f is None or not self.fuse_qkv_attention or frames != MotionLnFold.FRAMES:
            return None
        return f if ops.motion_qkv_takes(batch, frames, positions, self.heads, self.dim_head) else None

    def fold(self, i, M):
        """norm i's LnFold when its consumer GEMM runs folded over M rows, else None."""
        f = getattr(self, "_fold", {}).get(i)
        return f[0] if f is not None and f[0].runs(M, f[1]) else None

    def _out_norm(self, a, attn, i, h, mshape=None, **pe):
        """h' = to_out(a) + h and norm i of it: (h', n), or (h', None) when norm i folds into
        its consumer (the rows are then never normalised in memory).  mshape = (batch, frames,
        positions) of a temporal block: norm i (+ PE) may fold into the fused QKV attention."""
        folded = (self.fold(i, h.shape[0]) is not None if pe.get("pe") is None
                  else mshape is not None and self.temporal_fold(i, *mshape) is not None)
        if folded:
            return ops.gemm(a, attn._wo, bias=attn._bo, res=h), None
        return ops.gemm_ln(a, attn._wo, *self._nrm(i), bias=attn._bo, res=h, **pe)

    def _ff(self, h, n):
        f3 = self.fold(3, h.shape[0]) if n is None else None
        return self.ff.forward_rows(h if n is None else n, h, fold=f3)

    # spatial: tokens are (image, pixel) rows
    # run_*: `n` = norm1(h) when the caller's GEMM already produced it (ops.gemm_ln: the
    # LayerNorm fused into the epilogue of the GEMM writing h, or run right after it)
    def run_spatial(self, h, n_img, hw, ctx: Ctx, n=None, dup=False):
        """dup (the CFG dedup, UNetMotionModel.forward_rows): h holds ONE guidance half; everything
        before the cross-attention reads no text, so norm1 -> self-attention -> norm2 -> to_q run on
        it and h, q are duplicated for the cross-attention on both halves — planned as the whole
        batch (ops.plan_scaled), so the dedup changes no kernel choice and no bit of the result."""
        C = h.shape[1]
        d = self.dim_head
        with ops.plan_scaled(2) if dup else contextlib.nullcontext():
            f1 = self.fold(1, h.shape[0]) if n is None else None
            if f1 is not None:
                qkv = f1.gemm(h)
            else:
                if n is None:
                    n = ops.layer_norm(h, *self._nrm(1))
                qkv = ops.gemm(n, self.attn1._wqkv)
            a = ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], n_img, self.heads, hw, hw, d,
                              scale=self.attn1.attn_scale)
            h, n = self._out_norm(a, self.attn1, 2, h)
            q = self.fold(2, h.shape[0]).gemm(h) if n is None else ops.gemm(n, self.attn2._wq)
        kv = None if ctx.kv_cache is None else ctx.kv_cache.get(id(self.attn2))
        if kv is None:
            kv = self.attn2.project_kv(ctx.ehs_rows)
            if ctx.kv_cache is not None:
                ctx.kv_cache[id(self.attn2)] = kv
        if dup:  # the cross-attention of each guidance half on the shared q: no copy of q or h
            L, Mh = kv.shape[0] // 2, h.shape[0]
            a = torch.empty(2 * Mh, C, device=h.device, dtype=h.dtype)
            for g in range(2):
                ops.attention(q, kv[g * L:(g + 1) * L, :C], kv[g * L:(g + 1) * L, C:], n_img, self.heads, hw,
                              ctx.ctx_len, d, kv_div=ctx.frames, scale=self.attn2.attn_scale, out=a[g * Mh:(g + 1) * Mh])
            h, n = self._out_norm_dup(a, self.attn2, 3, h)
        else:
            a = ops.attention(q, kv[:, :C], kv[:, C:], n_img, self.heads, hw, ctx.ctx_len, d,
                              kv_div=ctx.frames, scale=self.attn2.attn_scale)
            h, n = self._out_norm(a, self.attn2, 3, h)
        return self._ff(h, n)

    def _out_norm_dup(self, a, attn, i, h):
        """_out_norm for both guidance halves of `a` on the one residual half h (the CFG dedup):
        one GEMM per half into the halves of the output, planned as the whole batch."""
        M, Mh = a.shape[0], h.shape[0]
        out = torch.empty(M, h.shape[1], device=h.device, dtype=h.dtype)
        folded = self.fold(i, M) is not None
        n = None if folded else torch.empty_like(out)
        with ops.plan_scaled(2):
            for g in range(2):
                sl = slice(g * Mh, (g + 1) * Mh)
                if folded:
                    ops.gemm(a[sl], attn._wo, bias=attn._bo, res=h, out=out[sl])
                else:
                    ops.gemm_ln(a[sl], attn._wo, *self._nrm(i), bias=attn._bo, res=h, out=out[sl], ln_out=n[sl])
        return out, n

    # temporal: tokens are (video, frame, position) rows; attention over frames
    def run_temporal(self, h, batch, frames, positions, n=None):
        C = h.shape[1]
        d = self.dim_head
        pe = self.pos_embed._pe
        mshape = (batch, frames, positions)
        for attn, i in ((self.attn1, 1), (self.attn2, 2)):
            # Q/K/V projection fused into the attention where the kernel takes the shape
            # (level 1: 16 frames, d 40), with norm i + PE folded in when the caller left the rows
            # un-normalised; else the norm, the QKV GEMM and the attention kernel
            tf = self.temporal_fold(i, *mshape) if n is None else None
            a = None
            if tf is not None and tf[0] == "m":
                mf = tf[1]
                a = ops.motion_qkv_attention(h, mf.w, batch, frames, positions, self.heads, d,
                                             scale=attn.attn_scale, ln_fold=(mf.tab, mf.eps))
            elif self.fuse_qkv_attention and tf is None:
                if n is None:
                    n = ops.layer_norm(h, *self._nrm(i), pe=pe, pe_div=positions, pe_period=frames)
                a = ops.motion_qkv_attention(n, attn._wqkv, batch, frames, positions, self.heads, d,
                                             scale=attn.attn_scale)
            if a is None:
                if tf is not None and tf[0] == "p":  # norm i + PE folded into the QKV GEMM
                    qkv = tf[1].gemm(h, pe_div=positions, pe_period=frames)
                else:
                    if n is None:
                        n = ops.layer_norm(h, *self._nrm(i), pe=pe, pe_div=positions, pe_period=frames)
                    qkv = ops.gemm(n, attn._wqkv)
                a = ops.temporal_attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], batch, frames,
                                           positions, self.heads, d, scale=attn.attn_scale)
            # norm2 (+ PE) after attn1, norm3 after attn2
            h, n = self._out_norm(a, attn, i + 1, h, mshape=mshape, pe=pe if i == 1 else None, pe_div=positions,
                                  pe_period=frames)
        return self._ff(h, n)

    def run_temporal_gathered(self, h, batch, frames_local, positions, dist):
        """run_temporal on a frame-sharded rank's rows (b, f_loc, p) under the K/V all-gather
        window (FrameShard(window="kv-gather")): q from the rank's own frames, K/V of every
        frame all-gathered over the frame shards; the positional encoding indexed by the
        global frame rank*f_loc + f."""
        C = h.shape[1]
        d = self.dim_head
        pe_off = dist.rank * frames_local
        pe = self.pos_embed._pe[pe_off:]
        frames = frames_local * dist.world
        M = h.shape[0]

        def pfold(i):  # norm i + PE folded into the Q and the K/V GEMM (the QKV GEMM's fold, sliced)
            tf = self.temporal_fold(i, batch, frames_local, positions)
            if tf is None or tf[0] != "p":
                return None
            if i not in self._pfold_split:
                self._pfold_split[i] = (tf[1].slice(0, C), tf[1].slice(C, 3 * C))
            fq, fkv = self._pfold_split[i]
            return (fq, fkv) if fq.runs(M) and fkv.runs(M) else None

        n = None
        if pfold(1) is None:
            n = ops.layer_norm(h, *self._nrm(1), pe=pe, pe_div=positions, pe_period=frames_local)
        for attn, i in ((self.attn1, 1), (self.attn2, 2)):
            pf = pfold(i) if n is None else None
            if pf is not None:
                q = pf[0].gemm(h, pe_div=positions, pe_period=frames_local, pe_off=pe_off)
                kv = pf[1].gemm(h, pe_div=positions, pe_period=frames_local, pe_off=pe_off)
            else:
                q = ops.gemm(n, attn._wqkv[:C])
                kv = ops.gemm(n, attn._wqkv[C:])
            kv = dist.gather_kv_frames(kv, batch, frames_local, positions, ops.block_transpose)
            a = ops.temporal_attention_kv(q, kv[:, :C], kv[:, C:], batch, frames_local, frames, positions,
                                          self.heads, d, scale=attn.attn_scale)
            if i == 1 and pfold(2) is not None:  # norm2 folds into attn2's Q / K/V GEMMs
                h, n = ops.gemm(a, attn._wo, bias=attn._bo, res=h), None
            else:
                h, n = self._out_norm(a, attn, i + 1, h, pe=pe if i == 1 else None, pe_div=positions,
                                      pe_period=frames_local)
        return self._ff(h, n)

    def forward(self, hidden_states, attention_mask=None, encoder_hidden_states=None,
                encoder_attention_mask=None, timestep=None, cross_attention_kwargs=None,
                class_labels=None, added_cond_kwargs=None):
        """diffusers BasicTransformerBlock.forward over (N, S, C) tokens."""
        n = self.norm1(hidden_states)
        if self.pos_embed is not None:
            n = self.pos_embed(n)
        h = add(self.attn1(n, attention_mask=attention_mask), hidden_states)
        n = self.norm2(h)
        if self.pos_embed is not None:
            n = self.pos_embed(n)
        ctx = encoder_hidden_states if self.attn2.is_cross else None
        h = add(self.attn2(n, encoder_hidden_states=ctx), h)
        return add(self.ff(self.norm3(h)), h)


class Transformer2DModel(nn.Module):
    """Legacy SD-1.5 Transformer2DModel (use_linear_projection=False)."""

    def __init__(self, heads, dim_head, in_channels, cross_attention_dim, groups=32):
        super().__init__()
        inner = heads * dim_head
        self.groups = groups
        self.norm = GroupNorm(groups, in_channels, eps=1e-6, affine=True)
        self.proj_in = Conv2d(in_channels, inner, 1)
        self.transformer_blocks = nn.ModuleList(
            [BasicTransformerBlock(inner, heads, dim_head, cross_attention_dim=cross_attention_dim)])
        self.proj_out = Conv2d(inner, in_channels, 1)

    def run(self, x: Act, ctx: Ctx, half: Act = None) -> Act:
        """half (the CFG dedup): x's first guidance half (x = [half; half]): the block runs on it up
        to the cross-attention (BasicTransformerBlock.run_spatial dup)."""
        hw = x.h * x.w
        src = x if half is None else half
        blk = self.transformer_blocks[0]
        with ops.plan_scaled(2) if half is not None else contextlib.nullcontext():
            hn = ops.group_norm(src.t, src.n, hw, self.groups, 1e-6, self.norm._g, self.norm._b)
            fold1 = blk.fold(1, hn.shape[0]) is not None  # norm1 folds into the QKV GEMM
            if fold1:
                h, n = ops.gemm(hn, self.proj_in._w, bias=self.proj_in._b), None
            else:
                h, n = ops.gemm_ln(hn, self.proj_in._w, *blk._nrm(1), bias=self.proj_in._b)
        h = blk.run_spatial(h, src.n, hw, ctx, n=n, dup=half is not None)
        if half is None:
            out = ops.gemm(h, self.proj_out._w, bias=self.proj_out._b, res=x.t)
        else:  # the residual is the one half for both guidance halves (x = [half; half] is never built)
            Mh = half.t.shape[0]
            out = torch.empty(2 * Mh, half.t.shape[1], device=h.device, dtype=h.dtype)
            with ops.plan_scaled(2):
                for g in range(2):
                    ops.gemm(h[g * Mh:(g + 1) * Mh], self.proj_out._w, bias=self.proj_out._b, res=half.t,
                             out=out[g * Mh:(g + 1) * Mh])
        return Act(out, x.n, x.h, x.w)

    def forward(self, hidden_states, encoder_hidden_states=None, timestep=None, added_cond_kwargs=None,
                class_labels=None, cross_attention_kwargs=None, attention_mask=None,
                encoder_attention_mask=None, return_dict: bool = True):
        n, c, hh, ww = hidden_states.shape
        h = self.proj_in(self.norm(hidden_states))
        tok = fmap_rows(h).view(n, hh * ww, -1)          # permute(0,2,3,1).reshape(n, hw, c): a view
        for blk in self.transformer_blocks:
            tok = blk(tok, encoder_hidden_states=encoder_hidden_states, timestep=timestep,
                      cross_attention_kwargs=cross_attention_kwargs, class_labels=class_labels)
        h = self.proj_out(rows_fmap(token_rows(tok), (n, tok.shape[-1], hh, ww)))
        out = add(h, hidden_states)
        return Transformer2DModelOutput(out) if return_dict else (out,)


class AnimateDiffTransformer3D(nn.Module):
    """diffusers:AnimateDiffTransformer3D (motion module).  GroupNorm statistics
    span all F frames of a video; attention runs over frames per position."""

    def __init__(self, heads, dim_head, in_channels, groups=32, max_seq_length=32):
        super().__init__()
        inner = heads * dim_head
        self.groups = groups
        self.norm = GroupNorm(groups, in_channels, eps=1e-6, affine=True)
        self.proj_in = Linear(in_channels, inner)
        self.transformer_blocks = nn.ModuleList([BasicTransformerBlock(
            inner, heads, dim_head, double_self_attention=True, positional_embeddings="sinusoidal",
            num_positional_embeddings=max_seq_length)])
        self.proj_out = Linear(inner, in_channels)

    def run(self, x: Act, ctx: Ctx) -> Act:
        hw = x.h * x.w
        B, Fl = ctx.batch, ctx.frames
        dist = ctx.dist
        # the motion norm's records (C <= 2560: per-group) all-gathered rank-major, no transpose copy
        gather = dist.gather_gn_records if dist is not None else None
        blk = self.transformer_blocks[0]
        if dist is not None and dist.fused_ok(B, Fl, hw):
            # the fused re-shard (FrameShard.send_perm): norm -> send order, one all-to-all, the
            # block on the received (frame, video, position) rows, one all-to-all back, proj_out
            # writing the returned rows into this rank's layout with the residual
            pl = hw // dist.world
            F = Fl * dist.world
            hn = ops.group_norm(x.t, B, Fl * hw, self.groups, 1e-6, self.norm._g, self.norm._b, gather=gather,
                                two_pass=False, n_split=Fl * ops.gn_splits_per_frame(hw),
                                rev3=dist.send_perm(B, Fl, hw))
            recv = dist.exchange(hn)                                   # rows (f, b, j)
            if blk.temporal_fold(1, 1, F, B * pl) is not None:  # norm1 + PE fold into the QKV attention / GEMM
                h, n = ops.gemm(recv, self.proj_in._w, bias=self.proj_in._b), None
            else:
                h, n = ops.gemm_ln(recv, self.proj_in._w, *blk._nrm(1), bias=self.proj_in._b, pe=blk.pos_embed._pe,
                                   pe_div=B * pl, pe_period=F)
            h = blk.run_temporal(h, 1, F, B * pl, n=n)
            back = dist.exchange(h)                                    # rows (r', f_loc, b, j)
            out = ops.gemm(back, self.proj_out._w, bias=self.proj_out._b, res=x.t,
                           rmap=dist.return_perm(B, Fl, hw))
            return Act(out, x.n, x.h, x.w)
        hn = ops.group_norm(x.t, B, Fl * hw, self.groups, 1e-6, self.norm._g, self.norm._b, gather=gather,
                            two_pass=False, n_split=Fl * ops.gn_splits_per_frame(hw))
        if dist is None:  # norm1 (+ PE by frame) fused into proj_in's epilogue, or folded into the QKV attention
            if blk.temporal_fold(1, B, Fl, hw) is not None:
                h, n = ops.gemm(hn, self.proj_in._w, bias=self.proj_in._b), None
            else:
                h, n = ops.gemm_ln(hn, self.proj_in._w, *blk._nrm(1), bias=self.proj_in._b, pe=blk.pos_embed._pe,
                                   pe_div=hw, pe_period=Fl)
            h = blk.run_temporal(h, B, Fl, hw, n=n)
        else:
            h = ops.gemm(hn, self.proj_in._w, bias=self.proj_in._b)
            if dist.window == "kv-gather":
                h = blk.run_temporal_gathered(h, B, Fl, hw, dist)
            else:
                h = dist.temporal_window(h, B, Fl, hw, ops.block_transpose, blk.run_temporal)
        out = ops.gemm(h, self.proj_out._w, bias=self.proj_out._b, res=x.t)
        return Act(out, x.n, x.h, x.w)

    def forward(self, hidden_states, encoder_hidden_states=None, timestep=None, class_labels=None,
                num_frames: int = 1, cross_attention_kwargs=None):
        """diffusers AnimateDiffTransformer3D.forward: hidden_states (B*F, C, H, W) with
        num_frames = F (experiments/03_trace_forward_pass.py:182 calls it this way)."""
        if hidden_states.dim() != 4:
            raise ValueError(f"expected (batch*frames, C, H, W) with num_frames=F, got shape "
                             f"{tuple(hidden_states.shape)} (the diffusers calling convention)")
        bf_, c, hh, ww = hidden_states.shape
        if bf_ % num_frames:
            raise ValueError(f"batch*frames {bf_} is not a multiple of num_frames={num_frames}")
        b = bf_ // num_frames
        hw = hh * ww
        x5 = hidden_states.reshape(b, num_frames, c, hh, ww).permute(0, 2, 1, 3, 4)   # (B, C, F, H, W)
        hn = fmap_rows(self.norm(x5))                                                # rows (b, f, p)
        tok = torch.empty_like(hn)
        for i in range(b):  # permute(0,3,4,2,1): rows (b, f, p) -> tokens (b, p, f)
            ops.block_transpose(hn[i * num_frames * hw:(i + 1) * num_frames * hw], num_frames, hw, 1,
                                out=tok[i * num_frames * hw:(i + 1) * num_frames * hw])
        h = self.proj_in(tok.view(b * hw, num_frames, c))
        for blk in self.transformer_blocks:
            h = blk(h, encoder_hidden_states=encoder_hidden_states, timestep=timestep)
        h = token_rows(self.proj_out(h))
        back = torch.empty_like(h)
        for i in range(b):  # tokens (b, p, f) -> rows (b, f, p)
            ops.block_transpose(h[i * num_frames * hw:(i + 1) * num_frames * hw], hw, num_frames, 1,
                                out=back[i * num_frames * hw:(i + 1) * num_frames * hw])
        return add(rows_fmap(back, (bf_, c, hh, ww)), hidden_states)


class _MotionBlockBase(nn.Module):
    def _run_layers(self, x, ctx, skips_in=None, res0=None):
        """res0 = (full, half): resnets[0]'s output computed by the caller on one guidance half
        (UNetMotionModel's CFG dedup) and duplicated; attentions[0] runs on the half up to its
        cross-attention."""
        outs = []
        attns = getattr(self, "attentions", None)
        for i, res in enumerate(self.resnets):
            skip = skips_in.pop() if skips_in is not None else None
            dup = i == 0 and res0 is not None
            if dup:  # res0 = (the full batch's shape, its first guidance half)
                x = res0[0] if attns is not None else Act(torch.cat([res0[1].t, res0[1].t]), res0[0].n, res0[0].h,
                                                           res0[0].w)
            else:
                x = res.run(x, ctx, skip=skip)
            if attns is not None:
                x = attns[i].run(x, ctx, half=res0[1] if dup else None)
            x = self.motion_modules[i].run(x, ctx)
            outs.append(x)
        return x, outs

    def _forward_layers(self, h, temb, ehs, num_frames, res_tuple=None):
        attns = getattr(self, "attentions", None)
        outs = ()
        for i, res in enumerate(self.resnets):
            if res_tuple is not None:
                h = concat_channels(h, res_tuple[-1])
                res_tuple = res_tuple[:-1]
            h = res(h, temb)
            if attns is not None:
                h = attns[i](h, encoder_hidden_states=ehs, return_dict=False)[0]
            h = self.motion_modules[i](h, num_frames=num_frames)
            outs = outs + (h,)
        return h, outs


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

    def run(self, x, ctx, res0=None):
        x, outs = self._run_layers(x, ctx, res0=res0)
        if self.downsamplers is not None:
            x = self.downsamplers[0].run(x)
            outs.append(x)
        return x, outs

    def forward(self, hidden_states, temb=None, encoder_hidden_states=None, attention_mask=None,
                num_frames: int = 1, encoder_attention_mask=None, cross_attention_kwargs=None,
                additional_residuals=None):
        h, outs = self._forward_layers(hidden_states, temb, encoder_hidden_states, num_frames)
        if self.downsamplers is not None:
            for d in self.downsamplers:
                h = d(h)
            outs = outs + (h,)
        return h, outs


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

    def forward(self, hidden_states, temb=None, num_frames: int = 1, *args, **kwargs):
        return super().forward(hidden_states, temb, None, num_frames=num_frames)


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

    def run(self, x, ctx, skips):
        x, _ = self._run_layers(x, ctx, skips_in=skips)
        if self.upsamplers is not None:
            x = self.upsamplers[0].run(x)
        return x

    def forward(self, hidden_states, res_hidden_states_tuple, temb=None, encoder_hidden_states=None,
                cross_attention_kwargs=None, upsample_size=None, attention_mask=None,
                encoder_attention_mask=None, num_frames: int = 1):
        h, _ = self._forward_layers(hidden_states, temb, encoder_hidden_states, num_frames,
                                    res_tuple=tuple(res_hidden_states_tuple))
        if self.upsamplers is not None:
            for u in self.upsamplers:
                h = u(h)
        return h


class UpBlockMotion(CrossAttnUpBlockMotion):
    def __init__(self, resnet_in, out_channels, temb_channels, motion_heads, add_upsample, groups,
                 eps, max_seq_length):
        super().__init__(resnet_in, out_channels, temb_channels, None, None, motion_heads, add_upsample,
                         groups, eps, max_seq_length, with_attn=False)

    def forward(self, hidden_states, res_hidden_states_tuple, temb=None, upsample_size=None,
                num_frames: int = 1, *args, **kwargs):
        return super().forward(hidden_states, res_hidden_states_tuple, temb, None, num_frames=num_frames)


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

    def run(self, x, ctx):
        x = self.resnets[0].run(x, ctx)
        x = self.attentions[0].run(x, ctx)
        if self.motion_modules is not None:
            x = self.motion_modules[0].run(x, ctx)
        return self.resnets[1].run(x, ctx)

    def forward(self, hidden_states, temb=None, encoder_hidden_states=None, attention_mask=None,
                cross_attention_kwargs=None, encoder_attention_mask=None, num_frames: int = 1):
        h = self.resnets[0](hidden_states, temb)
        h = self.attentions[0](h, encoder_hidden_states=encoder_hidden_states, return_dict=False)[0]
        if self.motion_modules is not None:
            h = self.motion_modules[0](h, num_frames=num_frames)
        return self.resnets[1](h, temb)
