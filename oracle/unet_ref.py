"""ORACLE — test infrastructure only.  Never imported by the product path.

fp32 PyTorch-CPU restatement of the denoiser the reference drives through
`diffusers:UNetMotionModel` (SD-1.5 + animatediff-motion-adapter-v1-5-2):
the reference calls it at experiments/03_trace_forward_pass.py:109-115 and,
inside `AnimateDiffPipeline.__call__`, from
experiments/05_grid_search_ablation.py:158-167.

diffusers itself (pinned `diffusers>=0.25.0`, requirements.txt:6; the
`AnimateDiffTransformer3D` name in docs/02_video_diffusion_architecture.md:52
dates the code to the 0.30-0.36 line) is NOT vendored in /root/reference and
is not installed here, so this file restates its published algorithm op by
op.  PARITY STATUS: numerics vs diffusers are
**unpinned** (no reference tensors exist anywhere in the reference); the
module tree is pinned by the reference's published structural known-answers
(1,312,730,244 parameters and 639 temporal / 32 spatial modules,
docs/02_video_diffusion_architecture.md:86-91, computed by
experiments/02_architecture_inspection.py:38-60) — see tests/test_structure.py.

All functions take a state dict keyed by diffusers parameter names and a
diffusers-style config dict.  `rnd` is an optional hook applied to every
activation a fused HIP kernel would store to HBM (identity for pure fp32;
bf16 rounding to emulate the device path's storage precision).

act modes of unet_forward (test instrumentation for the device's precision):
  "fp32" — the reference semantics in fp32 (what parity is measured against);
  "bf16" — + bf16 rounding at every point the device stores an activation;
  "dev"  — + the device's attention arithmetic: the softmax scale d^-1/2 * log2(e)
           folded into a bf16 copy of to_q.weight (vdiff Attention.prepare), so q is
           stored as bf16(x W_q'^T) and scores are in log2 units, and the probabilities
           P = 2^(s - max) rounded to bf16 before P V, with the row sum taken over the
           same bf16 P (the flash kernels' ones-column / row-sum arithmetic).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

_ident = lambda x: x  # noqa: E731


def _bf16_round(x):
    return x.to(torch.bfloat16).to(torch.float32)


def _bf16_dev(x):
    return x.to(torch.bfloat16).to(torch.float32)


_bf16_dev.device_attention = True  # marks the "dev" mode (see module docstring)

ROUNDERS = {"fp32": _ident, "bf16": _bf16_round, "dev": _bf16_dev}


# ---------------------------------------------------------------- primitives
def timestep_embedding(t: torch.Tensor, dim: int) -> torch.Tensor:
    """diffusers:embeddings.get_timestep_embedding with flip_sin_to_cos=True,
    downscale_freq_shift=0, scale=1, max_period=1e4."""
    half = dim // 2
    exponent = -math.log(10000.0) * torch.arange(half, dtype=torch.float32) / half
    freqs = torch.exp(exponent)
    args = t.float()[:, None] * freqs[None, :]
    emb = torch.cat([torch.sin(args), torch.cos(args)], dim=-1)
    return torch.cat([emb[:, half:], emb[:, :half]], dim=-1)  # flip -> [cos, sin]


def sinusoidal_pe(max_len: int, dim: int) -> torch.Tensor:
    """diffusers:embeddings.SinusoidalPositionalEmbedding buffer `pe` (App. A.4)."""
    pos = torch.arange(max_len, dtype=torch.float32).unsqueeze(1)
    div = torch.exp(torch.arange(0, dim, 2, dtype=torch.float32) * (-math.log(10000.0) / dim))
    pe = torch.zeros(1, max_len, dim)
    pe[0, :, 0::2] = torch.sin(pos * div)
    pe[0, :, 1::2] = torch.cos(pos * div)
    return pe


def linear(sd, p, x, bias=True):
    return F.linear(x, sd[p + ".weight"], sd.get(p + ".bias") if bias else None)


def conv(sd, p, x, stride=1, padding=1):
    return F.conv2d(x, sd[p + ".weight"], sd.get(p + ".bias"), stride=stride, padding=padding)


def group_norm(sd, p, x, groups, eps):
    return F.group_norm(x, groups, sd[p + ".weight"], sd[p + ".bias"], eps)


def layer_norm(sd, p, x, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], eps)


def folded_linear(sd, norm_p, x, w, b=None, eps=1e-5, pe=None):
    """The device's folded LayerNorm -> Linear ("dev" mode; vdiff.models.layers.LnFold and
    vd_gemm_desc.ln_fold_s): W' = bf16(W∘gamma), s = Σ_k W'[n][k], b' = W·beta + b and
    rstd·(x·W'^T − mean·s) + b' over the UN-normalised rows x — the same function as
    Linear(LayerNorm(x)) up to the rounding of W' (the normalised rows are never rounded).
    pe (1, F, C): the motion block's PE added after the norm, folded as W·pe[f] per frame
    (vdiff.models.layers.MotionLnFold); x is then (rows, F, C)."""
    g, be = sd[norm_p + ".weight"].double(), sd[norm_p + ".bias"].double()
    wd = w.double()
    wf = (wd * g[None, :]).to(torch.bfloat16).double()
    bp = wd @ be + (b.double() if b is not None else 0.0)
    if pe is not None:
        bp = bp + pe[:, : x.shape[1]].double() @ wd.T
    xd = x.double()
    mean = xd.mean(-1, keepdim=True)
    rstd = (xd.var(-1, unbiased=False, keepdim=True) + eps).rsqrt()
    return (rstd * (xd @ wf.T - mean * wf.sum(1)) + bp).float()


def attention(sd, p, x, ctx, heads, rnd=_ident, fold_norm=None, pe=None):
    """diffusers:Attention + AttnProcessor2_0 (App. A.5): q/k/v without bias,
    softmax(q k^T / sqrt(d)) v, to_out.0 with bias, no residual inside.  fold_norm ("dev" mode):
    x is the un-normalised input of that LayerNorm, folded into q (and k / v of a
    self-attention) as the device does (folded_linear)."""
    ctx = x if ctx is None else ctx
    dev = getattr(rnd, "device_attention", False)
    wq = sd[p + ".to_q.weight"]
    d = wq.shape[0] // heads
    if fold_norm is not None:  # vdiff BasicTransformerBlock.prepare: LnFold of the scaled q rows
        q = rnd(folded_linear(sd, fold_norm, x, wq.float() * (d ** -0.5 * math.log2(math.e)), pe=pe))
        self_attn = ctx is x
        k = rnd(folded_linear(sd, fold_norm, x, sd[p + ".to_k.weight"], pe=pe) if self_attn
                else linear(sd, p + ".to_k", ctx, bias=False))
        v = rnd(folded_linear(sd, fold_norm, x, sd[p + ".to_v.weight"], pe=pe) if self_attn
                else linear(sd, p + ".to_v", ctx, bias=False))
    else:
        if dev:  # vdiff Attention.prepare: bf16(W_q * d^-1/2 * log2 e); scores in log2 units
            wq = _bf16_round(wq * (d ** -0.5 * math.log2(math.e)))
        q = rnd(F.linear(x, wq))
        k = rnd(linear(sd, p + ".to_k", ctx, bias=False))
        v = rnd(linear(sd, p + ".to_v", ctx, bias=False))
    b, s, c = q.shape
    q = q.view(b, s, heads, d).transpose(1, 2)
    k = k.view(b, -1, heads, d).transpose(1, 2)
    v = v.view(b, -1, heads, d).transpose(1, 2)
    # batch chunks bound the score matrix to ~2^28 floats (the full config's level-1
    # self-attention would otherwise hold 32 x 8 x 4096^2 fp32 scores = 17 GB at once)
    step = max(1, (1 << 28) // (heads * s * k.shape[2]))
    outs = []
    for i in range(0, b, step):
        qi, ki, vi = q[i:i + step], k[i:i + step], v[i:i + step]
        if dev:
            sc = qi @ ki.transpose(-1, -2)
            pr = _bf16_round(torch.exp2(sc - sc.amax(-1, keepdim=True)))
            outs.append((pr @ vi) / pr.sum(-1, keepdim=True))
        else:
            outs.append(torch.softmax((qi @ ki.transpose(-1, -2)) * (d ** -0.5), dim=-1) @ vi)
    o = torch.cat(outs).transpose(1, 2).reshape(b, s, c)
    return linear(sd, p + ".to_out.0", rnd(o))


def feed_forward(sd, p, x, rnd=_ident, fold_norm=None):
    """diffusers:FeedForward(activation_fn='geglu'): GEGLU(C->4C) -> Linear(4C->C) (App. A.5).
    fold_norm: x un-normalised, that LayerNorm folded into the GEGLU projection (folded_linear)."""
    if fold_norm is not None:
        hg = folded_linear(sd, fold_norm, x, sd[p + ".net.0.proj.weight"], sd[p + ".net.0.proj.bias"])
    else:
        hg = linear(sd, p + ".net.0.proj", x)
    h, g = hg.chunk(2, dim=-1)
    a = rnd(h * F.gelu(g, approximate="none"))
    return linear(sd, p + ".net.2", a)


def basic_transformer_block(sd, p, x, ehs, heads, pe=None, double_self=False, rnd=_ident):
    """diffusers:BasicTransformerBlock, norm_type='layer_norm' (App. A.3 / A.4).  A "dev"-mode
    rounder may carry ln_fold(i, C, rows, motion) -> bool, the device's choice of folding norm i
    into its consuming GEMM (vdiff BasicTransformerBlock.fold); those norms then follow the
    device's folded arithmetic (folded_linear)."""
    fold = getattr(rnd, "ln_fold", None)
    rows = x.shape[0] * x.shape[1]

    def folds(i):
        return fold is not None and fold(i, x.shape[-1], rows, pe is not None, x.shape[1])

    if folds(1):
        x = rnd(attention(sd, p + ".attn1", x, None, heads, rnd, fold_norm=p + ".norm1", pe=pe) + x)
    else:
        n = layer_norm(sd, p + ".norm1", x)
        if pe is not None:
            n = n + pe[:, : x.shape[1]]
        x = rnd(attention(sd, p + ".attn1", rnd(n), None, heads, rnd) + x)
    ctx = None if double_self else ehs
    if folds(2):
        x = rnd(attention(sd, p + ".attn2", x, ctx, heads, rnd, fold_norm=p + ".norm2", pe=pe) + x)
    else:
        n = layer_norm(sd, p + ".norm2", x)
        if pe is not None:
            n = n + pe[:, : x.shape[1]]
        x = rnd(attention(sd, p + ".attn2", rnd(n), ctx, heads, rnd) + x)
    if folds(3):
        x = rnd(feed_forward(sd, p + ".ff", x, rnd, fold_norm=p + ".norm3") + x)
    else:
        n = layer_norm(sd, p + ".norm3", x)
        x = rnd(feed_forward(sd, p + ".ff", rnd(n), rnd) + x)
    return x


# ---------------------------------------------------------------- blocks
def resnet(sd, p, x, temb_silu, groups, eps=1e-5, rnd=_ident):
    """diffusers:ResnetBlock2D (App. A.2), output_scale_factor 1, pre_norm."""
    h = rnd(F.silu(group_norm(sd, p + ".norm1", x, groups, eps)))
    h = conv(sd, p + ".conv1", h)
    h = rnd(h + linear(sd, p + ".time_emb_proj", temb_silu)[:, :, None, None])
    h = rnd(F.silu(group_norm(sd, p + ".norm2", h, groups, eps)))
    h = conv(sd, p + ".conv2", h)
    sc = x
    if (p + ".conv_shortcut.weight") in sd:
        sc = rnd(conv(sd, p + ".conv_shortcut", x, padding=0))
    return rnd(sc + h)


def transformer2d(sd, p, x, ehs, heads, groups, rnd=_ident):
    """diffusers:Transformer2DModel, legacy SD-1.5 form (use_linear_projection=False) (App. A.3)."""
    n, c, hh, ww = x.shape
    h = rnd(group_norm(sd, p + ".norm", x, groups, 1e-6))
    h = rnd(conv(sd, p + ".proj_in", h, padding=0))
    h = h.permute(0, 2, 3, 1).reshape(n, hh * ww, c)
    h = basic_transformer_block(sd, p + ".transformer_blocks.0", h, ehs, heads, rnd=rnd)
    h = h.reshape(n, hh, ww, c).permute(0, 3, 1, 2)
    return rnd(conv(sd, p + ".proj_out", h, padding=0) + x)


def motion_module(sd, p, x, num_frames, heads, groups, max_len, rnd=_ident):
    """diffusers:AnimateDiffTransformer3D (App. A.4).  GroupNorm statistics span
    (C/G, F, H, W); tokens are (B*H*W, F, C) as the reference observes at
    experiments/03_trace_forward_pass.py:160-169."""
    bf, c, hh, ww = x.shape
    b = bf // num_frames
    h = x.reshape(b, num_frames, c, hh, ww).permute(0, 2, 1, 3, 4)
    h = rnd(group_norm(sd, p + ".norm", h, groups, 1e-6))
    h = h.permute(0, 3, 4, 2, 1).reshape(b * hh * ww, num_frames, c)
    h = rnd(linear(sd, p + ".proj_in", h))
    pe = sinusoidal_pe(max_len, c)
    h = basic_transformer_block(sd, p + ".transformer_blocks.0", h, None, heads, pe=pe,
                                double_self=True, rnd=rnd)
    h = linear(sd, p + ".proj_out", h)
    h = h.reshape(b, hh, ww, num_frames, c).permute(0, 3, 4, 1, 2).reshape(bf, c, hh, ww)
    return rnd(h + x)


# ---------------------------------------------------------------- model
def _down_plan(cfg):
    boc = list(cfg["block_out_channels"])
    out = boc[0]
    plan = []
    for i, bt in enumerate(cfg["down_block_types"]):
        inn, out = out, boc[i]
        ins = [inn if j == 0 else out for j in range(cfg["layers_per_block"])]
        plan.append((ins, bt.startswith("CrossAttn"), i != len(boc) - 1))
    return plan


def _up_plan(cfg):
    rev = list(cfg["block_out_channels"])[::-1]
    nl = cfg["layers_per_block"] + 1
    out = rev[0]
    plan = []
    for i, bt in enumerate(cfg["up_block_types"]):
        prev, out = out, rev[i]
        inn = rev[min(i + 1, len(rev) - 1)]
        ins = [(prev if j == 0 else out) + (inn if j == nl - 1 else out) for j in range(nl)]
        plan.append((ins, bt.startswith("CrossAttn"), i != len(rev) - 1))
    return plan


def unet_forward(sd, cfg, sample, timestep, encoder_hidden_states, act="fp32"):
    """diffusers:UNetMotionModel.forward(...).sample (App. A.1).

    sample (B, C, F, H, W); timestep int / 0-d / (B,); encoder_hidden_states (B, 77, D).
    Returns (B, out_channels, F, H, W) fp32.
    """
    rnd = ROUNDERS[act]
    g = cfg["norm_num_groups"]
    eps = cfg["norm_eps"]
    heads = cfg["num_attention_heads"]
    mheads = cfg["motion_num_attention_heads"]
    mlen = cfg["motion_max_seq_length"]
    sample = sample.float()
    b, _, nf, hh, ww = sample.shape
    t = torch.as_tensor(timestep)
    if t.ndim == 0:
        t = t[None]
    t = t.expand(b)
    temb = rnd(timestep_embedding(t, cfg["block_out_channels"][0]))
    temb = rnd(F.silu(linear(sd, "time_embedding.linear_1", temb)))
    temb = linear(sd, "time_embedding.linear_2", temb)
    temb_silu = rnd(F.silu(temb)).repeat_interleave(nf, 0)
    ehs = rnd(encoder_hidden_states.float()).repeat_interleave(nf, 0)

    x = rnd(sample).permute(0, 2, 1, 3, 4).reshape(b * nf, -1, hh, ww)
    x = rnd(conv(sd, "conv_in", x))
    skips = [x]
    for i, (ins, has_attn, down) in enumerate(_down_plan(cfg)):
        for j in range(len(ins)):
            p = f"down_blocks.{i}"
            x = resnet(sd, f"{p}.resnets.{j}", x, temb_silu, g, eps, rnd)
            if has_attn:
                x = transformer2d(sd, f"{p}.attentions.{j}", x, ehs, heads, g, rnd)
            x = motion_module(sd, f"{p}.motion_modules.{j}", x, nf, mheads, g, mlen, rnd)
            skips.append(x)
        if down:
            x = rnd(conv(sd, f"down_blocks.{i}.downsamplers.0.conv", x, stride=2, padding=1))
            skips.append(x)
    x = resnet(sd, "mid_block.resnets.0", x, temb_silu, g, eps, rnd)
    x = transformer2d(sd, "mid_block.attentions.0", x, ehs, heads, g, rnd)
    if cfg.get("use_motion_mid_block", True):
        x = motion_module(sd, "mid_block.motion_modules.0", x, nf, mheads, g, mlen, rnd)
    x = resnet(sd, "mid_block.resnets.1", x, temb_silu, g, eps, rnd)
    for i, (ins, has_attn, up) in enumerate(_up_plan(cfg)):
        p = f"up_blocks.{i}"
        for j in range(len(ins)):
            x = torch.cat([x, skips.pop()], dim=1)
            x = resnet(sd, f"{p}.resnets.{j}", x, temb_silu, g, eps, rnd)
            if has_attn:
                x = transformer2d(sd, f"{p}.attentions.{j}", x, ehs, heads, g, rnd)
            x = motion_module(sd, f"{p}.motion_modules.{j}", x, nf, mheads, g, mlen, rnd)
        if up:
            x = F.interpolate(x, scale_factor=2.0, mode="nearest")
            x = rnd(conv(sd, f"{p}.upsamplers.0.conv", x))
    x = rnd(F.silu(group_norm(sd, "conv_norm_out", x, g, eps)))
    x = conv(sd, "conv_out", x)
    return x.reshape(b, nf, -1, hh, ww).permute(0, 2, 1, 3, 4).contiguous()
