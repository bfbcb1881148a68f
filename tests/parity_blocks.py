"""Block-by-block parity of the fused path vs the oracle (test helper; also run by
tools/parity_probe.py).

Each block of a UNet runs on the device from the device's own input, and the oracle block
(fp32 and act="dev", the device-emulating mode) runs on the SAME input, so per-block
errors do not accumulate.  End to end, two bf16 realisations of the network decorrelate to
~1.3 % rel-L2 from ANY fp32-level difference (tests/test_oracle.py::
test_bf16_realisation_floor), so the end-to-end bound cannot be tighter than that floor;
per block, the device must agree with the emulation to a fraction of one bf16 rounding.
"""
import math

import numpy as np
import torch

from oracle import unet_ref
from vdiff import ops
from vdiff.models.blocks import CrossAttnDownBlockMotion
from vdiff.models.layers import Act


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm()).item()


def nchw(act: Act):
    return act.t.float().cpu().reshape(act.n, act.h, act.w, -1).permute(0, 3, 1, 2)


def device_rounder(unet):
    """The oracle's "dev" rounder plus the device's LayerNorm-fold decisions (ln_fold hook of
    unet_ref.basic_transformer_block): norm i of a block with C channels over `rows` rows folds
    exactly when the device's block of that kind would fold it (BasicTransformerBlock.fold,
    i.e. the library's own plan)."""
    from vdiff.models.blocks import BasicTransformerBlock
    blocks = {}
    for m in unet.modules():
        if isinstance(m, BasicTransformerBlock):
            blocks.setdefault((m.norm1.normalized_shape[0], m.pos_embed is not None), m)

    def dev(x):
        return unet_ref.ROUNDERS["dev"](x)

    def ln_fold(i, C, rows, motion, frames=1):
        b = blocks.get((C, motion))
        if b is None:
            return False
        if motion and i < 3:  # norm1 / norm2 + PE fold into the fused QKV attention or the QKV GEMM
            return b.temporal_fold(i, 1, frames, rows // frames) is not None
        return b.fold(i, rows) is not None

    dev.device_attention = True
    dev.ln_fold = ln_fold
    return dev


def block_errors(unet, lat, ehs, t=961, log=None):
    """-> [(block name, rel-L2 vs fp32 oracle, rel-L2 vs device-emulating oracle)]."""
    rows_out = []

    cfg = unet.config
    sd = {k: v.detach().float().cpu() for k, v in unet.state_dict().items()}
    x_in = torch.cat([lat, lat])
    L = ehs.shape[1]
    B, _, F, H, W = x_in.shape
    g, eps = cfg["norm_num_groups"], cfg["norm_eps"]
    heads, mheads, mlen = cfg["num_attention_heads"], cfg["motion_num_attention_heads"], cfg["motion_max_seq_length"]
    R = {"fp32": unet_ref.ROUNDERS["fp32"], "dev": device_rounder(unet)}
    # device context
    tt = torch.full((B,), float(t), device="cuda")
    te = ops.timestep_embed(tt, unet.time_proj.num_channels)
    ehs_rows = ehs.to("cuda", torch.bfloat16).reshape(B * L, -1)
    ctx = unet.make_ctx(te, ehs_rows, B, F, L)
    # oracle temb per mode
    temb_silu, ehs_rep = {}, ehs.repeat_interleave(F, 0)
    for m, r in R.items():
        e = r(unet_ref.timestep_embedding(torch.full((B,), t), cfg["block_out_channels"][0]))
        e = r(torch.nn.functional.silu(unet_ref.linear(sd, "time_embedding.linear_1", e)))
        e = unet_ref.linear(sd, "time_embedding.linear_2", e)
        temb_silu[m] = r(torch.nn.functional.silu(e)).repeat_interleave(F, 0)
    rows = ops.pack_latents(x_in.cuda(), dup=1, cpad=8)
    tconv, _, _ = ops.conv3x3(rows, B * F, H, W, unet.conv_in._w, bias=unet.conv_in._b)
    x = Act(tconv, B * F, H, W)
    xin = unet_ref.ROUNDERS["dev"](x_in).permute(0, 2, 1, 3, 4).reshape(B * F, 4, H, W)
    rows_out.append(("conv_in", rel(nchw(x), unet_ref.conv(sd, "conv_in", xin)),
                     rel(nchw(x), R["dev"](unet_ref.conv(sd, "conv_in", xin)))))

    def probe(name, dev_out, fn):
        got = nchw(dev_out)
        errs = {m: rel(got, fn(r, m)) for m, r in R.items()}
        rows_out.append((name, errs["fp32"], errs["dev"]))
        if log:
            log(f"{name:44s} fp32 {errs['fp32']:.5f}  dev {errs['dev']:.5f}")

    skips = [x]
    for i, blk in enumerate(unet.down_blocks):
        p = f"down_blocks.{i}"
        for j, res in enumerate(blk.resnets):
            xi = nchw(x)
            y = res.run(x, ctx)
            probe(f"{p}.resnets.{j}", y, lambda r, m: unet_ref.resnet(sd, f"{p}.resnets.{j}", xi, temb_silu[m], g, eps, r))
            x = y
            if isinstance(blk, CrossAttnDownBlockMotion) and hasattr(blk, "attentions"):
                xi = nchw(x)
                y = blk.attentions[j].run(x, ctx)
                probe(f"{p}.attentions.{j}", y, lambda r, m: unet_ref.transformer2d(sd, f"{p}.attentions.{j}", xi, ehs_rep, heads, g, r))
                x = y
            xi = nchw(x)
            y = blk.motion_modules[j].run(x, ctx)
            probe(f"{p}.motion_modules.{j}", y, lambda r, m: unet_ref.motion_module(sd, f"{p}.motion_modules.{j}", xi, F, mheads, g, mlen, r))
            x = y
            skips.append(x)
        if blk.downsamplers is not None:
            xi = nchw(x)
            y = blk.downsamplers[0].run(x)
            probe(f"{p}.downsamplers.0", y, lambda r, m: r(unet_ref.conv(sd, f"{p}.downsamplers.0.conv", xi, stride=2)))
            x = y
            skips.append(x)
    mb = unet.mid_block
    xi = nchw(x)
    y = mb.resnets[0].run(x, ctx)
    probe("mid_block.resnets.0", y, lambda r, m: unet_ref.resnet(sd, "mid_block.resnets.0", xi, temb_silu[m], g, eps, r))
    x = y
    xi = nchw(x)
    y = mb.attentions[0].run(x, ctx)
    probe("mid_block.attentions.0", y, lambda r, m: unet_ref.transformer2d(sd, "mid_block.attentions.0", xi, ehs_rep, heads, g, r))
    x = y
    xi = nchw(x)
    y = mb.motion_modules[0].run(x, ctx)
    probe("mid_block.motion_modules.0", y, lambda r, m: unet_ref.motion_module(sd, "mid_block.motion_modules.0", xi, F, mheads, g, mlen, r))
    x = y
    xi = nchw(x)
    y = mb.resnets[1].run(x, ctx)
    probe("mid_block.resnets.1", y, lambda r, m: unet_ref.resnet(sd, "mid_block.resnets.1", xi, temb_silu[m], g, eps, r))
    x = y
    for i, blk in enumerate(unet.up_blocks):
        p = f"up_blocks.{i}"
        for j, res in enumerate(blk.resnets):
            sk = skips.pop()
            xi = torch.cat([nchw(x), nchw(sk)], 1)
            y = res.run(x, ctx, skip=sk)
            probe(f"{p}.resnets.{j}", y, lambda r, m: unet_ref.resnet(sd, f"{p}.resnets.{j}", xi, temb_silu[m], g, eps, r))
            x = y
            if getattr(blk, "attentions", None) is not None:
                xi = nchw(x)
                y = blk.attentions[j].run(x, ctx)
                probe(f"{p}.attentions.{j}", y, lambda r, m: unet_ref.transformer2d(sd, f"{p}.attentions.{j}", xi, ehs_rep, heads, g, r))
                x = y
            xi = nchw(x)
            y = blk.motion_modules[j].run(x, ctx)
            probe(f"{p}.motion_modules.{j}", y, lambda r, m: unet_ref.motion_module(sd, f"{p}.motion_modules.{j}", xi, F, mheads, g, mlen, r))
            x = y
        if blk.upsamplers is not None:
            xi = nchw(x)
            y = blk.upsamplers[0].run(x)
            probe(f"{p}.upsamplers.0", y, lambda r, m: r(unet_ref.conv(
                sd, f"{p}.upsamplers.0.conv", torch.nn.functional.interpolate(xi, scale_factor=2.0, mode="nearest"))))
            x = y
    return rows_out


# ------------------------------------------------------------------ stage-by-stage (teacher-forced)
def _d(t):
    return t.detach().to("cpu", torch.float64)


def _bf(x):
    return x.to(torch.bfloat16).to(torch.float64)


def _ln(x, g, b, eps=1e-5):
    m = x.mean(1, keepdim=True)
    return (x - m) / torch.sqrt(x.var(1, unbiased=False, keepdim=True) + eps) * g + b


def _folded(x, w, s, b, eps=1e-5):
    """rstd·(x·W'^T − mean·s) + b' in fp64 (LnFold / MotionLnFold arithmetic, exact statistics)."""
    m = x.mean(1, keepdim=True)
    rstd = (x.var(1, unbiased=False, keepdim=True) + eps).rsqrt()
    return rstd * (x @ w.T - m * s) + b


def _tattn(qkv, B, Fr, P, heads, d):
    """The device's temporal attention on bf16 q|k|v rows (b, f, p): log2-unit scores (the scale
    is in W_q), P = bf16(2^(s − max)), O = (P·V) / ΣP."""
    C = heads * d
    q, k, v = (qkv[:, i * C:(i + 1) * C].reshape(B, Fr, P, heads, d).permute(0, 2, 3, 1, 4) for i in range(3))
    s = q @ k.transpose(-1, -2)
    p = _bf(torch.exp2(s - s.amax(-1, keepdim=True)))
    return ((p @ v) / p.sum(-1, keepdim=True)).permute(0, 3, 1, 2, 4).reshape(B * Fr * P, C)


def motion_stages(mm, x: Act, ctx, log=None):
    """One motion module (AnimateDiffTransformer3D.run, unsharded), re-run stage by stage on the
    device, each stage FROM THE DEVICE'S OWN INPUT to it, against fp64 of the same stage on the
    same input: "emu" = rounded to bf16 where the device stores (the device-emulating oracle's
    arithmetic), "exact" = unrounded.  -> [(stage, rel-L2 vs emu, rel-L2 vs exact, fraction of
    stored bf16 values that differ from emu)].  Teacher forcing keeps one stage's rounding flips
    out of the next stage's reference, so each number isolates one kernel's arithmetic."""
    out = []

    def rep(name, got, exact):
        got, exact = _d(got), exact.to(torch.float64)
        emu, nrm = _bf(exact), exact.norm().item()
        r = (name, ((got - emu).norm() / nrm).item(), ((got - exact).norm() / nrm).item(),
             (got != emu).double().mean().item())
        out.append(r)
        if log:
            log(f"  {name:36s} vs emu {r[1]:.6f}  vs exact {r[2]:.6f}  flips {r[3]:.5f}")

    hw, B, Fl = x.h * x.w, ctx.batch, ctx.frames
    blk = mm.transformer_blocks[0]
    C, heads, d = x.t.shape[1], blk.heads, blk.dim_head
    M = x.t.shape[0]
    frame = (torch.arange(M) // hw) % Fl
    pe = _d(blk.pos_embed._pe)[:Fl]
    xin = _d(x.t)
    G = mm.groups
    hn = ops.group_norm(x.t, B, Fl * hw, G, 1e-6, mm.norm._g, mm.norm._b, two_pass=False,
                        n_split=Fl * ops.gn_splits_per_frame(hw))
    xv = xin.reshape(B, Fl * hw, G, C // G)
    gn = ((xv - xv.mean((1, 3), keepdim=True)) / torch.sqrt(xv.var((1, 3), unbiased=False, keepdim=True) + 1e-6))
    rep("groupnorm", hn, gn.reshape(M, C) * _d(mm.norm._g) + _d(mm.norm._b))
    pin = _d(hn) @ _d(mm.proj_in._w).T + _d(mm.proj_in._b)
    if blk.temporal_fold(1, B, Fl, hw) is not None:
        h, n = ops.gemm(hn, mm.proj_in._w, bias=mm.proj_in._b), None
        rep("proj_in", h, pin)
    else:
        h, n = ops.gemm_ln(hn, mm.proj_in._w, *blk._nrm(1), bias=mm.proj_in._b, pe=blk.pos_embed._pe,
                           pe_div=hw, pe_period=Fl)
        rep("proj_in", h, pin)
        rep("  norm1 + pe (epilogue)", n, _ln(_d(h), *(_d(t) for t in blk._nrm(1))) + pe[frame])
    for attn, i in ((blk.attn1, 1), (blk.attn2, 2)):
        tf = blk.temporal_fold(i, B, Fl, hw) if n is None else None
        hd = _d(h)
        a = qkv = None
        c = d ** -0.5 * math.log2(math.e)
        wqkv = torch.cat([_d(attn.to_q.weight.float()) * c, _d(attn.to_k.weight.float()),
                          _d(attn.to_v.weight.float())], 0)
        gi, bi = (_d(t) for t in blk._nrm(i))
        if tf is not None and tf[0] == "m":  # level 1: norm i + PE folded into the fused QKV attention
            mf = tf[1]
            a = ops.motion_qkv_attention(h, mf.w, B, Fl, hw, heads, d, scale=attn.attn_scale, ln_fold=(mf.tab, mf.eps))
            wf = _d(mf.w)
            qkv = _bf(_folded(hd, wf, wf.sum(1), ((bi[None, :] + pe) @ wqkv.T)[frame], mf.eps))
            rep(f"attn{i} fused qkv+attention (folded)", a, _tattn(qkv, B, Fl, hw, heads, d))
        elif tf is not None and tf[0] == "p":  # levels 2-4: norm i + PE folded into the QKV GEMM
            f = tf[1]
            qkv = f.gemm(h, pe_div=hw, pe_period=Fl)
            rep(f"attn{i} qkv (norm{i}+pe folded)", qkv,
                _folded(hd, _d(f.w), _d(f.s), _d(f.b), f.eps) + _d(f.pe_b)[frame])
        else:
            if n is None:
                n = ops.layer_norm(h, *blk._nrm(i), pe=blk.pos_embed._pe, pe_div=hw, pe_period=Fl)
                rep(f"norm{i} + pe", n, _ln(hd, gi, bi) + pe[frame])
            if blk.fuse_qkv_attention:
                a = ops.motion_qkv_attention(n, attn._wqkv, B, Fl, hw, heads, d, scale=attn.attn_scale)
            if a is not None:
                rep(f"attn{i} fused qkv+attention", a,
                    _tattn(_bf(_d(n) @ _d(attn._wqkv).T), B, Fl, hw, heads, d))
            else:
                qkv = ops.gemm(n, attn._wqkv)
                rep(f"attn{i} qkv", qkv, _d(n) @ _d(attn._wqkv).T)
        if a is None:
            a = ops.temporal_attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], B, Fl, hw, heads, d,
                                       scale=attn.attn_scale)
            rep(f"attn{i} core", a, _tattn(_d(qkv), B, Fl, hw, heads, d))
        h2, n = blk._out_norm(a, attn, i + 1, h, mshape=(B, Fl, hw), pe=blk.pos_embed._pe if i == 1 else None,
                              pe_div=hw, pe_period=Fl)
        rep(f"attn{i} to_out + res", h2, _d(a) @ _d(attn._wo).T + _d(attn._bo) + hd)
        if n is not None:
            rep(f"  norm{i + 1} (epilogue)", n,
                _ln(_d(h2), *(_d(t) for t in blk._nrm(i + 1))) + (pe[frame] if i == 1 else 0.0))
        h = h2
    hd = _d(h)
    f3 = blk.fold(3, M) if n is None else None
    ff = blk.ff
    wg, bg = _d(ff.net[0].proj.weight.float()), _d(ff.net[0].proj.bias.float())
    if f3 is not None:
        g = f3.gemm(h, act=ops.ACT_GEGLU)
        g3, b3 = (_d(t) for t in blk._nrm(3))
        wf = _bf(wg * g3[None, :])
        hg = _folded(hd, wf, wf.sum(1), wg @ b3 + bg)
    else:
        g = ops.gemm(n, ff.net[0]._w, bias=ff.net[0]._b, act=ops.ACT_GEGLU)
        hg = _d(n) @ wg.T + bg
    hh, gg = hg.chunk(2, -1)
    rep("geglu" + (" (norm3 folded)" if f3 is not None else ""), g, hh * 0.5 * gg * (1 + torch.erf(gg / math.sqrt(2))))
    o = ops.gemm(g, ff._w2, bias=ff._b2, res=h)
    rep("ff2 + res", o, _d(g) @ _d(ff._w2).T + _d(ff._b2) + hd)
    fin = ops.gemm(o, mm.proj_out._w, bias=mm.proj_out._b, res=x.t)
    rep("proj_out + res", fin, _d(o) @ _d(mm.proj_out._w).T + _d(mm.proj_out._b) + xin)
    assert torch.equal(mm.run(x, ctx).t, fin), "the staged chain is not the module's run()"
    return out


def ulp_flip(x: torch.Tensor, frac: float = 2e-4, seed: int = 0) -> torch.Tensor:
    """bf16-valued x with a random `frac` of its elements moved by one bf16 ulp (up or down): the
    size of the difference one device stage leaves against its emulation (motion_stages: 1e-4 -
    3e-4 of the stored values differ, by one ulp each)."""
    g = torch.Generator().manual_seed(seed)
    b = x.to(torch.bfloat16).contiguous()
    bits = b.view(torch.int16).clone()
    pick = torch.rand(bits.shape, generator=g) < frac
    step = torch.where(torch.rand(bits.shape, generator=g) < 0.5, 1, -1).to(torch.int16)
    bits[pick] += step[pick]
    return bits.view(torch.bfloat16).float()


def noisy_rounder(base, frac=2e-4, seed=0):
    """`base` (a "dev" rounder) followed by ulp_flip at every store: an emulation that differs
    from itself by one ulp at `frac` of the stored values of EVERY stage — the rate at which the
    device's stages differ from their emulation (motion_stages) — so rel(noisy, dev) is the bf16
    realisation floor of a chain of stores at that rate."""
    count = [seed]

    def r(x):
        count[0] += 1
        return ulp_flip(base(x), frac, count[0])

    r.device_attention = True
    r.ln_fold = getattr(base, "ln_fold", None)
    return r


def motion_floor(unet, name, x: Act, frames, frac=2e-4):
    """-> (dev, noisy, fp32): the device-emulating oracle of motion module `name` on the device's
    input x, the same oracle with `frac` of every stage's stored values moved by one ulp
    (noisy_rounder), and the fp32 oracle.  rel(noisy, dev) is the block's bf16 realisation floor at
    the device's per-stage flip rate: how far two faithful bf16 realisations of this chain of
    stores drift apart."""
    cfg = unet.config
    sd = {k: v.detach().float().cpu() for k, v in unet.state_dict().items() if k.startswith(name + ".")}
    xi = nchw(x)
    args = (frames, cfg["motion_num_attention_heads"], cfg["norm_num_groups"], cfg["motion_max_seq_length"])
    dev = device_rounder(unet)
    with torch.no_grad():
        d0 = unet_ref.motion_module(sd, name, xi, *args, dev)
        d1 = unet_ref.motion_module(sd, name, xi, *args, noisy_rounder(dev, frac))
        f0 = unet_ref.motion_module(sd, name, xi, *args, unet_ref.ROUNDERS["fp32"])
    return d0, d1, f0
