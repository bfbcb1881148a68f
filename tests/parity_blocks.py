"""Block-by-block parity of the fused path vs the oracle (test helper; also run by
tools/parity_probe.py).

Each block of a UNet runs on the device from the device's own input, and the oracle block
(fp32 and act="dev", the device-emulating mode) runs on the SAME input, so per-block
errors do not accumulate.  End to end, two bf16 realisations of the network decorrelate to
~1.3 % rel-L2 from ANY fp32-level difference (tests/test_oracle.py::
test_bf16_realisation_floor), so the end-to-end bound cannot be tighter than that floor;
per block, the device must agree with the emulation to a fraction of one bf16 rounding.
"""
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
