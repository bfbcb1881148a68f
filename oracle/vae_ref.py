"""ORACLE — test infrastructure only.  Never imported by the product path.

fp32 PyTorch-CPU restatement of the VAE decode the reference runs once per video:
`diffusers:AnimateDiffPipeline.decode_latents` -> `AutoencoderKL.decode` of SD-1.5's
`vae` (loaded with the pipeline at experiments/05_grid_search_ablation.py:130-134,
sliced per frame by `pipe.enable_vae_slicing()` at :143).

diffusers is absent, so this restates its published algorithm
(0.25-0.36 semantics, unchanged across them for this model):
  * decode_latents: z = latents / scaling_factor (0.18215); (B, C, F, h, w) ->
    (B*F, C, h, w) frame-major; image = vae.decode(z).sample; back to (B, 3, F, H, W);
  * AutoencoderKL.decode: z = post_quant_conv(z) (1x1); decoder(z);
  * Decoder: conv_in 3x3 (4 -> C_last); mid_block = UNetMidBlock2D(resnet,
    attention(heads = C / attention_head_dim = 1, GroupNorm 32 eps 1e-6, q/k/v/out with
    bias, residual, rescale 1), resnet); up_blocks = UpDecoderBlock2D over the reversed
    block_out_channels, layers_per_block + 1 resnets each, nearest-x2 Upsample2D(conv)
    on all but the last; conv_norm_out GroupNorm(32, eps 1e-6), SiLU, conv_out 3x3 -> 3;
  * ResnetBlock2D(temb_channels=None, eps 1e-6): GN -> SiLU -> conv1 -> GN -> SiLU ->
    conv2, + (1x1 conv_shortcut if Cin != Cout) x, output_scale_factor 1.
PARITY STATUS: unpinned against diffusers (no VAE weights or reference tensors exist);
the module tree follows diffusers' parameter names (tests/test_structure.py).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .unet_ref import _ident, conv, group_norm, linear


def resnet(sd, p, x, groups, eps=1e-6, rnd=_ident):
    h = rnd(F.silu(group_norm(sd, p + ".norm1", x, groups, eps)))
    h = rnd(conv(sd, p + ".conv1", h))
    h = rnd(F.silu(group_norm(sd, p + ".norm2", h, groups, eps)))
    h = conv(sd, p + ".conv2", h)
    sc = x
    if (p + ".conv_shortcut.weight") in sd:
        sc = rnd(conv(sd, p + ".conv_shortcut", x, padding=0))
    return rnd(sc + h)


def attention(sd, p, x, groups, eps=1e-6, rnd=_ident):
    """diffusers:Attention as the VAE mid block builds it (single head, group_norm,
    biased projections, residual_connection=True, rescale_output_factor=1)."""
    b, c, h, w = x.shape
    t = rnd(group_norm(sd, p + ".group_norm", x, groups, eps)).reshape(b, c, h * w).transpose(1, 2)
    q = rnd(linear(sd, p + ".to_q", t))
    k = rnd(linear(sd, p + ".to_k", t))
    v = rnd(linear(sd, p + ".to_v", t))
    wgt = torch.softmax((q @ k.transpose(-1, -2)) * (c ** -0.5), dim=-1)
    o = rnd(wgt @ v)
    o = linear(sd, p + ".to_out.0", o)
    return rnd(o.transpose(1, 2).reshape(b, c, h, w) + x)


def decoder(sd, cfg, z, rnd=_ident):
    g = cfg["norm_num_groups"]
    ch = list(reversed(cfg["block_out_channels"]))
    x = rnd(conv(sd, "decoder.conv_in", z))
    x = resnet(sd, "decoder.mid_block.resnets.0", x, g, rnd=rnd)
    x = attention(sd, "decoder.mid_block.attentions.0", x, g, rnd=rnd)
    x = resnet(sd, "decoder.mid_block.resnets.1", x, g, rnd=rnd)
    for i in range(len(ch)):
        for j in range(cfg["layers_per_block"] + 1):
            x = resnet(sd, f"decoder.up_blocks.{i}.resnets.{j}", x, g, rnd=rnd)
        if i < len(ch) - 1:
            x = F.interpolate(x, scale_factor=2.0, mode="nearest")
            x = rnd(conv(sd, f"decoder.up_blocks.{i}.upsamplers.0.conv", x))
    x = rnd(F.silu(group_norm(sd, "decoder.conv_norm_out", x, g, 1e-6)))
    return conv(sd, "decoder.conv_out", x)


def vae_decode(sd, cfg, z, rnd=_ident):
    """AutoencoderKL.decode(z).sample for z (N, latent_channels, h, w)."""
    z = F.conv2d(z, sd["post_quant_conv.weight"], sd["post_quant_conv.bias"])
    return decoder(sd, cfg, z, rnd=rnd)


def decode_latents(sd, cfg, latents, rnd=_ident):
    """AnimateDiffPipeline.decode_latents: (B, C, F, h, w) latents -> (B, 3, F, H, W) video."""
    B, C, Fr, h, w = latents.shape
    z = (latents / cfg["scaling_factor"]).permute(0, 2, 1, 3, 4).reshape(B * Fr, C, h, w)
    img = vae_decode(sd, cfg, z, rnd=rnd)
    return img[None].reshape((B, Fr) + img.shape[1:]).permute(0, 2, 1, 3, 4).float()
