"""AutoencoderKL decoder — the VAE decode of `diffusers:AnimateDiffPipeline.decode_latents`
(SURVEY.md §8f rank 1): SD-1.5's `vae` as the reference loads it with the pipeline
(experiments/05_grid_search_ablation.py:130-134) and slices it per frame
(`pipe.enable_vae_slicing()`, :143).  Module tree and parameter names are diffusers'
(`post_quant_conv`, `decoder.conv_in`, `decoder.mid_block.{resnets,attentions}`,
`decoder.up_blocks[i].{resnets,upsamplers}`, `decoder.conv_norm_out`, `decoder.conv_out`),
so diffusers-keyed safetensors load with vdiff.load_diffusers_state_dict; the encoder
(`quant_conv`, `encoder.*`) is not on the text-to-video path and is not built.

MI355X layout: frames are decoded in chunks of `frames_per_chunk` (default 8: one
chunk's 512x512x256 activation is 1 GiB, inside the GEMM's 32-bit buffer offsets; the
reference's slicing decodes 1 frame at a time on a 12 GB GPU), every activation is NHWC
bf16 rows over (frame, y, x), and each op is a vdiff kernel:
  * every conv (3x3, nearest-x2 upsample folded into the loader, 1x1 shortcut) is the
    implicit-GEMM MFMA kernel with bias / residual fused into its epilogue;
  * GroupNorm(+SiLU) is the partial / finalize / apply trio of the UNet;
  * the single-head (d = 512) mid-block attention: q,k,v = one GEMM over the normed rows
    (softmax scale * log2 e folded into q's weight and bias), then ONE flash pass over every
    frame (vd_attention with d = 512 -> flash512_kernel, csrc/attention_d512.hip: no score
    matrix in memory; round 2 materialised a 64 MB fp32 S per frame and ran GEMM ->
    vd_softmax_rows -> GEMM), out = O.W_o^T + b_o + x.
"""
from __future__ import annotations

import copy
import math
from collections import namedtuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .layers import Act, bf, f32, pack_conv3x3

DecoderOutput = namedtuple("DecoderOutput", ["sample"])

VAE_FULL = dict(  # SD-1.5 vae/config.json
    in_channels=3,
    out_channels=3,
    latent_channels=4,
    block_out_channels=(128, 256, 512, 512),
    layers_per_block=2,
    norm_num_groups=32,
    sample_size=512,
    scaling_factor=0.18215,
)

VAE_TINY = dict(VAE_FULL, block_out_channels=(64, 64), layers_per_block=1, sample_size=32)

VAE_CONFIGS = {"full": VAE_FULL, "tiny": VAE_TINY}


class VAEResnetBlock2D(nn.Module):
    """diffusers:ResnetBlock2D(temb_channels=None, eps=1e-6, groups=32) as the VAE builds it."""

    def __init__(self, in_channels, out_channels, groups=32, eps=1e-6):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.groups, self.eps = groups, eps
        self.norm1 = nn.GroupNorm(groups, in_channels, eps=eps, affine=True)
        self.conv1 = nn.Conv2d(in_channels, out_channels, 3, padding=1)
        self.norm2 = nn.GroupNorm(groups, out_channels, eps=eps, affine=True)
        self.dropout = nn.Dropout(0.0)
        self.conv2 = nn.Conv2d(out_channels, out_channels, 3, padding=1)
        self.nonlinearity = nn.SiLU()
        self.conv_shortcut = (nn.Conv2d(in_channels, out_channels, 1) if in_channels != out_channels
                              else None)

    def prepare(self):
        self._g1, self._b1 = f32(self.norm1.weight), f32(self.norm1.bias)
        self._g2, self._b2 = f32(self.norm2.weight), f32(self.norm2.bias)
        self._w1, self._c1 = pack_conv3x3(self.conv1.weight), f32(self.conv1.bias)
        self._w2, self._c2 = pack_conv3x3(self.conv2.weight), f32(self.conv2.bias)
        if self.conv_shortcut is not None:
            self._ws = bf(self.conv_shortcut.weight.reshape(self.out_channels, self.in_channels))
            self._bs = f32(self.conv_shortcut.bias)

    def forward(self, x: Act) -> Act:
        hw = x.h * x.w
        h = ops.group_norm(x.t, x.n, hw, self.groups, self.eps, self._g1, self._b1, silu=True)
        h, _, _ = ops.conv3x3(h, x.n, x.h, x.w, self._w1, bias=self._c1)
        h = ops.group_norm(h, x.n, hw, self.groups, self.eps, self._g2, self._b2, silu=True)
        sc = ops.gemm(x.t, self._ws, bias=self._bs) if self.conv_shortcut is not None else x.t
        out, _, _ = ops.conv3x3(h, x.n, x.h, x.w, self._w2, bias=self._c2, res=sc)
        return Act(out, x.n, x.h, x.w)


class VAEAttention(nn.Module):
    """diffusers:Attention of the VAE mid block: heads = 1 (dim_head = C), group_norm
    (32, eps 1e-6), biased to_q/to_k/to_v/to_out.0, residual_connection, rescale 1."""

    def __init__(self, channels, groups=32, eps=1e-6):
        super().__init__()
        self.channels, self.groups, self.eps = channels, groups, eps
        self.heads = 1
        self.group_norm = nn.GroupNorm(groups, channels, eps=eps, affine=True)
        self.to_q = nn.Linear(channels, channels)
        self.to_k = nn.Linear(channels, channels)
        self.to_v = nn.Linear(channels, channels)
        self.to_out = nn.ModuleList([nn.Linear(channels, channels), nn.Dropout(0.0)])

    def prepare(self):
        c = self.channels ** -0.5 * math.log2(math.e)  # softmax scale in log2 units, folded into q
        self._gg, self._gb = f32(self.group_norm.weight), f32(self.group_norm.bias)
        self._wqkv = bf(torch.cat([self.to_q.weight.float() * c, self.to_k.weight.float(),
                                   self.to_v.weight.float()], 0))
        self._bqkv = f32(torch.cat([self.to_q.bias.float() * c, self.to_k.bias.float(),
                                    self.to_v.bias.float()], 0))
        self._wo, self._bo = bf(self.to_out[0].weight), f32(self.to_out[0].bias)

    def forward(self, x: Act) -> Act:
        C, hw = self.channels, x.h * x.w
        n = ops.group_norm(x.t, x.n, hw, self.groups, self.eps, self._gg, self._gb)
        qkv = ops.gemm(n, self._wqkv, bias=self._bqkv)             # [n*hw, 3C], q pre-scaled
        # one flash pass over every frame (vd_attention d = 512: flash512_kernel); the scale
        # (C^-1/2 log2 e) is already in q, so the kernel's exp2 argument is the score itself
        o = ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], x.n, 1, hw, hw, C,
                          scale=1.0 / math.log2(math.e))
        out = ops.gemm(o, self._wo, bias=self._bo, res=x.t)
        return Act(out, x.n, x.h, x.w)


class UNetMidBlock2D(nn.Module):
    def __init__(self, channels, groups=32):
        super().__init__()
        self.attentions = nn.ModuleList([VAEAttention(channels, groups)])
        self.resnets = nn.ModuleList([VAEResnetBlock2D(channels, channels, groups),
                                      VAEResnetBlock2D(channels, channels, groups)])

    def forward(self, x: Act) -> Act:
        x = self.resnets[0](x)
        x = self.attentions[0](x)
        return self.resnets[1](x)


class Upsample2D(nn.Module):
    def __init__(self, channels):
        super().__init__()
        self.conv = nn.Conv2d(channels, channels, 3, padding=1)

    def prepare(self):
        self._w, self._b = pack_conv3x3(self.conv.weight), f32(self.conv.bias)

    def forward(self, x: Act) -> Act:
        t, h, w = ops.conv3x3(x.t, x.n, x.h, x.w, self._w, upsample=True, bias=self._b)
        return Act(t, x.n, h, w)


class UpDecoderBlock2D(nn.Module):
    def __init__(self, in_channels, out_channels, num_layers, add_upsample, groups=32):
        super().__init__()
        self.resnets = nn.ModuleList([VAEResnetBlock2D(in_channels if i == 0 else out_channels, out_channels,
                                                       groups) for i in range(num_layers)])
        self.upsamplers = nn.ModuleList([Upsample2D(out_channels)]) if add_upsample else None

    def forward(self, x: Act) -> Act:
        for r in self.resnets:
            x = r(x)
        if self.upsamplers is not None:
            x = self.upsamplers[0](x)
        return x


class Decoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        ch = list(reversed(cfg["block_out_channels"]))
        g = cfg["norm_num_groups"]
        self.groups = g
        self.conv_in = nn.Conv2d(cfg["latent_channels"], ch[0], 3, padding=1)
        self.mid_block = UNetMidBlock2D(ch[0], g)
        blocks, prev = [], ch[0]
        for i, c in enumerate(ch):
            blocks.append(UpDecoderBlock2D(prev, c, cfg["layers_per_block"] + 1, i < len(ch) - 1, g))
            prev = c
        self.up_blocks = nn.ModuleList(blocks)
        self.conv_norm_out = nn.GroupNorm(g, ch[-1], eps=1e-6, affine=True)
        self.conv_act = nn.SiLU()
        self.conv_out = nn.Conv2d(ch[-1], cfg["out_channels"], 3, padding=1)

    def prepare(self):
        self._gn, self._bn = f32(self.conv_norm_out.weight), f32(self.conv_norm_out.bias)
        # conv_out's 3 output channels padded to 4 (zero rows): fp32 NHWC rows of 16 bytes
        co = self.conv_out.out_channels
        self._cout = co
        self._w_out = pack_conv3x3(F.pad(self.conv_out.weight.detach().float(), (0, 0, 0, 0, 0, 0, 0, 4 - co)))
        self._b_out = f32(F.pad(self.conv_out.bias.detach().float(), (0, 4 - co)))

    def forward(self, x: Act) -> torch.Tensor:
        t, _, _ = ops.conv3x3(x.t, x.n, x.h, x.w, self._w_in, bias=self._b_in)
        x = self.mid_block(Act(t, x.n, x.h, x.w))
        for blk in self.up_blocks:
            x = blk(x)
        h = ops.group_norm(x.t, x.n, x.h * x.w, self.groups, 1e-6, self._gn, self._bn, silu=True)
        out, _, _ = ops.conv3x3(h, x.n, x.h, x.w, self._w_out, bias=self._b_out, out_f32=True)
        return out, x.h, x.w


class AutoencoderKL(nn.Module):
    """Decode side of diffusers:AutoencoderKL: `decode(z).sample`, `.config`, `.dtype`, `.device`."""

    def __init__(self, config="full"):
        super().__init__()
        cfg = copy.deepcopy(VAE_CONFIGS[config] if isinstance(config, str) else dict(config))
        self.config = cfg
        self.post_quant_conv = nn.Conv2d(cfg["latent_channels"], cfg["latent_channels"], 1)
        self.decoder = Decoder(cfg)
        self.frames_per_chunk = 8
        self._prepared = False

    @property
    def dtype(self):
        return next(self.parameters()).dtype

    @property
    def device(self):
        return next(self.parameters()).device

    def enable_slicing(self):  # diffusers API; chunked decoding is always on
        pass

    def prepare(self):
        """Pack device operands (bf16 weights, fp32 biases/affines, latent channels padded
        to 8 so the packed latent rows are 16-byte chunks, as in the UNet's conv_in)."""
        for m in reversed(list(self.modules())):
            if m is not self and hasattr(m, "prepare"):
                m.prepare()
        lc = self.config["latent_channels"]
        wq = torch.zeros(8, 8)
        wq[:lc, :lc] = self.post_quant_conv.weight.detach().float().reshape(lc, lc)
        self._w_pq = bf(wq.to(self.device))
        self._b_pq = f32(F.pad(self.post_quant_conv.bias.detach().float(), (0, 8 - lc)))
        d = self.decoder
        d._w_in = pack_conv3x3(d.conv_in.weight, cin_pad=8)
        d._b_in = f32(d.conv_in.bias)
        self._prepared = True
        return self

    def decode_rows(self, z_rows, n, h, w):
        """Packed latent rows [n*h*w, 8] (channels >= latent_channels zero) -> fp32 rows
        [n*H*W, 4] (channel 3 is padding)."""
        zq = ops.gemm(z_rows, self._w_pq, bias=self._b_pq)  # post_quant_conv (1x1), pad channels stay 0
        return self.decoder(Act(zq, n, h, w))

    @torch.no_grad()
    def decode(self, z: torch.Tensor, return_dict: bool = True):
        """z (N, latent_channels, h, w) -> DecoderOutput(sample=(N, 3, 8h, 8w) fp32)."""
        if not self._prepared:
            self.prepare()
        N, C, h, w = z.shape
        outs = []
        for i in range(0, N, self.frames_per_chunk):
            zc = z[i:i + self.frames_per_chunk].to(self.device, torch.float32)
            n = zc.shape[0]
            rows = ops.pack_latents(zc.permute(1, 0, 2, 3)[None].contiguous(), dup=1, cpad=8)
            out, H, W = self.decode_rows(rows, n, h, w)
            outs.append(ops.unpack_nhwc(out, 1, self.decoder._cout, n, H, W)[0].permute(1, 0, 2, 3))
        img = torch.cat(outs, 0)
        return DecoderOutput(img) if return_dict else (img,)
