"""ORACLE — test infrastructure only.  Never imported by the product path.

fp32 PyTorch-CPU restatement of the build-defined DiT-style video denoiser of SURVEY.md
§8f rank 3 / BASELINE config 5 ("DiT-style transformer denoiser (patchified 3D latents)").
The reference has NO DiT (its only denoiser is diffusers' UNetMotionModel), so this model
is defined by the build and its parity is "parity unpinned" with respect to any external
implementation; it follows the public DiT / Latte recipe:

  * patch embed: Conv3d(C_in, D, kernel (1, p, p), stride (1, p, p)) over (B, C, F, H, W)
    -> tokens (b, f, hp, wp) x D;
  * timestep: sinusoidal(256, [cos, sin], diffusers' get_timestep_embedding with
    flip_sin_to_cos=True, shift 0) -> Linear(256, D) -> SiLU -> Linear(D, D) = c;
  * `depth` blocks alternating spatial (even index: attention over the Hp*Wp tokens of
    one frame, 2-D RoPE on (h, w)) and temporal (odd index: attention over the F frames
    of one patch position, 1-D RoPE on f), each
        shift1, scale1, gate1, shift2, scale2, gate2 = Linear(SiLU(c)) (adaLN-Zero layout)
        x = x + gate1 * SelfAttn(RoPE)(LN(x) * (1 + scale1) + shift1)
        x = x + CrossAttn(LN(x), text)                 (per video, text K/V)
        x = x + gate2 * MLP(LN(x) * (1 + scale2) + shift2),  MLP = fc2(gelu_erf(fc1))
    with LN = LayerNorm(D, eps 1e-6, no affine), heads of width d = D / heads;
  * final: shift, scale = Linear(SiLU(c)); out = Linear(LN(x)*(1+scale)+shift) to
    p*p*C_out features ordered (ph, pw, c), unpatchified to (B, C_out, F, H, W).
RoPE: rotate-half pairs (i, i + S/2) inside a section of width S at angle
pos * theta^(-2i/S); spatial sections are the two halves of a head (h, then w).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

EPS = 1e-6


def timestep_embedding(t: torch.Tensor, dim: int) -> torch.Tensor:
    half = dim // 2
    freqs = torch.exp(-math.log(10000.0) * torch.arange(half, dtype=torch.float32) / half)
    arg = t.float()[:, None] * freqs[None]
    return torch.cat([torch.cos(arg), torch.sin(arg)], dim=1)


def rope(x: torch.Tensor, pos: torch.Tensor, theta: float) -> torch.Tensor:
    """x (..., S) rotated by pos (broadcast over the leading dims), rotate-half pairing."""
    S = x.shape[-1]
    half = S // 2
    inv = theta ** (-(2.0 * torch.arange(half, dtype=torch.float64)) / S)
    ang = (pos.double()[..., None] * inv).float()
    cs, sn = torch.cos(ang), torch.sin(ang)
    a, b = x[..., :half], x[..., half:]
    return torch.cat([a * cs - b * sn, b * cs + a * sn], dim=-1)


def _ln(x):
    return F.layer_norm(x, (x.shape[-1],), eps=EPS)


def _lin(x, sd, key):
    return F.linear(x, sd[key + ".weight"], sd[key + ".bias"])


def _attn(q, k, v, heads):
    """q (N, Sq, D), k/v (N, Sk, D) -> (N, Sq, D), softmax attention per head."""
    N, Sq, D = q.shape
    d = D // heads
    q = q.view(N, Sq, heads, d).transpose(1, 2)
    k = k.view(N, k.shape[1], heads, d).transpose(1, 2)
    v = v.view(N, v.shape[1], heads, d).transpose(1, 2)
    o = F.scaled_dot_product_attention(q, k, v)
    return o.transpose(1, 2).reshape(N, Sq, D)


def forward(sd: dict, cfg: dict, sample: torch.Tensor, timestep, ehs: torch.Tensor) -> torch.Tensor:
    sd = {k: v.float() for k, v in sd.items()}
    B, Cin, Fr, H, W = sample.shape
    p, D, heads = cfg["patch_size"], cfg["hidden_size"], cfg["num_heads"]
    d = D // heads
    Hp, Wp = H // p, W // p
    S = Hp * Wp
    theta = cfg["rope_theta"]
    t = torch.as_tensor(timestep, dtype=torch.float32).reshape(-1).expand(B)
    # patch embed (Conv3d (1,p,p)) -> x[b, f, s, D]
    pe = F.conv3d(sample.float(), sd["patch_embed.weight"], sd["patch_embed.bias"], stride=(1, p, p))
    x = pe.permute(0, 2, 3, 4, 1).reshape(B, Fr, S, D)
    c = _lin(F.silu(_lin(timestep_embedding(t, cfg["freq_dim"]), sd, "t_embedder.linear_1")), sd,
             "t_embedder.linear_2")
    sc = F.silu(c)
    hpos = torch.arange(S) // Wp
    wpos = torch.arange(S) % Wp
    fpos = torch.arange(Fr)
    for i in range(cfg["depth"]):
        pre = f"blocks.{i}."
        mod = _lin(sc, sd, pre + "adaLN_modulation")  # (B, 6D)
        sh1, sc1, g1, sh2, sc2, g2 = [m[:, None, None, :] for m in mod.chunk(6, dim=1)]
        h = _ln(x) * (1 + sc1) + sh1
        q, k, v = _lin(h, sd, pre + "attn.to_qkv").chunk(3, dim=-1)
        if i % 2 == 0:  # spatial: sequences = frames, 2-D RoPE
            def rot(z):
                z = z.view(B, Fr, S, heads, 2, d // 2)
                zh = rope(z[..., 0, :].transpose(2, 3), hpos, theta).transpose(2, 3)
                zw = rope(z[..., 1, :].transpose(2, 3), wpos, theta).transpose(2, 3)
                return torch.stack([zh, zw], dim=4).reshape(B, Fr, S, D)
            q, k = rot(q), rot(k)
            o = _attn(q.reshape(B * Fr, S, D), k.reshape(B * Fr, S, D), v.reshape(B * Fr, S, D), heads)
            o = o.view(B, Fr, S, D)
        else:  # temporal: sequences = patch positions, 1-D RoPE over frames
            def rot(z):
                z = z.view(B, Fr, S, heads, d).permute(0, 2, 3, 1, 4)  # b s h f d
                return rope(z, fpos, theta).permute(0, 3, 1, 2, 4).reshape(B, Fr, S, D)
            q, k = rot(q), rot(k)
            tq = lambda z: z.permute(0, 2, 1, 3).reshape(B * S, Fr, D)
            o = _attn(tq(q), tq(k), tq(v), heads).view(B, S, Fr, D).permute(0, 2, 1, 3)
        x = x + g1 * _lin(o, sd, pre + "attn.to_out")
        h = _ln(x)
        q = _lin(h, sd, pre + "cross.to_q").reshape(B, Fr * S, D)
        kk, vv = _lin(ehs.float(), sd, pre + "cross.to_kv").chunk(2, dim=-1)
        o = _attn(q, kk, vv, heads).view(B, Fr, S, D)
        x = x + _lin(o, sd, pre + "cross.to_out")
        h = _ln(x) * (1 + sc2) + sh2
        m = F.gelu(_lin(h, sd, pre + "mlp.fc1"))
        x = x + g2 * _lin(m, sd, pre + "mlp.fc2")
    shf, scf = [m[:, None, None, :] for m in _lin(sc, sd, "final.adaLN_modulation").chunk(2, dim=1)]
    out = _lin(_ln(x) * (1 + scf) + shf, sd, "final.linear")  # (B, F, S, p*p*C)
    Co = cfg["out_channels"]
    out = out.view(B, Fr, Hp, Wp, p, p, Co).permute(0, 6, 1, 2, 4, 3, 5)
    return out.reshape(B, Co, Fr, H, W)
