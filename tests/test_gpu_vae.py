"""VAE decode on the MI355X against the CPU oracle (oracle/vae_ref.py).

Tolerances: the device path stores bf16 activations; the tiny decoder is compared by
relative L2 against the fp32 oracle fixture (bound 3%: the bf16-storage-emulating oracle
itself lands at 1.6%) and the mid-block attention alone, with sharpened weights so the
softmax is far from uniform, at 2.5%.  Parity to diffusers is unpinned (oracle header).
"""
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import vae_ref
from vdiff import AnimateDiffPipeline, AutoencoderKL, init_synthetic_, ops
from vdiff.models.layers import Act
from vdiff.models.vae import VAE_TINY, VAEAttention

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"


def rel_l2(got, want):
    got, want = got.double().cpu(), want.double().cpu()
    return ((got - want).norm() / want.norm()).item()


@pytest.fixture(scope="module")
def tiny_vae(cuda):
    return init_synthetic_(AutoencoderKL("tiny"), seed=0).to("cuda", torch.bfloat16).prepare()


def test_softmax_rows_matches_torch(cuda):
    for rows, cols in ((7, 4096), (300, 256), (3, 12)):
        s = torch.randn(rows, cols, device=cuda) * 6
        p = ops.softmax_rows(s)
        want = torch.softmax(s.double() * np.log(2.0), -1)
        torch.testing.assert_close(p.double(), want, rtol=2 ** -7, atol=1e-6)
    big = torch.randn(4, 8192, device=cuda)[:, :4096]  # strided rows
    torch.testing.assert_close(ops.softmax_rows(big).double(), torch.softmax(big.double() * np.log(2.0), -1),
                               rtol=2 ** -7, atol=1e-6)


def _flash512_emulated(q, k, v, n, S, m_mode):
    """fp64 restatement of flash512_kernel's arithmetic: per query the offset m is the first
    32-key tile's row max (m_mode "tile0") or the exact row max (the block's exact rerun,
    "exact"); e = 2^(s - m), P = bf16(e) for P.V, the row sum l over the unrounded e.  The
    one freedom left is the last ulps of s (fp32 MFMA accumulation) and of v_exp_f32: where e
    lies within 2^-15 (relative) of a bf16 rounding midpoint the kernel's P may round the other
    way; `slack` is exactly what those flips can move O by (as the d = 40 real-valued test)."""
    outs, slacks = [], []
    for i in range(n):
        r = slice(i * S, (i + 1) * S)
        s = q[r].double() @ k[r].double().T                   # log2 units (scale folded into q)
        m = s[:, :32].amax(1, keepdim=True) if m_mode == "tile0" else s.amax(1, keepdim=True)
        e = torch.exp2(s - m)
        del s
        p = e.float().to(torch.bfloat16).double()
        l = e.sum(1, keepdim=True)
        vd = v[r].double()
        want = (p @ vd) / l
        _, ex = torch.frexp(e)
        ulp = torch.ldexp(torch.full_like(e, 2.0 ** -8), ex)
        mid = (torch.floor(e / ulp) + 0.5) * ulp
        dp = torch.where((e - mid).abs() <= e * 2.0 ** -15, ulp, torch.zeros_like(e))
        slacks.append((dp @ vd.abs()) / l)
        outs.append(want)
    return torch.cat(outs), torch.cat(slacks)


@pytest.mark.parametrize("S", [4096, 1000, 96])
def test_flash512_matches_fp64(cuda, S):
    """vd_attention at d = 512 (flash512_kernel, the VAE mid-block attention) with fp32 output
    against the fp64 emulation of its rounding points, at the north-star tolerance rtol 1e-3 /
    atol 1e-4: S = 4096 (the decode's 64x64 latents), a ragged 1000 (last key tile masked, last
    query block partial) and a single query block (96)."""
    n, d = 2, 512
    g = torch.Generator(device=cuda).manual_seed(11)
    qkv = torch.randn(n * S, 3 * d, device=cuda, generator=g)
    qkv[:, :d] *= 0.06   # scores of a few log2 units, as the model's folded q gives
    qkv = qkv.to(torch.bfloat16)
    q, k, v = qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:]
    scale = 1.0 / np.log2(np.e)
    got = ops.attention(q, k, v, n, 1, S, S, d, scale=scale, out_f32=True).double().cpu()
    want, slack = _flash512_emulated(q.cpu(), k.cpu(), v.cpu(), n, S, "tile0")
    err = (got - want).abs()
    print(f"flash512 S={S}: max |O - O_ref(bf16 P)| {err.max().item():.2e}, max flip allowance "
          f"{slack.max().item():.2e}, |O| max {want.abs().max().item():.3f}")
    assert torch.all(err <= 1e-4 + 1e-3 * want.abs() + slack), (err - 1e-3 * want.abs() - slack).max().item()
    # the bf16-output kernel rounds the same values once
    got16 = ops.attention(q, k, v, n, 1, S, S, d, scale=scale).double().cpu()
    assert torch.all((got16 - want).abs() <= 1e-4 + 2 ** -8 * want.abs() + slack)


def test_flash512_exact_rerun(cuda):
    """A key far above every query's first-tile max (+40 log2 units: P would reach 2^40 against
    the fast pass's fixed offset) sends the block through the exact rerun (QK-only max sweep,
    then the flash sweep with the true row max); the result matches the emulation with m =
    the exact row max."""
    n, S, d = 1, 512, 512
    g = torch.Generator(device=cuda).manual_seed(5)
    u = torch.randn(d, device=cuda, generator=g)
    u = u / u.norm()
    q = torch.randn(n * S, d, device=cuda, generator=g) * 0.02 + u
    k = torch.randn(n * S, d, device=cuda, generator=g) * 0.02
    k[300] = 40.0 * u
    v = torch.randn(n * S, d, device=cuda, generator=g)
    q, k, v = (t.to(torch.bfloat16) for t in (q, k, v))
    got = ops.attention(q, k, v, n, 1, S, S, d, scale=1.0 / np.log2(np.e), out_f32=True).double().cpu()
    want, slack = _flash512_emulated(q.cpu(), k.cpu(), v.cpu(), n, S, "exact")
    err = (got - want).abs()
    assert torch.all(err <= 1e-4 + 1e-3 * want.abs() + slack), (err - 1e-3 * want.abs() - slack).max().item()


def test_vae_attention_block_matches_oracle(cuda):
    C, n, h, w = 64, 2, 16, 16
    g = torch.Generator().manual_seed(3)
    m = VAEAttention(C)
    with torch.no_grad():
        for name, p in m.named_parameters():
            std = 0.3 if name.startswith(("to_q", "to_k")) else 0.1
            r = torch.randn(p.shape, generator=g) * std + (1.0 if name == "group_norm.weight" else 0.0)
            p.copy_(r.to(torch.bfloat16).float())
    sd = {f"a.{k}": v.float() for k, v in m.state_dict().items()}
    m = m.to("cuda", torch.bfloat16)
    m.prepare()
    x = (torch.randn(n, C, h, w, generator=g) + 0.3).to(torch.bfloat16).float()
    rows = x.permute(0, 2, 3, 1).reshape(-1, C).to("cuda", torch.bfloat16).contiguous()
    out = m(Act(rows, n, h, w)).t.float().cpu().reshape(n, h, w, C).permute(0, 3, 1, 2)
    want = vae_ref.attention(sd, "a", x, 32)
    assert rel_l2(out - x, want - x) < 0.025  # the attention branch itself, not the residual


def test_tiny_vae_decode_matches_oracle(tiny_vae):
    gold = np.load(GOLD / "vae_tiny.npz")
    lat = torch.from_numpy(gold["latents"]).cuda()
    pipe = AnimateDiffPipeline.__new__(AnimateDiffPipeline)
    pipe.vae = tiny_vae
    video = pipe.decode_latents(lat)
    assert video.shape == (1, 3, 2, 32, 32) and video.dtype == torch.float32
    assert rel_l2(video, torch.from_numpy(gold["video"])) < 0.03
    assert rel_l2(video, torch.from_numpy(gold["video_bf16emu"])) < 0.03
    # chunked decoding (1 frame per chunk, the reference's enable_vae_slicing) gives the same frames
    tiny_vae.frames_per_chunk = 1
    try:
        torch.testing.assert_close(pipe.decode_latents(lat), video, rtol=0, atol=0)
    finally:
        tiny_vae.frames_per_chunk = 8
    pt = pipe.postprocess_video(video, "pt")
    assert pt.shape == (1, 2, 3, 32, 32) and float(pt.min()) >= 0 and float(pt.max()) <= 1


def test_pipeline_end_to_end_with_vae(cuda):
    """prompt -> 2 DDIM steps on the tiny UNet -> VAE decode, output_type "np" (the
    reference's pipe(...).frames[0] surface with frames as arrays instead of PIL)."""
    pipe = AnimateDiffPipeline.from_config("tiny", vae="tiny")
    out = pipe(prompt="a cat", negative_prompt="", num_frames=2, height=64, width=64, num_inference_steps=2,
               guidance_scale=7.5, generator=torch.Generator().manual_seed(42), output_type="np")
    frames = out.frames[0]
    assert frames.shape == (2, 16, 16, 3) and np.isfinite(frames).all()  # tiny VAE: one x2 upsample of 8x8 latents
    assert frames.min() >= 0 and frames.max() <= 1


def test_full_vae_one_frame_matches_oracle(cuda):
    """The FULL SD-1.5 decoder shapes (49.5M params: 64x64 latents -> 512x512, the d = 512
    mid-block attention over 4096 tokens, the 512^2 x 128-channel convs) on one frame against
    the fp32 oracle on the same bf16 weights (~3 s of host CPU).  Bound: rel-L2 3 %."""
    from vdiff.models.vae import VAE_FULL
    vae = init_synthetic_(AutoencoderKL("full"), seed=0).to("cuda", torch.bfloat16).prepare()
    pipe = AnimateDiffPipeline.__new__(AnimateDiffPipeline)
    pipe.vae = vae
    lat = (torch.randn((1, 4, 1, 64, 64), generator=torch.Generator().manual_seed(6)) * 0.18215)
    got = pipe.decode_latents(lat.cuda()).cpu()
    sd = {k: v.detach().float().cpu() for k, v in vae.state_dict().items()}
    with torch.no_grad():
        want = vae_ref.decode_latents(sd, VAE_FULL, lat)
    err = rel_l2(got, want)
    print(f"full VAE decode (1 frame) rel-L2 vs oracle: {err:.4f}")
    assert got.shape == (1, 3, 1, 512, 512) and err < 0.03, err
