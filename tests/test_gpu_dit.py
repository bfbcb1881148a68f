"""DiT-style denoiser (BASELINE config 5) on the MI355X against the
CPU oracle (oracle/dit_ref.py) and plain fp32 torch references of each new kernel.

Tolerances: patchify / unpatchify move values (bit-exact up to the bf16 rounding of the
patch rows); RoPE and the adaLN row pass compute in fp32 from bf16 inputs and store bf16
(2^-7 relative); the tiny model and its 3-step CFG DDIM loop are compared by relative L2
against the fp32 oracle fixture (3 % / 1 %, the bounds the UNet uses).  Parity of the DiT
to any external implementation is unpinned (the reference has none).
"""
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import dit_ref
from vdiff import ops
from vdiff.models.dit import DIT_TINY, DiT3DModel, DiTDenoiseLoop, init_dit_state_dict
from vdiff.sched.ddim import DDIMScheduler

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"


def rel_l2(got, want):
    got, want = got.double().cpu(), want.double().cpu()
    return ((got - want).norm() / want.norm()).item()


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD / "dit_tiny.npz")


@pytest.fixture(scope="module")
def tiny_dit(cuda):
    return DiT3DModel(DIT_TINY, init_dit_state_dict(DIT_TINY, seed=0), device=cuda)


@pytest.mark.parametrize("shape,p,dup", [((1, 4, 4, 16, 16), 2, 2), ((2, 4, 3, 12, 20), 2, 1),
                                         ((1, 3, 2, 9, 6), 3, 1)])
def test_patchify_unpatchify(cuda, shape, p, dup):
    g = torch.Generator().manual_seed(0)
    lat = torch.randn(shape, generator=g)
    B, C, F, H, W = shape
    kpad = (C * p * p + 7) // 8 * 8
    tok = ops.patchify(lat.cuda(), p, kpad, dup=dup, in_div=2.0).float().cpu()
    ref = lat.reshape(B, C, F, H // p, p, W // p, p).permute(0, 2, 3, 5, 1, 4, 6)
    ref = (ref.reshape(-1, C * p * p) / 2.0).to(torch.bfloat16).float()
    n = ref.shape[0]
    assert tok.shape == (dup * n, kpad)
    assert torch.equal(tok[:n, :C * p * p], ref) and not tok[:, C * p * p:].any()
    if dup == 2:
        assert torch.equal(tok[n:], tok[:n])
    # unpatchify of token rows [(n,hp,wp)][(ph,pw,c)] -> NHWC pixel rows
    src = torch.randn(B * F * (H // p) * (W // p), p * p * C + 4, generator=g)
    pix = ops.unpatchify(src.cuda()[:, :p * p * C], B * F, H, W, p, C).cpu()
    want = src[:, :p * p * C].reshape(B * F, H // p, W // p, p, p, C).permute(0, 1, 3, 2, 4, 5)
    assert torch.equal(pix, want.reshape(-1, C))


@pytest.mark.parametrize("mode", [0, 1])
def test_rope_kernel_matches_oracle(cuda, mode):
    g = torch.Generator().manual_seed(1)
    B, F, Hp, Wp, heads, d = 2, 5, 6, 7, 3, 64
    D = heads * d
    rows = B * F * Hp * Wp
    qkv = (torch.randn(rows, 3 * D + 8, generator=g)).to(torch.bfloat16)
    x = qkv.cuda()
    ops.rope_qk(x, 2 * D, d, mode, F, Hp, Wp, 10000.0)
    got = x.float().cpu()
    r = torch.arange(rows)
    z = qkv.float()[:, :2 * D].reshape(rows, 2 * heads, d)
    if mode == 0:
        zh = dit_ref.rope(z[..., :d // 2].transpose(0, 1), (r // Wp) % Hp, 10000.0).transpose(0, 1)
        zw = dit_ref.rope(z[..., d // 2:].transpose(0, 1), r % Wp, 10000.0).transpose(0, 1)
        want = torch.cat([zh, zw], -1)
    else:
        want = dit_ref.rope(z.transpose(0, 1), (r // (Hp * Wp)) % F, 10000.0).transpose(0, 1)
    torch.testing.assert_close(got[:, :2 * D].reshape(rows, 2 * heads, d), want, rtol=2 ** -7, atol=2e-2)
    assert torch.equal(got[:, 2 * D:], qkv.float()[:, 2 * D:])  # v and padding untouched


@pytest.mark.parametrize("C", [128, 320, 1152, 2048])
@pytest.mark.parametrize("with_y", [True, False])
def test_res_ln_mod_matches_torch(cuda, C, with_y):
    g = torch.Generator().manual_seed(C)
    rows, B = 70, 2
    x = torch.randn(rows, C, generator=g).to(torch.bfloat16)
    y = torch.randn(rows, C, generator=g).to(torch.bfloat16)
    mod = torch.randn(B, 3 * C + 4, generator=g) * 0.5
    gate, shift, scale = mod[:, :C], mod[:, C:2 * C], mod[:, 2 * C:3 * C]
    xc = x.cuda().clone()
    modc = mod.cuda()
    h = ops.res_ln_mod(xc, y=y.cuda() if with_y else None, gate=modc[:, :C] if with_y else None,
                       shift=modc[:, C:2 * C], scale=modc[:, 2 * C:3 * C], rows_per_b=35,
                       x_out=xc if with_y else None)
    b = torch.arange(rows) // 35
    xn = x.float() + gate[b] * y.float() if with_y else x.float()
    if with_y:
        torch.testing.assert_close(xc.float().cpu(), xn, rtol=2 ** -7, atol=1e-2)
        xn = xc.float().cpu()  # the kernel normalises the stored (bf16) residual
    want = torch.nn.functional.layer_norm(xn, (C,), eps=1e-6) * (1 + scale[b]) + shift[b]
    torch.testing.assert_close(h.float().cpu(), want, rtol=2 ** -7, atol=2e-2)


def test_gemm_gelu_epilogue(cuda):
    g = torch.Generator().manual_seed(2)
    for M, N, K in ((300, 256, 128), (4096, 1152, 1152), (2, 4608, 1152)):
        a = torch.randn(M, K, generator=g).to(torch.bfloat16)
        w = (torch.randn(N, K, generator=g) * 0.05).to(torch.bfloat16)
        bias = torch.randn(N, generator=g) * 0.1
        out = ops.gemm(a.cuda(), w.cuda(), bias=bias.cuda(), act=ops.ACT_GELU).float().cpu()
        want = torch.nn.functional.gelu(a.float() @ w.float().t() + bias)
        torch.testing.assert_close(out, want, rtol=2 ** -6, atol=2e-2)


@pytest.mark.parametrize("F", [4, 16, 17, 27, 32])
@pytest.mark.parametrize("d", [40, 64, 80, 160])
def test_temporal_attention_mfma_up_to_32_frames(cuda, F, d):
    """The full DiT config attends over 32 frames with d = 64: temporal_mfma32_kernel for
    17..32 frames, temporal_mfma_kernel (now also d = 64) up to 16, ragged frame counts."""
    g = torch.Generator().manual_seed(5 + F + d)
    B, P, heads = 2, 12, 3
    D = heads * d
    qkv = torch.randn(B * F * P, 3 * D, generator=g).to(torch.bfloat16)
    c = qkv.cuda()
    o = ops.temporal_attention(c[:, :D], c[:, D:2 * D], c[:, 2 * D:], B, F, P, heads, d).float().cpu()
    t = qkv.float().reshape(B, F, P, 3, heads, d).permute(3, 0, 2, 4, 1, 5)  # qkv b p h f d
    want = torch.nn.functional.scaled_dot_product_attention(t[0], t[1], t[2])
    want = want.permute(0, 3, 1, 2, 4).reshape(B * F * P, D)
    torch.testing.assert_close(o, want, rtol=2 ** -6, atol=1e-2)


@pytest.mark.parametrize("t", [961, 500])
def test_tiny_dit_matches_oracle(tiny_dit, gold, t):
    lat = torch.from_numpy(gold["latents"]).cuda()
    ehs = torch.from_numpy(gold["ehs"]).cuda()
    out = tiny_dit(torch.cat([lat, lat]), t, encoder_hidden_states=ehs).sample
    assert out.shape == (2, 4, 4, 16, 16) and out.dtype == torch.float32
    err = rel_l2(out, torch.from_numpy(gold[f"eps_t{t}"]))
    assert err < 0.03, err


@pytest.mark.parametrize("use_graph", [True, False])
def test_dit_denoise_loop_matches_oracle(tiny_dit, gold, use_graph):
    lat = torch.from_numpy(gold["latents"]).cuda()
    ehs = torch.from_numpy(gold["ehs"]).cuda()
    s = DDIMScheduler(beta_schedule="linear", steps_offset=1, clip_sample=False)
    s.set_timesteps(50)
    loop = DiTDenoiseLoop(tiny_dit, s, lat, ehs, 7.5, use_graph=use_graph).prime()
    assert (loop.graph is not None) == use_graph
    x = loop.run(3)
    assert int(loop.step_idx.item()) == 3
    err = rel_l2(x, torch.from_numpy(gold["loop3_x"]))
    assert err < 0.01, err
