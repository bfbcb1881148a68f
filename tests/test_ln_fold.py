"""LayerNorm folded into its consuming GEMM (round 5; vd_gemm_desc.ln_fold_s, LnFold) — CPU side:
the algebra of the fold, the plan's decisions (vd_gemm_plan is host-only: no launch), and the
device-emulating oracle's folded form against diffusers' LayerNorm -> Linear.  The kernel itself is
tested on the GPU (tests/test_gpu_kernels.py::test_gemm_ln_fold)."""
import ctypes

import pytest
import torch

from oracle import unet_ref
from vdiff import _lib as L
from vdiff import ops
from vdiff.models.layers import LnFold, pack_geglu


def _ln(K, seed=0):
    g = torch.Generator().manual_seed(seed)
    n = torch.nn.LayerNorm(K)
    with torch.no_grad():
        n.weight.copy_(1 + 0.2 * torch.randn(K, generator=g))
        n.bias.copy_(0.1 * torch.randn(K, generator=g))
    return n


def _folded_eval(fold, x):
    """fp64 of the arithmetic the kernel performs: rstd (x W'^T - mean s) + b'."""
    xd = x.double()
    mean = xd.mean(1, keepdim=True)
    rstd = (xd.var(1, unbiased=False, keepdim=True) + fold.eps).rsqrt()
    return rstd * (xd @ fold.w.double().T - mean * fold.s.double()) + fold.b.double()


@pytest.mark.parametrize("offset", [0.0, 30.0])
def test_fold_equals_layernorm_linear(offset):
    """r(x W'^T - mean s) + b' == W (gamma∘(x - mean) r + beta) + b: to fp64 roundoff with W' kept
    in fp64, and within the bf16 rounding of W' as the product stores it — including rows whose
    mean is 30 std (the cancellation the kernel's fp32 accumulators must carry)."""
    K, N, M = 320, 96, 64
    g = torch.Generator().manual_seed(1)
    norm = _ln(K)
    w = torch.randn(N, K, generator=g) * K ** -0.5
    b = torch.randn(N, generator=g) * 0.1
    x = torch.randn(M, K, generator=g) + offset + 0.5 * torch.randn(M, 1, generator=g)
    want = torch.nn.functional.linear(torch.nn.functional.layer_norm(x.double(), (K,), norm.weight.double(),
                                                                     norm.bias.double(), norm.eps), w.double(), b.double())
    fold = LnFold(norm, w, b)
    # exact algebra: the same identity with W' unrounded
    wf = w.double() * norm.weight.double()
    xd = x.double()
    mean = xd.mean(1, keepdim=True)
    rstd = (xd.var(1, unbiased=False, keepdim=True) + norm.eps).rsqrt()
    exact = rstd * (xd @ wf.T - mean * wf.sum(1)) + (w.double() @ norm.bias.double() + b.double())
    assert (exact - want).abs().max().item() < 1e-9 * (1 + offset)
    got = _folded_eval(fold, x)
    err = ((got - want).norm() / want.norm()).item()
    assert err < 4e-3, err  # bf16 W' (2^-9 relative per weight), not the row offset
    assert fold.w.dtype == torch.bfloat16 and fold.s.dtype == torch.float32 and fold.b.dtype == torch.float32
    assert torch.equal(fold.s, fold.w.double().sum(1).float())


def test_fold_geglu_packing_commutes():
    """pack_geglu after folding: the packed W', s and b' are the row permutation of the unpacked
    ones, so the GEGLU epilogue's (hidden, gate) pairing is unchanged."""
    K, N = 320, 2 * 64
    g = torch.Generator().manual_seed(2)
    norm = _ln(K, 3)
    w = torch.randn(N, K, generator=g) * K ** -0.5
    b = torch.randn(N, generator=g)
    plain, packed = LnFold(norm, w, b), LnFold(norm, w, b, pack=pack_geglu)
    assert torch.equal(packed.w, pack_geglu(plain.w))
    assert torch.equal(packed.b, pack_geglu(plain.b))
    assert torch.equal(packed.s, pack_geglu(plain.s))


def test_oracle_folded_linear_matches_layernorm_linear():
    """The device-emulating oracle's folded form (unet_ref.folded_linear) is LayerNorm -> Linear
    up to the bf16 rounding of W∘gamma."""
    K, N, M = 320, 64, 50
    g = torch.Generator().manual_seed(4)
    norm = _ln(K, 5)
    sd = {"n.weight": norm.weight.detach(), "n.bias": norm.bias.detach()}
    w = torch.randn(N, K, generator=g) * K ** -0.5
    b = torch.randn(N, generator=g)
    x = torch.randn(3, M, K, generator=g) * 2 + 1
    got = unet_ref.folded_linear(sd, "n", x, w, b)
    want = torch.nn.functional.linear(unet_ref.layer_norm(sd, "n", x), w, b)
    assert ((got - want).norm() / want.norm()).item() < 4e-3


def _desc(M, N, K=320, act=0, path=0, plan_m=0, **kw):
    nout = N // 2 if act == ops.ACT_GEGLU else N
    d = L.GemmDesc(a0=256, lda0=K, k0=K, a_mode=0, w=256, ldw=K, M=M, N=N, K=K, bias=256, act=act, out=256,
                   ldc=nout, ln_fold_s=256, ln_fold_eps=1e-5, path=path, plan_m=plan_m)
    for k, v in kw.items():
        setattr(d, k, v)
    return d


def _plan(d):
    k, sp = ctypes.c_int32(-1), ctypes.c_int32(-1)
    assert L.lib().vd_gemm_plan(ctypes.byref(d), ctypes.byref(k), ctypes.byref(sp)) == 0
    return k.value, sp.value


def test_gn_small_rule_mirrors_library():
    """vd_gn_small decides from (pix, C, groups) before reading any operand: with null pointers it
    returns VD_EUNSUPPORTED exactly where vdiff.ops.gn_small_chunk says 0, and VD_EINVAL (the
    null operands) where the mirror takes the shape; the UNet's levels 3-4 / mid norms are taken,
    levels 1-2 (C / groups = 10, 20) are not."""
    cases = [(pix, C) for pix in (16, 64, 256, 1024, 4096, 100) for C in (320, 640, 960, 1280, 1920, 2560)]
    for pix, C in cases:
        rc = L.lib().vd_gn_small(None, C, C, None, 0, C, 4, pix, 32, 1e-5, None, None, 1, None, C, None)
        taken = ops.gn_small_chunk(pix, C, 32)
        assert rc == (1000 if taken else 1001), (pix, C, rc, taken)
    assert ops.gn_small_chunk(256, 1280, 32) == 80 and ops.gn_small_chunk(64, 1280, 32) == 320
    assert ops.gn_small_chunk(64, 2560, 32) == 320 and ops.gn_small_chunk(256, 2560, 32) == 80
    assert ops.gn_small_chunk(4096, 320, 32) == 0 and ops.gn_small_chunk(1024, 640, 32) == 0
    assert ops.gn_small_chunk(256, 1920, 32) == 0   # C / groups = 60: a piece would straddle groups


def test_plan_skinny_m_v9_forced_only():
    """vd_gemm_plan: M <= 16 dense rows (the time-embedding MLP, M = the UNet batch) run on v1 in
    the product plan and on v9 (bit-identical to v1) only when forced (path 9; round 6: v9's
    rank-step gain and 16-frame loss come from the same M = 2 GEMMs); a forced v9 on a GEGLU, a
    folded LayerNorm or M = 17 keeps the automatic plan."""
    d = _desc(2, 1280, K=1280)
    d.ln_fold_s = None
    assert _plan(d)[0] == 1
    d.path = 9
    assert _plan(d) == (9, 1)
    d.M = 16
    assert _plan(d) == (9, 1)
    d.M = 17
    assert _plan(d)[0] == 1
    d.M, d.path = 2, 1
    assert _plan(d)[0] == 1
    g = _desc(2, 2560, K=1280, act=ops.ACT_GEGLU)
    g.ln_fold_s = None
    g.path = 9
    assert _plan(g)[0] == 1
    assert _plan(_desc(2, 1280, K=1280))[0] == 0  # a fold at M = 2: no kernel, the unfolded form


def test_plan_folds_on_v8_and_unsplit_v6():
    """vd_gemm_plan: a folded LayerNorm runs on v8 where the automatic plan would take v8
    (M >= 16384, K = 320, N a multiple of 160) or where v8 is forced (path 8, M >= 4096), and on
    v6 wherever the plain GEMM's plan is an unsplit v6 (the small M of a frame shard); every other
    shape — v2 / v3 plans, split K — reports kernel 0: vd_gemm refuses it and the model keeps the
    unfolded form."""
    assert _plan(_desc(16384, 960)) == (8, 1)
    assert _plan(_desc(131072, 2560, act=ops.ACT_GEGLU)) == (8, 1)
    assert _plan(_desc(8192, 320)) == (6, 1)          # below the automatic v8 range: v6
    assert _plan(_desc(8192, 320, path=8))[0] == 8    # forced
    assert _plan(_desc(1024, 3840, K=1280)) == (6, 1)  # L3 QKV at 4 images
    assert _plan(_desc(256, 10240, K=1280, act=ops.ACT_GEGLU)) == (6, 1)
    assert _plan(_desc(4096, 1920, K=640))[0] == 0    # the plain plan is v2
    assert _plan(_desc(32768, 1920, K=640))[0] == 0   # the plain plan is v3
    assert _plan(_desc(1024, 1280, K=1280, path=6))[0] == 0  # forced v6 splits K: no fold
    assert _plan(_desc(131072, 320, plan_m=8192)) == (6, 1)  # planned as a small shard: v6
    d = _desc(16384, 320)
    d.ln_fold_s = None
    assert _plan(d)[0] == 8                           # the unfolded GEMM itself is still v8


def test_fold_shape_gate_and_refusal():
    assert ops.ln_fold_shape_ok(960, 320) and ops.ln_fold_shape_ok(2560, 320, act=ops.ACT_GEGLU)
    assert ops.ln_fold_shape_ok(3840, 1280) and ops.ln_fold_shape_ok(10240, 1280, act=ops.ACT_GEGLU)
    assert not ops.ln_fold_shape_ok(320, 328)         # K not a multiple of 32: v1 only
    # vd_gemm refuses a fold no kernel takes, before any launch (argument checks are host-side)
    d = _desc(32768, 1920, K=640)
    assert L.lib().vd_gemm(ctypes.byref(d), None) == 1001  # VD_EUNSUPPORTED
    d = _desc(16384, 320, res=256, ld_res=320)
    assert L.lib().vd_gemm(ctypes.byref(d), None) == 1000  # VD_EINVAL: no residual with a fold
