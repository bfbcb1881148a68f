"""Kernel parity on the MI355X: every HIP entry point vs a plain PyTorch
fp32/fp64 reference of the same op on the same bf16-rounded inputs.

Tolerances (written per test): fp32-output kernels must meet the north-star
rtol=1e-3 / atol=1e-4 (scaled by the output's magnitude where noted);
bf16-output kernels are allowed one bf16 rounding of the output
(rel 2^-8) plus a small absolute floor.
"""
import math

import pytest
import torch
import torch.nn.functional as F
import torch.nn.functional as F_

from vdiff import ops
from vdiff._lib import GemmDesc
from vdiff.dist import block_transpose_reference, rev3_reference
from vdiff.models.layers import LnFold, pack_conv3x3, pack_geglu

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def bf(x):
    return x.to(BF)


def close_bf16(got, want, rel=1 / 128, abs_frac=2e-3):
    want = want.double().cpu()
    got = got.double().cpu()
    scale = want.abs().max().item() + 1e-12
    err = (got - want).abs()
    bound = rel * want.abs() + abs_frac * scale
    bad = (err > bound).sum().item()
    assert bad == 0, f"{bad} / {want.numel()} elements out of tolerance; max err {err.max().item():.3e} (scale {scale:.3e})"


def close_f32(got, want, rtol=1e-3, atol=1e-4):
    torch.testing.assert_close(got.double().cpu(), want.double().cpu(), rtol=rtol, atol=atol)


def rnd(*shape, std=1.0, dev="cuda"):
    return bf(torch.randn(*shape, device=dev) * std)


# ---------------------------------------------------------------- GEMM
@pytest.mark.parametrize("M,N,K", [(300, 320, 640), (128, 64, 64), (1000, 160, 128), (2, 1280, 1280),
                                   (154, 640, 768), (4096, 1280, 320)])
def test_gemm_fp32_out_bias(cuda, M, N, K):
    a, w = rnd(M, K), rnd(N, K, std=K ** -0.5)
    b = torch.randn(N, device=cuda)
    got = ops.gemm(a, w, bias=b, out_f32=True)
    want = a.double() @ w.double().T + b.double()
    close_f32(got, want, rtol=1e-3, atol=1e-4)


def test_gemm_epilogues(cuda):
    M, N, K = 520, 320, 192
    a, a1, w = rnd(M, 128), rnd(M, 64), rnd(N, K, std=0.1)
    b = torch.randn(N, device=cuda)
    temb = torch.randn(3, 400, device=cuda)[:, 40:40 + N]       # column-slice view, like Ctx.temb_all
    res = rnd(M, N)
    rb_div = 200
    got = ops.gemm(a, w, a1=a1, bias=b, rowbias=temb, rb_div=rb_div, res=res)
    x = torch.cat([a, a1], 1).double()
    idx = torch.arange(M, device=cuda) // rb_div
    want = x @ w.double().T + b.double() + temb.double()[idx] + res.double()
    close_bf16(got, want)
    got = ops.gemm(a, w, a1=a1, bias=b, act=ops.ACT_SILU)
    close_bf16(got, F.silu(x @ w.double().T + b.double()))


@pytest.mark.parametrize("N,out_view", [(100, False), (328, False), (488, True), (1288, False)])
def test_gemm_epilogue_widths(cuda, gemm_path, N, out_view):
    """16-B (permlane16-paired) epilogue vs its 8-B fallback: N % 8 == 4 and an output /
    residual whose row stride is not a multiple of 8 take the narrow path; N = 328 / 1288
    leave a partial last column tile on the wide one."""
    M, K = 700, 320
    a, w = rnd(M, K), rnd(N, K, std=K ** -0.5)
    b = torch.randn(N, device=cuda)
    if out_view:
        out = torch.empty(M, N + 4, device=cuda, dtype=torch.bfloat16)[:, :N]
        res = rnd(M, N + 4)[:, :N]
    else:
        out, res = None, rnd(M, N)
    got = ops.gemm(a, w, bias=b, res=res, out=out)
    close_bf16(got, a.double() @ w.double().T + b.double() + res.double())


def test_gemm_geglu(cuda):
    M, C = 333, 64
    n = rnd(M, C)
    w = rnd(8 * C, C, std=0.2)
    b = torch.randn(8 * C, device=cuda) * 0.1
    got = ops.gemm(n, pack_geglu(w), bias=pack_geglu(b), act=ops.ACT_GEGLU)
    hg = n.double() @ w.double().T + b.double()
    h, g = hg.chunk(2, -1)
    close_bf16(got, h * F.gelu(g))


# ---------------------------------------------------------------- v2 (LDS-DMA) paths
@pytest.fixture(params=["v6", "v5", "v3", "v2", "v1"])
def gemm_path(request, cuda):
    """Force one GEMM kernel per call (vd_gemm_desc.path; v3 only takes dense A, other shapes
    fall back to the automatic plan)."""
    with ops.gemm_plan(path={"auto": 0, "v1": 1, "v2": 2, "v3": 3, "v5": 5, "v6": 6}[request.param]):
        yield request.param


def test_gemm_large_dense(gemm_path):
    """Shapes large enough for the 256-row LDS-DMA kernel (v2) and the same on v1."""
    M, N = 32768, 320
    a, a1 = rnd(M, 256), rnd(M, 384)
    w = rnd(N, 640, std=0.04)
    b = torch.randn(N, device="cuda")
    temb = torch.randn(4, N, device="cuda")
    res = rnd(M, N)
    got = ops.gemm(a, w, a1=a1, bias=b, rowbias=temb, rb_div=M // 4, res=res)
    x = torch.cat([a, a1], 1).float()
    want = x @ w.float().T + b + temb.repeat_interleave(M // 4, 0) + res.float()
    close_bf16(got, want)
    got = ops.gemm(a1, w[:, :384].contiguous(), bias=b, out_f32=True)
    close_f32(got, a1.float() @ w[:, :384].float().T + b, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("M,N,K,k0", [(256, 256, 64, 64), (300, 512, 128, 64), (513, 1000, 192, 192),
                                      (2048, 1280, 2560, 2560), (8192, 768, 640, 320), (1024, 256, 5120, 5120)])
def test_gemm_v3_shapes(cuda, M, N, K, k0):
    """v3 pipeline edges: 1-3 K-tiles (prologue / drain), ragged M and N, the a0|a1 channel
    concat split at k0, few tiles (split-K), bias + residual epilogue."""
    with ops.gemm_plan(path=3):
        a = rnd(M, k0)
        a1 = rnd(M, K - k0) if K > k0 else None
        w = rnd(N, K, std=K ** -0.5)
        b = torch.randn(N, device=cuda)
        res = rnd(M, N)
        got = ops.gemm(a, w, a1=a1, bias=b, res=res)
        x = a if a1 is None else torch.cat([a, a1], 1)
        close_bf16(got, x.float() @ w.float().T + b + res.float())


@pytest.mark.parametrize("M,N,K,k0", [(256, 160, 32, 32), (300, 128, 96, 64), (513, 1000, 192, 160),
                                      (2048, 1280, 2560, 2560), (8192, 480, 640, 320), (1024, 320, 5120, 5120),
                                      (131072, 320, 320, 320)])
@pytest.mark.parametrize("path", [5, 0])
def test_gemm_v5_shapes(cuda, path, M, N, K, k0):
    """v5 (BK 32 ring; path 0 = automatic, which takes v5 for k0 % 64 != 0) pipeline edges: 1-3 k-steps (shorter than the ring), ragged M and
    N, the a0|a1 concat split at k0 (a multiple of 32, not of 64), few tiles (split-K), and
    the L1 shape whose units wrap the persistent grid several times."""
    with ops.gemm_plan(path=path):
        a = rnd(M, k0)
        a1 = rnd(M, K - k0) if K > k0 else None
        w = rnd(N, K, std=K ** -0.5)
        b = torch.randn(N, device=cuda)
        res = rnd(M, N)
        got = ops.gemm(a, w, a1=a1, bias=b, res=res)
        x = a if a1 is None else torch.cat([a, a1], 1)
        close_bf16(got, x.float() @ w.float().T + b + res.float())


@pytest.mark.parametrize("M,N,K", [(131072, 960, 320), (1000, 328, 96), (4096, 640, 32), (300, 2560, 640)])
@pytest.mark.parametrize("epi", ["bias", "nobias", "silu", "geglu"])
@pytest.mark.parametrize("path", [5])
def test_gemm_v5_load_free_epilogue(cuda, path, M, N, K, epi):
    """v5's load-free epilogue (bias DMA'd into an LDS slot per unit, unconditional buffer
    stores with out-of-range lanes dropped, the stores left in flight across the next
    k-steps' counted waits): ragged M and N, one-k-step units, every activation."""
    with ops.gemm_plan(path=path):
        a = rnd(M, K)
        if epi == "geglu":
            N = N // 32 * 32
        w = rnd(N, K, std=K ** -0.5)
        b = None if epi == "nobias" else torch.randn(N, device=cuda)
        if epi == "geglu":
            got = ops.gemm(a, pack_geglu(w), bias=pack_geglu(b), act=ops.ACT_GEGLU)
            h, g = (a.float() @ w.float().T + b).chunk(2, -1)
            close_bf16(got, h * F.gelu(g))
        else:
            got = ops.gemm(a, w, bias=b, act=ops.ACT_SILU if epi == "silu" else ops.ACT_NONE)
            want = a.float() @ w.float().T + (b if b is not None else 0)
            close_bf16(got, F.silu(want) if epi == "silu" else want)


@pytest.mark.parametrize("M,N,kind", [(131072, 320, "res"), (65536 + 37, 960, "nobias"), (70000 + 5, 320, "res"),
                                      (65536, 640, "silu"), (65600, 160, "gelu"), (98304, 5120, "bias"),
                                      (65536 + 16 * 5 + 3, 2560, "geglu")])
def test_gemm_v8_weight_stationary(cuda, M, N, kind):
    """v8 (one 160 x 320 W tile + bias resident in LDS per workgroup, A streamed into registers,
    output staged through LDS):
    ragged M (a partial last 32-row block, unequal XCD ranges), 1 / 2 / 4 / 6 / 32 column tiles
    per XCD (idle workgroups when 32 % tiles != 0), every epilogue it takes — and bit-equal to
    v2, whose k-order per output and epilogue arithmetic it keeps."""
    K = 320
    a = rnd(M, K)
    w = rnd(N, K, std=K ** -0.5)
    bias = None if kind == "nobias" else torch.randn(N, device=cuda)
    kw = {}
    if kind == "geglu":
        w, bias = pack_geglu(w), pack_geglu(bias)
        kw["act"] = ops.ACT_GEGLU
    elif kind == "res":
        kw["res"] = rnd(M, N)
    elif kind in ("silu", "gelu"):
        kw["act"] = ops.ACT_SILU if kind == "silu" else ops.ACT_GELU
    with ops.gemm_plan(path=8):
        got = ops.gemm(a, w, bias=bias, **kw)
    with ops.gemm_plan(path=2):
        ref = ops.gemm(a, w, bias=bias, **kw)
    torch.cuda.synchronize()
    assert torch.equal(got, ref), f"v8 != v2 bits: max |diff| {(got.float() - ref.float()).abs().max().item()}"
    x = a.float() @ w.float().T + (bias if bias is not None else 0)
    if kind == "res":
        x = x + kw["res"].float()
    elif kind == "silu":
        x = F.silu(x)
    elif kind == "gelu":
        x = F.gelu(x)
    elif kind == "geglu":  # packed: (hidden block i, gate block i) 16-column pairs
        x = x.view(M, -1, 2, 16)
        x = x[:, :, 0].reshape(M, -1) * F.gelu(x[:, :, 1].reshape(M, -1))
    close_bf16(got, x)


@pytest.mark.parametrize("M,N,K,kind", [(2, 1280, 320, "silu"), (2, 1280, 1280, "bias"), (2, 20160, 1280, "f32"),
                                        (1, 52, 264, "res"), (5, 1292, 776, "rowbias"), (16, 4096, 2560, "gelu"),
                                        (3, 640, 96, "nobias")])
def test_gemm_v9_skinny(cuda, M, N, K, kind):
    """v9 (M <= 16: the time-embedding MLP and the resnets' concatenated time_emb_proj; forced,
    path 9): every epilogue it carries, a partial last 16-column block (N = 52, 1292) and a
    partial last 32-k step (K = 264, 776, 96); bit-equal to v1, whose MFMA chain it keeps, and
    within bf16 output rounding of fp32."""
    with ops.gemm_plan(path=9):
        assert ops.gemm_plan_of(GemmDesc(a0=256, lda0=K, k0=K, a_mode=0, w=256, ldw=K, M=M, N=N, K=K, out=256,
                                         ldc=N))[0] == 9
    a = rnd(M, K)
    w = rnd(N, K, std=K ** -0.5)
    bias = None if kind == "nobias" else torch.randn(N, device=cuda)
    kw = {}
    if kind in ("silu", "gelu"):
        kw["act"] = ops.ACT_SILU if kind == "silu" else ops.ACT_GELU
    elif kind == "f32":
        kw["out_f32"] = True
    elif kind == "res":
        kw["res"] = rnd(M, N)
    elif kind == "rowbias":
        kw["rowbias"], kw["rb_div"] = torch.randn(M, N, device=cuda), 1
    with ops.gemm_plan(path=9):
        got = ops.gemm(a, w, bias=bias, **kw)
    with ops.gemm_plan(path=1):
        ref = ops.gemm(a, w, bias=bias, **kw)
    torch.cuda.synchronize()
    assert torch.equal(got, ref), f"v9 != v1 bits: max |diff| {(got.float() - ref.float()).abs().max().item()}"
    x = a.float() @ w.float().T + (bias if bias is not None else 0)
    if kind == "res":
        x = x + kw["res"].float()
    elif kind == "rowbias":
        x = x + kw["rowbias"]
    elif kind == "silu":
        x = F.silu(x)
    elif kind == "gelu":
        x = F.gelu(x)
    if kind == "f32":
        close_f32(got, x, rtol=1e-4, atol=1e-4)
    else:
        close_bf16(got, x)


def test_gemm_v8_strided_operands(cuda):
    """v8 on column-slice views: A with lda0 = 384, out and residual slices of wider
    buffers (ldc = ld_res = N + 160) — v8's own A / store / residual address arithmetic — bit-equal
    to v2 on the same views."""
    M, N, K = 8192, 320, 320
    abuf = rnd(M, 384)
    a = abuf[:, 32:32 + K]
    w = rnd(N, K, std=K ** -0.5)
    bias = torch.randn(N, device=cuda)
    rbuf = rnd(M, N + 160)
    res = rbuf[:, 80:80 + N]
    outs = []
    for path in (8, 2):
        obuf = torch.full((M, N + 160), 7.0, device=cuda, dtype=torch.bfloat16)
        with ops.gemm_plan(path=path):
            ops.gemm(a, w, bias=bias, res=res, out=obuf[:, 160:])
        outs.append(obuf)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]), "v8 != v2 on strided views"
    assert torch.all(outs[0][:, :160] == 7.0), "v8 wrote outside its column slice"
    close_bf16(outs[0][:, 160:], a.float() @ w.float().T + bias + res.float())


@pytest.mark.parametrize("M,N,K,kind,offset,kern", [
    (16384, 960, 320, "plain", 0.0, 8), (16384 + 37, 320, 320, "plain", 30.0, 8),
    (65536 + 16 * 5 + 3, 2560, 320, "geglu", 0.0, 8), (20000, 2560, 320, "geglu", 30.0, 8),
    (131072, 960, 320, "plain", 0.0, 8),
    # rows offset by 100 / 300 std: the exact second pass of the ill-conditioned variance
    (16384 + 37, 320, 320, "plain", 100.0, 8), (20000, 2560, 320, "geglu", 300.0, 8),
    # the unsplit v6 of a frame shard's small M (L2-L4 at 4 images per rank)
    (1024, 3840, 1280, "plain", 0.0, 6), (4096 + 37, 640, 640, "plain", 30.0, 6),
    (256, 10240, 1280, "geglu", 0.0, 6), (700, 2560, 640, "geglu", 30.0, 6), (256, 1280, 1280, "plain", 0.0, 6),
    (4096 + 37, 640, 640, "plain", 300.0, 6), (700, 2560, 640, "geglu", 100.0, 6)])
def test_gemm_ln_fold(cuda, M, N, K, kind, offset, kern):
    """vd_gemm_desc.ln_fold_s (round 5): Linear(LayerNorm(x)) as ONE GEMM over the un-normalised
    rows (LnFold: W' = W∘gamma in bf16, s = its row sums, b' = b + W·beta; each row's mean / rstd
    from the A fragments by two extra MFMAs per X fragment, on v8 and v6).  Within bf16 output
    rounding of fp64 of the same folded arithmetic; within the unfolded path's own rounding (bf16
    normalised rows) of fp64 LayerNorm -> Linear and of the unfolded device path (vd_layernorm +
    GEMM); rows whose mean is 30 std exercise the fp32 one-pass variance, 100 / 300 std the exact
    second pass it falls back to past 16 std (round 6, ADVICE r05: E[x²] − mean² alone loses
    ~1e-7·(mean/std)² of the variance); ragged M (partial row block, unequal XCD ranges / a
    partial 64-row tile)."""
    g = torch.Generator(device=cuda).manual_seed(0)
    x = bf(1.7 * (torch.randn(M, K, device=cuda, generator=g) + offset
                  + 0.5 * torch.randn(M, 1, device=cuda, generator=g)))
    norm = torch.nn.LayerNorm(K).to(cuda)
    with torch.no_grad():
        norm.weight.copy_(1 + 0.2 * torch.randn(K, device=cuda, generator=g))
        norm.bias.copy_(0.1 * torch.randn(K, device=cuda, generator=g))
    w = torch.randn(N, K, device=cuda, generator=g) * K ** -0.5
    b = 0.1 * torch.randn(N, device=cuda, generator=g)
    geglu = kind == "geglu"
    act = ops.ACT_GEGLU if geglu else ops.ACT_NONE
    fold = LnFold(norm, w, b, pack=pack_geglu if geglu else None)
    assert fold.runs(M, act), "the plan does not fold this shape"
    nout = N // 2 if geglu else N
    assert ops.gemm_plan_of(GemmDesc(a0=256, lda0=K, k0=K, a_mode=0, w=fold.w.data_ptr(), ldw=K, M=M, N=N, K=K,
                                     bias=256, act=act, out=256, ldc=nout, ln_fold_s=fold.s.data_ptr(),
                                     ln_fold_eps=1e-5)) == (kern, 1)
    got = fold.gemm(x, act=act)

    def epi(y):  # packed GEGLU pairs -> h * gelu(g)
        if not geglu:
            return y
        y = y.reshape(M, -1, 2, 16)
        return y[:, :, 0].reshape(M, -1) * F.gelu(y[:, :, 1].reshape(M, -1))

    xd = x.double()
    mean = xd.mean(1, keepdim=True)
    rstd = (xd.var(1, unbiased=False, keepdim=True) + fold.eps).rsqrt()
    same = epi(rstd * (xd @ fold.w.double().T - mean * fold.s.double()) + fold.b.double())
    close_bf16(got, same)
    wp = pack_geglu(w) if geglu else w
    bp = pack_geglu(b) if geglu else b
    ln = F.layer_norm(xd, (K,), norm.weight.double(), norm.bias.double(), norm.eps)
    ref = epi(ln @ wp.double().T + bp.double())
    unfolded = ops.gemm(ops.layer_norm(x, norm.weight.detach().float().contiguous(),
                                       norm.bias.detach().float().contiguous()), bf(wp).contiguous(), bias=bp, act=act)
    e_ref = ((got.double() - ref).norm() / ref.norm()).item()
    e_unf = ((unfolded.double() - ref).norm() / ref.norm()).item()
    e_dev = ((got.double() - unfolded.double()).norm() / ref.norm()).item()
    print(f"M={M} N={N} {kind} offset {offset}: folded vs fp64 {e_ref:.5f}, unfolded vs fp64 {e_unf:.5f}, "
          f"folded vs unfolded {e_dev:.5f}")
    assert e_ref < 5e-3 and e_dev < 7e-3
    assert e_ref < 1.5 * e_unf + 1e-3  # no worse than the unfolded path's own bf16 rounding


@pytest.mark.parametrize("B,F,P,C,kern", [(2, 16, 32, 1280, 6), (2, 16, 8, 1280, 6), (1, 16, 37, 1280, 6),
                                          (2, 16, 64, 640, 6)])
def test_gemm_ln_fold_pe_rowbias(cuda, B, F, P, C, kern):
    """The motion block's norm + sinusoidal PE folded into its levels-2-4 QKV GEMM (LnFold(pe=...)):
    rows (video, frame, position), PE[frame] added after the norm = the row bias W·pe[(m / P) % F]
    after the fold (v6: the rank's levels 3-4).  Within bf16 output rounding of
    fp64 LayerNorm + PE -> Linear, no worse than the unfolded device path."""
    g = torch.Generator(device=cuda).manual_seed(1)
    M, N, K = B * F * P, 3 * C, C
    x = bf(1.3 * torch.randn(M, K, device=cuda, generator=g) + 0.4 * torch.randn(M, 1, device=cuda, generator=g))
    norm = torch.nn.LayerNorm(K).to(cuda)
    with torch.no_grad():
        norm.weight.copy_(1 + 0.2 * torch.randn(K, device=cuda, generator=g))
        norm.bias.copy_(0.1 * torch.randn(K, device=cuda, generator=g))
    pe = 0.5 * torch.randn(32, K, device=cuda, generator=g)
    w = torch.randn(N, K, device=cuda, generator=g) * K ** -0.5
    fold = LnFold(norm, w, pe=pe)
    assert fold.runs(M), "the plan does not fold this shape"
    assert ops.gemm_plan_of(GemmDesc(a0=256, lda0=K, k0=K, a_mode=0, w=fold.w.data_ptr(), ldw=K, M=M, N=N, K=K,
                                     bias=256, rowbias=256, ld_rb=N, rb_div=P, out=256, ldc=N,
                                     ln_fold_s=fold.s.data_ptr(), ln_fold_eps=1e-5)) == (kern, 1)
    got = fold.gemm(x, pe_div=P, pe_period=F)
    xd = x.double()
    frame = (torch.arange(M, device=cuda) // P) % F
    ln = F_.layer_norm(xd, (K,), norm.weight.double(), norm.bias.double(), norm.eps) + pe.double()[frame]
    ref = ln @ w.double().T
    unfolded = ops.gemm(ops.layer_norm(x, norm.weight.detach().float().contiguous(),
                                       norm.bias.detach().float().contiguous(), pe=pe.float().contiguous(),
                                       pe_div=P, pe_period=F), bf(w).contiguous())
    e_ref = ((got.double() - ref).norm() / ref.norm()).item()
    e_unf = ((unfolded.double() - ref).norm() / ref.norm()).item()
    print(f"B={B} F={F} P={P} C={C}: folded vs fp64 {e_ref:.5f}, unfolded vs fp64 {e_unf:.5f}")
    assert e_ref < 5e-3 and e_ref < 1.5 * e_unf + 1e-3


def test_gemm_ln_fold_refused_off_plan(cuda):
    """A fold no kernel takes (here the v3 plan of M 32768 x N 1920 x K 640) is refused
    (VD_EUNSUPPORTED), never run on another kernel."""
    K, M = 640, 32768
    norm = torch.nn.LayerNorm(K).to(cuda)
    fold = LnFold(norm, torch.randn(1920, K, device=cuda) * K ** -0.5)
    assert not fold.runs(M)
    with pytest.raises(Exception, match="unsupported|1001"):
        fold.gemm(rnd(M, K))


@pytest.mark.parametrize("path,M,N,K", [(0, 16384, 320, 320), (8, 4096, 320, 320), (0, 4096, 640, 640),
                                        (6, 1024, 1280, 1280), (0, 256, 1280, 1280), (1, 512, 320, 192)])
def test_gemm_row_map(cuda, path, M, N, K):
    """vd_gemm_desc.rmap_* (round 5, the frame-sharded motion module's proj_out): product row m and
    its residual live at row rev3(m) — rows (r', f_loc, b, j) of the returning all-to-all written
    into a rank's (b, f_loc, r', j) layout (8 ranks, 2 frames, CFG batch 2).  The plan carries
    the map on v8 (residual), v6 (split where forced) and v1; each case is bit-equal to the same
    kernel without the map on pre-permuted residual rows, and within bf16 of fp32."""
    n1, n2, world = 2, 2, 8
    inner = M // (world * n1 * n2)
    a = rnd(M, K)
    w = rnd(N, K, std=K ** -0.5)
    bias = torch.randn(N, device=cuda)
    res = rnd(M, N)                                   # in the destination layout
    res_src = rev3_reference(res, n1, world, inner)   # residual rows in product order
    with ops.gemm_plan(path=path):
        got = ops.gemm(a, w, bias=bias, res=res, rmap=(n1, n2, inner))
        plain = ops.gemm(a, w, bias=bias, res=res_src)
    torch.cuda.synchronize()
    want = rev3_reference(plain, n1, n2, inner)
    assert torch.equal(got, want), f"row map != permuted plain GEMM: max {(got.float() - want.float()).abs().max()}"
    close_bf16(got, rev3_reference(a.float() @ w.float().T + bias, n1, n2, inner) + res.float())


@pytest.mark.parametrize("n,pix,C,c0,silu", [(4, 256, 1280, 1280, True), (4, 64, 1280, 1280, True),
                                           (2, 64, 2560, 1280, True), (3, 256, 2560, 1280, True),
                                           (4, 256, 1280, 1280, False), (1, 100, 1280, 1280, True)])
def test_gn_small_one_launch(cuda, n, pix, C, c0, silu):
    """vd_gn_small (the one-launch GroupNorm of levels 3-4 / mid, incl. the up blocks' skip concat
    x0 | x1 and a ragged row count) against fp64 GroupNorm (+SiLU) at bf16 output rounding, and
    against the two-launch path it replaces."""
    G, eps = 32, 1e-5
    assert ops.gn_small_chunk(pix, C, G)
    x0 = bf(torch.randn(n * pix, c0, device=cuda) * 1.5 + 0.7)
    x1 = bf(torch.randn(n * pix, C - c0, device=cuda) - 0.3) if c0 < C else None
    g = 1 + 0.2 * torch.randn(C, device=cuda)
    b = 0.2 * torch.randn(C, device=cuda)
    got = ops.group_norm(x0, n, pix, G, eps, g, b, silu=silu, x1=x1)
    two = ops.group_norm_2pass(x0, n, pix, G, eps, g, b, silu=silu, x1=x1)
    torch.cuda.synchronize()
    x = (torch.cat([x0, x1], 1) if x1 is not None else x0).double().view(n, pix, G, C // G)
    mean, var = x.mean((1, 3), keepdim=True), x.var((1, 3), unbiased=False, keepdim=True)
    ref = ((x - mean) / (var + eps).sqrt()).view(n * pix, C) * g.double() + b.double()
    if silu:
        ref = F.silu(ref)
    close_bf16(got, ref)
    close_bf16(two, ref)
    assert (got.float() - two.float()).abs().max().item() <= 2 * 2 ** -7 * ref.abs().max().item()


def test_gn_finalize_group_records(cuda):
    """vd_gn_finalize_g (the motion norm on vd_gn_partial_g's per-group records): fp64 GroupNorm
    statistics over (C/G, F, H, W) within fp32 rounding, and the records of a video's frames made
    in two frame halves and concatenated along the split axis — what a 2-way frame-sharded
    all-gather hands over — give the whole video's scale / shift bit for bit."""
    B, F, HW, C, G, eps = 2, 4, 1024, 640, 32, 1e-6
    x = bf(torch.randn(B * F * HW, C, device=cuda) * 2 + 0.5)
    g = 1 + 0.1 * torch.randn(C, device=cuda)
    b = 0.1 * torch.randn(C, device=cuda)
    sp = ops.gn_splits_per_frame(HW)
    ss = ops.gn_finalize_g(ops.gn_partial_g(x, C, B, F * HW, F * sp, G), C, eps, g, b)
    xv = x.view(B, F, HW, C)
    halves = [xv[:, i * F // 2:(i + 1) * F // 2].reshape(-1, C).contiguous() for i in range(2)]
    ws2 = torch.cat([ops.gn_partial_g(h, C, B, F // 2 * HW, F // 2 * sp, G) for h in halves], 1)
    ss2 = ops.gn_finalize_g(ws2, C, eps, g, b)
    torch.cuda.synchronize()
    assert torch.equal(ss, ss2)
    xd = x.double().view(B, F * HW, G, C // G)
    mean = xd.mean((1, 3))
    rstd = (xd.var((1, 3), unbiased=False) + eps).rsqrt()
    a = (rstd[:, :, None] * g.double().view(G, C // G)).reshape(B, C)
    sh = b.double() - mean.repeat_interleave(C // G, 1) * a
    torch.testing.assert_close(ss[..., 0].double(), a, rtol=2e-5, atol=0)
    torch.testing.assert_close(ss[..., 1].double(), sh, rtol=0, atol=2e-5 * a.abs().max().item())


@pytest.mark.parametrize("ranks", [1, 2, 4])
def test_gn_finalize_rank_major_records(cuda, ranks):
    """vd_gn_finalize_g_ranks (round 6): the frame-sharded ranks' records in the
    all-gather's rank-major order [rank, video, split, group] — no transpose copy — give the same
    scale / shift bits as vd_gn_finalize_g on the split-concatenated records."""
    B, F, HW, C, G, eps = 2, 8, 256, 1280, 32, 1e-6
    x = bf(torch.randn(B * F * HW, C, device=cuda) * 1.5 - 0.2)
    g = 1 + 0.1 * torch.randn(C, device=cuda)
    b = 0.1 * torch.randn(C, device=cuda)
    sp = ops.gn_splits_per_frame(HW)
    Fl = F // ranks
    xv = x.view(B, F, HW, C)
    parts = [ops.gn_partial_g(xv[:, r * Fl:(r + 1) * Fl].reshape(-1, C).contiguous(), C, B, Fl * HW, Fl * sp, G)
             for r in range(ranks)]
    ss_cat = ops.gn_finalize_g(torch.cat(parts, 1), C, eps, g, b)
    ss_rm = ops.gn_finalize_g(torch.stack(parts, 0), C, eps, g, b)
    ss_one = ops.gn_finalize_g(ops.gn_partial_g(x, C, B, F * HW, F * sp, G), C, eps, g, b)
    torch.cuda.synchronize()
    assert torch.equal(ss_rm, ss_cat)
    assert torch.equal(ss_rm, ss_one)


def test_gn_apply_rev3(cuda):
    """vd_gn_apply_rev3: the motion norm writing the all-to-all's send order directly equals the
    plain apply followed by the row permutation, bit for bit."""
    B, Fl, HW, C, world = 2, 2, 1024, 320, 8
    x = rnd(B * Fl * HW, C) + 0.3
    g = 1 + 0.1 * torch.randn(C, device=cuda)
    b = 0.1 * torch.randn(C, device=cuda)
    ws = ops.gn_partial(x, C, B, Fl * HW, Fl * ops.gn_splits_per_frame(HW))
    ss = ops.gn_finalize(ws, 32, 1e-6, g, b)
    perm = (Fl, world, HW // world)
    got = ops.gn_apply(x, ss, Fl * HW, False, rev3=perm)
    plain = ops.gn_apply(x, ss, Fl * HW, False)
    torch.cuda.synchronize()
    assert torch.equal(got, rev3_reference(plain, *perm))


@pytest.mark.parametrize("M,N,K,kind", [(256, 1280, 1280, "res"), (1024, 1280, 5120, "rowbias"), (100, 320, 2560, "silu"),
                                       (256, 2560, 1280, "geglu"), (4096, 640, 640, "f32"), (64, 1280, 23040, "res")])
def test_gemm_v6_small_m_splitk(cuda, M, N, K, kind):
    """v6 (64 x 64 tiles, split K reduced in-kernel by the last-arriving K-slice): small M
    with long K (the split path), every epilogue flavour, and a second launch on the
    same workspace (the counters were reset)."""
    with ops.gemm_plan(path=6):
        a = rnd(M, K)
        w = rnd(N, K, std=K ** -0.5)
        b = torch.randn(N, device=cuda)
        x = a.float()
        for _ in range(2):
            if kind == "geglu":
                got = ops.gemm(a, pack_geglu(w), bias=pack_geglu(b), act=ops.ACT_GEGLU)
                h, g = (x @ w.float().T + b).chunk(2, -1)
                close_bf16(got, h * F.gelu(g))
            elif kind == "res":
                res = rnd(M, N)
                close_bf16(ops.gemm(a, w, bias=b, res=res), x @ w.float().T + b + res.float())
            elif kind == "rowbias":
                rb = torch.randn(4, N, device=cuda)
                got = ops.gemm(a, w, bias=b, rowbias=rb, rb_div=M // 4)
                close_bf16(got, x @ w.float().T + b + rb.repeat_interleave(M // 4, 0))
            elif kind == "silu":
                close_bf16(ops.gemm(a, w, bias=b, act=ops.ACT_SILU), F.silu(x @ w.float().T + b))
            else:
                close_f32(ops.gemm(a, w, bias=b, out_f32=True), x.double() @ w.double().T + b.double(),
                          rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("case", ["l3", "l4cat"])
def test_conv3x3_v6_splitk(cuda, case):
    """Small-M implicit-GEMM conv on v6 with split K (L3/L4 shapes at 2 frames per GPU),
    including the up-block channel concat."""
    with ops.gemm_plan(path=6):
        n, hw, c0, c1, co = (4, 16, 640, 0, 640) if case == "l3" else (4, 8, 1280, 1280, 1280)
        x0 = rnd(n * hw * hw, c0)
        x1 = rnd(n * hw * hw, c1) if c1 else None
        wt = bf(torch.randn(co, c0 + c1, 3, 3, device="cuda") * (9 * (c0 + c1)) ** -0.5)
        b = torch.randn(co, device="cuda")
        res = rnd(n * hw * hw, co)
        out, _, _ = ops.conv3x3(x0, n, hw, hw, pack_conv3x3(wt), x1=x1, bias=b, res=res)
        xin = x0 if x1 is None else torch.cat([x0, x1], 1)
        img = xin.float().reshape(n, hw, hw, -1).permute(0, 3, 1, 2)
        want = F.conv2d(img, wt.float(), b, padding=1).permute(0, 2, 3, 1).reshape(-1, co) + res.float()
        close_bf16(out, want)


def test_gemm_large_geglu(gemm_path):
    M, C = 32768, 64
    n = rnd(M, 256)
    w = rnd(8 * C, 256, std=0.06)
    bb = torch.randn(8 * C, device="cuda") * 0.1
    got = ops.gemm(n, pack_geglu(w), bias=pack_geglu(bb), act=ops.ACT_GEGLU)
    hg = n.float() @ w.float().T + bb
    h, g = hg.chunk(2, -1)
    close_bf16(got, h * F.gelu(g))


@pytest.mark.parametrize("case", ["s1", "s2", "up", "concat"])
def test_conv3x3_large(gemm_path, case):
    n, co = 8, 320
    h = w = 128 if case == "s2" else (32 if case == "up" else 64)
    c0, c1 = 64, (64 if case == "concat" else 0)
    x0 = rnd(n * h * w, c0)
    x1 = rnd(n * h * w, c1) if c1 else None
    wt = bf(torch.randn(co, c0 + c1, 3, 3, device="cuda") * 0.04)
    b = torch.randn(co, device="cuda")
    stride = 2 if case == "s2" else 1
    out, ho, wo = ops.conv3x3(x0, n, h, w, pack_conv3x3(wt), x1=x1, stride=stride, upsample=case == "up",
                              bias=b)
    assert ho * wo * n == 32768
    xin = x0 if x1 is None else torch.cat([x0, x1], 1)
    img = xin.float().reshape(n, h, w, -1).permute(0, 3, 1, 2)
    if case == "up":
        img = F.interpolate(img, scale_factor=2.0, mode="nearest")
    want = F.conv2d(img, wt.float(), b, stride=stride, padding=1).permute(0, 2, 3, 1).reshape(-1, co)
    close_bf16(out, want)


@pytest.mark.parametrize("co,out_f32,M", [(4, True, 32768), (4, False, 1000), (24, False, 32768), (32, True, 600)])
def test_conv3x3_small_n(cuda, co, out_f32, M):
    """conv_out-shaped convs (N <= 32: the 256 x 32 v2 tiles; M < 256 falls back to v1):
    ragged M, N % 8 == 4, fp32 output (the UNet's eps), bias."""
    n = 8 if M == 32768 else 1
    h = w = 64 if M == 32768 else (32 if M == 1000 else 24)
    if M == 1000:
        n, h, w = 1, 25, 40
    if M == 600:
        n, h, w = 1, 20, 30
    ci = 320
    x0 = rnd(n * h * w, ci)
    wt = bf(torch.randn(co, ci, 3, 3, device="cuda") * 0.02)
    b = torch.randn(co, device="cuda")
    out = torch.empty(n * h * w, co, device="cuda", dtype=torch.float32 if out_f32 else torch.bfloat16)
    ops.conv3x3(x0, n, h, w, pack_conv3x3(wt), bias=b, out=out, out_f32=out_f32)
    img = x0.double().reshape(n, h, w, -1).permute(0, 3, 1, 2)
    want = F.conv2d(img, wt.double(), b.double(), padding=1).permute(0, 2, 3, 1).reshape(-1, co)
    if out_f32:
        close_f32(out, want, rtol=1e-3, atol=1e-4)
    else:
        close_bf16(out, want)


@pytest.mark.parametrize("M,N,res,pe", [(32768 + 77, 320, True, False), (131072, 320, False, True),
                                         (40000, 320, True, True), (3000, 320, True, True), (32768, 640, True, False)])
def test_gemm_ln(cuda, M, N, res, pe):
    """vd_gemm with ln_out: the LayerNorm fused into the 256 x 320 GEMM epilogue (N = 320,
    >= 128 row tiles, M < 65536; forced with path 5) or run after the GEMM (v8 at M >= 65536,
    smaller M, other N): out equals the plain GEMM
    and ln_out the LayerNorm of out (+ PE by frame) to bf16 rounding."""
    from vdiff._lib import lib
    K, frames, pos = 320, 16, 64
    a = rnd(M, K)
    w = rnd(N, K, std=K ** -0.5)
    b = torch.randn(N, device=cuda) * 0.1
    r = rnd(M, N) if res else None
    g = 1 + 0.1 * torch.randn(N, device=cuda)
    be = 0.1 * torch.randn(N, device=cuda)
    pet = torch.randn(32, N, device=cuda) if pe else None
    kw = dict(pe=pet, pe_div=pos, pe_period=frames) if pe else {}
    out, ln = ops.gemm_ln(a, w, g, be, bias=b, res=r, **kw)
    plain = ops.gemm(a, w, bias=b, res=r)
    assert torch.equal(out, plain)
    want = ops.layer_norm(plain, g, be, **kw)
    close_bf16(ln, want)
    x = plain.double()
    ref = F.layer_norm(x, (N,), g.double(), be.double(), eps=1e-5)
    if pe:
        ref = ref + pet.double()[(torch.arange(M, device=cuda) // pos) % frames]
    close_bf16(ln, ref)
    with ops.gemm_plan(path=2):  # unfused reference path: GEMM + vd_layernorm
        out2, ln2 = ops.gemm_ln(a, w, g, be, bias=b, res=r, **kw)
    assert torch.equal(ln2, want)
    assert (ln.float() - ln2.float()).abs().max().item() <= 2 ** -6 * (ln2.float().abs().max().item() + 1)
    with ops.gemm_plan(path=5):  # the fused epilogue itself (at M >= 65536 the automatic plan takes v8 + vd_layernorm)
        out5, ln5 = ops.gemm_ln(a, w, g, be, bias=b, res=r, **kw)
    close_bf16(out5, plain.float())
    assert (ln5.float() - ln2.float()).abs().max().item() <= 2 ** -6 * (ln2.float().abs().max().item() + 1)


def test_gemm_splitk_dense(cuda):
    """Few output tiles + long K (the 8x8 level): split-K slabs + reduce epilogue."""
    M, N, K = 2048, 1280, 2560
    a, w = rnd(M, K), rnd(N, K, std=K ** -0.5)
    b = torch.randn(N, device=cuda)
    temb = torch.randn(2, N, device=cuda)
    res = rnd(M, N)
    got = ops.gemm(a, w, bias=b, rowbias=temb, rb_div=M // 2, res=res)
    want = a.float() @ w.float().T + b + temb.repeat_interleave(M // 2, 0) + res.float()
    close_bf16(got, want)
    got = ops.gemm(a, w, bias=b, act=ops.ACT_SILU, out_f32=True)
    close_f32(got, F.silu(a.double() @ w.double().T + b.double()), rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("case", ["dense", "dense_f32_silu", "geglu", "conv", "conv_concat_rowbias"])
def test_gemm_splitk_deterministic(cuda, case):
    """Split-K launches (slabs + gemm_splitk_reduce, which applies every epilogue form) at the
    shapes of a 2-frame rank: the fp64 reference to bf16 / fp32 tolerance, and the same bits run
    after run (fixed slice order, no atomics).  (Round 4 tried reducing in the v2 kernel — the
    tile's last K slice summing the slabs — and measured it slower at every such shape,
    profiles/r04_gemm_splitk_inkernel_refuted.txt; it is gone.)"""
    torch.manual_seed(17)
    if case.startswith("conv"):
        n, h, w, ci, co = 4, 16, 16, 640, 640           # level 3 at 2 frames per rank: 32 tiles -> split
        c1 = 320 if "concat" in case else 0
        x0, x1 = rnd(n * h * w, ci - c1), (rnd(n * h * w, c1) if c1 else None)
        wt = bf(torch.randn(co, ci, 3, 3, device=cuda) * (9 * ci) ** -0.5)
        b = torch.randn(co, device=cuda)
        rb = torch.randn(n, co, device=cuda) if "rowbias" in case else None

        def run():
            return ops.conv3x3(x0, n, h, w, pack_conv3x3(wt), x1=x1, bias=b, rowbias=rb, rb_div=h * w)[0]
        img = (x0 if x1 is None else torch.cat([x0, x1], 1)).double().reshape(n, h, w, ci).permute(0, 3, 1, 2)
        want = F.conv2d(img.cpu(), wt.double().cpu(), b.double().cpu(), padding=1).permute(0, 2, 3, 1).reshape(-1, co)
        want = want.to(cuda) + (rb.double().repeat_interleave(h * w, 0) if rb is not None else 0)
    else:
        M, N, K = (2048, 1280, 5120) if case != "geglu" else (1024, 1024, 2560)
        a, wm = rnd(M, K), rnd(N, K, std=K ** -0.5)
        b = torch.randn(N, device=cuda) * 0.1
        if case == "geglu":
            def run():
                return ops.gemm(a, pack_geglu(wm), bias=pack_geglu(b), act=ops.ACT_GEGLU)
            hh, gg = (a.double() @ wm.double().T + b.double()).chunk(2, -1)
            want = hh * F.gelu(gg)
        elif case == "dense":
            res = rnd(M, N)

            def run():
                return ops.gemm(a, wm, bias=b, res=res)
            want = a.double() @ wm.double().T + b.double() + res.double()
        else:
            def run():
                return ops.gemm(a, wm, bias=b, act=ops.ACT_SILU, out_f32=True)
            want = F.silu(a.double() @ wm.double().T + b.double())
    ref = run()
    got, again = run(), run()
    assert torch.equal(got, ref) and torch.equal(again, ref)
    if ref.dtype == torch.float32:
        close_f32(got, want, rtol=1e-3, atol=1e-3)
    else:
        close_bf16(got, want)


def test_gemm_splitk_geglu(cuda):
    M, C, K = 1024, 128, 1280
    n = rnd(M, K)
    w = rnd(8 * C, K, std=K ** -0.5)
    bb = torch.randn(8 * C, device=cuda) * 0.1
    got = ops.gemm(n, pack_geglu(w), bias=pack_geglu(bb), act=ops.ACT_GEGLU)
    h, g = (n.float() @ w.float().T + bb).chunk(2, -1)
    close_bf16(got, h * F.gelu(g))


def test_conv3x3_splitk(cuda):
    n, h, w, ci, co = 32, 8, 8, 256, 1280
    x = rnd(n * h * w, ci)
    wt = bf(torch.randn(co, ci, 3, 3, device=cuda) * 0.02)
    b = torch.randn(co, device=cuda)
    res = rnd(n * h * w, co)
    out, _, _ = ops.conv3x3(x, n, h, w, pack_conv3x3(wt), bias=b, res=res)
    img = x.float().reshape(n, h, w, ci).permute(0, 3, 1, 2)
    want = F.conv2d(img, wt.float(), b, padding=1).permute(0, 2, 3, 1).reshape(-1, co) + res.float()
    close_bf16(out, want)


# ---------------------------------------------------------------- conv
@pytest.mark.parametrize("case", ["s1", "s2", "up", "concat", "cin8", "cout4", "m128"])
def test_conv3x3(cuda, case):
    """m128: fewer output rows than one 256-row tile (a 1-2 image rank's level 4) -> 64x64 tiles."""
    torch.manual_seed(1)
    n, h, w = 3, 12, 10
    c0, c1, co = 64, 0, 128
    if case == "m128":
        n, h, w, c0, co = 2, 8, 8, 256, 320
    stride, up = 1, False
    if case == "s2":
        stride = 2
    if case == "up":
        up = True
    if case == "concat":
        c1 = 32
    if case == "cin8":
        c0, co = 8, 64
    if case == "cout4":
        co = 4
    x0 = rnd(n * h * w, c0)
    x1 = rnd(n * h * w, c1) if c1 else None
    wt = bf(torch.randn(co, c0 + c1, 3, 3, device=cuda) * 0.05)
    b = torch.randn(co, device=cuda)
    out, ho, wo = ops.conv3x3(x0, n, h, w, pack_conv3x3(wt), x1=x1, stride=stride, upsample=up, bias=b,
                              out_f32=True)
    xin = x0 if x1 is None else torch.cat([x0, x1], 1)
    img = xin.double().reshape(n, h, w, -1).permute(0, 3, 1, 2)
    if up:
        img = F.interpolate(img, scale_factor=2.0, mode="nearest")
    want = F.conv2d(img.cpu(), wt.double().cpu(), b.double().cpu(), stride=stride, padding=1)
    want = want.permute(0, 2, 3, 1).reshape(-1, co)
    assert out.shape == want.shape
    close_f32(out, want, rtol=1e-3, atol=1e-4 * max(1.0, want.abs().max().item()))


@pytest.mark.parametrize("kt,ks,stride,path", [(3, 3, 1, 0), (3, 3, 2, 0), (3, 1, 1, 0), (1, 3, 1, 0),
                                                (3, 3, 1, 1), (3, 1, 1, 1), (3, 3, 1, 2)])
def test_conv3d_temporal_taps(cuda, kt, ks, stride, path):
    """The north star's 3-D / (2+1)D conv over (B, C, T, H, W): kernel (3,3,3), the temporal
    half (3,1,1) and the reference's per-frame (1,3,3), spatial stride 1 / 2, temporal zero
    padding at the video's ends, fp32 output vs fp64 F.conv3d at rtol 1e-3 / atol 1e-4
    (scaled by the output's magnitude); path 0 = automatic (v2 LDS-DMA), 1 = v1, 2 = v2 split."""
    from vdiff._lib import lib
    from vdiff.models.layers import pack_conv3d
    torch.manual_seed(3)
    B, T, h, w, ci, co = 2, 5, 16, 12, 64, 160
    x = rnd(B * T * h * w, ci)
    wt = bf(torch.randn(co, ci, kt, ks, ks, device=cuda) * 0.05)
    b = torch.randn(co, device=cuda)
    with ops.gemm_plan(path=path):
        out, ho, wo = ops.conv3d(x, B, T, h, w, pack_conv3d(wt), kt=kt, ks=ks, stride=stride, bias=b, out_f32=True)
    vid = x.double().reshape(B, T, h, w, ci).permute(0, 4, 1, 2, 3).cpu()
    want = F.conv3d(vid, wt.double().cpu(), b.double().cpu(), stride=(1, stride, stride),
                    padding=(kt // 2, ks // 2, ks // 2))
    want = want.permute(0, 2, 3, 4, 1).reshape(-1, co)
    assert out.shape == want.shape
    close_f32(out, want, rtol=1e-3, atol=1e-4 * max(1.0, want.abs().max().item()))


def test_conv3d_halo_form_matches_full_video(cuda):
    """A frame-sharded rank's call: its frames plus one halo frame each side (frames_in =
    frames_out + 2, t_off = 1, no temporal padding needed inside) gives exactly the full
    video's conv on those frames."""
    from vdiff.models.layers import pack_conv3d
    torch.manual_seed(4)
    B, T, h, w, ci, co = 2, 8, 8, 8, 64, 128
    x = rnd(B * T * h * w, ci)
    wp = pack_conv3d(bf(torch.randn(co, ci, 3, 3, 3, device=cuda) * 0.05))
    full, _, _ = ops.conv3d(x, B, T, h, w, wp, out_f32=True)
    v = x.view(B, T, h * w, ci)
    f0, fl = 3, 2                                           # this "rank" holds frames 3, 4
    halo = v[:, f0 - 1:f0 + fl + 1].reshape(-1, ci).contiguous()
    part, _, _ = ops.conv3d(halo, B, fl + 2, h, w, wp, frames_out=fl, t_off=1, out_f32=True)
    want = full.view(B, T, h * w, co)[:, f0:f0 + fl].reshape(-1, co)
    assert torch.equal(part, want)


def test_conv3d_module_on_videos(cuda):
    """vdiff Conv3d (torch.nn.Conv3d subclass) on a (B, C, T, H, W) video, (2+1)D factorised:
    (1,3,3) then (3,1,1), against torch's conv3d in fp64 on the same bf16 values."""
    from vdiff.models.layers import Conv3d
    torch.manual_seed(5)
    sp, tp = Conv3d(64, 64, (1, 3, 3), padding=(0, 1, 1)), Conv3d(64, 64, (3, 1, 1), padding=(1, 0, 0))
    for m in (sp, tp):
        with torch.no_grad():
            m.weight.mul_(0.5)
        m.to("cuda", BF).prepare()
    x = rnd(2, 64, 6, 10, 10)
    y = tp(sp(x))
    assert y.shape == (2, 64, 6, 10, 10)
    with torch.no_grad():
        ref = F.conv3d(x.double(), sp.weight.double(), sp.bias.double(), padding=(0, 1, 1))
        ref = F.conv3d(ref.to(BF).double(), tp.weight.double(), tp.bias.double(), padding=(1, 0, 0))
    close_bf16(y, ref)


# ---------------------------------------------------------------- norms
@pytest.mark.parametrize("kind", ["image", "video", "concat"])
def test_group_norm(cuda, kind):
    torch.manual_seed(2)
    frames = 4 if kind == "video" else 1
    n_img, hw, C = 8, 96, 320
    c0 = 192 if kind == "concat" else C
    x = rnd(n_img * hw, c0) * 3 + 1.5          # non-zero mean: exercises the shifted statistics
    x1 = rnd(n_img * hw, C - c0) if kind == "concat" else None
    g = torch.rand(C, device=cuda) + 0.5
    be = torch.randn(C, device=cuda)
    n_inst, pix = n_img // frames, frames * hw
    got = ops.group_norm(x, n_inst, pix, 32, 1e-5, g, be, silu=True, x1=x1)
    xx = x if x1 is None else torch.cat([x, x1], 1)
    t = xx.double().reshape(n_inst, pix, C).permute(0, 2, 1)             # (inst, C, pix)
    want = F.silu(F.group_norm(t, 32, g.double(), be.double(), 1e-5)).permute(0, 2, 1).reshape(-1, C)
    close_bf16(got, want)


@pytest.mark.parametrize("n_inst,pix,C,c0,silu", [(4, 64, 1280, 1280, True), (2, 4096, 320, 320, False),
                                                   (4, 64, 2560, 1280, True), (3, 100, 640, 640, True),
                                                   (1, 7, 64, 32, False), (32, 1024, 640, 640, True)])
@pytest.mark.parametrize("path", ["2pass", "4pass"])
def test_group_norm_paths(cuda, n_inst, pix, C, c0, silu, path):
    """The two-launch image GroupNorm (per-group records, finalize in the apply prologue) and
    the partial/finalize/apply path the motion module takes (forced by an identity `gather`),
    over L4-like small instances, a whole 64x64 image, the 2560-channel up-block concat,
    ragged row blocks and a 7-pixel instance."""
    torch.manual_seed(3)
    x = rnd(n_inst * pix, c0) * 3 + 1.5
    x1 = rnd(n_inst * pix, C - c0) - 0.7 if c0 < C else None
    g = torch.rand(C, device=cuda) + 0.5
    be = torch.randn(C, device=cuda)
    if path == "2pass":  # the two-launch kernels directly (the policy picks them for large norms only)
        got = ops.group_norm_2pass(x, n_inst, pix, 32, 1e-6, g, be, silu=silu, x1=x1)
    else:
        got = ops.group_norm(x, n_inst, pix, 32, 1e-6, g, be, silu=silu, x1=x1, two_pass=False)
    xx = x if x1 is None else torch.cat([x, x1], 1)
    t = xx.double().reshape(n_inst, pix, C).permute(0, 2, 1)
    want = F.group_norm(t, 32, g.double(), be.double(), 1e-6)
    want = (F.silu(want) if silu else want).permute(0, 2, 1).reshape(-1, C)
    close_bf16(got, want)


@pytest.mark.parametrize("C,rows", [(320, 4 * 16 * 24 + 5), (640, 1000), (1280, 333), (64, 77), (128, 301),
                                    (1152, 129), (2048, 65)])
def test_layer_norm_kernels(cuda, C, rows):
    """Both LayerNorm kernels (several rows per wave for C in 320/640/1280, one row per wave
    otherwise: 64 / 128 the tiny config, 1152 the DiT, 2048 the widest row) with ragged row counts
    and the motion block's sinusoidal PE."""
    x = rnd(rows, C) * 2 + 0.3
    g, b = torch.rand(C, device=cuda) + 0.5, torch.randn(C, device=cuda)
    pe = torch.randn(16, C, device=cuda)
    got = ops.layer_norm(x, g, b, pe=pe, pe_div=24, pe_period=16)
    plain = ops.layer_norm(x, g, b)
    f = (torch.arange(rows, device=cuda) // 24) % 16
    ref = F.layer_norm(x.double(), (C,), g.double(), b.double(), 1e-5)
    close_bf16(got, ref + pe.double()[f])
    close_bf16(plain, ref)


def test_layer_norm_pe(cuda):
    rows, C, frames, pos = 4 * 16 * 24, 320, 16, 24
    x = rnd(rows, C) * 2 + 0.3
    g, b = torch.rand(C, device=cuda) + 0.5, torch.randn(C, device=cuda)
    pe = torch.randn(32, C, device=cuda)
    got = ops.layer_norm(x, g, b, pe=pe, pe_div=pos, pe_period=frames)
    f = (torch.arange(rows, device=cuda) // pos) % frames
    want = F.layer_norm(x.double(), (C,), g.double(), b.double(), 1e-5) + pe.double()[f]
    close_bf16(got, want)
    got = ops.layer_norm(x, g, b)
    close_bf16(got, F.layer_norm(x.double(), (C,), g.double(), b.double(), 1e-5))


# ---------------------------------------------------------------- attention
def sdpa_ref(q, k, v, batch, heads, sq, skv, d, kv_div=1, scale=None):
    q = q.double().reshape(batch, sq, heads, d).transpose(1, 2)
    kb = k.double().reshape(batch // kv_div, skv, heads, d).transpose(1, 2).repeat_interleave(kv_div, 0)
    vb = v.double().reshape(batch // kv_div, skv, heads, d).transpose(1, 2).repeat_interleave(kv_div, 0)
    w = torch.softmax(q @ kb.transpose(-1, -2) * (d ** -0.5 if scale is None else scale), -1)
    return (w @ vb).transpose(1, 2).reshape(batch * sq, heads * d)


@pytest.fixture(params=["flash40", "flash32", "v1"])
def attn_path(request, cuda):
    """d = 40, per call (vd_attention_ex's kernel): "flash40" (round 3's two-group ping-pong over
    an LDS-DMA ring, wherever it applies: >= 2 key tiles; the automatic choice from 4), "flash32"
    (the 4-wave 32x32x16 kernel), "v1" (the 16x16x32 one).  Other head widths take their one
    kernel whatever is asked."""
    return request.param


@pytest.mark.parametrize("d", [32, 40, 64, 80, 128, 160])
@pytest.mark.parametrize("sq", [64, 300, 1024])
def test_flash_attention_self(cuda, d, sq):
    torch.manual_seed(3)
    batch, heads = 2, 3
    C = heads * d
    qkv = rnd(batch * sq, 3 * C, std=1.5)     # fused-QKV row layout, like the product path
    q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
    got = ops.attention(q, k, v, batch, heads, sq, sq, d)
    close_bf16(got, sdpa_ref(q, k, v, batch, heads, sq, sq, d))


@pytest.mark.parametrize("d", [40, 80, 160])
def test_flash_attention_cross(cuda, d):
    frames, videos, heads, sq, L = 4, 2, 2, 256, 77
    C = heads * d
    q = rnd(videos * frames * sq, C, std=1.5)
    kv = rnd(videos * L, 2 * C, std=1.5)
    got = ops.attention(q, kv[:, :C], kv[:, C:], videos * frames, heads, sq, L, d, kv_div=frames)
    close_bf16(got, sdpa_ref(q, kv[:, :C], kv[:, C:], videos * frames, heads, sq, L, d, kv_div=frames))


def test_flash_attention_rescale_spike(cuda):
    """Force the online-softmax rescale branch: one key in a LATE tile dominates
    (cdna_hip_programming.md §5.4 rule 26)."""
    batch, heads, sq, d = 1, 1, 128, 64
    q = rnd(sq, d)
    k = rnd(sq, d) * 0.1
    v = rnd(sq, d)
    k[100] = bf(q[5].float() * 4)   # spike for query 5 at key 100 (tile 1)
    got = ops.attention(q, k, v, batch, heads, sq, sq, d)
    close_bf16(got, sdpa_ref(q, k, v, batch, heads, sq, sq, d))


@pytest.mark.parametrize("sq,skv", [(256, 256), (300, 77), (1000, 333), (64, 1)])
def test_flash_attention_d40_paths(attn_path, sq, skv):
    """Both d = 40 kernels over aligned, ragged and single-key shapes (queries past sq,
    keys past skv), fused-QKV strides for self and separate K/V otherwise."""
    torch.manual_seed(11)
    batch, heads, d = 2, 8, 40
    C = heads * d
    q = rnd(batch * sq, 3 * C, std=1.5)[:, :C]
    kv = rnd(batch * skv, 2 * C, std=1.5)
    got = ops.attention(q, kv[:, :C], kv[:, C:], batch, heads, sq, skv, d, kernel=attn_path)
    close_bf16(got, sdpa_ref(q, kv[:, :C], kv[:, C:], batch, heads, sq, skv, d))


def _deferred_max_case(kind, sq=256, skv=640, d=40):
    """Score patterns that drive the deferred-max branch (§5.4 rule 26): the branch
    is data-dependent, so each case forces a different decision sequence.  Scores run
    along a fixed unit direction u: s*log2(e)/sqrt(d) grows by about 2.7*alpha per
    64-key tile for q = 12u, k = alpha*tile*u (threshold THR = 6 in those units)."""
    g = torch.Generator(device="cuda").manual_seed(5)
    q = torch.randn(sq, d, device="cuda", generator=g)
    k = torch.randn(skv, d, device="cuda", generator=g)
    v = torch.randn(skv, d, device="cuda", generator=g)
    u = torch.randn(d, device="cuda", generator=g)
    u = u / u.norm()
    tile = (torch.arange(skv, device="cuda") // 64).float()[:, None]
    if kind == "ramp":          # each tile's max beats the last by ~8 > THR: rescale every tile
        q, k = 12 * u + 0.3 * q, 3.0 * tile * u + 0.1 * k
    elif kind == "creep":       # growth ~3 < THR per tile: deferred, P accumulates up to 2^THR
        q, k = 12 * u + 0.3 * q, 1.1 * tile * u + 0.1 * k
    elif kind == "late_spike":  # one query's max jumps in the last tile only (mixed lanes)
        k = 0.1 * k
        k[skv - 3] = q[37] * 6
    elif kind == "huge_spike":  # a jump of ~180 (log2) in a late tile: exp2 would overflow -> exact rerun
        k = 0.1 * k
        k[skv - 70] = q[37] * 20
    elif kind == "offset":      # all scores ~ +70 (mu far from 0: bf16 rounding of mu)
        q, k = 8 * u + 0.3 * q, 40 * u + 0.1 * k
    elif kind == "negative":    # all scores ~ -70: the first tile's mu must come from the data
        q, k = 8 * u + 0.3 * q, -40 * u + 0.1 * k
    return bf(q), bf(k), bf(v)


@pytest.mark.parametrize("kind", ["ramp", "creep", "late_spike", "huge_spike", "offset", "negative"])
def test_flash_attention_deferred_max(attn_path, kind):
    q, k, v = _deferred_max_case(kind)
    sq, skv, d = q.shape[0], k.shape[0], q.shape[1]
    got = ops.attention(q, k, v, 1, 1, sq, skv, d, kernel=attn_path)
    assert torch.isfinite(got.float()).all()
    # O is a convex combination of V rows and P is rounded to bf16 (relative 2^-9) before
    # PV, so the absolute error scales with |V|, not |O| (these cases concentrate the
    # weights on a few keys and |O| << |V|); a mis-scaled tile shows up as errors >= 0.1.
    close_bf16(got, sdpa_ref(q, k, v, 1, 1, sq, skv, d), abs_frac=2e-3 * v.float().abs().max().item()
               / sdpa_ref(q, k, v, 1, 1, sq, skv, d).abs().max().item())


@pytest.mark.parametrize("kind", ["ramp", "creep", "late_spike", "huge_spike", "offset", "negative"])
def test_flash_attention_deferred_max_unit_scale(attn_path, kind):
    """The same score patterns through the unit-scale fast pass (the model's call, softmax
    scale folded into q; its row-sum check runs one tile late)."""
    q, k, v = _deferred_max_case(kind)
    sq, skv, d = q.shape[0], k.shape[0], q.shape[1]
    q = bf(q.float() * d ** -0.5 * math.log2(math.e))  # scores in log2 units
    got = ops.attention(q, k, v, 1, 1, sq, skv, d, scale=1.0 / math.log2(math.e), kernel=attn_path)
    assert torch.isfinite(got.float()).all()
    want = sdpa_ref(q, k, v, 1, 1, sq, skv, d, scale=1.0 / math.log2(math.e))
    close_bf16(got, want, abs_frac=2e-3 * v.float().abs().max().item() / want.abs().max().item())


@pytest.mark.parametrize("kind", ["ramp", "creep", "late_spike", "huge_spike", "offset", "negative"])
@pytest.mark.parametrize("unit", [False, True])
def test_flash80_deferred_max(cuda, kind, unit):
    """flash80 (round 6: the level-2 d = 80 self-attention on flash40's schedule, exact deferred max
    decided on P = exp2(S)) through the deferred-max score patterns at d = 80, prescaled and on the
    model's unit scale: "huge_spike" sends a P to inf (the rare branch recomputes it from the exact
    tile max), "ramp" rescales every tile, "negative" needs mu from the data — no fix-up pass."""
    q, k, v = _deferred_max_case(kind, d=80)
    sq, skv, d = q.shape[0], k.shape[0], q.shape[1]
    sc = None
    if unit:
        q = bf(q.float() * d ** -0.5 * math.log2(math.e))
        sc = 1.0 / math.log2(math.e)
    got = ops.attention(q, k, v, 1, 1, sq, skv, d, scale=sc, kernel="flash40")
    assert torch.isfinite(got.float()).all()
    want = sdpa_ref(q, k, v, 1, 1, sq, skv, d, scale=sc)
    close_bf16(got, want, abs_frac=2e-3 * v.float().abs().max().item() / want.abs().max().item())


@pytest.mark.parametrize("sq,skv,batch,kv_div", [(1024, 1024, 2, 1), (300, 300, 3, 1), (777, 640, 2, 2),
                                               (1024, 128, 1, 1)])
def test_flash80_matches_fp64(cuda, sq, skv, batch, kv_div):
    """flash80 on the model's real-valued level-2 inputs (q, k, v ~ N(0, 1.5^2), fused-QKV row
    strides, the softmax scale folded into q), ragged query blocks (sq not a multiple of its 256),
    ragged key tiles, a K/V shared by kv_div query batches and the 2-tile minimum: bf16 output
    within bf16 rounding of fp64 SDPA, and the automatic choice equal to the forced one."""
    torch.manual_seed(sq + skv + 80)
    heads, d = 8, 80
    C = heads * d
    q = rnd(batch * sq, 3 * C, std=1.5)[:, :C]
    q = bf(q.float() * d ** -0.5 * math.log2(math.e))
    kv = rnd(batch // kv_div * skv, 2 * C, std=1.5)
    sc = 1.0 / math.log2(math.e)
    got = ops.attention(q, kv[:, :C], kv[:, C:], batch, heads, sq, skv, d, kv_div=kv_div, scale=sc, kernel="flash40")
    close_bf16(got, sdpa_ref(q, kv[:, :C], kv[:, C:], batch, heads, sq, skv, d, kv_div=kv_div, scale=sc))
    if skv >= 256:
        auto = ops.attention(q, kv[:, :C], kv[:, C:], batch, heads, sq, skv, d, kv_div=kv_div, scale=sc)
        assert torch.equal(auto, got)


def test_flash_attention_unit_scale(cuda):
    """c = scale*log2(e) == 1 exactly skips the in-kernel Q prescale (callers that fold
    the softmax scale into the Q projection); must equal the prescaled path's math."""
    torch.manual_seed(2)
    sq, d = 512, 40
    q, k, v = rnd(sq, d, std=3.0), rnd(sq, d), rnd(sq, d)
    got = ops.attention(q, k, v, 1, 1, sq, sq, d, scale=1.0 / math.log2(math.e))
    qd, kd, vd = q.double(), k.double(), v.double()
    want = torch.softmax(qd @ kd.T / math.log2(math.e), -1) @ vd
    close_bf16(got, want)


@pytest.mark.parametrize("d,sq,skv,batch,kv_div", [(40, 4096, 4096, 2, 1), (40, 1000, 333, 2, 1), (40, 777, 77, 4, 4),
                                                  (80, 1024, 1024, 2, 1), (160, 256, 256, 3, 1), (64, 300, 300, 2, 1),
                                                  (32, 200, 77, 2, 2), (128, 130, 130, 1, 1)])
def test_attention_fp32_out_north_star_tolerance(attn_path, d, sq, skv, batch, kv_div):
    """vd_attention_f32 against fp64 softmax(q k^T / log2 e) v at the north star's rtol 1e-3 /
    atol 1e-4.  Scores are integers (q, k in {-1, 0, 1}) and the scale is the model path's
    unit c, so every P = 2^(s - max) is exactly representable in bf16: what is checked is the
    kernels' tiling, online softmax, ragged tails, row sums and fp32 accumulation — the one
    rounding the product path adds on purpose (P to bf16 before PV, and O to bf16) is the
    subject of the bf16-output tests above."""
    torch.manual_seed(d + sq)
    heads = 2
    C = heads * d
    q = bf(torch.randint(-1, 2, (batch * sq, C), device="cuda").float())
    k = bf(torch.randint(-1, 2, (batch // kv_div * skv, C), device="cuda").float())
    v = rnd(batch // kv_div * skv, C)
    got = ops.attention(q, k, v, batch, heads, sq, skv, d, kv_div=kv_div, scale=1.0 / math.log2(math.e), out_f32=True,
                        kernel=attn_path)
    assert got.dtype == torch.float32
    qd = q.double().reshape(batch, sq, heads, d).transpose(1, 2)
    kd = k.double().reshape(batch // kv_div, skv, heads, d).transpose(1, 2).repeat_interleave(kv_div, 0)
    vd = v.double().reshape(batch // kv_div, skv, heads, d).transpose(1, 2).repeat_interleave(kv_div, 0)
    s = qd @ kd.transpose(-1, -2)
    p = torch.exp2(s - s.amax(-1, keepdim=True))
    want = ((p @ vd) / p.sum(-1, keepdim=True)).transpose(1, 2).reshape(batch * sq, C)
    err = (got.double() - want).abs()
    print(f"d={d} sq={sq} skv={skv}: max |O - O_fp64| {err.max().item():.2e}")
    assert torch.all(err <= 1e-4 + 1e-3 * want.abs()), err.max().item()


def _flash40_vs_flash32(q, k, v, batch, heads, sq, skv, d, kv_div=1, scale=None, out_f32=False):
    a = ops.attention(q, k, v, batch, heads, sq, skv, d, kv_div=kv_div, scale=scale, out_f32=out_f32, kernel="flash40")
    b = ops.attention(q, k, v, batch, heads, sq, skv, d, kv_div=kv_div, scale=scale, out_f32=out_f32, kernel="flash32")
    return a, b


@pytest.mark.parametrize("sq,skv,batch,kv_div,out_f32", [(4096, 4096, 2, 1, False), (512, 128, 1, 1, False),
                                                         (1000, 333, 2, 1, True), (777, 4100, 2, 2, False),
                                                         (300, 640, 3, 1, True)])
def test_flash40_bit_identical_to_flash32(cuda, sq, skv, batch, kv_div, out_f32):
    """flash40 (round 3: ping-pong schedule, LDS-DMA ring, data-driven ragged tail, out-of-line
    exact pass) keeps flash32's arithmetic tile for tile: the same MFMA chains in the same order,
    the same mu decisions at the same points, and keys past skv contribute an exact 0 (zero V
    row and ones column) where flash32 masks them to -inf.  So the outputs are equal BIT FOR BIT,
    on the model's unit-scale path and the prescaled one, bf16 and fp32 outputs, ragged sq (not
    a multiple of the 512-query block) and skv, and a K/V shared by kv_div query batches."""
    torch.manual_seed(sq + skv)
    heads, d = 4, 40
    C = heads * d
    q = rnd(batch * sq, 3 * C, std=1.5)[:, :C]
    q_unit = bf(q.float() * d ** -0.5 * math.log2(math.e))
    kv = rnd(batch // kv_div * skv, 2 * C, std=1.5)
    for qq, sc in ((q_unit, 1.0 / math.log2(math.e)), (q, None)):
        a, b = _flash40_vs_flash32(qq, kv[:, :C], kv[:, C:], batch, heads, sq, skv, d, kv_div=kv_div, scale=sc,
                                   out_f32=out_f32)
        assert torch.isfinite(a.float()).all()
        assert torch.equal(a, b), (a.float() - b.float()).abs().max().item()


@pytest.mark.parametrize("kind", ["ramp", "creep", "late_spike", "huge_spike", "offset", "negative"])
def test_flash40_deferred_max_cases_bit_identical(cuda, kind):
    """The deferred-max score patterns (§5.4 rule 26) through flash40 and flash32: "huge_spike"
    sends flash40's block through its NaN flag and flash32's exact fix-up launch, the others
    through the fast pass's rescale decisions — all bit-identical to flash32."""
    q, k, v = _deferred_max_case(kind)
    sq, skv, d = q.shape[0], k.shape[0], q.shape[1]
    qu = bf(q.float() * d ** -0.5 * math.log2(math.e))
    for qq, sc in ((qu, 1.0 / math.log2(math.e)), (q, None)):
        a, b = _flash40_vs_flash32(qq, k, v, 1, 1, sq, skv, d, scale=sc)
        assert torch.isfinite(a.float()).all()
        assert torch.equal(a, b), (a.float() - b.float()).abs().max().item()


@pytest.mark.parametrize("sq,skv,batch", [(4096, 4096, 2), (1000, 333, 2), (300, 77, 3)])
def test_attention_d40_real_valued_north_star_tolerance(attn_path, sq, skv, batch):
    """The roofline kernel (d = 40, the model's unit scale) on REAL-valued inputs as the model
    produces them (q, k, v ~ N(0, 1.5^2), softmax scale * log2 e folded into q), fp32 output,
    at the north star's rtol 1e-3 / atol 1e-4 against an fp64 reference that rounds P to bf16
    where the kernel does: P = bf16(2^(s - mu)) with mu = bf16(max of the row's scores over the
    first 64-key tile) (the fast pass's running offset; its 2^32 row-sum rescale is not reached
    at this logit range, asserted below), O = (P V) / sum(P), the sum over the same bf16 P.
    The one freedom left is the last ulps of x = s - mu and of v_exp_f32: where 2^(s - mu) lies within 2^-17
    (relative) of a bf16 rounding midpoint, the kernel's P may round the other way; the bound
    adds exactly what those flips can move O by, |P_alt - P| |v - O| / l summed over the flagged
    scores.  Printed: that ambiguity term and the distance to exact fp64 softmax (what the bf16
    P rounding itself costs)."""
    if attn_path == "v1":
        pytest.skip("the 16x16x32 kernel tracks a per-tile running max (another mu); bf16-output tests cover it")
    torch.manual_seed(sq + skv)
    heads, d = 2, 40
    C = heads * d
    q = bf(torch.randn(batch * sq, C, device="cuda") * 1.5 * d ** -0.5 * math.log2(math.e))
    k = bf(torch.randn(batch * skv, C, device="cuda") * 1.5)
    v = bf(torch.randn(batch * skv, C, device="cuda") * 1.5)
    got = ops.attention(q, k, v, batch, heads, sq, skv, d, scale=1.0 / math.log2(math.e), out_f32=True,
                        kernel=attn_path)
    qd = q.double().reshape(batch, sq, heads, d).transpose(1, 2)
    kd = k.double().reshape(batch, skv, heads, d).transpose(1, 2)
    vd = v.double().reshape(batch, skv, heads, d).transpose(1, 2)
    s = qd @ kd.transpose(-1, -2)                                     # log2 units
    mu = s[..., :64].amax(-1, keepdim=True).float().to(torch.bfloat16).double()
    e = torch.exp2(s - mu)
    del s
    assert (e.sum(-1) < 2.0 ** 32).all()                              # no fast-pass rescale
    p = e.float().to(torch.bfloat16).double()
    l = p.sum(-1, keepdim=True)
    want = (p @ vd) / l
    # bf16 neighbours of e: the rounding midpoint nearest e and the value on its other side
    m, ex = torch.frexp(e)                                            # e = m 2^ex, m in [0.5, 1)
    ulp = torch.ldexp(torch.full_like(e, 2.0 ** -8), ex)              # bf16 spacing at e
    mid = (torch.floor(e / ulp) + 0.5) * ulp                          # the rounding midpoint of e's cell
    amb = (e - mid).abs() <= e * 2.0 ** -17
    alt = torch.where(p >= e, p - ulp, p + ulp)
    dp = torch.where(amb, (alt - p).abs(), torch.zeros_like(p))
    del m, ex, ulp, mid, amb, alt, e
    slack = (dp @ vd.abs() + dp.sum(-1, keepdim=True) * want.abs()) / l
    want = want.transpose(1, 2).reshape(batch * sq, C)
    slack = slack.transpose(1, 2).reshape(batch * sq, C)
    pe = torch.exp2(qd @ kd.transpose(-1, -2) - mu)
    exact = ((pe @ vd) / pe.sum(-1, keepdim=True)).transpose(1, 2).reshape(batch * sq, C)
    err = (got.double() - want).abs()
    print(f"d=40 real-valued [{attn_path}] sq={sq} skv={skv}: max|O - O_ref(bf16 P)| {err.max().item():.2e}, "
          f"max exp2-flip allowance {slack.max().item():.2e}, max|O - O_fp64 exact| "
          f"{(got.double() - exact).abs().max().item():.2e}")
    assert torch.all(err <= 1e-4 + 1e-3 * want.abs() + slack), (err - 1e-3 * want.abs() - slack).max().item()


@pytest.fixture(params=["mfma", "valu"])
def temporal_path(request, cuda):
    """frames <= 16 with d in {40, 80, 160} run on the MFMA kernel; "valu" runs every shape on the
    VALU kernel (vd_temporal_attention_valu)."""
    return request.param


@pytest.mark.parametrize("frames,d,scale", [(16, 40, None), (16, 80, None), (16, 160, None), (5, 40, None),
                                            (1, 80, None), (12, 160, None), (16, 40, "unit"), (4, 32, None),
                                            (16, 32, None), (32, 80, None), (5, 64, None)])
def test_temporal_attention(temporal_path, frames, d, scale):
    batch, pos, heads = 2, 37, 3
    C = heads * d
    qkv = rnd(batch * frames * pos, 3 * C, std=1.5)
    q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
    sc = 1.0 / math.log2(math.e) if scale == "unit" else None   # the model's call (scale folded into to_q)
    got = ops.temporal_attention(q, k, v, batch, frames, pos, heads, d, scale=sc, valu=temporal_path == "valu")
    if sc is not None:
        q = q.double() * (sc * math.sqrt(d))   # sdpa_ref applies d^-0.5

    def tok(t):  # rows (b, f, p) -> (b*p, f, C)
        return t.double().reshape(batch, frames, pos, C).permute(0, 2, 1, 3).reshape(batch * pos, frames, C)

    want = sdpa_ref(tok(q), tok(k), tok(v), batch * pos, heads, frames, frames, d)
    want = want.reshape(batch, pos, frames, C).permute(0, 2, 1, 3).reshape(-1, C)
    close_bf16(got, want)


@pytest.mark.parametrize("d", [32, 40, 80, 160])
@pytest.mark.parametrize("frames,qf,f0", [(16, 2, 6), (16, 4, 12), (8, 8, 0), (16, 1, 15)])
def test_temporal_attention_kv(cuda, frames, qf, f0, d):
    """vd_temporal_attention_kv (the K/V all-gather window): a rank's qf query frames
    [f0, f0 + qf) in their own rows against all frames' K/V equals those frames' rows of the
    full self-attention bit for bit (same MFMA operands and order), and fp64 SDPA."""
    batch, pos, heads = 2, 37, 2
    C = heads * d
    qkv = rnd(batch * frames * pos, 3 * C, std=1.5)
    q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
    full = ops.temporal_attention(q, k, v, batch, frames, pos, heads, d)
    mine = lambda t: t.reshape(batch, frames, pos, -1)[:, f0:f0 + qf].reshape(-1, t.shape[1]).contiguous()
    kv = torch.cat([k, v], 1)   # the gathered [rows][2C] buffer
    got = ops.temporal_attention_kv(mine(q), kv[:, :C], kv[:, C:], batch, qf, frames, pos, heads, d)
    assert torch.equal(got, mine(full))

    def tok(t, f):
        return t.double().reshape(batch, f, pos, C).permute(0, 2, 1, 3).reshape(batch * pos, f, C)

    want = sdpa_ref(tok(mine(q), qf), tok(k, frames), tok(v, frames), batch * pos, heads, qf, frames, d)
    close_bf16(got, want.reshape(batch, pos, qf, C).permute(0, 2, 1, 3).reshape(-1, C))


@pytest.mark.parametrize("batch,positions,unit", [(2, 4096, True), (1, 4100, False), (3, 1373, True),
                                                   (1, 2048, False)])
def test_motion_qkv_attention(cuda, batch, positions, unit):
    """vd_motion_qkv_attention (the level-1 motion module's Q/K/V projection fused into its
    temporal attention) equals vd_gemm + vd_temporal_attention bit for bit — ragged position
    counts (the last workgroup's idle waves), both softmax-scale forms — and fp64 SDPA of the
    bf16 projection to bf16 rounding.  The first three shapes take two positions per wave, the
    last (256 workgroups at one, 128 at two) one."""
    C, d, heads, F = 320, 40, 8, 16
    x = rnd(batch * F * positions, C)
    w = rnd(3 * C, C, std=C ** -0.5 * 2.0)
    sc = 1.0 / math.log2(math.e) if unit else None
    got = ops.motion_qkv_attention(x, w, batch, F, positions, heads, d, scale=sc)
    assert got is not None
    qkv = ops.gemm(x, w)
    want = ops.temporal_attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], batch, F, positions, heads, d, scale=sc)
    assert torch.equal(got, want)
    q, k, v = qkv[:, :C].double(), qkv[:, C:2 * C].double(), qkv[:, 2 * C:].double()
    if unit:
        q = q * (sc * math.sqrt(d))   # sdpa_ref applies d^-0.5

    def tok(t):  # rows (b, f, p) -> (b*p, f, C)
        return t.reshape(batch, F, positions, C).permute(0, 2, 1, 3).reshape(batch * positions, F, C)

    ref = sdpa_ref(tok(q), tok(k), tok(v), batch * positions, heads, F, F, d)
    close_bf16(got, ref.reshape(batch, positions, F, C).permute(0, 2, 1, 3).reshape(-1, C))
    assert ops.motion_qkv_attention(x[:, :320], w[:, :320], batch, 8, positions * 2, heads, d) is None  # 8 frames
    assert ops.motion_qkv_attention(x[:16 * 64], w, 1, F, 64, heads, d) is None  # 8 workgroups: unfused path
    assert ops.motion_qkv_takes(batch, F, positions, heads, d) and not ops.motion_qkv_takes(1, F, 64, heads, d)


@pytest.mark.parametrize("batch,positions,offset", [(2, 4096, 0.0), (1, 4100, 30.0), (1, 2048, 0.0),
                                                     (1, 2048, 300.0)])
def test_motion_qkv_attention_ln_fold(cuda, batch, positions, offset):
    """vd_motion_qkv_attention with ln_fold_tab (round 5): the motion block's LayerNorm + PE by
    frame folded into the fused QKV attention (MotionLnFold: W' = W∘gamma, per head the row sums
    and W·(beta + pe[f])), over the UN-normalised rows — against the unfolded device path
    (vd_layernorm with PE, then the same kernel on bf16(W)) within the two paths' bf16 roundings,
    and against fp64 LayerNorm + PE -> QKV -> SDPA; rows offset by 30 std (one-pass variance) and
    300 std (its exact second pass); both PW forms."""
    from vdiff.models.layers import MotionLnFold
    C, d, heads, NF = 320, 40, 8, 16
    g = torch.Generator(device=cuda).manual_seed(3)
    x = bf(1.3 * (torch.randn(batch * NF * positions, C, device=cuda, generator=g) + offset))
    norm = torch.nn.LayerNorm(C).to(cuda)
    with torch.no_grad():
        norm.weight.copy_(1 + 0.2 * torch.randn(C, device=cuda, generator=g))
        norm.bias.copy_(0.1 * torch.randn(C, device=cuda, generator=g))
    pe = torch.randn(32, C, device=cuda, generator=g) * 0.5
    w = torch.randn(3 * C, C, device=cuda, generator=g) * C ** -0.5 * 2.0
    sc = 1.0 / math.log2(math.e)
    mf = MotionLnFold(norm, w, pe, heads, d)
    got = ops.motion_qkv_attention(x, mf.w, batch, NF, positions, heads, d, scale=sc, ln_fold=(mf.tab, mf.eps))
    assert got is not None
    gamma, beta = norm.weight.detach().float().contiguous(), norm.bias.detach().float().contiguous()
    n = ops.layer_norm(x, gamma, beta, pe=pe.float().contiguous(), pe_div=positions, pe_period=NF)
    unf = ops.motion_qkv_attention(n, bf(w).contiguous(), batch, NF, positions, heads, d, scale=sc)
    xd = x.double()
    ln = F.layer_norm(xd, (C,), norm.weight.double(), norm.bias.double(), norm.eps)
    ln = ln + pe.double()[(torch.arange(x.shape[0], device=cuda) // positions) % NF]
    qkv = ln @ w.double().T
    q, k, v = qkv[:, :C] * (sc * math.sqrt(d)), qkv[:, C:2 * C], qkv[:, 2 * C:]

    def tok(t):  # rows (b, f, p) -> (b*p, f, C)
        return t.reshape(batch, NF, positions, C).permute(0, 2, 1, 3).reshape(batch * positions, NF, C)

    ref = sdpa_ref(tok(q), tok(k), tok(v), batch * positions, heads, NF, NF, d)
    ref = ref.reshape(batch, positions, NF, C).permute(0, 2, 1, 3).reshape(-1, C)
    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()  # noqa: E731
    e_ref, e_unf, e_dev = rel(got, ref), rel(unf, ref), rel(got, unf)
    print(f"batch {batch} positions {positions} offset {offset}: folded vs fp64 {e_ref:.5f}, unfolded vs fp64 "
          f"{e_unf:.5f}, folded vs unfolded {e_dev:.5f}")
    assert e_ref < 2.5e-2 and e_dev < 3e-2  # the attention of bf16 q / k at this weight scale: ~1.5 % either way
    assert e_ref < 1.5 * e_unf + 1e-3


# ---------------------------------------------------------------- step glue
def test_timestep_embed(cuda):
    from oracle.unet_ref import timestep_embedding
    ts = torch.tensor([961.0, 1.0, 500.0], device=cuda)
    got = ops.timestep_embed(ts, 320)
    close_bf16(got, timestep_embedding(ts.cpu(), 320))
    step = torch.tensor([2], device=cuda, dtype=torch.int32)
    got = ops.timestep_embed(ts, 320, step_idx=step, batch=2)
    close_bf16(got, timestep_embedding(torch.tensor([500.0, 500.0]), 320))


def test_pack_unpack_roundtrip(cuda):
    x = torch.randn(2, 4, 3, 8, 6, device=cuda)
    rows = ops.pack_latents(x, dup=2, cpad=8)
    assert rows.shape == (2 * 2 * 3 * 48, 8)
    assert torch.all(rows[:, 4:] == 0)
    back = ops.unpack_nhwc(rows[: 2 * 3 * 48], 2, 4, 3, 8, 6)
    close_bf16(back, x)
    back2 = ops.unpack_nhwc(rows[2 * 3 * 48:], 2, 4, 3, 8, 6)
    assert torch.equal(back, back2)


def test_ddim_cfg_step_matches_oracle(cuda):
    from oracle import ddim_ref
    acp = ddim_ref.alphas_cumprod()
    B, Cc, Fr, H, W = 1, 4, 3, 8, 8
    lat = torch.randn(B, Cc, Fr, H, W, device=cuda)
    eps_rows = torch.randn(2 * Fr * H * W, 4, device=cuda)
    t, n = 961, 50
    prev = t - 1000 // n
    sq = ddim_ref._sqrt  # correctly rounded fp32 sqrt, as the product host tables
    coef = torch.stack([sq(acp[t]), sq(1 - acp[t]), sq(acp[prev]), sq(1 - acp[prev])]).float()
    x = lat.clone()
    x0 = torch.empty_like(x)
    nxt = torch.empty(2 * Fr * H * W, 8, device=cuda, dtype=BF)
    ops.ddim_cfg_step(eps_rows, 2, 7.5, x, coef.to(cuda), x0_out=x0, next_in=nxt)
    e = eps_rows.cpu().reshape(2, Fr, H, W, 4).permute(0, 4, 1, 2, 3)
    want, want0 = ddim_ref.ddim_step(ddim_ref.cfg_combine(e, 7.5), t, lat.cpu(), n, acp)
    # one rounding per op in diffusers' order (no contraction, correctly rounded division)
    assert torch.equal(x.cpu(), want)
    assert torch.equal(x0.cpu(), want0)
    close_bf16(ops.unpack_nhwc(nxt[: Fr * H * W], 1, 4, Fr, H, W), want)


def test_step_index_is_clamped_to_the_tables(cuda):
    """a device step counter past the end of its timestep / coefficient table
    (a replay beyond the schedule) reads the table's last row, never memory past it."""
    ts = torch.tensor([961.0, 941.0], device=cuda)
    lat = torch.randn(1, 4, 2, 8, 8, device=cuda)
    eps_rows = torch.randn(2 * 8 * 8, 4, device=cuda)
    coef = torch.tensor([[0.05, 0.99, 0.06, 0.98], [0.3, 0.9, 0.4, 0.8]], device=cuda)
    for idx, row in ((5, 1), (-3, 0), (1, 1)):
        st = torch.tensor([idx], device=cuda, dtype=torch.int32)
        te = ops.timestep_embed(ts, 320, step_idx=st, batch=1)
        assert torch.equal(te, ops.timestep_embed(ts[row:row + 1].contiguous(), 320))
        a, b = lat.clone(), lat.clone()
        ops.ddim_cfg_step(eps_rows, 1, 1.0, a, coef, step_idx=st)
        ops.ddim_cfg_step(eps_rows, 1, 1.0, b, coef[row:row + 1].contiguous())
        assert torch.equal(a, b)


@pytest.mark.parametrize("ncfg", [2, 1])
def test_euler_cfg_step_matches_oracle(cuda, ncfg):
    """CFG + EulerDiscreteScheduler.step in diffusers' fp32 operation order: bit-exact against
    the oracle on the same inputs (no FMA contraction in the kernel); the packed next input is
    scale_model_input(x, sigma_next) rounded once to bf16."""
    from oracle import euler_ref
    _, sig = euler_ref.set_timesteps(25)
    B, Cc, Fr, H, W = 1, 4, 3, 8, 8
    for i in (0, 11, 24):  # first, interior, last (sigma_next = 0, divisor 1)
        s, sn = sig[i], sig[i + 1]
        coef = torch.stack([s, sn, (sn ** 2 + 1) ** 0.5, torch.zeros(())]).float()
        lat = torch.randn(B, Cc, Fr, H, W, device=cuda) * float(s)
        eps_rows = torch.randn(ncfg * Fr * H * W, 4, device=cuda)
        x = lat.clone()
        x0 = torch.empty_like(x)
        nxt = torch.empty(ncfg * Fr * H * W, 8, device=cuda, dtype=BF)
        ops.euler_cfg_step(eps_rows, ncfg, 7.5, x, coef.to(cuda), x0_out=x0, next_in=nxt)
        e = eps_rows.cpu().reshape(ncfg, Fr, H, W, 4).permute(0, 4, 1, 2, 3)
        e = e[0:1] + 7.5 * (e[1:2] - e[0:1]) if ncfg == 2 else e
        want, want0 = euler_ref.euler_step(e, lat.cpu(), s, sn)
        close_f32(x, want, rtol=1e-6, atol=1e-6)
        close_f32(x0, want0, rtol=1e-6, atol=1e-6)
        close_bf16(ops.unpack_nhwc(nxt[: Fr * H * W], 1, 4, Fr, H, W), euler_ref.scale_model_input(want, sn))


def test_pack_latents_input_divisor(cuda):
    x = torch.randn(1, 4, 2, 8, 8, device=cuda) * 25.0
    rows = ops.pack_latents(x, dup=1, cpad=8, in_div=25.17)
    close_bf16(ops.unpack_nhwc(rows, 1, 4, 2, 8, 8), x / 25.17)


def test_step_advance_and_block_transpose(cuda):
    s = torch.zeros(1, device=cuda, dtype=torch.int32)
    ops.step_advance(s)
    ops.step_advance(s)
    assert s.item() == 2
    src = rnd(2 * 3 * 5, 16)
    close_bf16(ops.block_transpose(src, 2, 3, 5), block_transpose_reference(src.cpu(), 2, 3, 5))
