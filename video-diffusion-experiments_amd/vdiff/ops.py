"""Tensor-level wrappers over the C ABI (include/vdiff.h).

Every function launches HIP kernels on torch's current stream (so it is
hipGraph-capturable) and never falls back to a CPU or torch implementation:
non-CUDA tensors are rejected and a missing library raises.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import math

import torch

from ._lib import VD_EUNSUPPORTED, GemmDesc, check, lib

ACT_NONE, ACT_SILU, ACT_GEGLU, ACT_GELU = 0, 1, 2, 3
A_DENSE, A_CONV3X3 = 0, 1
BF16 = torch.bfloat16


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _p(t):
    return None if t is None else t.data_ptr()


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("vdiff ops run on the GPU only (got a CPU tensor); no CPU fallback")


def _rows(t, dtype=BF16):
    """Validate a 2-D row-major operand (unit inner stride) and return its row stride."""
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"expected a 2-D row-major tensor, got shape {tuple(t.shape)} strides {t.stride()}")
    if t.dtype != dtype:
        raise ValueError(f"expected {dtype}, got {t.dtype}")
    return t.stride(0)


# ---------------------------------------------------------------- GEMM / conv
class _GemmPlan:
    path = 0       # vd_gemm_desc.path for the GEMMs issued (0 = the automatic plan)
    plan_div = 0   # > 0: plan every GEMM whose M it divides as if M were M / plan_div
    plan_mul = 1   # > 1: plan every GEMM as if M were M * plan_mul (before plan_div)


_PLAN = _GemmPlan()


@contextlib.contextmanager
def plan_scaled(mul: int):
    """Plan every GEMM (and the fused-kernel shape questions) inside the block as if its M were
    `mul` times larger: the motion block run on one of `mul` position chunks
    (FrameShard(overlap_chunks=mul)) then makes every kernel, split-K and LayerNorm-fold decision
    the whole block would, so chunking changes the launch count, never the arithmetic."""
    old = _PLAN.plan_mul
    _PLAN.plan_mul = old * int(mul)
    try:
        yield
    finally:
        _PLAN.plan_mul = old


@contextlib.contextmanager
def gemm_plan(path: int = 0, plan_div: int = 0):
    """Test / benchmark hook on the Python side only — the C ABI takes both values per call in
    vd_gemm_desc and keeps no state.  Inside the block every vd_gemm carries `path` (1 v1, 2 v2,
    3 v3, 5 v5, 6 v6, 8 v8: forced where that kernel takes the shape) and, with plan_div = N, plan_m =
    M / N for each GEMM whose M N divides: an unsharded model planned like one of N frame shards
    (same kernels, split-K and LayerNorm fusion, so the same summation order), which makes the
    sharded-vs-unsharded comparison of tests/test_gpu_dist2.py bit-exact under the product plan."""
    old = (_PLAN.path, _PLAN.plan_div)
    _PLAN.path, _PLAN.plan_div = int(path), int(plan_div)
    try:
        yield
    finally:
        _PLAN.path, _PLAN.plan_div = old


def _plan_controls(d):
    d.path = _PLAN.path
    m = d.M * _PLAN.plan_mul
    if _PLAN.plan_div > 1 and m % _PLAN.plan_div == 0:
        m //= _PLAN.plan_div
    if m != d.M:
        d.plan_m = m


def gemm_plan_of(d):
    """(kernel, split) vd_gemm would run for descriptor d under the current gemm_plan controls
    (vd_gemm_plan; kernel 0 = refused)."""
    _plan_controls(d)
    k, sp = C.c_int32(0), C.c_int32(0)
    check(lib().vd_gemm_plan(C.byref(d), C.byref(k), C.byref(sp)), "vd_gemm_plan")
    return k.value, sp.value


def ln_fold_runs(M, w, s, *, act=ACT_NONE, rowbias=False):
    """True when vd_gemm runs Linear(LayerNorm(x)) over M rows of x with the norm folded into
    the GEMM (vd_gemm_desc.ln_fold_s: w = W∘gamma, s = its row sums) — the v8 plan (K = 320) or
    an unsplit v6 (the small M of a frame shard); the caller otherwise writes the normalised rows
    and runs the plain GEMM.  Decided by the library's own plan (with plan_div, so a frame shard
    and its unsharded replay decide alike)."""
    N, K = w.shape
    nout = N // 2 if act == ACT_GEGLU else N
    d = GemmDesc(a0=256, lda0=K, k0=K, a_mode=A_DENSE, w=_p(w), ldw=_rows(w), M=M, N=N, K=K, bias=256,
                 act=act, out=256, ldc=nout, ln_fold_s=_p(s), ln_fold_eps=1e-5)
    if rowbias:  # the motion block's PE by frame (LnFold(pe=...)): no v8 / v5 plan takes a row bias
        d.rowbias, d.ld_rb, d.rb_div = 256, N, 1
    return gemm_plan_of(d)[0] != 0


# row counts a folded LayerNorm is asked about at prepare time: the UNet's levels at 2-32 images
LN_FOLD_PROBE_M = (256, 1024, 4096, 16384, 32768, 131072)


def ln_fold_shape_ok(N, K, *, act=ACT_NONE, rowbias=False):
    """Whether a folded LayerNorm (ln_fold_s) can run for an N x K Linear at any of the row counts
    the UNet gives it (LN_FOLD_PROBE_M, automatic plan): decides at prepare time which folded
    weights to build."""
    nout = N // 2 if act == ACT_GEGLU else N
    for M in LN_FOLD_PROBE_M:
        d = GemmDesc(a0=256, lda0=K, k0=K, a_mode=A_DENSE, w=256, ldw=K, M=M, N=N, K=K, bias=256, act=act,
                     out=256, ldc=nout, ln_fold_s=256, ln_fold_eps=1e-5)
        if rowbias:
            d.rowbias, d.ld_rb, d.rb_div = 256, N, 1
        k, sp = C.c_int32(0), C.c_int32(0)
        check(lib().vd_gemm_plan(C.byref(d), C.byref(k), C.byref(sp)), "vd_gemm_plan")
        if k.value != 0:
            return True
    return False


def _run_gemm(d, device, what):
    """Attach the split-K workspace the C side asks for (if any), then launch."""
    _plan_controls(d)
    nbytes = lib().vd_gemm_ws_bytes(C.byref(d))
    ws = None
    if nbytes > 0:
        ws = torch.empty(nbytes // 4, device=device, dtype=torch.float32)
        d.ws, d.ws_bytes = ws.data_ptr(), nbytes
    check(lib().vd_gemm(C.byref(d), _stream()), what)
    return ws  # keep alive until the launch is enqueued (stream-ordered reuse is safe)


def gemm(a, w, *, a1=None, bias=None, rowbias=None, rb_div=1, res=None, act=ACT_NONE,
         out=None, out_f32=False, rmap=None, ln_fold=None):
    """out[m, n] = epi(sum_k cat(a, a1)[m, k] * w[n, k]); a/a1/w bf16, bias/rowbias fp32.
    rmap = (n1, n2, inner): product row m is written (and its residual read) at row rev3(m)
    (vd_gemm_desc.rmap_*, vdiff.dist.frame_shard.rev3_reference).
    ln_fold = (s, eps): a is the UN-normalised input of a LayerNorm folded into this GEMM —
    w = W∘gamma, bias = b + W·beta, s = w's fp32 row sums (vd_gemm_desc.ln_fold_s,
    vdiff.models.layers.LnFold); raises when the plan cannot take it (see ln_fold_runs)."""
    _dev(a, w, a1, bias, rowbias, res, out)
    M = a.shape[0]
    N, K = w.shape
    lda0 = _rows(a)
    k0 = a.shape[1]
    lda1 = _rows(a1) if a1 is not None else 0
    if a1 is not None and (a1.shape[0] != M or k0 + a1.shape[1] != K):
        raise ValueError("concat operand shapes do not add up to K")
    if a1 is None and k0 != K:
        raise ValueError(f"A has {k0} columns, W has K={K}")
    nout = N // 2 if act == ACT_GEGLU else N
    if out is None:
        out = torch.empty(M, nout, device=a.device, dtype=torch.float32 if out_f32 else BF16)
    d = GemmDesc(a0=_p(a), lda0=lda0, k0=k0, a1=_p(a1), lda1=lda1, a_mode=A_DENSE,
                 w=_p(w), ldw=_rows(w), M=M, N=N, K=K,
                 bias=_p(bias), rowbias=_p(rowbias),
                 ld_rb=rowbias.stride(0) if rowbias is not None else 0, rb_div=rb_div,
                 res=_p(res), ld_res=_rows(res) if res is not None else 0, act=act,
                 out=_p(out), ldc=_rows(out, torch.float32 if out_f32 else BF16),
                 out_f32=int(out_f32))
    if rmap is not None:
        d.rmap_n1, d.rmap_n2, d.rmap_inner = (int(v) for v in rmap)
    if ln_fold is not None:
        s, eps = ln_fold
        _dev(s)
        if s.dtype != torch.float32 or not s.is_contiguous() or s.numel() != N:
            raise ValueError("ln_fold s must be a contiguous fp32 vector of N entries")
        d.ln_fold_s, d.ln_fold_eps = _p(s), float(eps)
    _run_gemm(d, a.device, "vd_gemm")
    return out


def gemm_ln(a, w, gamma, beta, *, eps=1e-5, pe=None, pe_div=1, pe_period=1, bias=None, res=None, out=None,
            ln_out=None):
    """(out, ln_out): out = a @ w^T (+ bias) (+ res) in bf16 and ln_out = LayerNorm(out)
    (+ pe[(m / pe_div) % pe_period]) — the GEMM producing a transformer block's residual
    stream with the next norm fused into its epilogue where one tile owns whole rows."""
    _dev(a, w, gamma, beta, pe, bias, res, out, ln_out)
    M = a.shape[0]
    N, K = w.shape
    if a.shape[1] != K:
        raise ValueError(f"A has {a.shape[1]} columns, W has K={K}")
    if out is None:
        out = torch.empty(M, N, device=a.device, dtype=BF16)
    if ln_out is None:
        ln_out = torch.empty(M, N, device=a.device, dtype=BF16)
    d = GemmDesc(a0=_p(a), lda0=_rows(a), k0=K, a1=None, lda1=0, a_mode=A_DENSE,
                 w=_p(w), ldw=_rows(w), M=M, N=N, K=K, bias=_p(bias), rowbias=None, ld_rb=0, rb_div=1,
                 res=_p(res), ld_res=_rows(res) if res is not None else 0, act=ACT_NONE,
                 out=_p(out), ldc=_rows(out), out_f32=0,
                 ln_gamma=_p(gamma), ln_beta=_p(beta), ln_eps=eps, ln_pe=_p(pe), ln_pe_div=pe_div,
                 ln_pe_period=pe_period, ln_out=_p(ln_out), ld_ln=_rows(ln_out))
    _run_gemm(d, a.device, "vd_gemm(ln)")
    return out, ln_out


def conv3x3(x, n_img, h_in, w_in, w, *, x1=None, stride=1, upsample=False, bias=None,
            rowbias=None, rb_div=1, res=None, act=ACT_NONE, out=None, out_f32=False):
    """3x3 pad-1 conv over NHWC rows x (+ channel-concat x1); w packed [Cout][3][3][Cin]."""
    _dev(x, w, x1, bias, rowbias, res, out)
    N, K = w.shape
    c0 = x.shape[1]
    if K % 9 or (c0 + (x1.shape[1] if x1 is not None else 0)) * 9 != K:
        raise ValueError("conv weight K does not match input channels")
    if upsample:
        h_out, w_out = 2 * h_in, 2 * w_in
    else:
        h_out, w_out = (h_in - 1) // stride + 1, (w_in - 1) // stride + 1
    M = n_img * h_out * w_out
    if x.shape[0] != n_img * h_in * w_in:
        raise ValueError("conv input rows != n_img*h*w")
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=torch.float32 if out_f32 else BF16)
    d = GemmDesc(a0=_p(x), lda0=_rows(x), k0=c0, a1=_p(x1),
                 lda1=_rows(x1) if x1 is not None else 0, a_mode=A_CONV3X3,
                 n_img=n_img, h_in=h_in, w_in=w_in, h_out=h_out, w_out=w_out,
                 stride=stride, upsample=int(bool(upsample)),
                 w=_p(w), ldw=_rows(w), M=M, N=N, K=K,
                 bias=_p(bias), rowbias=_p(rowbias),
                 ld_rb=rowbias.stride(0) if rowbias is not None else 0, rb_div=rb_div,
                 res=_p(res), ld_res=_rows(res) if res is not None else 0, act=act,
                 out=_p(out), ldc=_rows(out, torch.float32 if out_f32 else BF16),
                 out_f32=int(out_f32))
    _run_gemm(d, x.device, "vd_gemm(conv3x3)")
    return out, h_out, w_out


def conv3d(x, batch, frames_in, h_in, w_in, w, *, kt=3, ks=3, frames_out=None, t_off=0, stride=1, bias=None,
           rowbias=None, rb_div=1, res=None, act=ACT_NONE, out=None, out_f32=False):
    """kt x ks x ks conv (pad kt/2, ks/2; spatial stride 1/2, temporal stride 1) over the frames
    of each video: x = NHWC rows of batch*frames_in images, w packed [Cout][kt][ks][ks][Cin]
    (K = (dt*ks*ks + tap)*Cin + ci, pack_conv3d).  Output frame f of a video reads input frames
    f + t_off + dt - kt/2 (zero outside [0, frames_in)): frames_out = frames_in, t_off = 0 is
    the plain 3-D conv; a frame-sharded rank passes halo'd frames (frames_in = frames_out + 2,
    t_off = 1).  ks = 1, kt = 3 is the temporal half of a (2+1)D conv."""
    _dev(x, w, bias, rowbias, res, out)
    frames_out = frames_in if frames_out is None else frames_out
    N, K = w.shape
    cin = x.shape[1]
    if K != kt * ks * ks * cin:
        raise ValueError(f"conv3d weight K={K} != kt*ks*ks*Cin = {kt * ks * ks * cin}")
    if x.shape[0] != batch * frames_in * h_in * w_in:
        raise ValueError("conv3d input rows != batch*frames_in*h*w")
    h_out, w_out = (h_in - 1) // stride + 1, (w_in - 1) // stride + 1
    n_img = batch * frames_out
    M = n_img * h_out * w_out
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=torch.float32 if out_f32 else BF16)
    d = GemmDesc(a0=_p(x), lda0=_rows(x), k0=cin, a1=None, lda1=0, a_mode=A_CONV3X3,
                 n_img=n_img, h_in=h_in, w_in=w_in, h_out=h_out, w_out=w_out, stride=stride, upsample=0,
                 w=_p(w), ldw=_rows(w), M=M, N=N, K=K, bias=_p(bias), rowbias=_p(rowbias),
                 ld_rb=rowbias.stride(0) if rowbias is not None else 0, rb_div=rb_div,
                 res=_p(res), ld_res=_rows(res) if res is not None else 0, act=act,
                 out=_p(out), ldc=_rows(out, torch.float32 if out_f32 else BF16), out_f32=int(out_f32),
                 kt=kt, ks=ks, frames_in=frames_in, frames_out=frames_out, t_off=t_off)
    _run_gemm(d, x.device, "vd_gemm(conv3d)")
    return out, h_out, w_out


# ---------------------------------------------------------------- norms
def gn_splits(n_inst: int, pix: int) -> int:
    """Pixel splits per instance for vd_gn_partial: ~2048 partial blocks in total, at
    most 256 per instance (the finalize pass combines n_split x C/groups records per
    group)."""
    return max(1, min(pix // 16, math.ceil(2048 / n_inst), 256))


def gn_splits_per_frame(hw: int) -> int:
    """Splits per frame of the motion-module norm (instance = a whole video): a function of the
    frame size alone, so a frame-sharded rank's records for its frames are exactly the
    unsharded run's records for those frames and the all-gathered set equals the unsharded one
    record for record — the sharded norm is bit-identical (at F = 16 this is the same 256 / 64
    splits per video as gn_splits)."""
    return max(1, min(hw // 16, 16))


def gn_partial(x, C, n_inst, pix, n_split, x1=None):
    _dev(x, x1)
    ws = torch.empty(n_inst, n_split, C, 4, device=x.device, dtype=torch.float32)
    check(lib().vd_gn_partial(_p(x), _rows(x), x.shape[1], _p(x1), _rows(x1) if x1 is not None else 0,
                              C, n_inst, pix, n_split, _p(ws), _stream()), "vd_gn_partial")
    return ws


def gn_finalize(ws, groups, eps, gamma, beta):
    n_inst, n_split, C, _ = ws.shape
    ss = torch.empty(n_inst, C, 2, device=ws.device, dtype=torch.float32)
    check(lib().vd_gn_finalize(_p(ws), n_inst, n_split, C, groups, eps, _p(gamma), _p(beta), _p(ss),
                               _stream()), "vd_gn_finalize")
    return ss


def gn_partial_g(x, C, n_inst, pix, n_split, groups, x1=None):
    """vd_gn_partial_g: one {n, mean, M2} record per (instance, split, group)."""
    _dev(x, x1)
    ws = torch.empty(n_inst, n_split, groups, 4, device=x.device, dtype=torch.float32)
    x1p, ld1 = (_p(x1), _rows(x1)) if x1 is not None else (None, 0)
    check(lib().vd_gn_partial_g(_p(x), _rows(x), x.shape[1], x1p, ld1, C, n_inst, pix, n_split, groups, _p(ws),
                                _stream()), "vd_gn_partial_g")
    return ws


def gn_finalize_g(ws, C, eps, gamma, beta):
    """ws: [inst, splits, groups, 4] records, or rank-major [ranks, inst, splits of a rank, groups, 4]
    (FrameShard.gather_gn_records: the all-gather output as it lands, vd_gn_finalize_g_ranks)."""
    if ws.dim() == 5:
        n_ranks, n_inst, nsl, groups, _ = ws.shape
        ss = torch.empty(n_inst, C, 2, device=ws.device, dtype=torch.float32)
        check(lib().vd_gn_finalize_g_ranks(_p(ws), n_inst, n_ranks, nsl, C, groups, eps, _p(gamma), _p(beta),
                                           _p(ss), _stream()), "vd_gn_finalize_g_ranks")
        return ss
    n_inst, n_split, groups, _ = ws.shape
    ss = torch.empty(n_inst, C, 2, device=ws.device, dtype=torch.float32)
    check(lib().vd_gn_finalize_g(_p(ws), n_inst, n_split, C, groups, eps, _p(gamma), _p(beta), _p(ss),
                                 _stream()), "vd_gn_finalize_g")
    return ss


def gn_apply(x, ss, pix, silu, x1=None, out=None, rev3=None):
    """rev3 = (n1, n2, inner): input row m lands at output row rev3(m) (vd_gn_apply_rev3)."""
    _dev(x, x1, ss)
    n_inst, C, _ = ss.shape
    if out is None:
        out = torch.empty(x.shape[0], C, device=x.device, dtype=BF16)
    n1, n2, inner = rev3 if rev3 is not None else (1, 1, 0)
    check(lib().vd_gn_apply_rev3(_p(x), _rows(x), x.shape[1], _p(x1), _rows(x1) if x1 is not None else 0,
                                 C, n_inst, pix, _p(ss), int(silu), _p(out), _rows(out), n1, n2, inner,
                                 _stream()), "vd_gn_apply_rev3")
    return out


def group_norm(x, n_inst, pix, groups, eps, gamma, beta, silu=False, x1=None, gather=None, two_pass=True,
               n_split=None, rev3=None):
    """GroupNorm(+SiLU) over NHWC rows; instance = `pix` consecutive rows.
    Image-instance norms (two_pass): per-group partial records, and an apply that finalizes
    them itself (two launches).  The motion-module norm (two_pass=False: its instance is a
    whole video, so it needs hundreds of splits) runs partial / [gather] / finalize / apply,
    where `gather(ws) -> ws'` merges the partial statistics across frame-sharded ranks.
    Image instances always take the two-launch path, whose splits depend on the image size
    alone: a frame-sharded rank normalises its images bit-identically to the unsharded run
    (round 3; the four-launch path was 1-2 us faster on a 2-frame rank's few deep-level
    instances, tools/gn_bench.py).  A one-launch form (blocks waiting for their image's other
    blocks on an arrival counter) was slower at every image norm of the step and is gone
    (round 4, profiles/r04_gn_one_launch_refuted.txt).  Round 5: small image instances (levels
    3-4, the mid block) take vd_gn_small instead — one workgroup per (image, whole-group chunk),
    no cross-block wait, chosen from (pix, C, groups) alone, so the sharded run still matches."""
    C = x.shape[1] + (x1.shape[1] if x1 is not None else 0)
    grec = C <= 2560 and 256 % groups == 0
    if two_pass and gather is None and rev3 is None:
        if gn_small_chunk(pix, C, groups):  # round 5: one launch at the small levels
            return gn_small(x, n_inst, pix, groups, eps, gamma, beta, silu=silu, x1=x1)
        if grec:
            return group_norm_2pass(x, n_inst, pix, groups, eps, gamma, beta, silu=silu, x1=x1)
    n_split = n_split or gn_splits(n_inst, pix)
    if grec:  # per-group records (round 5: C/groups times fewer for the gather and the finalize)
        ws = gn_partial_g(x, C, n_inst, pix, n_split, groups, x1=x1)
        if gather is not None:
            ws = gather(ws)  # [inst, ranks*splits, G, 4], or rank-major [ranks, inst, splits, G, 4]
        ss = gn_finalize_g(ws, C, eps, gamma, beta)
    else:
        ws = gn_partial(x, C, n_inst, pix, n_split, x1=x1)
        if gather is not None:
            ws = gather(ws)
            if ws.dim() == 5:  # rank-major records: vd_gn_finalize takes [inst, ranks*splits, C, 4]
                ws = ws.transpose(0, 1).reshape(n_inst, -1, C, 4).contiguous()
        ss = gn_finalize(ws, groups, eps, gamma, beta)
    return gn_apply(x, ss, pix, silu, x1=x1, rev3=rev3)


GNS_NT, GNS_MAXR, GNS_GMAX = 256, 16, 32


def gn_small_chunk(pix: int, C: int, groups: int) -> int:
    """The channel chunk vd_gn_small takes for this image norm (0 = not taken): the widest whole-group
    chunk dividing C whose rows fit 16 pieces of 8 channels per thread, C / groups a multiple of 8
    (csrc/norm.hip gn_small_chunk; tests/test_ln_fold.py checks the mirror against the library)."""
    if groups <= 0 or C <= 0 or C % groups or pix <= 0 or pix > GNS_NT * GNS_MAXR:
        return 0
    cpg = C // groups
    if cpg % 8:
        return 0
    for cg in range((C // cpg) * cpg, cpg - 1, -cpg):
        if C % cg or cg // 8 > GNS_NT or cg // cpg > GNS_GMAX:
            continue
        rpt = GNS_NT // (cg // 8)
        if -(-pix // rpt) <= GNS_MAXR:
            return cg
    return 0


def gn_small(x, n_inst, pix, groups, eps, gamma, beta, silu=False, x1=None, out=None):
    """vd_gn_small: the one-launch GroupNorm of a small image instance."""
    _dev(x, x1, gamma, beta, out)
    C = x.shape[1] + (x1.shape[1] if x1 is not None else 0)
    if out is None:
        out = torch.empty(x.shape[0], C, device=x.device, dtype=BF16)
    x1p, ld1 = (_p(x1), _rows(x1)) if x1 is not None else (None, 0)
    check(lib().vd_gn_small(_p(x), _rows(x), x.shape[1], x1p, ld1, C, n_inst, pix, groups, eps, _p(gamma), _p(beta),
                            int(silu), _p(out), _rows(out), _stream()), "vd_gn_small")
    return out


def gn_image_splits(pix: int) -> int:
    """Partial records per image instance of vd_gn_partial_g: a function of the image size alone
    (frame-sharded ranks then match the unsharded run bit for bit), at most 32 (the apply prologue
    merges splits x groups records)."""
    return max(1, min(pix // 16, 32))


def gn_apply_blocks(n_inst: int, pix: int, C: int) -> int:
    """Apply blocks per instance of vd_gn_apply_g: ~1024 in all.  Each block re-merges the
    instance's records in its prologue, so a block's rows set how far that prologue is amortised;
    the choice changes no bit (the apply is elementwise on the same {a, b})."""
    return max(1, min(pix, math.ceil(1024 / n_inst)))


def group_norm_2pass(x, n_inst, pix, groups, eps, gamma, beta, silu=False, x1=None, out=None, n_split=None):
    """vd_gn_partial_g + vd_gn_apply_g.  Splits: <= 32 per instance (the apply prologue reads
    splits x groups records); the split count is a function of the image size alone (the same
    records whatever the instance count: frame-sharded ranks match the unsharded run bit for bit);
    ~1024 apply blocks in all (tools/gn_bench.py).  n_split: override (the motion norm's splits
    per frame x frames)."""
    _dev(x, x1, gamma, beta, out)
    C = x.shape[1] + (x1.shape[1] if x1 is not None else 0)
    n_split = n_split or gn_image_splits(pix)
    ws = gn_partial_g(x, C, n_inst, pix, n_split, groups, x1=x1)
    x1p, ld1 = (_p(x1), _rows(x1)) if x1 is not None else (None, 0)
    if out is None:
        out = torch.empty(x.shape[0], C, device=x.device, dtype=BF16)
    rows_per_blk = math.ceil(pix / gn_apply_blocks(n_inst, pix, C))
    check(lib().vd_gn_apply_g(_p(x), _rows(x), x.shape[1], x1p, ld1, C, n_inst, pix, _p(ws), n_split, groups, eps,
                              _p(gamma), _p(beta), int(silu), _p(out), _rows(out), rows_per_blk, _stream()),
          "vd_gn_apply_g")
    return out


def layer_norm(x, gamma, beta, eps=1e-5, pe=None, pe_div=1, pe_period=1, out=None):
    _dev(x, gamma, beta, pe)
    rows, Cc = x.shape
    if out is None:
        out = torch.empty(rows, Cc, device=x.device, dtype=BF16)
    check(lib().vd_layernorm(_p(x), _rows(x), rows, Cc, _p(gamma), _p(beta), eps, _p(pe), pe_div,
                             pe_period, _p(out), _rows(out), _stream()), "vd_layernorm")
    return out


# ---------------------------------------------------------------- attention
ATTN_KERNELS = {"auto": 0, "v1": 1, "flash32": 2, "flash40": 3}
ATTN_TAP = None  # bench hook: callable(q, k, v, batch, heads, sq, skv, d, scale) seen by every attention call


def attention(q, k, v, batch, heads, sq, skv, d, kv_div=1, scale=None, out=None, out_f32=False, kernel="auto"):
    """q/k/v: 2-D row views (may be column slices of a fused QKV buffer).  out_f32: O in fp32
    (the tests' north-star-tolerance mode).  kernel: "auto" (the product choice) or, for the
    parity tests, "v1" / "flash32" / "flash40" (vd_attention_ex)."""
    _dev(q, k, v, out)
    if out is None:
        out = torch.empty(batch * sq, heads * d, device=q.device, dtype=torch.float32 if out_f32 else BF16)
    scale = d ** -0.5 if scale is None else scale
    if ATTN_TAP is not None:
        ATTN_TAP(q, k, v, batch, heads, sq, skv, d, scale)
    check(lib().vd_attention_ex(_p(q), q.stride(0), _p(k), k.stride(0), _p(v), v.stride(0), _p(out), out.stride(0),
                                batch, heads, sq, skv, d, kv_div, scale, int(out_f32), ATTN_KERNELS[kernel],
                                _stream()), "vd_attention_ex")
    return out


def temporal_attention(q, k, v, batch, frames, positions, heads, d, scale=None, out=None, rope_theta=None,
                       valu=False):
    """rope_theta: apply the temporal 1-D RoPE (rope_qk mode 1) to q/k inside the kernel
    (vd_temporal_attention_rope: d = 64, 17..32 frames); q and k are read un-rotated.
    valu: the VALU kernel for every shape (vd_temporal_attention_valu; parity tests)."""
    _dev(q, k, v, out)
    if not (q.stride(0) == k.stride(0) == v.stride(0)):
        raise ValueError("q/k/v must share a row stride")
    if out is None:
        out = torch.empty(q.shape[0], heads * d, device=q.device, dtype=BF16)
    scale = d ** -0.5 if scale is None else scale
    if rope_theta is not None:
        if not valu:
            check(lib().vd_temporal_attention_rope(_p(q), _p(k), _p(v), q.stride(0), _p(out), out.stride(0), batch,
                                                   frames, positions, heads, d, scale, rope_theta, _stream()),
                  "vd_temporal_attention_rope")
            return out
        # the VALU kernel has no fused RoPE: rotate a COPY of q|k (the caller's buffer stays
        # un-rotated, as the fused kernel leaves it), then attend on the copy
        C = heads * d
        qkv = torch.empty(q.shape[0], 3 * C, device=q.device, dtype=BF16)
        qkv[:, :C].copy_(q[:, :C])
        qkv[:, C:2 * C].copy_(k[:, :C])
        qkv[:, 2 * C:].copy_(v[:, :C])
        rope_qk(qkv, 2 * C, d, 1, frames, 1, positions, rope_theta)
        q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
    fn = lib().vd_temporal_attention_valu if valu else lib().vd_temporal_attention
    check(fn(_p(q), _p(k), _p(v), q.stride(0), _p(out), out.stride(0), batch, frames, positions, heads, d, scale,
             _stream()), "vd_temporal_attention")
    return out


def motion_qkv_takes(batch, frames, positions, heads, d):
    """Whether vd_motion_qkv_attention takes this shape (vd_motion_qkv_attention_takes; no launch).
    Under gemm_plan(plan_div=N) the question is asked for one of N frame shards (batch 1, the
    positions divided by N), so an unsharded replay folds the motion norms exactly where a shard would."""
    positions *= _PLAN.plan_mul
    if _PLAN.plan_div > 1 and (batch * positions) % _PLAN.plan_div == 0:
        batch, positions = 1, batch * positions // _PLAN.plan_div
    return bool(lib().vd_motion_qkv_attention_takes(batch, frames, positions, heads, d))


def motion_qkv_attention(x, wqkv, batch, frames, positions, heads, d, scale=None, out=None, ln_fold=None):
    """Temporal attention over frames with the fused Q/K/V projection folded in
    (vd_motion_qkv_attention): x = normed rows (b, f, p), wqkv = [3C][C].  Returns None where
    the fused kernel does not take the shape (the caller runs gemm + temporal_attention).
    ln_fold = (table, eps): x holds the UN-normalised rows and the block's LayerNorm + PE are
    folded in (wqkv = W∘gamma; vdiff.models.blocks.MotionLnFold builds the table)."""
    _dev(x, wqkv, out)
    C = heads * d
    if out is None:
        out = torch.empty(x.shape[0], C, device=x.device, dtype=BF16)
    scale = d ** -0.5 if scale is None else scale
    tab, eps = (None, 0.0) if ln_fold is None else ln_fold
    if tab is not None:
        _dev(tab)
        if tab.dtype != torch.float32 or not tab.is_contiguous() or tab.numel() != 8 * 2048:
            raise ValueError("ln_fold table must be a contiguous fp32 [8][2048]")
    rc = lib().vd_motion_qkv_attention(_p(x), _rows(x), _p(wqkv), _rows(wqkv), _p(out), _rows(out), batch, frames,
                                       positions, heads, d, scale, _p(tab), float(eps), _stream())
    if rc == VD_EUNSUPPORTED:
        return None
    check(rc, "vd_motion_qkv_attention")
    return out


def temporal_attention_kv(q, k, v, batch, qframes, kframes, positions, heads, d, scale=None, out=None):
    """A rank's own `qframes` query frames (rows (b, qframes, p) of q) against `kframes` key
    frames (rows (b, kframes, p) of k/v, e.g. all-gathered from every frame shard)."""
    _dev(q, k, v, out)
    if k.stride(0) != v.stride(0):
        raise ValueError("k/v must share a row stride")
    if out is None:
        out = torch.empty(q.shape[0], heads * d, device=q.device, dtype=BF16)
    scale = d ** -0.5 if scale is None else scale
    check(lib().vd_temporal_attention_kv(_p(q), q.stride(0), _p(k), _p(v), k.stride(0), _p(out), out.stride(0),
                                         batch, qframes, kframes, positions, heads, d, scale, _stream()),
          "vd_temporal_attention_kv")
    return out


def softmax_rows(s, out=None):
    """fp32 scores [rows, cols] in log2 units -> bf16 probabilities (row softmax)."""
    _dev(s, out)
    rows, cols = s.shape
    if out is None:
        out = torch.empty(rows, cols, device=s.device, dtype=BF16)
    check(lib().vd_softmax_rows(_p(s), s.stride(0), rows, cols, _p(out), out.stride(0), _stream()),
          "vd_softmax_rows")
    return out


# ---------------------------------------------------------------- step glue
def timestep_embed(ts, dim, step_idx=None, batch=None, out=None):
    _dev(ts, step_idx)
    B = ts.numel() if step_idx is None else batch
    if out is None:
        out = torch.empty(B, dim, device=ts.device, dtype=BF16)
    check(lib().vd_timestep_embed(_p(ts), ts.numel(), _p(step_idx), B, dim, _p(out), _stream()), "vd_timestep_embed")
    return out


def pack_latents(x, dup=1, cpad=8, out=None, in_div=1.0):
    _dev(x, out)
    x = x.contiguous().float()
    B, Cc, Fr, H, W = x.shape
    if out is None:
        out = torch.empty(dup * B * Fr * H * W, cpad, device=x.device, dtype=BF16)
    check(lib().vd_pack_latents(_p(x), B, Cc, Fr, H, W, dup, _p(out), cpad, float(in_div), _stream()), "vd_pack_latents")
    return out


def unpack_nhwc(src, B, Cc, Fr, H, W, out=None):
    _dev(src, out)
    if out is None:
        out = torch.empty(B, Cc, Fr, H, W, device=src.device, dtype=torch.float32)
    check(lib().vd_unpack_nhwc(_p(src), int(src.dtype == torch.float32), src.stride(0), B, Cc, Fr, H, W,
                               _p(out), _stream()), "vd_unpack_nhwc")
    return out


def ddim_cfg_step(eps, ncfg, guidance, latents, coef, step_idx=None, x0_out=None, next_in=None):
    _dev(eps, latents, coef, step_idx, x0_out, next_in)
    if latents.dtype != torch.float32 or not latents.is_contiguous():
        raise ValueError("latents must be contiguous fp32")
    B, Cc, Fr, H, W = latents.shape
    check(lib().vd_ddim_cfg_step(_p(eps), eps.stride(0), ncfg, guidance, _p(latents), B, Cc, Fr, H, W,
                                 _p(coef), coef.numel() // 4, _p(step_idx), _p(x0_out), _p(next_in),
                                 next_in.shape[1] if next_in is not None else 0, _stream()),
          "vd_ddim_cfg_step")


def euler_cfg_step(eps, ncfg, guidance, latents, coef, step_idx=None, x0_out=None, next_in=None):
    """CFG combine + EulerDiscreteScheduler.step (+ next input's scale_model_input), fused."""
    _dev(eps, latents, coef, step_idx, x0_out, next_in)
    if latents.dtype != torch.float32 or not latents.is_contiguous():
        raise ValueError("latents must be contiguous fp32")
    B, Cc, Fr, H, W = latents.shape
    check(lib().vd_euler_cfg_step(_p(eps), eps.stride(0), ncfg, guidance, _p(latents), B, Cc, Fr, H, W,
                                  _p(coef), coef.numel() // 4, _p(step_idx), _p(x0_out), _p(next_in),
                                  next_in.shape[1] if next_in is not None else 0, _stream()),
          "vd_euler_cfg_step")


SCHED_STEP = {"ddim": ddim_cfg_step, "euler": euler_cfg_step}


def step_advance(step_idx):
    _dev(step_idx)
    check(lib().vd_step_advance(_p(step_idx), _stream()), "vd_step_advance")


def block_transpose(src, nb, na, nc, out=None):
    """dst[(a*nb + b)*nc + c] = src[(b*na + a)*nc + c] over bf16 rows."""
    _dev(src, out)
    width = src.shape[1]
    if out is None:
        out = torch.empty_like(src)
    check(lib().vd_block_transpose(_p(src), _p(out), nb, na, nc, width, _stream()), "vd_block_transpose")
    return out


# ---------------------------------------------------------------- module-level path (rows.hip)
def rows_add(x, y, y_div=1, y_period=None, out=None):
    """out[r] = (x[r] if x is not None else 0) + y[(r // y_div) % y_period]: bf16 rows x, y bf16 or
    fp32 rows.  `out` may be a column slice of a wider buffer (channel concat)."""
    _dev(x, y, out)
    rows = out.shape[0] if out is not None else x.shape[0]
    C = y.shape[1] if x is None else x.shape[1]
    if out is None:
        out = torch.empty(rows, C, device=y.device, dtype=BF16)
    y_f32 = y.dtype == torch.float32
    period = y.shape[0] if y_period is None else y_period
    check(lib().vd_rows_eltwise(0, _p(x), _rows(x) if x is not None else 0, _p(y), _rows(y, y.dtype), int(y_f32),
                                y_div, period, rows, C, _p(out), _rows(out), _stream()), "vd_rows_eltwise(add)")
    return out


def silu_rows(x, out=None):
    _dev(x, out)
    if out is None:
        out = torch.empty_like(x)
    check(lib().vd_rows_eltwise(1, _p(x), _rows(x), None, 0, 0, 1, 1, x.shape[0], x.shape[1], _p(out),
                                _rows(out), _stream()), "vd_rows_eltwise(silu)")
    return out


def upsample2x_rows(x, n_img, h, w, out=None):
    _dev(x, out)
    if out is None:
        out = torch.empty(n_img * 4 * h * w, x.shape[1], device=x.device, dtype=BF16)
    check(lib().vd_upsample_nearest2x(_p(x), _rows(x), n_img, h, w, x.shape[1], _p(out), _rows(out), _stream()),
          "vd_upsample_nearest2x")
    return out


# ---------------------------------------------------------------- DiT (§8f rank 3)
def patchify(lat, p, kpad, dup=1, in_div=1.0, out=None):
    """latents fp32 (B,C,F,H,W) -> bf16 token rows [(b,f,hp,wp)][kpad] (x dup for CFG)."""
    _dev(lat, out)
    if lat.dtype != torch.float32 or not lat.is_contiguous():
        raise ValueError("patchify expects contiguous fp32 latents")
    B, Cc, F, H, W = lat.shape
    rows = B * F * (H // p) * (W // p)
    if out is None:
        out = torch.empty(dup * rows, kpad, device=lat.device, dtype=BF16)
    check(lib().vd_patchify(_p(lat), B, Cc, F, H, W, p, dup, in_div, _p(out), kpad, _stream()), "vd_patchify")
    return out


def unpatchify(src, n_img, H, W, p, Cc, out=None):
    """fp32 token rows [(n,hp,wp)][(ph,pw,c)] -> fp32 NHWC pixel rows [(n,h,w)][c]."""
    _dev(src, out)
    if src.dtype != torch.float32:
        raise ValueError("unpatchify expects fp32 rows")
    if out is None:
        out = torch.empty(n_img * H * W, Cc, device=src.device, dtype=torch.float32)
    check(lib().vd_unpatchify(_p(src), _rows(src, torch.float32), n_img, H, W, p, Cc, _p(out), _stream()),
          "vd_unpatchify")
    return out


def rope_qk(x, ncols, d, mode, F, Hp, Wp, theta=10000.0):
    """In-place rotary embedding on columns [0, ncols) of bf16 token rows x."""
    _dev(x)
    check(lib().vd_rope_qk(_p(x), _rows(x), x.shape[0], ncols, d, mode, F, Hp, Wp, theta, _stream()),
          "vd_rope_qk")
    return x


def res_ln_mod(x, *, y=None, gate=None, shift=None, scale=None, rows_per_b=None, x_out=None,
               eps=1e-6, out=None):
    """h = LN(x + gate*y) * (1 + scale) + shift per row group b = row // rows_per_b;
    x_out (may be x) receives x + gate*y.  gate/shift/scale: fp32 [B, >= C] row views."""
    _dev(x, y, gate, shift, scale, x_out, out)
    rows, Cc = x.shape
    mods = [t for t in (gate, shift, scale) if t is not None]
    ld_mod = mods[0].stride(0) if mods else 0
    for t in mods:
        if t.dtype != torch.float32 or t.stride(1) != 1 or t.stride(0) != ld_mod:
            raise ValueError("gate/shift/scale must be fp32 row views sharing one row stride")
    if out is None:
        out = torch.empty(rows, Cc, device=x.device, dtype=BF16)
    check(lib().vd_res_ln_mod(_p(x), _rows(x), _p(y), _rows(y) if y is not None else 0, _p(gate), _p(shift),
                              _p(scale), ld_mod, rows_per_b or rows, _p(x_out),
                              _rows(x_out) if x_out is not None else 0, _p(out), _rows(out), rows, Cc, eps,
                              _stream()), "vd_res_ln_mod")
    return out


def attention_fp8_quant(q, k, v, batch, heads, sq, skv, d=64, rope=None, q_scale=1.0):
    """bf16 q/k/v row views -> the fp8 operands of vd_attention_fp8 (a dict of buffers).
    rope=(Hp, Wp, theta): apply the spatial 2-D RoPE (rope_qk mode 0) to q and k inside the
    quantization pass (vd_attention_fp8_quant_rope); q and k are read un-rotated.
    q_scale: q is multiplied by it before quantization (attention_fp8 folds the softmax scale x
    log2 e there); ws["q_scale"] records it."""
    _dev(q, k, v)
    dev = q.device
    ld8 = (heads * d + 15) // 16 * 16
    u8 = torch.uint8
    ws = {"q8": torch.empty(batch * sq, ld8, device=dev, dtype=u8),
          "k8": torch.empty(batch * skv, ld8, device=dev, dtype=u8),
          "vt8": torch.empty(batch * heads * d, skv, device=dev, dtype=u8),
          "qs": torch.empty(batch * sq, heads, device=dev, dtype=u8),
          "ks": torch.empty(batch * skv, heads, device=dev, dtype=u8),
          "vs": torch.empty(batch * heads, max(1, skv // 64), device=dev, dtype=u8),
          "ld8": ld8, "batch": batch, "heads": heads, "sq": sq, "skv": skv, "d": d, "q_scale": float(q_scale)}
    if rope is not None:
        if sq != skv:
            raise ValueError("fused RoPE quantization needs sq == skv (self-attention)")
        Hp, Wp, theta = rope
        check(lib().vd_attention_fp8_quant_rope(
            _p(q), q.stride(0), _p(k), k.stride(0), _p(v), v.stride(0), batch, heads, sq, d, Hp, Wp, theta,
            _p(ws["q8"]), _p(ws["k8"]), ld8, _p(ws["vt8"]), _p(ws["qs"]), _p(ws["ks"]), _p(ws["vs"]), float(q_scale),
            _stream()), "vd_attention_fp8_quant_rope")
        return ws
    check(lib().vd_attention_fp8_quant(_p(q), q.stride(0), _p(k), k.stride(0), _p(v), v.stride(0), batch, heads,
                                       sq, skv, d, _p(ws["q8"]), _p(ws["k8"]), ld8, _p(ws["vt8"]), _p(ws["qs"]),
                                       _p(ws["ks"]), _p(ws["vs"]), float(q_scale), _stream()), "vd_attention_fp8_quant")
    return ws


LOG2E = 1.4426950408889634


def attention_fp8_run(ws, out, scale=None):
    """vd_attention_fp8 on operands from attention_fp8_quant.  `scale` multiplies the scores of
    the dequantized q8 (default d^-1/2 / ws["q_scale"]: the softmax scale q_scale did not fold;
    1 / log2 e after attention_fp8's full fold selects the kernel's folded form)."""
    d = ws["d"]
    if scale is None:
        scale = d ** -0.5 / ws["q_scale"]
    check(lib().vd_attention_fp8(_p(ws["q8"]), _p(ws["k8"]), ws["ld8"], _p(ws["qs"]), _p(ws["ks"]), _p(ws["vt8"]),
                                 _p(ws["vs"]), _p(out), out.stride(0), ws["batch"], ws["heads"], ws["sq"], ws["skv"],
                                 d, scale, _stream()), "vd_attention_fp8")
    return out


def attention_fp8(q, k, v, batch, heads, sq, skv, d=64, scale=None, out=None, rope=None):
    """fp8 (e4m3, block-scaled MFMA) self-attention, d = 64: quantize (optionally with the
    spatial RoPE fused, see attention_fp8_quant) with the softmax scale x log2 e folded into q,
    then attend (the kernel's folded form: no per-score multiply)."""
    scale = d ** -0.5 if scale is None else scale
    ws = attention_fp8_quant(q, k, v, batch, heads, sq, skv, d, rope=rope, q_scale=scale * LOG2E)
    if out is None:
        out = torch.empty(batch * sq, heads * d, device=q.device, dtype=BF16)
    _dev(out)
    return attention_fp8_run(ws, out, scale=1.0 / LOG2E)
