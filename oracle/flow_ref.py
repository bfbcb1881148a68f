"""ORACLE — test infrastructure only.  Never imported by the product path.

Restatement of the optical-flow and warp-error metrics of
experiments/06_measure_grid_search.py:

* OpticalFlowEstimator.compute_flow (06:157-188): grey = uint8(mean_c(frame) * 255), then
  cv2.calcOpticalFlowFarneback(grey1, grey2, None, pyr_scale=0.5, levels=3, winsize=15,
  iterations=3, poly_n=5, poly_sigma=1.2, flags=0);
* compute_flow_stats (06:190-199): magnitude mean / std / max / median;
* warp_frame (06:259-284): backward warp of frame1 by the flow, grid_sample bilinear, border
  padding, align_corners=True; warp_error = compute_mse(warped, frame2) (06:333-335).

OpenCV is not installed here and the reference does not vendor it: the third-party
algorithm is OpenCV's Farneback (opencv >= 4 `modules/video/src/optflowgf.cpp`,
`calcOpticalFlowFarneback` with its helpers FarnebackPolyExp / FarnebackPrepareGaussian /
FarnebackUpdateMatrices / FarnebackUpdateFlow_Blur, plus GaussianBlur / getGaussianKernel and
resize(INTER_LINEAR)), restated below step by step in numpy with OpenCV's border rules,
coefficient tables and float32/float64 split.  PARITY is pinned by the reference's own
records — `outputs/06_grid_search_metrics/*_metrics.json` hold per-pair
flow_magnitude_mean / flow_magnitude_std / warp_error computed by the reference from the
frames in `outputs/05_grid_search/*/frames`; tests/golden/make_metrics_golden.py runs this
restatement over all 78 measured videos and records the largest relative deviation per field
in tests/golden/metrics/oracle_vs_reference.json (~1e-6: OpenCV's SIMD summation order is not
reproduced bit for bit), and tests/test_flow_oracle.py re-checks the committed video.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

F32 = np.float32


# ---------------------------------------------------------------- OpenCV primitives
def cv_round(x: float) -> int:
    """cvRound: round half to even (the SSE2 cvtsd2si path)."""
    return int(np.rint(x))


_SMALL_GAUSS = {1: [1.0], 3: [0.25, 0.5, 0.25], 5: [0.0625, 0.25, 0.375, 0.25, 0.0625],
                7: [0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125]}


def gaussian_kernel(n: int, sigma: float) -> np.ndarray:
    """getGaussianKernel(n, sigma, CV_32F)."""
    fixed = _SMALL_GAUSS.get(n) if sigma <= 0 else None
    sx = sigma if sigma > 0 else ((n - 1) * 0.5 - 1) * 0.3 + 0.8
    scale2 = -0.5 / (sx * sx)
    cf = np.empty(n, F32)
    s = 0.0
    for i in range(n):
        x = i - (n - 1) * 0.5
        t = fixed[i] if fixed is not None else math.exp(scale2 * x * x)
        cf[i] = F32(t)
        s += float(cf[i])
    s = 1.0 / s
    return np.array([F32(float(c) * s) for c in cf], F32)


def _reflect101(idx, n):
    idx = np.abs(idx)
    return np.where(idx >= n, 2 * (n - 1) - idx, idx)


def gaussian_blur(img: np.ndarray, ksize: int, sigma: float) -> np.ndarray:
    """GaussianBlur(img, (ksize, ksize), sigma, sigma) on float32, BORDER_REFLECT_101,
    separable: rows then columns, float32 sums."""
    k = gaussian_kernel(ksize, sigma)
    r = ksize // 2
    h, w = img.shape
    cols = _reflect101(np.arange(-r, w + r), w)
    src = img[:, cols]
    tmp = np.zeros((h, w), F32)
    for i in range(ksize):
        tmp = tmp + k[i] * src[:, i:i + w]
    rows = _reflect101(np.arange(-r, h + r), h)
    src = tmp[rows]
    out = np.zeros((h, w), F32)
    for i in range(ksize):
        out = out + k[i] * src[i:i + h]
    return out


def _linear_coeffs(dsize, ssize):
    scale = ssize / dsize
    fx = ((np.arange(dsize) + 0.5) * scale - 0.5).astype(F32)
    sx = np.floor(fx).astype(np.int64)
    fx = (fx - sx).astype(F32)
    lo = sx < 0
    fx[lo], sx[lo] = 0, 0
    hi = sx >= ssize - 1
    fx[hi], sx[hi] = 0, ssize - 1
    sx1 = np.minimum(sx + 1, ssize - 1)
    return sx, sx1, (F32(1) - fx).astype(F32), fx


def resize_linear(img: np.ndarray, h: int, w: int) -> np.ndarray:
    """resize(img, (w, h), INTER_LINEAR) for float images (any trailing channels)."""
    sh, sw = img.shape[:2]
    x0, x1, ax0, ax1 = _linear_coeffs(w, sw)
    y0, y1, ay0, ay1 = _linear_coeffs(h, sh)
    ex = (slice(None),) + (None,) * (img.ndim - 2)
    row = img[:, x0] * ax0[ex] + img[:, x1] * ax1[ex]                       # horizontal pass
    ey = (slice(None), None) + (None,) * (img.ndim - 2)
    return (row[y0] * ay0[ey] + row[y1] * ay1[ey]).astype(F32)              # vertical pass


# ---------------------------------------------------------------- Farneback
def prepare_gaussian(n: int, sigma: float):
    """FarnebackPrepareGaussian -> g, xg, xxg (float32, index -n..n) and ig11, ig03, ig33, ig55."""
    if sigma < np.finfo(np.float32).eps:
        sigma = n * 0.3
    xs = np.arange(-n, n + 1)
    g = np.array([F32(math.exp(-x * x / (2 * sigma * sigma))) for x in xs], F32)
    s = 1.0 / float(np.sum(g.astype(np.float64)))
    g = np.array([F32(float(v) * s) for v in g], F32)
    xg = (xs * g).astype(F32)
    xxg = (xs * xs * g).astype(F32)
    G = np.zeros((6, 6))
    gd = g.astype(np.float64)
    for yi, y in enumerate(xs):
        for xi, x in enumerate(xs):
            w = gd[yi] * gd[xi]
            G[0, 0] += w
            G[1, 1] += w * x * x
            G[3, 3] += w * x ** 4
            G[5, 5] += w * x * x * y * y
    G[2, 2] = G[0, 3] = G[0, 4] = G[3, 0] = G[4, 0] = G[1, 1]
    G[4, 4] = G[3, 3]
    G[3, 4] = G[4, 3] = G[5, 5]
    iG = np.linalg.inv(G)
    return g, xg, xxg, iG[1, 1], iG[0, 3], iG[3, 3], iG[5, 5]


def poly_exp(src: np.ndarray, n: int = 5, sigma: float = 1.2) -> np.ndarray:
    """FarnebackPolyExp: float32 [h, w] -> float32 [h, w, 5] (the channel order OpenCV stores:
    0 = y-linear, 1 = x-linear, 2 = yy, 3 = xx, 4 = xy coefficients)."""
    g, xg, xxg, ig11, ig03, ig33, ig55 = prepare_gaussian(n, sigma)
    h, w = src.shape
    c = n  # index of offset 0
    # vertical part (float32, rows clamped)
    r0 = src * g[c]
    r1 = np.zeros_like(src)
    r2 = np.zeros_like(src)
    for k in range(1, n + 1):
        s0 = src[np.maximum(np.arange(h) - k, 0)]
        s1 = src[np.minimum(np.arange(h) + k, h - 1)]
        p = (s0 + s1).astype(F32)
        r0 = (r0 + g[c + k] * p).astype(F32)
        r1 = (r1 + xg[c + k] * (s1 - s0)).astype(F32)
        r2 = (r2 + xxg[c + k] * p).astype(F32)
    # horizontal part (float64 accumulators, columns replicated)
    cols = np.clip(np.arange(-n, w + n), 0, w - 1)
    R0, R1, R2 = (r.astype(np.float64)[:, cols] for r in (r0, r1, r2))
    b1 = R0[:, n:n + w] * float(g[c])
    b3 = R1[:, n:n + w] * float(g[c])
    b5 = R2[:, n:n + w] * float(g[c])
    b2 = np.zeros((h, w))
    b4 = np.zeros((h, w))
    b6 = np.zeros((h, w))
    for k in range(1, n + 1):
        pk, mk = slice(n + k, n + k + w), slice(n - k, n - k + w)
        tg = R0[:, pk] + R0[:, mk]
        b1 += tg * float(g[c + k])
        b4 += tg * float(xxg[c + k])
        b2 += (R0[:, pk] - R0[:, mk]) * float(xg[c + k])
        b3 += (R1[:, pk] + R1[:, mk]) * float(g[c + k])
        b6 += (R1[:, pk] - R1[:, mk]) * float(xg[c + k])
        b5 += (R2[:, pk] + R2[:, mk]) * float(g[c + k])
    out = np.empty((h, w, 5), F32)
    out[..., 1] = b2 * ig11
    out[..., 0] = b3 * ig11
    out[..., 3] = b1 * ig03 + b4 * ig33
    out[..., 2] = b1 * ig03 + b5 * ig33
    out[..., 4] = b6 * ig55
    return out


_BORDER = np.array([0.14, 0.14, 0.4472, 0.4472, 0.4472], F32)


def update_matrices(R0, R1, flow):
    """FarnebackUpdateMatrices over the whole image -> M float32 [h, w, 5]."""
    h, w = flow.shape[:2]
    dx, dy = flow[..., 0], flow[..., 1]
    xs = np.arange(w, dtype=F32)[None, :]
    ys = np.arange(h, dtype=F32)[:, None]
    fx = (xs + dx).astype(F32)
    fy = (ys + dy).astype(F32)
    x1 = np.floor(fx).astype(np.int64)
    y1 = np.floor(fy).astype(np.int64)
    fx = (fx - x1).astype(F32)
    fy = (fy - y1).astype(F32)
    inside = (x1 >= 0) & (x1 < w - 1) & (y1 >= 0) & (y1 < h - 1)
    xc, yc = np.clip(x1, 0, w - 2), np.clip(y1, 0, h - 2)
    a00 = ((1 - fx) * (1 - fy)).astype(F32)
    a01 = (fx * (1 - fy)).astype(F32)
    a10 = ((1 - fx) * fy).astype(F32)
    a11 = (fx * fy).astype(F32)
    r = (a00[..., None] * R1[yc, xc] + a01[..., None] * R1[yc, xc + 1] + a10[..., None] * R1[yc + 1, xc]
         + a11[..., None] * R1[yc + 1, xc + 1]).astype(F32)
    r2, r3, r4, r5, r6 = (r[..., i] for i in range(5))
    r4 = np.where(inside, (R0[..., 2] + r4) * F32(0.5), R0[..., 2]).astype(F32)
    r5 = np.where(inside, (R0[..., 3] + r5) * F32(0.5), R0[..., 3]).astype(F32)
    r6 = np.where(inside, (R0[..., 4] + r6) * F32(0.25), R0[..., 4] * F32(0.5)).astype(F32)
    r2 = np.where(inside, r2, F32(0))
    r3 = np.where(inside, r3, F32(0))
    r2 = ((R0[..., 0] - r2) * F32(0.5)).astype(F32)
    r3 = ((R0[..., 1] - r3) * F32(0.5)).astype(F32)
    r2 = (r2 + r4 * dy + r6 * dx).astype(F32)
    r3 = (r3 + r6 * dy + r5 * dx).astype(F32)
    bx = np.ones(w, F32)
    by = np.ones(h, F32)
    bx[:5] *= _BORDER
    bx[w - 5:] *= _BORDER[::-1]
    by[:5] *= _BORDER
    by[h - 5:] *= _BORDER[::-1]
    sc = (by[:, None] * bx[None, :]).astype(F32)
    r2, r3, r4, r5, r6 = (v * sc for v in (r2, r3, r4, r5, r6))
    M = np.empty((h, w, 5), F32)
    M[..., 0] = r4 * r4 + r6 * r6
    M[..., 1] = (r4 + r5) * r6
    M[..., 2] = r5 * r5 + r6 * r6
    M[..., 3] = r4 * r2 + r6 * r3
    M[..., 4] = r6 * r2 + r5 * r3
    return M


def box_blur_replicate(M: np.ndarray, k: int) -> np.ndarray:
    """Sum over a k x k box (replicate borders) in float64, as FarnebackUpdateFlow_Blur's
    running vertical / horizontal sums."""
    m = k // 2
    h, w = M.shape[:2]
    P = np.pad(M.astype(np.float64), ((m, m), (m, m), (0, 0)), mode="edge")
    c = np.cumsum(P, axis=0)
    c = np.concatenate([np.zeros((1,) + c.shape[1:]), c], 0)
    v = c[k:k + h] - c[:h]
    c = np.cumsum(v, axis=1)
    c = np.concatenate([np.zeros((h, 1, c.shape[2])), c], 1)
    return c[:, k:k + w] - c[:, :w]


def update_flow_blur(M: np.ndarray, k: int) -> np.ndarray:
    s = box_blur_replicate(M, k) * (1.0 / (k * k))
    g11, g12, g22, h1, h2 = (s[..., i] for i in range(5))
    idet = 1.0 / (g11 * g22 - g12 * g12 + 1e-3)
    return np.stack([(g11 * h2 - g12 * h1) * idet, (g22 * h1 - g12 * h2) * idet], -1).astype(F32)


def farneback(prev: np.ndarray, nxt: np.ndarray, pyr_scale=0.5, levels=3, winsize=15, iterations=3,
              poly_n=5, poly_sigma=1.2) -> np.ndarray:
    """cv2.calcOpticalFlowFarneback(prev, next, None, ...) with flags = 0 -> flow [H, W, 2] float32."""
    H, W = prev.shape
    min_size = 32
    scale = 1.0
    k = 0
    while k < levels:
        scale *= pyr_scale
        if W * scale < min_size or H * scale < min_size:
            break
        k += 1
    levels = k
    prev_flow = None
    for k in range(levels, -1, -1):
        scale = 1.0
        for _ in range(k):
            scale *= pyr_scale
        sigma = (1.0 / scale - 1) * 0.5
        smooth = max(cv_round(sigma * 5) | 1, 3)
        w, h = cv_round(W * scale), cv_round(H * scale)
        if prev_flow is None:
            flow = np.zeros((h, w, 2), F32)
        else:
            flow = (resize_linear(prev_flow, h, w) * F32(1.0 / pyr_scale)).astype(F32)
        R = [poly_exp(resize_linear(gaussian_blur(im.astype(F32), smooth, sigma), h, w), poly_n, poly_sigma)
             for im in (prev, nxt)]
        M = update_matrices(R[0], R[1], flow)
        for it in range(iterations):
            flow = update_flow_blur(M, winsize)
            if it < iterations - 1:
                M = update_matrices(R[0], R[1], flow)
        prev_flow = flow
    return prev_flow


# ---------------------------------------------------------------- 06's metric functions
def grey_u8(frame: torch.Tensor) -> np.ndarray:
    """06:173-174: (frame.mean(dim=0) * 255).numpy().astype(np.uint8), frame [C, H, W] in [0, 1]."""
    return (frame.mean(dim=0) * 255).numpy().astype(np.uint8)


def flow_stats(flow: np.ndarray) -> dict:
    mag = np.sqrt(flow[..., 0] ** 2 + flow[..., 1] ** 2)
    return {"magnitude_mean": float(mag.mean()), "magnitude_std": float(mag.std()),
            "magnitude_max": float(mag.max()), "magnitude_median": float(np.median(mag))}


def warp_frame(frame: torch.Tensor, flow: np.ndarray) -> torch.Tensor:
    """06:259-284."""
    C, H, W = frame.shape
    gy, gx = np.mgrid[0:H, 0:W].astype(np.float32)
    sx = 2 * (gx + flow[..., 0]) / (W - 1) - 1
    sy = 2 * (gy + flow[..., 1]) / (H - 1) - 1
    grid = torch.stack([torch.from_numpy(sx), torch.from_numpy(sy)], dim=-1).unsqueeze(0)
    return F.grid_sample(frame.unsqueeze(0), grid, mode="bilinear", padding_mode="border",
                         align_corners=True).squeeze(0)


def pair_metrics(f1: torch.Tensor, f2: torch.Tensor) -> dict:
    """flow_magnitude_mean / std and warp_error of one frame pair (06:330-335)."""
    flow = farneback(grey_u8(f1), grey_u8(f2))
    st = flow_stats(flow)
    warped = warp_frame(f1, flow)
    return {"flow_magnitude_mean": st["magnitude_mean"], "flow_magnitude_std": st["magnitude_std"],
            "warp_error": F.mse_loss(warped, f2).item(), "flow": flow}


def video_flow_metrics(frames_u8: np.ndarray) -> dict:
    """Flow / warp part of 06's measure_video_metrics (06:320-383) over [F, H, W, 3] uint8
    frames (05's PNGs as 06:97-113 loads them: float / 255, [C, H, W])."""
    fr = torch.from_numpy(frames_u8).permute(0, 3, 1, 2).float() / 255
    pairs = [pair_metrics(fr[i], fr[i + 1]) for i in range(len(fr) - 1)]
    mags = [p["flow_magnitude_mean"] for p in pairs]
    warps = [p["warp_error"] for p in pairs]
    return {"frame_metrics": [{k: p[k] for k in ("flow_magnitude_mean", "flow_magnitude_std", "warp_error")}
                              for p in pairs],
            "mean_flow_magnitude": float(np.mean(mags)), "flow_magnitude_variance": float(np.var(mags)),
            "mean_warp_error": float(np.mean(warps)), "warp_error_variance": float(np.var(warps))}
