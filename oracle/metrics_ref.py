"""ORACLE — test infrastructure only.  Never imported by the product path.

Restatement of the reference's temporal-consistency metrics that need no network
weights or OpenCV, experiments/06_measure_grid_search.py:
  * load_frames (:97-113): sorted frame_*.png, PIL RGB, float /255, [F, C, H, W];
  * compute_mse (:209-211): F.mse_loss(frame_i, frame_i+1) over all C*H*W values;
  * compute_psnr (:214-218): 100 if mse < 1e-10 else 10*log10(1/mse);
  * compute_flicker_index (:221-235): mean over t of mean|I_t - 2 I_t+1 + I_t+2|;
  * measure_video aggregates (:366-385): mean/std (population) of the pair MSEs,
    mean PSNR; temporal_consistency_score (:238-256) from MSE and LPIPS values.
Frames are uint8, so the pair sum of squared differences and the triplet sum of
absolute second differences are exact integers here (the reference accumulates them in
fp32; the two agree to ~1e-6 relative).  LPIPS (AlexNet weights) and the Farneback flow
/ warp error (cv2) are not restated: no weights and no OpenCV in this image.
PARITY STATUS: pinned — tests/test_oracle.py checks this file against the reference's own
outputs/06_grid_search_metrics JSON for the committed frames (tests/golden/metrics/), and
tests/golden/make_metrics_golden.py against all 78 experiments when /root/reference exists.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np


def load_frames_u8(frame_dir) -> np.ndarray:
    """[F, H, W, 3] uint8, sorted *.png (else *.jpg) as experiments/06:97-113 reads them."""
    from PIL import Image
    d = Path(frame_dir)
    files = sorted(d.glob("*.png")) or sorted(d.glob("*.jpg"))
    if not files:
        raise ValueError(f"No frames found in {d}")
    return np.stack([np.array(Image.open(f).convert("RGB")) for f in files])


def pair_sse(frames: np.ndarray) -> np.ndarray:
    """[F-1] exact sum over C*H*W of (a - b)^2 for consecutive uint8 frames."""
    x = frames.astype(np.int64)
    return ((x[1:] - x[:-1]) ** 2).reshape(len(frames) - 1, -1).sum(1)


def triplet_sad(frames: np.ndarray) -> np.ndarray:
    """[F-2] exact sum over C*H*W of |a - 2b + c|."""
    x = frames.astype(np.int64)
    return np.abs(x[:-2] - 2 * x[1:-1] + x[2:]).reshape(len(frames) - 2, -1).sum(1)


def psnr(mse: float) -> float:
    return 100.0 if mse < 1e-10 else float(10 * np.log10(1.0 / mse))


def metrics_from_sums(sse, sad, n_values: int, lpips=None) -> dict:
    """The reference's per-video record from the integer sums (n_values = C*H*W)."""
    mse = [float(s) / (255.0 ** 2 * n_values) for s in sse]
    ps = [psnr(m) for m in mse]
    out = {"num_frames": len(mse) + 1, "mean_mse": float(np.mean(mse)), "std_mse": float(np.std(mse)),
           "mean_psnr": float(np.mean(ps)),
           "flicker_index": float(np.mean([float(s) / (255.0 * n_values) for s in sad])) if len(sad) else 0.0,
           "frame_metrics": [{"frame_idx": i, "mse": m, "psnr": p} for i, (m, p) in enumerate(zip(mse, ps))]}
    if lpips is not None:
        out["temporal_consistency_score"] = consistency_score(mse, lpips)
    return out


def consistency_score(mse, lpips) -> float:
    """experiments/06:238-256."""
    return (float(np.var(mse)) * 1000 + float(np.mean(mse)) * 100 + float(np.mean(lpips)) * 50
            + float(np.var(lpips)) * 500)


def measure_frames(frames: np.ndarray, lpips=None) -> dict:
    return metrics_from_sums(pair_sse(frames), triplet_sad(frames), int(np.prod(frames.shape[1:])), lpips)
