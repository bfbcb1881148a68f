"""Temporal-consistency metrics of generated videos on the GPU.

Mirrors the reference's measurement (experiments/06_measure_grid_search.py): frames are
read like its load_frames (:97-113: sorted frame_*.png, PIL RGB), and per video the
consecutive-pair MSE / PSNR (:209-218), their mean / population std, and the flicker
index (:221-235) are reported under the reference's JSON keys.  The pixel work — every
byte of every frame, for a whole batch of videos — is one pass of the HIP kernel
vd_frame_metrics (exact integer sums); the host only forms the scalars.  LPIPS (AlexNet
weights) and the Farneback flow / warp error (OpenCV) have no offline counterpart here:
their fields are None, and temporal_consistency_score is formed only when per-pair LPIPS
values are supplied.
"""
from __future__ import annotations

from pathlib import Path
from typing import Optional, Sequence

import numpy as np
import torch

from ._lib import check, lib


def load_frames(frame_dir) -> np.ndarray:
    """[F, H, W, 3] uint8 — experiments/06:97-113 without its /255."""
    from PIL import Image
    d = Path(frame_dir)
    files = sorted(d.glob("*.png")) or sorted(d.glob("*.jpg"))
    if not files:
        raise ValueError(f"No frames found in {d}")
    return np.stack([np.array(Image.open(f).convert("RGB")) for f in files])


def frame_sums(videos_u8: torch.Tensor):
    """uint8 [V, F, H, W, 3] on the GPU -> (sse [V, F-1], sad [V, F-2]) int64 on the GPU."""
    if not videos_u8.is_cuda or videos_u8.dtype != torch.uint8:
        raise ValueError("frame_sums takes a uint8 CUDA tensor (no CPU fallback)")
    x = videos_u8.contiguous()
    V, Fr = x.shape[:2]
    nb = x[0, 0].numel()
    sse = torch.empty(V, Fr - 1, device=x.device, dtype=torch.int64)
    sad = torch.empty(V, max(Fr - 2, 0), device=x.device, dtype=torch.int64)
    stream = torch.cuda.current_stream().cuda_stream
    check(lib().vd_frame_metrics(x.data_ptr(), V, Fr, nb, sse.data_ptr(), sad.data_ptr() if Fr > 2 else None,
                                 stream), "vd_frame_metrics")
    return sse, sad


def _psnr(mse: float) -> float:
    return 100.0 if mse < 1e-10 else float(10 * np.log10(1.0 / mse))


def video_metrics(sse, sad, n_values: int, lpips: Optional[Sequence[float]] = None) -> dict:
    """One video's record, keys as the reference's <experiment>_metrics.json."""
    mse = [float(s) / (255.0 ** 2 * n_values) for s in sse]
    psnr = [_psnr(m) for m in mse]
    rec = {
        "num_frames": len(mse) + 1,
        "mean_mse": float(np.mean(mse)), "std_mse": float(np.std(mse)),
        "mean_psnr": float(np.mean(psnr)),
        "mean_lpips": float(np.mean(lpips)) if lpips is not None else None,
        "std_lpips": float(np.std(lpips)) if lpips is not None else None,
        "mean_flow_magnitude": None, "flow_magnitude_variance": None,
        "mean_warp_error": None, "warp_error_variance": None,
        "temporal_consistency_score": None,
        "flicker_index": float(np.mean([float(s) / (255.0 * n_values) for s in sad])) if len(sad) else 0.0,
        "frame_metrics": [{"frame_idx": i, "mse": m, "psnr": p,
                           "lpips": float(lpips[i]) if lpips is not None else None}
                          for i, (m, p) in enumerate(zip(mse, psnr))],
    }
    if lpips is not None:  # experiments/06:238-256
        rec["temporal_consistency_score"] = (float(np.var(mse)) * 1000 + float(np.mean(mse)) * 100
                                             + float(np.mean(lpips)) * 50 + float(np.var(lpips)) * 500)
    return rec


def measure_videos(videos_u8: torch.Tensor, lpips=None) -> list:
    """uint8 [V, F, H, W, 3] (GPU) -> one record per video."""
    sse, sad = frame_sums(videos_u8)
    sse, sad = sse.cpu().tolist(), sad.cpu().tolist()
    n = int(np.prod(videos_u8.shape[2:]))
    return [video_metrics(sse[v], sad[v], n, None if lpips is None else lpips[v]) for v in range(len(sse))]


def frames_from_video(video: torch.Tensor) -> torch.Tensor:
    """Pipeline output (B, F, 3, H, W) in [0, 1] -> uint8 [B, F, H, W, 3] as the reference saves
    its PNG frames (numpy_to_pil: (x * 255).round())."""
    return (video.permute(0, 1, 3, 4, 2) * 255).round().to(torch.uint8)
