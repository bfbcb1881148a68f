"""Temporal-consistency metrics of generated videos on the GPU.

Mirrors the reference's measurement (experiments/06_measure_grid_search.py): frames are
read like its load_frames (:97-113: sorted frame_*.png, PIL RGB), and per video the
consecutive-pair MSE / PSNR (:209-218), their mean / population std, and the flicker
index (:221-235) are reported under the reference's JSON keys.  The pixel work — every
byte of every frame, for a whole batch of videos — is one pass of the HIP kernel
vd_frame_metrics (exact integer sums); the host only forms the scalars.  The optical-flow
fields (06:163-199 Farneback flow magnitude, :259-284 warp error) come from the HIP
Farneback pipeline vd_farneback_flow + vd_flow_warp_stats over every pair of the batch.
LPIPS (AlexNet weights) has no offline counterpart here: its fields are None, and
temporal_consistency_score is formed only when per-pair LPIPS values are supplied.
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


# OpticalFlowEstimator.compute_flow's cv2 arguments (06:176-186)
FARNEBACK = dict(pyr_scale=0.5, levels=3, winsize=15, iterations=3, poly_n=5, poly_sigma=1.2)


def _u8_videos(videos_u8: torch.Tensor) -> torch.Tensor:
    if not videos_u8.is_cuda or videos_u8.dtype != torch.uint8 or videos_u8.dim() != 5 or videos_u8.shape[-1] != 3:
        raise ValueError("takes a uint8 CUDA tensor [videos, frames, H, W, 3] (no CPU fallback)")
    return videos_u8.contiguous()


def farneback_flow(videos_u8: torch.Tensor, **params) -> torch.Tensor:
    """uint8 [V, F, H, W, 3] on the GPU -> flow fp32 [V, F-1, H, W, 2]: cv2.calcOpticalFlowFarneback
    of every consecutive grey pair (06:163-188), parameters as 06 passes them unless overridden."""
    x = _u8_videos(videos_u8)
    V, Fr, H, W = x.shape[:4]
    p = {**FARNEBACK, **params}
    ws_bytes = lib().vd_farneback_workspace(V, Fr, H, W)
    if ws_bytes < 0:
        raise ValueError(f"bad video shape {tuple(x.shape)}")
    ws = torch.empty(ws_bytes, device=x.device, dtype=torch.uint8)
    flow = torch.empty(V, Fr - 1, H, W, 2, device=x.device, dtype=torch.float32)
    stream = torch.cuda.current_stream().cuda_stream
    check(lib().vd_farneback_flow(x.data_ptr(), V, Fr, H, W, p["pyr_scale"], p["levels"], p["winsize"],
                                  p["iterations"], p["poly_n"], p["poly_sigma"], flow.data_ptr(), ws.data_ptr(),
                                  ws_bytes, stream), "vd_farneback_flow")
    return flow


def flow_sums(videos_u8: torch.Tensor, flow: torch.Tensor) -> torch.Tensor:
    """-> fp64 [V, F-1, 3] = {sum |flow|, sum |flow|^2, sum (warp_frame(f, flow) - f')^2}."""
    x = _u8_videos(videos_u8)
    V, Fr, H, W = x.shape[:4]
    if tuple(flow.shape) != (V, Fr - 1, H, W, 2) or flow.dtype != torch.float32 or not flow.is_cuda:
        raise ValueError("flow must be fp32 CUDA [V, F-1, H, W, 2]")
    flow = flow.contiguous()
    ws_bytes = lib().vd_flow_warp_workspace(V, Fr)
    ws = torch.empty(ws_bytes, device=x.device, dtype=torch.uint8)
    stats = torch.empty(V, Fr - 1, 3, device=x.device, dtype=torch.float64)
    stream = torch.cuda.current_stream().cuda_stream
    check(lib().vd_flow_warp_stats(x.data_ptr(), flow.data_ptr(), V, Fr, H, W, stats.data_ptr(), ws.data_ptr(),
                                   ws_bytes, stream), "vd_flow_warp_stats")
    return stats


def flow_fields(stats, hw: int) -> dict:
    """One video's [F-1, 3] flow sums -> the per-pair and aggregate flow / warp fields of the
    reference's record (06:190-199 magnitude mean / population std, :336-338, :379-383)."""
    mag_mean = [s[0] / hw for s in stats]
    mag_std = [float(np.sqrt(max(s[1] / hw - (s[0] / hw) ** 2, 0.0))) for s in stats]
    warp = [s[2] / (3 * hw) for s in stats]
    return {"mean_flow_magnitude": float(np.mean(mag_mean)), "flow_magnitude_variance": float(np.var(mag_mean)),
            "mean_warp_error": float(np.mean(warp)), "warp_error_variance": float(np.var(warp)),
            "pairs": [{"flow_magnitude_mean": m, "flow_magnitude_std": sd, "warp_error": w}
                      for m, sd, w in zip(mag_mean, mag_std, warp)]}


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


FLOW_WORKSPACE_CAP = 2 << 30   # bytes of Farneback workspace per group of videos


def measure_videos(videos_u8: torch.Tensor, lpips=None, flow: bool = True,
                   workspace_cap: int = FLOW_WORKSPACE_CAP) -> list:
    """uint8 [V, F, H, W, 3] (GPU) -> one record per video (flow fields from the HIP Farneback
    pipeline unless flow=False).  The flow pass runs over groups of videos whose workspace
    (~112 B per pixel-frame) stays under `workspace_cap`, so the reference's 78-video grid does
    not need ~37 GB at once; videos too short or small for Farneback (fewer than 2 frames,
    H or W < 8) keep their flow fields None, as 06 leaves them when it has no pair."""
    sse, sad = frame_sums(videos_u8)
    sse, sad = sse.cpu().tolist(), sad.cpu().tolist()
    n = int(np.prod(videos_u8.shape[2:]))
    recs = [video_metrics(sse[v], sad[v], n, None if lpips is None else lpips[v]) for v in range(len(sse))]
    V, Fr, H, W = videos_u8.shape[:4]
    if flow and Fr >= 2 and H >= 8 and W >= 8:
        hw = int(H * W)
        per_video = max(int(lib().vd_farneback_workspace(1, Fr, H, W)), 1)
        group = max(1, min(V, workspace_cap // per_video))
        st = []
        for v0 in range(0, V, group):
            part = videos_u8[v0:v0 + group]
            st += flow_sums(part, farneback_flow(part)).cpu().tolist()
        for rec, s in zip(recs, st):
            ff = flow_fields(s, hw)
            for fm, pm in zip(rec["frame_metrics"], ff.pop("pairs")):
                fm.update(pm)
            rec.update(ff)
    return recs


def frames_from_video(video: torch.Tensor) -> torch.Tensor:
    """Pipeline output (B, F, 3, H, W) in [0, 1] -> uint8 [B, F, H, W, 3] as the reference saves
    its PNG frames (numpy_to_pil: (x * 255).round())."""
    return (video.permute(0, 1, 3, 4, 2) * 255).round().to(torch.uint8)
