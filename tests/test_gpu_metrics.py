"""Temporal-consistency metrics on the MI355X.

Pinned parity: the reference's own outputs — the committed frames of one grid-search
experiment and its outputs/06_grid_search_metrics record (tests/golden/metrics/) — and the
oracle (oracle/metrics_ref.py, itself checked against all 78 reference records by
tests/golden/make_metrics_golden.py).  The kernel's integer sums must equal the oracle's
exactly; the scalar metrics must match the reference's fp32 results to 1e-6 relative.
"""
import json
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import metrics_ref
from vdiff import metrics

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden" / "metrics" / "portrait_cfg9.0_steps25"


def test_reference_video_matches_reference_record(cuda):
    frames = metrics.load_frames(GOLD / "frames")
    ref = json.loads((GOLD / "metrics.json").read_text())
    x = torch.from_numpy(frames)[None].to(cuda)
    sse, sad = metrics.frame_sums(x)
    assert sse[0].cpu().tolist() == metrics_ref.pair_sse(frames).tolist()
    assert sad[0].cpu().tolist() == metrics_ref.triplet_sad(frames).tolist()
    rec = metrics.measure_videos(x, lpips=[[m["lpips"] for m in ref["frame_metrics"]]])[0]
    for k in ("mean_mse", "std_mse", "mean_psnr", "flicker_index", "temporal_consistency_score"):
        assert rec[k] == pytest.approx(ref[k], rel=1e-6), k
    for a, b in zip(rec["frame_metrics"], ref["frame_metrics"]):
        assert a["mse"] == pytest.approx(b["mse"], rel=1e-6) and a["psnr"] == pytest.approx(b["psnr"], rel=1e-6)


@pytest.mark.parametrize("V,F,H,W", [(3, 16, 64, 48), (1, 2, 16, 16), (2, 3, 8, 32), (1, 32, 32, 32), (5, 7, 48, 16)])
def test_frame_sums_exact_against_oracle(cuda, V, F, H, W):
    g = torch.Generator().manual_seed(V * 100 + F)
    x = torch.randint(0, 256, (V, F, H, W, 3), generator=g, dtype=torch.uint8)
    x[0, 0] = 255  # extreme values: max squared / second differences
    x[0, 1 % F] = 0
    sse, sad = metrics.frame_sums(x.to(cuda))
    for v in range(V):
        assert sse[v].cpu().tolist() == metrics_ref.pair_sse(x[v].numpy()).tolist()
        if F > 2:
            assert sad[v].cpu().tolist() == metrics_ref.triplet_sad(x[v].numpy()).tolist()


def test_identical_frames_and_psnr_cap(cuda):
    x = torch.full((1, 4, 16, 16, 3), 77, dtype=torch.uint8, device=cuda)
    rec = metrics.measure_videos(x)[0]
    assert rec["mean_mse"] == 0.0 and rec["mean_psnr"] == 100.0 and rec["flicker_index"] == 0.0


def test_large_frame_batch_sums(cuda):
    """512x512 frames (the reference's size), 4 videos, against the oracle."""
    g = torch.Generator().manual_seed(9)
    x = torch.randint(0, 256, (4, 16, 512, 512, 3), generator=g, dtype=torch.uint8)
    sse, sad = metrics.frame_sums(x.to(cuda))
    for v in range(4):
        assert sse[v].cpu().tolist() == metrics_ref.pair_sse(x[v].numpy()).tolist()
        assert sad[v].cpu().tolist() == metrics_ref.triplet_sad(x[v].numpy()).tolist()
