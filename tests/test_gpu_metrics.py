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


# ---------------------------------------------------------------- Farneback flow / warp error
# Parity: the reference's records (flow_magnitude_mean / _std / warp_error per pair, computed
# by cv2 + torch in experiments/06) and oracle/flow_ref.py (the OpenCV restatement, within
# ~1e-5 of all 78 records: tests/golden/metrics/oracle_vs_reference.json).  The kernels follow
# the oracle's fp32/fp64 operation order; only the box-filter sums are summed directly instead
# of by running sums, so flows agree to last-bit noise carried through the fixed-point
# iterations — bounds below: 1e-3 px on the flow, 1e-4 relative on the per-pair fields.
def _flow_oracle(frames_u8, pairs):
    from oracle import flow_ref
    fr = torch.from_numpy(frames_u8).permute(0, 3, 1, 2).float() / 255
    return [flow_ref.pair_metrics(fr[i], fr[i + 1]) for i in pairs]


def test_reference_video_flow_matches_reference_record(cuda):
    frames = metrics.load_frames(GOLD / "frames")
    ref = json.loads((GOLD / "metrics.json").read_text())
    x = torch.from_numpy(frames)[None].to(cuda)
    rec = metrics.measure_videos(x)[0]
    worst = 0.0
    for a, b in zip(rec["frame_metrics"], ref["frame_metrics"]):
        for k in ("flow_magnitude_mean", "flow_magnitude_std", "warp_error"):
            worst = max(worst, abs(a[k] - b[k]) / abs(b[k]))
    print(f"worst per-pair relative deviation from the reference record: {worst:.2e}")
    assert worst < 1e-4
    for k in ("mean_flow_magnitude", "mean_warp_error"):
        assert rec[k] == pytest.approx(ref[k], rel=1e-5), k
    for k in ("flow_magnitude_variance", "warp_error_variance"):
        assert rec[k] == pytest.approx(ref[k], rel=2e-3), k


def test_reference_video_flow_field_against_oracle(cuda):
    frames = metrics.load_frames(GOLD / "frames")[:4]
    flow = metrics.farneback_flow(torch.from_numpy(frames)[None].to(cuda))[0].cpu().numpy()
    for i, o in zip((0, 2), _flow_oracle(frames, (0, 2))):
        d = np.abs(flow[i] - o["flow"])
        print(f"pair {i}: max |flow - oracle| {d.max():.2e} px, mean {d.mean():.2e}")
        assert d.max() < 1e-3 and d.mean() < 1e-6


def _smooth_video(g, V, F, H, W, shift):
    """Band-limited random texture translated by `shift` px per frame (known motion)."""
    base = torch.randn(V, 1, H + 8 * F, W + 8 * F, generator=g)
    base = torch.nn.functional.avg_pool2d(base, 5, 1, 2)
    base = torch.nn.functional.avg_pool2d(base, 5, 1, 2)
    frames = []
    for f in range(F):
        o = int(round(f * shift))
        crop = base[:, :, o:o + H, o:o + W]
        frames.append(crop)
    v = torch.stack(frames, 1)[:, :, 0]
    v = (v - v.amin()) / (v.amax() - v.amin())
    return (v[..., None].repeat(1, 1, 1, 1, 3) * 255).round().to(torch.uint8)


@pytest.mark.parametrize("V,F,H,W", [(2, 3, 64, 48), (1, 2, 100, 75), (1, 4, 130, 260)])
def test_flow_against_oracle_shapes(cuda, V, F, H, W):
    g = torch.Generator().manual_seed(H * W + F)
    x = _smooth_video(g, V, F, H, W, 1.0)
    x[0, -1, :4] = 255  # a saturated band
    flow = metrics.farneback_flow(x.to(cuda)).cpu().numpy()
    st = metrics.flow_sums(x.to(cuda), torch.from_numpy(flow).to(cuda)).cpu().numpy()
    for v in range(V):
        for i, o in enumerate(_flow_oracle(x[v].numpy(), range(F - 1))):
            d = np.abs(flow[v, i] - o["flow"])
            assert d.max() < 1e-3, (v, i, d.max())
            ff = metrics.flow_fields(st[v, i:i + 1].tolist(), H * W)
            assert ff["mean_flow_magnitude"] == pytest.approx(o["flow_magnitude_mean"], rel=1e-4)
            assert ff["pairs"][0]["flow_magnitude_std"] == pytest.approx(o["flow_magnitude_std"], rel=1e-4)
            assert ff["mean_warp_error"] == pytest.approx(o["warp_error"], rel=1e-4, abs=1e-9)


def test_flow_identical_frames_and_known_shift(cuda):
    x = torch.full((1, 3, 64, 64, 3), 90, dtype=torch.uint8, device=cuda)
    flow = metrics.farneback_flow(x)
    assert torch.count_nonzero(flow) == 0
    st = metrics.flow_sums(x, flow)
    assert torch.count_nonzero(st) == 0
    g = torch.Generator().manual_seed(3)
    y = _smooth_video(g, 1, 2, 128, 128, 2.0).to(cuda)  # content moves up-left by 2 px
    fl = metrics.farneback_flow(y)[0, 0, 16:-16, 16:-16]
    assert fl[..., 0].median().item() == pytest.approx(-2.0, abs=0.2)
    assert fl[..., 1].median().item() == pytest.approx(-2.0, abs=0.2)


def test_flow_rejects_bad_input(cuda):
    with pytest.raises(ValueError):
        metrics.farneback_flow(torch.zeros(1, 2, 16, 16, 3, dtype=torch.uint8))  # CPU tensor: no fallback
    with pytest.raises(ValueError):
        metrics.farneback_flow(torch.zeros(1, 2, 16, 16, 4, dtype=torch.uint8, device=cuda))
