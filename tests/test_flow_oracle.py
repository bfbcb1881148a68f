"""The Farneback flow / warp-error oracle (oracle/flow_ref.py) against the reference's own
records: the committed portrait_cfg9.0_steps25 frames and their
outputs/06_grid_search_metrics record, plus the all-videos pin that
tests/golden/make_metrics_golden.py wrote.  CPU only."""
import json
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import flow_ref, metrics_ref

GOLD = Path(__file__).resolve().parent / "golden" / "metrics"


def test_grey_conversion_is_torch_exact():
    """06:173 grey = uint8(mean_c(x / 255) * 255): the fp32 sequence the HIP kernel uses,
    ((r + g) + b) / 3 with IEEE divides, equals torch's for every RGB triple."""
    v = np.arange(256, dtype=np.uint8)
    r, g, b = (a.reshape(-1) for a in np.meshgrid(v, v, v[::7], indexing="ij"))
    frame = torch.from_numpy(np.stack([r, g, b]).reshape(3, 256, -1))
    want = flow_ref.grey_u8(frame.float() / 255)
    x = [c.astype(np.float32) / np.float32(255) for c in (r, g, b)]
    got = (((x[0] + x[1]) + x[2]) / np.float32(3) * np.float32(255)).astype(np.uint8)
    assert np.array_equal(got.reshape(want.shape), want)


def test_oracle_matches_reference_pairs():
    d = GOLD / "portrait_cfg9.0_steps25"
    ref = json.loads((d / "metrics.json").read_text())
    frames = metrics_ref.load_frames_u8(d / "frames")
    fr = torch.from_numpy(frames[:4]).permute(0, 3, 1, 2).float() / 255
    for i in range(3):
        got = flow_ref.pair_metrics(fr[i], fr[i + 1])
        want = ref["frame_metrics"][i]
        for k in ("flow_magnitude_mean", "flow_magnitude_std", "warp_error"):
            assert got[k] == pytest.approx(want[k], rel=1e-5), (i, k)


def test_oracle_pin_over_all_reference_videos():
    pin = json.loads((GOLD / "oracle_vs_reference.json").read_text())
    assert pin["experiments"] == 78
    dev = pin["max_relative_deviation"]
    for k in ("frame_flow_magnitude_mean", "frame_flow_magnitude_std", "frame_warp_error", "mean_flow_magnitude",
              "mean_warp_error"):
        assert dev[k] < 1e-4, k
    for k in ("flow_magnitude_variance", "warp_error_variance"):
        assert dev[k] < 1e-3, k


def test_farneback_zero_motion_and_levels():
    img = (np.random.default_rng(0).random((64, 80)) * 255).astype(np.uint8)
    flow = flow_ref.farneback(img, img)
    # OpenCV treats the outermost row / column as outside the image (UpdateMatrices), so
    # identical frames give a small flow at the border that the box filter spreads inward
    assert flow.shape == (64, 80, 2) and np.abs(flow).max() < 0.1 and np.abs(flow[16:-16, 16:-16]).max() < 1e-3
    const = np.full((64, 80), 90, np.uint8)
    assert np.abs(flow_ref.farneback(const, const)).max() == 0
    assert flow_ref.gaussian_kernel(3, 0).tolist() == [0.25, 0.5, 0.25]
    k = flow_ref.gaussian_kernel(19, 3.5)
    assert abs(float(k.sum()) - 1) < 1e-6 and k[9] == k.max()
