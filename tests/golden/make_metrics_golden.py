"""Temporal-consistency metric fixtures, run in the build container:

    python tests/golden/make_metrics_golden.py

* copies ONE experiment's frames and its metrics record — data the reference holds in
  outputs/05_grid_search/<id>/frames/*.png and outputs/06_grid_search_metrics/<id>_metrics.json —
  into tests/golden/metrics/ (the GPU parity test and the CPU oracle test use them; the GPU box
  has no /root/reference);
* runs oracle/metrics_ref.py and oracle/flow_ref.py (Farneback flow + warp error) over EVERY
  experiment the reference measured and writes the largest relative deviation per metric to
  tests/golden/metrics/oracle_vs_reference.json (the oracles' pin across all 78 videos).
"""
import json
import shutil
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path[:0] = [str(ROOT)]

from oracle import flow_ref, metrics_ref  # noqa: E402

REF = Path("/root/reference/outputs")
KEEP = "portrait_cfg9.0_steps25"
FIELDS = ("mean_mse", "std_mse", "mean_psnr", "flicker_index")
FLOW_FIELDS = ("mean_flow_magnitude", "flow_magnitude_variance", "mean_warp_error", "warp_error_variance")
PAIR_FLOW = ("flow_magnitude_mean", "flow_magnitude_std", "warp_error")


def main():
    dst = HERE / "metrics" / KEEP
    (dst / "frames").mkdir(parents=True, exist_ok=True)
    for f in sorted((REF / "05_grid_search" / KEEP / "frames").glob("*.png")):
        shutil.copyfile(f, dst / "frames" / f.name)
    shutil.copyfile(REF / "06_grid_search_metrics" / f"{KEEP}_metrics.json", dst / "metrics.json")

    worst = {k: 0.0 for k in FIELDS + ("frame_mse", "frame_psnr", "temporal_consistency_score")
             + FLOW_FIELDS + tuple("frame_" + k for k in PAIR_FLOW)}
    n = 0
    for js in sorted((REF / "06_grid_search_metrics").glob("*_metrics.json")):
        ref = json.loads(js.read_text())
        frames = metrics_ref.load_frames_u8(REF / "05_grid_search" / ref["experiment_id"] / "frames")
        got = metrics_ref.measure_frames(frames, lpips=[m["lpips"] for m in ref["frame_metrics"]])
        for k in FIELDS + ("temporal_consistency_score",):
            worst[k] = max(worst[k], abs(got[k] - ref[k]) / abs(ref[k]))
        for a, b in zip(got["frame_metrics"], ref["frame_metrics"]):
            worst["frame_mse"] = max(worst["frame_mse"], abs(a["mse"] - b["mse"]) / b["mse"])
            worst["frame_psnr"] = max(worst["frame_psnr"], abs(a["psnr"] - b["psnr"]) / b["psnr"])
        flow = flow_ref.video_flow_metrics(frames)
        for k in FLOW_FIELDS:
            worst[k] = max(worst[k], abs(flow[k] - ref[k]) / abs(ref[k]))
        for a, b in zip(flow["frame_metrics"], ref["frame_metrics"]):
            for k in PAIR_FLOW:
                worst["frame_" + k] = max(worst["frame_" + k], abs(a[k] - b[k]) / abs(b[k]))
        n += 1
        print(ref["experiment_id"], {k: f"{v:.1e}" for k, v in worst.items() if "flow" in k or "warp" in k},
              flush=True)
    out = {"experiments": n, "max_relative_deviation": worst,
           "note": "oracle/metrics_ref.py (exact integer sums) and oracle/flow_ref.py (Farneback "
                   "restated from OpenCV) vs the reference's fp32 torch / cv2 results"}
    (HERE / "metrics" / "oracle_vs_reference.json").write_text(json.dumps(out, indent=1))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
