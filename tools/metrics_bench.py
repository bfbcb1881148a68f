"""Metrics benchmark: vd_frame_metrics over a batch of 16-frame
512x512 uint8 videos (the reference's grid search measured 78 of them), 1x MI355X.

    python tools/metrics_bench.py [--videos 78] [--reps 20]

One JSON line: videos/s, the kernel's HBM roofline (algorithmic bytes = every frame byte
read once, per launch / average launch time from HIP events on the launch stream, vs
8 TB/s) and the CPU baseline (oracle/metrics_ref.py integer sums, numpy, 1 thread) on 2
videos scaled to the batch.
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]

import torch  # noqa: E402

from vdiff import metrics  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--videos", type=int, default=78)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randint(0, 256, (args.videos, 16, 512, 512, 3), device="cuda", dtype=torch.uint8, generator=g)
    s = torch.cuda.current_stream()
    for _ in range(3):
        metrics.frame_sums(x)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(args.reps):
        metrics.frame_sums(x)
    e1.record(s)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / args.reps
    byts = x.numel()
    from oracle import metrics_ref
    xc = x[:2].cpu().numpy()
    t0 = time.perf_counter()
    for v in range(2):
        metrics_ref.pair_sse(xc[v]), metrics_ref.triplet_sad(xc[v])
    tc = (time.perf_counter() - t0) / 2
    print(json.dumps({
        "metric": "temporal-consistency metric sums (pair MSE + flicker), videos/s",
        "value": round(args.videos / (ms * 1e-3), 1), "unit": "videos/s", "ms_per_launch": round(ms, 4),
        "config": {"workload": f"{args.videos} videos x 16 frames x 512x512x3 uint8 per launch"},
        "roofline": {"bound": "hbm", "achieved": round(byts / (ms * 1e-3) / 1e9, 1), "peak": 8000.0, "unit": "GB/s",
                     "frac": round(byts / (ms * 1e-3) / 1e9 / 8000.0, 4), "algorithmic_bytes_per_launch": byts},
        "cpu_baseline": {"value": round(1.0 / tc, 2), "unit": "videos/s", "cores": 1, "kind": "port",
                         "sample": f"2 videos through oracle/metrics_ref.py (numpy int64), {tc:.3f} s/video"}}))


if __name__ == "__main__":
    main()
