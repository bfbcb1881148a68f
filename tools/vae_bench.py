"""VAE decode benchmark: AnimateDiffPipeline.decode_latents of one
16-frame 512x512 video (latents (1, 4, 16, 64, 64)) through the SD-1.5 AutoencoderKL
decoder shapes (synthetic N(0, 0.02^2) weights), bf16, 1x MI355X.

    python tools/vae_bench.py [--frames 16] [--reps 3] [--chunk 8] [--cpu-frames 1]

Prints one JSON line: videos/s and frames/s, ms per video, the algorithmic TFLOP of the
decode (convs + attention, 2*M*N*K) and the MFMA fraction it reaches, plus the CPU oracle
(oracle/vae_ref.py, fp32, all host threads) on --cpu-frames frames scaled to the video.
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]

import torch  # noqa: E402

from vdiff import AnimateDiffPipeline, AutoencoderKL, init_synthetic_  # noqa: E402
from vdiff.models.vae import VAE_FULL  # noqa: E402

PEAK = 2500.0


def decode_flop(cfg, frames, h, w):
    """2*M*N*K over every conv / linear / attention product of the decoder."""
    ch = list(reversed(cfg["block_out_channels"]))
    f = 0.0
    hw = h * w

    def conv(cin, cout, pix, k=9):
        return 2.0 * frames * pix * cout * cin * k

    f += conv(4, 4, hw, 1) + conv(4, ch[0], hw)
    res = lambda cin, cout, pix: conv(cin, cout, pix) + conv(cout, cout, pix) + (conv(cin, cout, pix, 1) if cin != cout else 0)  # noqa: E731
    f += 2 * res(ch[0], ch[0], hw)
    f += frames * (2.0 * hw * ch[0] * ch[0] * 4 + 4.0 * hw * hw * ch[0])  # q,k,v,out + QK^T, PV
    prev, pix = ch[0], hw
    for i, c in enumerate(ch):
        for j in range(cfg["layers_per_block"] + 1):
            f += res(prev if j == 0 else c, c, pix)
        prev = c
        if i < len(ch) - 1:
            pix *= 4
            f += conv(c, c, pix)
    f += conv(ch[-1], 3, pix)
    return f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--chunk", type=int, default=8)
    ap.add_argument("--cpu-frames", type=int, default=1)
    args = ap.parse_args()
    vae = init_synthetic_(AutoencoderKL("full"), seed=0).to("cuda", torch.bfloat16).prepare()
    vae.frames_per_chunk = args.chunk
    pipe = AnimateDiffPipeline.__new__(AnimateDiffPipeline)
    pipe.vae = vae
    lat = torch.randn((1, 4, args.frames, 64, 64), generator=torch.Generator().manual_seed(42)).cuda() * 0.18215
    video = pipe.decode_latents(lat)  # warm-up (kernel loads, allocator)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        video = pipe.decode_latents(lat)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.reps
    assert torch.isfinite(video).all()
    flop = decode_flop(VAE_FULL, args.frames, 64, 64)
    cpu = None
    if args.cpu_frames:
        from oracle import vae_ref
        sd = {k: v.detach().float().cpu() for k, v in vae.state_dict().items()}
        with torch.no_grad():
            t0 = time.perf_counter()
            vae_ref.decode_latents(sd, VAE_FULL, lat[:, :, :args.cpu_frames].cpu().float())
            tc = time.perf_counter() - t0
        cpu = {"value": round(args.cpu_frames / tc, 4), "unit": "frames/s", "cores": torch.get_num_threads(),
               "kind": "port", "sample": f"{args.cpu_frames} frame(s) of the decode, fp32 oracle, {tc:.2f} s"}
    print(json.dumps({
        "metric": "VAE decode frames/s (16-frame 512x512 video, SD-1.5 AutoencoderKL decoder)",
        "value": round(args.frames / dt, 2), "unit": "frames/s", "ms_per_video": round(1e3 * dt, 2),
        "videos_per_s": round(1.0 / dt, 3), "dtype": "bf16", "data": "synthetic (latents randn seed 42, weights N(0,0.02^2))",
        "config": {"workload": "decode_latents (1, 4, 16, 64, 64) -> (1, 3, 16, 512, 512)", "frames_per_chunk": args.chunk},
        "algorithmic_tflop": round(flop / 1e12, 3),
        "mfma": {"achieved": round(flop / dt / 1e12, 1), "peak": PEAK, "unit": "TFLOP/s",
                 "frac": round(flop / dt / 1e12 / PEAK, 4)},
        "cpu_baseline": cpu}))


if __name__ == "__main__":
    main()
