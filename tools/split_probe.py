"""Split-K at a frame shard's small M: the automatic plan (v2 split-K + gemm_splitk_reduce, two
launches) against forced v6 (64 x 64 tiles, K split toward 2 workgroups per CU, the slices reduced
in-kernel by the last arriver: one launch), on the rank's split shapes (tools/gemm_inventory.py
--frames 2).  Timed back-to-back in a hipGraph of R launches per shape, so launch gaps count as in
the step.

    python tools/split_probe.py [--reps 20]
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]

import torch  # noqa: E402

from vdiff import ops  # noqa: E402

# (kind, n_img, h, w, N, Cin) for convs; (kind, M, N, K) for dense (+res)
SHAPES = [("conv+res", 4, 32, 32, 640, 640), ("conv+res", 4, 16, 16, 1280, 1280), ("conv+res", 4, 8, 8, 1280, 1280),
          ("conv", 4, 16, 16, 1280, 2560), ("conv", 4, 8, 8, 1280, 2560), ("conv", 4, 32, 32, 640, 1920),
          ("conv", 4, 64, 64, 320, 640), ("dense+res", 1024, 1280, 5120), ("dense+res", 256, 1280, 5120),
          ("dense", 256, 1280, 2560), ("dense", 1024, 1280, 2560)]


# the rank's unsplit v6 shapes (K <= 1280), where forced v6 splits K toward 2 workgroups per CU
V6_SHAPES = [("dense+res", 1024, 1280, 1280), ("dense", 1024, 1280, 1280), ("dense+res", 256, 1280, 1280),
             ("dense", 256, 3840, 1280), ("dense", 1024, 1280, 640), ("dense+res", 4096, 640, 640),
             ("dense", 256, 1280, 1280)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--set", default="split", choices=["split", "v6"])
    args = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    for sh in (SHAPES if args.set == "split" else V6_SHAPES):
        kind = sh[0]
        if kind.startswith("conv"):
            _, n, hh, ww, N, cin = sh
            x = (torch.randn(n * hh * ww, cin, device="cuda", generator=g)).to(torch.bfloat16)
            w = (torch.randn(N, 9 * cin, device="cuda", generator=g) * (9 * cin) ** -0.5).to(torch.bfloat16)
            res = torch.randn(n * hh * ww, N, device="cuda", generator=g).to(torch.bfloat16) if "res" in kind else None
            M, K = n * hh * ww, 9 * cin

            def run():
                return ops.conv3x3(x, n, hh, ww, w, res=res)[0]
        else:
            _, M, N, K = sh
            a = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
            w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
            res = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16) if "res" in kind else None

            def run():
                return ops.gemm(a, w, res=res)
        line = f"{kind:10s} M {M:6d} N {N:5d} K {K:6d}"
        outs = {}
        for path in (0, 6):
            with ops.gemm_plan(path=path):
                d = ops.GemmDesc(a0=256, lda0=K, k0=K, a_mode=1 if kind.startswith("conv") else 0, w=256, ldw=K,
                                 M=M, N=N, K=K, out=256, ldc=N)
                if kind.startswith("conv"):
                    d.n_img, d.h_in, d.w_in, d.h_out, d.w_out, d.stride = n, hh, ww, hh, ww, 1
                kern, split = ops.gemm_plan_of(d)
                outs[path] = run()
                torch.cuda.synchronize()
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    for _ in range(args.reps):
                        run()
                graph.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                graph.replay()
                e1.record()
                e1.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / args.reps
            line += f" | path {path}: v{kern}/s{split} {us:7.1f} us ({2 * M * N * K / us / 1e6:6.1f} TF/s)"
        err = ((outs[0].float() - outs[6].float()).norm() / outs[0].float().norm()).item()
        print(line + f" | rel diff {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
