"""Every vd_gemm call of one UNet forward, timed: which GEMM / conv shapes carry the step.

    python tools/gemm_inventory.py [--frames F] [--reps R]

One eager CFG forward of the full model at F frames (16 = BASELINE config 3, 2 = the 8-way
rank's images) records each vd_gemm descriptor (M, N, K, conv or dense, residual, activation,
the plan's kernel), then re-launches every recorded call R times between HIP events on the
same operands and prints the per-step time by shape, with TFLOP/s and the kernel family.
Launch-by-launch timing of a single kernel: no graph, so each number carries its launch's
own ramp, not the neighbours'."""
from __future__ import annotations

import argparse
import collections
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]

import torch  # noqa: E402

from vdiff import ops  # noqa: E402
from vdiff._lib import check, lib  # noqa: E402
from vdiff.weights import materialize_synthetic  # noqa: E402

KIND = {0: "dense", 1: "conv"}
ACT = {0: "", 1: "+silu", 2: "geglu", 3: "+gelu"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    unet = materialize_synthetic("full", device="cuda", seed=0)
    unet.prepare()
    calls = []
    orig = ops._run_gemm

    def rec(d, device, what):
        ws = orig(d, device, what)
        dd = type(d)()
        C.pointer(dd)[0] = d
        calls.append((dd, ws))
        return ws
    ops._run_gemm = rec
    x = torch.randn(2, 4, args.frames, 64, 64, device="cuda")
    ehs = torch.randn(2, 77, 768, device="cuda")
    with torch.no_grad():
        unet(x, 981, encoder_hidden_states=ehs)
    torch.cuda.synchronize()
    ops._run_gemm = orig
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    s = torch.cuda.current_stream().cuda_stream
    for d, _ in calls:
        for _ in range(2):
            check(lib().vd_gemm(C.byref(d), s), "vd_gemm")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            check(lib().vd_gemm(C.byref(d), s), "vd_gemm")
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.reps
        kind = KIND[d.a_mode] + ("+res" if d.res else "") + ACT.get(d.act, "") + ("+ln" if d.ln_out else "") + \
            ("+rb" if d.rowbias else "") + ("+fold" if d.ln_fold_s else "")
        kv, sp = C.c_int32(), C.c_int32()
        check(lib().vd_gemm_plan(C.byref(d), C.byref(kv), C.byref(sp)), "vd_gemm_plan")
        key = (kind, d.M, d.N, d.K, f"v{kv.value}" + (f"/s{sp.value}" if sp.value > 1 else ""))
        a = agg[key]
        a[0] += 1
        a[1] += us
        a[2] += 2.0 * d.M * d.N * d.K
    tot = sum(v[1] for v in agg.values())
    print(f"{len(calls)} vd_gemm calls, {tot / 1e3:.2f} ms per forward (launch-by-launch), frames {args.frames}")
    print(f"{'kind':18s} {'M':>7s} {'N':>5s} {'K':>6s} {'plan':>7s} {'calls':>5s} {'us/call':>8s} {'ms/step':>8s} "
          f"{'TF/s':>7s}")
    for key, (n, us, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{key[0]:18s} {key[1]:7d} {key[2]:5d} {key[3]:6d} {key[4]:>7s} {n:5d} {us / n:8.1f} {us / 1e3:8.3f} "
              f"{fl / (us * 1e-6) / 1e12:7.1f}")


if __name__ == "__main__":
    main()
