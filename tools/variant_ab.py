"""Same-process step A/B of a DIAGNOSTIC variant of the library (built with an extra -D define
that selects an experimental code path under #ifdef) against the product build.  Round 5 used it
for VD_G2_PRIO — the v2 GEMM's MFMA stretch at raised wave priority (s_setprio 1 around the
k-tile's MFMAs): 47.32 vs 46.79 ms at 16 frames, 12.19 vs 12.14 at 8-way, not kept
(profiles/r05_g2_prio_refuted.txt); and for VD_GN_BT=512 / 1024 (GroupNorm partial blocks of
512 / 1024 threads: slower at every shape, profiles/r05_gn_launch_shape_refuted.txt).  The
#ifdefs were removed with the results.

    python tools/variant_ab.py --build --define VD_SOMETHING [--name v]   # here (CPU): tools/diag_build/libvdiff_v.so
    python tools/variant_ab.py [--world 8] [--name v1,v2]                 # GPU box

Both libraries are loaded in one process (the variant with RTLD_LOCAL); vdiff's calls go through
vdiff._lib.lib(), whose handle is swapped while each arm's hipGraph is captured, then the two
graphs are replayed in alternating rounds (tools/ab_step.py's method)."""
from __future__ import annotations

import argparse
import ctypes as C
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "video-diffusion-experiments_amd"
OUT = ROOT / "tools" / "diag_build"


def lib_path(name):
    return OUT / f"libvdiff_{name}.so"


def load_variant(name):
    """The variant library loaded beside the product one, its ctypes signatures set."""
    from vdiff import _lib as L
    var = C.CDLL(str(lib_path(name)), mode=os.RTLD_NOW | os.RTLD_LOCAL)
    for fn_name, (argt, rest) in L.SIGNATURES.items():
        fn = getattr(var, fn_name)
        fn.argtypes, fn.restype = argt, rest
    return var


def build(define, name):
    sys.path.insert(0, str(PKG))
    import build_ext as B
    OUT.mkdir(exist_ok=True)
    defs = ['-DVD_BUILD_HASH="diag"', f'-DVD_BUILD_ARCH="{B.ARCH}"'] + [f"-D{d}" for d in define.split(",")]
    objs = []
    for src in sorted(B.CSRC.glob("*.hip")):
        obj = OUT / (src.stem + f"_{name}.o")
        subprocess.run([B.HIPCC, *B.CFLAGS, *defs, "-c", str(src), "-o", str(obj)], check=True)
        objs.append(str(obj))
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(lib_path(name)), *objs,
                    "-L/opt/rocm/lib", "-lrccl"], check=True)
    for o in objs:
        os.remove(o)
    print("built", lib_path(name))


def run(args):
    sys.path[:0] = [str(ROOT), str(PKG), str(ROOT / "tools")]
    import torch
    from vdiff import DDIMScheduler, DenoiseLoop
    from vdiff import _lib as L
    from vdiff.weights import materialize_synthetic
    base = L.lib()
    arms = [("base", base)] + [(n, load_variant(n)) for n in args.name.split(",")]
    unet = materialize_synthetic("full", device="cuda", seed=0)
    if args.world > 1:
        from rank_emulate import EmulatedShard
        unet.dist = EmulatedShard(args.world, 1, "copy")
    unet.prepare()
    fl = args.frames // args.world
    lat = torch.randn(1, 4, fl, 64, 64, device="cuda")
    ehs = torch.randn(2, 77, unet.config["cross_attention_dim"], device="cuda")
    s = DDIMScheduler(beta_schedule="linear", steps_offset=1, clip_sample=False)
    s.set_timesteps(50)
    ts = s.timesteps.repeat(1 + (args.rounds * args.steps + 10) // 50)
    loops = {}
    for arm, h in arms:
        L._lib = h
        lp = DenoiseLoop(unet, s, lat.clone(), ehs, 7.5, timesteps=ts, use_graph=True).prime()
        assert lp.graph is not None, lp.graph_error
        lp.run(3)
        loops[arm] = lp
    L._lib = base
    res = {a: [] for a in loops}
    for _ in range(args.rounds):
        for arm, lp in loops.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            lp.run(args.steps)
            torch.cuda.synchronize()
            res[arm].append(1e3 * (time.perf_counter() - t0) / args.steps)
    for arm, v in res.items():
        v = sorted(v)
        print(f"diag variant A/B {arm}: world {args.world} frames/rank {fl}: median {v[len(v) // 2]:.3f} ms/step, "
              f"min {v[0]:.3f} (rounds {len(v)})", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--define", default="VD_DIAG_VARIANT", help="the -D define(s) of the variant build, comma-separated")
    ap.add_argument("--name", default="variant", help="variant library name(s); several, comma-separated, at run time")
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    build(a.define, a.name) if a.build else run(a)
