"""GEMM plan sweep: every dense UNet shape (proj, qkv, ff2, GEGLU per level) on the forced paths
v2 / v3 / v5 / v6 and the automatic plan, interleaved over rounds in one process (min of the
rounds reported; a warm-up pass first so no case pays the clock ramp).

python tools/plan_sweep.py [images ...]   (default 32 4; SWEEP=dense / conv / dense,conv)"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import ops  # noqa: E402
from vdiff._lib import lib  # noqa: E402

PATHS = {"auto": 0, "v2": 2, "v3": 3, "v5": 5, "v6": 6, "v8": 8}
g = torch.Generator(device="cuda").manual_seed(0)


def rnd(*s, std=1.0):
    return (torch.randn(*s, device="cuda", generator=g) * std).to(torch.bfloat16)


def run(imgs):
    cases = []
    for lvl, (hw, C) in enumerate([(4096, 320), (1024, 640), (256, 1280), (64, 1280)]):
        M = imgs * hw
        cases += [(f"L{lvl+1} proj+res M={M} N={C} K={C}", M, C, C, True, False),
                  (f"L{lvl+1} proj     M={M} N={C} K={C}", M, C, C, False, False),
                  (f"L{lvl+1} qkv      M={M} N={3*C} K={C}", M, 3 * C, C, False, False),
                  (f"L{lvl+1} ff2+res  M={M} N={C} K={4*C}", M, C, 4 * C, True, False),
                  (f"L{lvl+1} geglu    M={M} N={8*C} K={C}", M, 8 * C, C, False, True)]
    fns = []
    for name, hw, ci, co in [("L1 conv 320->320", 64, 320, 320), ("L1 conv 640->320", 64, 640, 320),
                             ("L2 conv 640->640", 32, 640, 640), ("L2 conv 1280->640", 32, 1280, 640),
                             ("L3 conv 1280->1280", 16, 1280, 1280), ("L3 conv 2560->1280", 16, 2560, 1280),
                             ("L4 conv 1280->1280", 8, 1280, 1280), ("L4 conv 2560->1280", 8, 2560, 1280)]:
        if CONV:
            x, w = rnd(imgs * hw * hw, ci), rnd(co, 9 * ci, std=(9 * ci) ** -0.5)
            out = torch.empty(imgs * hw * hw, co, device="cuda", dtype=torch.bfloat16)
            fns.append((f"{name} M={imgs*hw*hw}", lambda x=x, w=w, out=out, hw=hw: ops.conv3x3(x, imgs, hw, hw, w, out=out)))
    for name, M, N, K, res, geglu in cases:
        if not DENSE:
            continue
        a, w = rnd(M, K), rnd(N, K, std=K ** -0.5)
        b = torch.zeros(N, device="cuda")
        r = rnd(M, N) if res else None
        out = torch.empty(M, N // 2 if geglu else N, device="cuda", dtype=torch.bfloat16)
        act = ops.ACT_GEGLU if geglu else ops.ACT_NONE
        fns.append((name, lambda a=a, w=w, b=b, r=r, act=act, out=out: ops.gemm(a, w, bias=b, res=r, act=act, out=out)))
    best = {}
    for rnd_i in range(4):  # round 0 = warm-up, not recorded
        for name, fn in fns:
            for path, code in PATHS.items():
                ops._PLAN.path = code  # per-call vd_gemm_desc.path
                try:
                    for _ in range(2):
                        fn()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(10):
                        fn()
                    e1.record()
                    e1.synchronize()
                    us = e0.elapsed_time(e1) / 10 * 1e3
                except Exception:  # noqa: BLE001  (a path that refuses the shape)
                    us = float("nan")
                if rnd_i:
                    best[(name, path)] = min(best.get((name, path), float("inf")), us)
        ops._PLAN.path = 0  # per-call vd_gemm_desc.path
    for name, _ in fns:
        row = "  ".join(f"{p} {best[(name, p)]:7.1f}" for p in PATHS)
        print(f"[{imgs:2d} img] {name:36s} {row}", flush=True)


import os  # noqa: E402
CONV = os.environ.get("SWEEP", "dense,conv").find("conv") >= 0
DENSE = os.environ.get("SWEEP", "dense,conv").find("dense") >= 0
for imgs in [int(x) for x in sys.argv[1:]] or [32, 4]:
    run(imgs)
