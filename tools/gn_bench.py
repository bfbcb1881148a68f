"""GroupNorm paths at the UNet's image-norm shapes: two-launch (per-group records, finalize in
the apply prologue) vs partial/finalize/apply.  python tools/gn_bench.py [--variant NAME,...]
(--variant: the two-launch path under the product library and under each diagnostic build of
tools/variant_ab.py, in one process)."""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd"), str(ROOT / "tools")]
import torch  # noqa: E402

from vdiff import _lib as L  # noqa: E402
from vdiff import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--variant", default="")
args = ap.parse_args()
arms = [("two-launch", True, L.lib()), ("four-launch", False, L.lib())]
if args.variant:
    from variant_ab import load_variant
    arms = [("base", True, L.lib())] + [(n, True, load_variant(n)) for n in args.variant.split(",")]

# (instances, pixels per instance, channels, motion-norm splits or 0 for an image norm)
SHAPES = [(32, 4096, 320, 0), (32, 1024, 640, 0), (32, 256, 1280, 0), (32, 64, 1280, 0), (32, 64, 2560, 0),
          (4, 4096, 320, 0), (4, 1024, 640, 0), (4, 256, 1280, 0), (4, 64, 2560, 0),
          (2, 16 * 4096, 320, 256), (2, 16 * 1024, 640, 256), (2, 2 * 4096, 320, 32), (2, 2 * 1024, 640, 32),
          (2, 2 * 256, 1280, 32)]
for n_inst, pix, C, msplit in SHAPES:
    x = torch.randn(n_inst * pix, C, device="cuda").to(torch.bfloat16)
    g, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
    res, outs = [], []
    for _, tp, h in arms:
        L._lib = h
        f = lambda: ops.group_norm(x, n_inst, pix, 32, 1e-5, g, b, silu=not msplit, two_pass=tp and not msplit,  # noqa: E731
                                   n_split=msplit or None)
        outs.append(f())
        for _ in range(3):
            f()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(20):
                f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        graph.replay()
        e0.record()
        graph.replay()
        e1.record()
        e1.synchronize()
        res.append(e0.elapsed_time(e1) / 20 * 1e3)
    L._lib = arms[0][2]
    diff = max((o.float() - outs[0].float()).abs().max().item() for o in outs)
    print(f"inst={n_inst:3d} pix={pix:5d} C={C:5d} {'motion' if msplit else 'image '} " + "   ".join(f"{a[0]} {t:7.1f} us" for a, t in zip(arms, res))
          + f"   max |diff| {diff:.2e}", flush=True)
