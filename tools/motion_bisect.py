"""Sub-block parity bisect of the FULL model's motion modules.

The full model runs on a 2-frame CFG batch (the 8-way rank's shapes, as
tests/test_gpu_unet.py::test_full_blocks_match_device_emulation); the named motion modules'
inputs are captured from the fused path, then tests/parity_blocks.py::motion_stages re-runs each
stage (GroupNorm, proj_in, the folded norm+PE QKV GEMM or fused QKV attention, the temporal
attention, to_out + residual, ..., ff2 + residual, proj_out + residual) FROM THE DEVICE'S OWN
INPUT to that stage against fp64 of the same stage ("emu": rounded where the device stores).
Then motion_floor: the whole block against the device-emulating oracle, and that oracle against
itself with 2e-4 of every stage's stored values moved by one ulp (its bf16 realisation floor).

    python tools/motion_bisect.py [frames] [module ...]   (frames: 2 = the 8-way rank's shapes, default)
"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd"), str(ROOT / "tests")]

from parity_blocks import motion_floor, motion_stages, nchw, rel  # noqa: E402
from vdiff.weights import materialize_synthetic  # noqa: E402


def main(names, frames=2):
    torch.manual_seed(0)
    unet = materialize_synthetic("full", device="cuda", seed=0)
    unet.prepare()
    mods = dict(unet.named_modules())
    caps = {}
    for nm in names:
        mm = mods[nm]

        def run(x, ctx, _nm=nm, _orig=mm.run):
            caps[_nm] = (x, ctx)
            return _orig(x, ctx)
        mm.run = run
    g = torch.Generator().manual_seed(42)
    lat = torch.randn((1, 4, frames, 64, 64), generator=g).to(torch.bfloat16).float()
    ehs = torch.randn((2, 77, 768), generator=torch.Generator().manual_seed(1)).to(torch.bfloat16).float()
    with torch.no_grad():
        unet(torch.cat([lat, lat]).cuda(), 500, encoder_hidden_states=ehs.cuda())
        for nm in names:
            mm = mods[nm]
            del mm.run
            x, ctx = caps[nm]
            print(f"== {nm}: rows {x.t.shape[0]}, C {x.t.shape[1]}, batch {ctx.batch}, frames {ctx.frames}", flush=True)
            motion_stages(mm, x, ctx, log=print)
            got = nchw(mm.run(x, ctx))
            d0, d1, f0 = motion_floor(unet, nm, x, ctx.frames)
            print(f"  block: device vs dev-oracle {rel(got, d0):.5f}, device vs fp32 {rel(got, f0):.5f}, "
                  f"dev-oracle vs fp32 {rel(d0, f0):.5f}; floor (dev-oracle with 2e-4 ulp flips per store) {rel(d1, d0):.5f}",
                  flush=True)


if __name__ == "__main__":
    args = sys.argv[1:]
    nf = int(args.pop(0)) if args and args[0].isdigit() else 2
    main(args or ["down_blocks.2.motion_modules.0", "down_blocks.2.motion_modules.1",
                          "up_blocks.1.motion_modules.0", "down_blocks.1.motion_modules.0",
                          "down_blocks.0.motion_modules.0", "up_blocks.3.motion_modules.2"], nf)
