"""Generate tests/golden/full_f16_t500.npz (CPU only, in the build container; ~minutes):

    python tests/golden/make_full_golden.py

BASELINE config 3 at its full workload shape, one UNet forward: the FULL UNetMotionModel
(SD-1.5 + motion-adapter-v1-5-2 shapes, 1.31B parameters) with synthetic weights
init_synthetic_(seed 0) drawn on the CPU generator (bf16-rounded N(0, 0.02^2)), F = 16
frames, CFG batch cat([x, x]) of latents randn seed 42 (1, 4, 16, 64, 64), text embeddings
randn seed 1 (2, 77, 768), both bf16-rounded (the device stores its inputs in bf16), t = 500.
Stored: eps of the fp32 oracle ("eps") and of the oracle emulating the device's storage and
attention arithmetic (act="dev", "eps_dev"), as fp32.  The motion modules see all 16 frames
(the reference's num_frames=16, experiments/05_grid_search_ablation.py:48).
"""
import sys
import time
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]

from oracle import unet_ref  # noqa: E402
from vdiff.config import get_config  # noqa: E402
from vdiff.models import UNetMotionModel  # noqa: E402
from vdiff.weights import init_synthetic_  # noqa: E402

FRAMES, T = 16, 500


def full_inputs(frames=FRAMES):
    lat = torch.randn((1, 4, frames, 64, 64), generator=torch.Generator().manual_seed(42))
    ehs = torch.randn((2, 77, 768), generator=torch.Generator().manual_seed(1))
    return lat.to(torch.bfloat16).float(), ehs.to(torch.bfloat16).float()


def main():
    torch.manual_seed(0)
    m = init_synthetic_(UNetMotionModel("full"), seed=0)
    sd = {k: v.float() for k, v in m.state_dict().items()}
    del m
    lat, ehs = full_inputs()
    x = torch.cat([lat, lat])
    out = {}
    with torch.no_grad():
        for key, act in (("eps", "fp32"), ("eps_dev", "dev")):
            t0 = time.time()
            out[key] = unet_ref.unet_forward(sd, get_config("full"), x, T, ehs, act=act).numpy()
            print(f"{key}: {time.time() - t0:.1f} s", flush=True)
    np.savez_compressed(HERE / "full_f16_t500.npz", **out)
    e = torch.from_numpy(out["eps"]).double()
    d = torch.from_numpy(out["eps_dev"]).double()
    print("dev-vs-fp32 rel-L2", ((d - e).norm() / e.norm()).item())


if __name__ == "__main__":
    main()
