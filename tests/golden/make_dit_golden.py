"""Generate tests/golden/dit_tiny.npz (CPU only, in the build container):

    python tests/golden/make_dit_golden.py

The build-defined DiT denoiser (oracle/dit_ref.py) at its tiny
config: synthetic weights init_dit_state_dict(DIT_TINY, seed 0) (bf16-rounded N(0, 0.02^2)),
latents randn seed 42 (1, 4, 4, 16, 16), text embeddings randn seed 1 (2, 77, 64), CFG
batch cat([x, x]); oracle eps at t in {961, 500}, and a 3-step CFG DDIM loop (50-step
schedule, guidance 7.5).  Parity of the DiT itself is unpinned: the reference has no DiT.
"""
import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]

from oracle import ddim_ref, dit_ref  # noqa: E402
from vdiff.models.dit import DIT_TINY, init_dit_state_dict  # noqa: E402


def main():
    torch.manual_seed(0)
    sd = init_dit_state_dict(DIT_TINY, seed=0)
    lat = torch.randn((1, 4, 4, 16, 16), generator=torch.Generator().manual_seed(42))
    ehs = torch.randn((2, 77, 64), generator=torch.Generator().manual_seed(1))
    fn = lambda x, t, e: dit_ref.forward(sd, DIT_TINY, x, t, e)
    out = {"latents": lat.numpy(), "ehs": ehs.numpy(),
           "weight_checksum": np.array(sum(float(v.double().sum()) for v in sd.values()))}
    for t in (961, 500):
        out[f"eps_t{t}"] = fn(torch.cat([lat, lat]), t, ehs).numpy()
    acp = ddim_ref.alphas_cumprod()
    out["loop3_x"] = ddim_ref.denoise_loop(fn, lat, ehs, 50, 7.5, acp, steps=3).numpy()
    np.savez_compressed(HERE / "dit_tiny.npz", **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
