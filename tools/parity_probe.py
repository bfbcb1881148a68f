"""Block-by-block parity probe of the fused path vs the oracle (tiny config); the logic
lives in tests/parity_blocks.py (also used by tests/test_gpu_unet.py).

    python tools/parity_probe.py
"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd"), str(ROOT / "tests")]

from parity_blocks import block_errors  # noqa: E402
from vdiff import UNetMotionModel, init_synthetic_  # noqa: E402

if __name__ == "__main__":
    gold = np.load(ROOT / "tests" / "golden" / "tiny_unet.npz")
    unet = init_synthetic_(UNetMotionModel("tiny"), seed=0).to("cuda", torch.bfloat16).prepare()
    with torch.no_grad():
        block_errors(unet, torch.from_numpy(gold["latents"]), torch.from_numpy(gold["ehs"]), log=print)
