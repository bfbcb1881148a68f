"""ORACLE — test infrastructure only.  Never imported by the product path.

Restatement of `diffusers:DDIMScheduler` as the reference configures it at
experiments/05_grid_search_ablation.py:136-141 (`from_config(sd15_cfg,
beta_schedule="linear", steps_offset=1, clip_sample=False)`), with the DDIM
update of docs/01_diffusion_fundamentals.md:109-124 and the CFG combine of
docs/01_diffusion_fundamentals.md:176-186.

Pinned by the alpha-bar check values in SURVEY.md App. A.7 (fp32 cumprod);
parity to diffusers itself is unpinned (diffusers is not present).
"""
from __future__ import annotations

import numpy as np
import torch


def alphas_cumprod(num_train_timesteps=1000, beta_start=0.00085, beta_end=0.012, schedule="linear"):
    if schedule == "linear":
        betas = torch.linspace(beta_start, beta_end, num_train_timesteps, dtype=torch.float32)
    elif schedule == "scaled_linear":
        betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_train_timesteps,
                               dtype=torch.float32) ** 2
    else:
        raise ValueError(schedule)
    return torch.cumprod(1.0 - betas, dim=0)


def _sqrt(x):
    """fp32 sqrt, correctly rounded whatever the host's fp32 vector sqrt does (through fp64)."""
    return torch.sqrt(torch.as_tensor(x).double()).float()


def timesteps_leading(n, num_train_timesteps=1000, steps_offset=1):
    ratio = num_train_timesteps // n
    ts = (np.arange(0, n) * ratio).round()[::-1].copy().astype(np.int64)
    return ts + steps_offset


def ddim_step(eps, t, x, n_steps, acp, final_alpha_cumprod=None, num_train_timesteps=1000):
    """eta = 0 DDIM update, epsilon prediction (App. A.7)."""
    fa = acp[0] if final_alpha_cumprod is None else final_alpha_cumprod
    prev = t - num_train_timesteps // n_steps
    a_t = acp[t]
    a_p = acp[prev] if prev >= 0 else fa
    x0 = (x - _sqrt(1 - a_t) * eps) / _sqrt(a_t)
    return _sqrt(a_p) * x0 + _sqrt(1 - a_p) * eps, x0


def cfg_combine(eps2, g):
    """noise_pred_uncond + g * (noise_pred_text - noise_pred_uncond); uncond first."""
    u, c = eps2.chunk(2)
    return u + g * (c - u)


def denoise_loop(unet_fn, latents, ehs2, n_steps, guidance, acp, steps=None):
    """The AnimateDiffPipeline.__call__ loop body,
    run for `steps` iterations (default: all)."""
    ts = timesteps_leading(n_steps)
    x = latents.float()
    for i, t in enumerate(ts[: steps if steps is not None else n_steps]):
        x_in = torch.cat([x, x]) if guidance > 1 else x
        eps = unet_fn(x_in, int(t), ehs2)
        if guidance > 1:
            eps = cfg_combine(eps, guidance)
        x, _ = ddim_step(eps, int(t), x, n_steps, acp)
    return x
