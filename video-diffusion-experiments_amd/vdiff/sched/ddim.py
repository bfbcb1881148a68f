"""DDIMScheduler — drop-in for diffusers:DDIMScheduler as the reference uses it
(experiments/05_grid_search_ablation.py:136-141: `DDIMScheduler.from_config(
pipe.scheduler.config, beta_schedule="linear", steps_offset=1, clip_sample=False)`;
SURVEY.md App. A.7).

Host side (numpy/torch-CPU, once per video): beta/alpha tables, timestep
spacing, per-step coefficient table.  Device side: `step()` runs the fused
HIP kernel vd_ddim_cfg_step (fp32, in one HBM pass); the pipeline's captured
graph reads the same coefficient table by a device step counter.
"""
from __future__ import annotations

import math
from collections import namedtuple

import numpy as np
import torch

from .. import ops

DDIMSchedulerOutput = namedtuple("DDIMSchedulerOutput", ["prev_sample", "pred_original_sample"])

# SD-1.5's scheduler_config.json (the `pipe.scheduler.config` the reference
# overrides), with DDIMScheduler's own defaults for the remaining fields.
DEFAULT_CONFIG = dict(
    num_train_timesteps=1000,
    beta_start=0.00085,
    beta_end=0.012,
    beta_schedule="scaled_linear",
    trained_betas=None,
    clip_sample=False,
    set_alpha_to_one=False,
    steps_offset=1,
    prediction_type="epsilon",
    thresholding=False,
    clip_sample_range=1.0,
    timestep_spacing="leading",
    rescale_betas_zero_snr=False,
)


def sqrt32(x: torch.Tensor) -> torch.Tensor:
    """Correctly rounded fp32 square root (through fp64), i.e. what IEEE fp32 `x ** 0.5` gives.
    Some hosts' torch fp32 sqrt is off by one ulp on ~20 % of inputs, which would make the
    scheduler tables depend on the machine."""
    return torch.sqrt(x.double()).float()


class _Cfg(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


class DDIMScheduler:
    order = 1
    kind = "ddim"  # selects the fused device update (ops.SCHED_STEP)
    init_noise_sigma = 1.0

    def __init__(self, **kwargs):
        cfg = dict(DEFAULT_CONFIG)
        unknown = set(kwargs) - set(cfg)
        cfg.update({k: v for k, v in kwargs.items() if k in cfg})
        self.config = _Cfg(cfg)
        self._ignored = sorted(unknown)
        n = cfg["num_train_timesteps"]
        if cfg["trained_betas"] is not None:
            betas = torch.tensor(cfg["trained_betas"], dtype=torch.float32)
        elif cfg["beta_schedule"] == "linear":
            betas = torch.linspace(cfg["beta_start"], cfg["beta_end"], n, dtype=torch.float32)
        elif cfg["beta_schedule"] == "scaled_linear":
            betas = torch.linspace(cfg["beta_start"] ** 0.5, cfg["beta_end"] ** 0.5, n, dtype=torch.float32) ** 2
        elif cfg["beta_schedule"] == "squaredcos_cap_v2":
            f = lambda t: math.cos((t + 0.008) / 1.008 * math.pi / 2) ** 2  # noqa: E731
            betas = torch.tensor([min(1 - f((i + 1) / n) / f(i / n), 0.999) for i in range(n)],
                                 dtype=torch.float32)
        else:
            raise NotImplementedError(cfg["beta_schedule"])
        if cfg["rescale_betas_zero_snr"]:
            raise NotImplementedError("rescale_betas_zero_snr")
        if cfg["prediction_type"] != "epsilon" or cfg["thresholding"] or cfg["clip_sample"]:
            raise NotImplementedError("only epsilon prediction without clipping/thresholding "
                                      "(the SD-1.5 configuration the reference runs)")
        self.betas = betas
        self.alphas = 1.0 - betas
        self.alphas_cumprod = torch.cumprod(self.alphas, dim=0)
        self.final_alpha_cumprod = torch.tensor(1.0) if cfg["set_alpha_to_one"] else self.alphas_cumprod[0]
        self.num_inference_steps = None
        self.timesteps = torch.from_numpy(np.arange(0, n)[::-1].copy().astype(np.int64))

    @classmethod
    def from_config(cls, config, **kwargs):
        base = dict(config) if config is not None else {}
        base.update(kwargs)
        return cls(**base)

    def set_timesteps(self, num_inference_steps: int, device=None):
        n = self.config.num_train_timesteps
        if num_inference_steps > n:
            raise ValueError("num_inference_steps > num_train_timesteps")
        self.num_inference_steps = num_inference_steps
        sp = self.config.timestep_spacing
        if sp == "leading":
            ratio = n // num_inference_steps
            ts = (np.arange(0, num_inference_steps) * ratio).round()[::-1].copy().astype(np.int64)
            ts += self.config.steps_offset
        elif sp == "trailing":
            ratio = n / num_inference_steps
            ts = np.round(np.arange(n, 0, -ratio)).astype(np.int64) - 1
        elif sp == "linspace":
            ts = np.linspace(0, n - 1, num_inference_steps).round()[::-1].copy().astype(np.int64)
        else:
            raise ValueError(sp)
        self.timesteps = torch.from_numpy(ts).to(device)

    def scale_model_input(self, sample, timestep=None):
        return sample

    def _alphas(self, timestep):
        t = int(timestep)
        prev = t - self.config.num_train_timesteps // self.num_inference_steps
        a_t = self.alphas_cumprod[t]
        a_p = self.alphas_cumprod[prev] if prev >= 0 else self.final_alpha_cumprod
        return a_t, a_p

    def coefficients(self, timestep) -> torch.Tensor:
        """fp32 {sqrt(a_t), sqrt(1-a_t), sqrt(a_prev), sqrt(1-a_prev)}: diffusers' fp32 torch math
        with every square root correctly rounded (`sqrt32`)."""
        a_t, a_p = self._alphas(timestep)
        return torch.stack([sqrt32(a_t), sqrt32(1 - a_t), sqrt32(a_p), sqrt32(1 - a_p)]).float()

    def coefficient_table(self, timesteps=None) -> torch.Tensor:
        ts = self.timesteps if timesteps is None else timesteps
        return torch.stack([self.coefficients(t) for t in ts.tolist()])

    def step(self, model_output, timestep, sample, eta: float = 0.0, use_clipped_model_output=False,
             generator=None, variance_noise=None, return_dict: bool = True):
        if self.num_inference_steps is None:
            raise ValueError("call set_timesteps() first")
        if eta != 0.0:
            raise NotImplementedError("eta > 0 (the reference pipeline runs eta = 0)")
        if not (model_output.is_cuda and sample.is_cuda):
            raise ValueError("DDIMScheduler.step runs the HIP kernel; tensors must be on the GPU")
        coef = self.coefficients(timestep).to(sample.device)
        x = sample.float().contiguous().clone()
        eps = model_output.float().contiguous()
        x0 = torch.empty_like(x)
        flat = lambda t: t.view(1, 1, 1, 1, t.numel())  # noqa: E731  elementwise view
        ops.ddim_cfg_step(eps.view(-1, 1), 1, 1.0, flat(x), coef, x0_out=flat(x0))
        prev, x0 = x.to(sample.dtype), x0.to(sample.dtype)
        if not return_dict:
            return (prev,)
        return DDIMSchedulerOutput(prev_sample=prev, pred_original_sample=x0)
