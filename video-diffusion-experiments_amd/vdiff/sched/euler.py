"""EulerDiscreteScheduler — drop-in for diffusers:EulerDiscreteScheduler as the reference
configures it (experiments/01_baseline_generation.py:76-80 and
experiments/03_trace_forward_pass.py:51-55: `EulerDiscreteScheduler.from_config(
pipe.scheduler.config, timestep_spacing="linspace", beta_schedule="linear")`;
SURVEY.md §8f rank 2), epsilon prediction, s_churn = 0 (the pipeline's defaults).

Host side (numpy, once per video): sigma table sqrt((1 - a_bar) / a_bar) interpolated
at the (float) inference timesteps, a trailing 0, and the per-step coefficient table
{sigma_i, sigma_{i+1}, sqrt(sigma_{i+1}^2 + 1), 0}.  Device side: `step()` runs the
fused HIP kernel vd_euler_cfg_step; the pipeline's captured graph reads the same
coefficient table by a device step counter and its kernel also writes the next
step's `scale_model_input` (x / sqrt(sigma^2 + 1)) as the packed bf16 UNet input.

Square roots of the tables are correctly rounded (`sqrt32`, via fp64).  This is a deliberate
divergence from diffusers, which takes torch fp32 `** 0.5` on the host CPU: on some hosts (the
round-3 build container) that is one ulp off on ~19 % of the 1000 training sigmas, so the
reference's own table depends on the host.  The correctly rounded table is host-independent;
the scheduler-table parity against diffusers is therefore UNPINNED at the 1-ulp level, and
tests/test_oracle.py bounds the difference from the `** 0.5` form at 1 ulp.
"""
from __future__ import annotations

from collections import namedtuple

import numpy as np
import torch

from .. import ops
from .ddim import DEFAULT_CONFIG as _SD15, _Cfg, sqrt32

EulerDiscreteSchedulerOutput = namedtuple("EulerDiscreteSchedulerOutput", ["prev_sample", "pred_original_sample"])

# SD-1.5's scheduler_config.json fields EulerDiscreteScheduler reads, plus its own defaults.
DEFAULT_CONFIG = dict(
    num_train_timesteps=_SD15["num_train_timesteps"],
    beta_start=_SD15["beta_start"],
    beta_end=_SD15["beta_end"],
    beta_schedule=_SD15["beta_schedule"],
    trained_betas=None,
    prediction_type="epsilon",
    interpolation_type="linear",
    use_karras_sigmas=False,
    timestep_spacing="linspace",
    timestep_type="discrete",
    steps_offset=_SD15["steps_offset"],
    rescale_betas_zero_snr=False,
    final_sigmas_type="zero",
)


class EulerDiscreteScheduler:
    order = 1
    kind = "euler"

    def __init__(self, **kwargs):
        cfg = dict(DEFAULT_CONFIG)
        cfg.update({k: v for k, v in kwargs.items() if k in cfg})
        self.config = _Cfg(cfg)
        n = cfg["num_train_timesteps"]
        if cfg["trained_betas"] is not None:
            betas = torch.tensor(cfg["trained_betas"], dtype=torch.float32)
        elif cfg["beta_schedule"] == "linear":
            betas = torch.linspace(cfg["beta_start"], cfg["beta_end"], n, dtype=torch.float32)
        elif cfg["beta_schedule"] == "scaled_linear":
            betas = torch.linspace(cfg["beta_start"] ** 0.5, cfg["beta_end"] ** 0.5, n, dtype=torch.float32) ** 2
        else:
            raise NotImplementedError(cfg["beta_schedule"])
        if (cfg["prediction_type"] != "epsilon" or cfg["use_karras_sigmas"] or cfg["rescale_betas_zero_snr"]
                or cfg["interpolation_type"] != "linear" or cfg["final_sigmas_type"] != "zero"):
            raise NotImplementedError("only the SD-1.5 epsilon / linear-interpolation configuration the "
                                      "reference runs")
        self.betas = betas
        self.alphas = 1.0 - betas
        self.alphas_cumprod = torch.cumprod(self.alphas, dim=0)
        sig = sqrt32((1 - self.alphas_cumprod) / self.alphas_cumprod).numpy()
        self._sigmas_train = sig
        # diffusers' __init__ state (before set_timesteps): the full training schedule
        self.sigmas = torch.from_numpy(np.concatenate([sig[::-1], [0.0]]).astype(np.float32))
        self.timesteps = torch.from_numpy(np.linspace(0, n - 1, n, dtype=np.float32)[::-1].copy())
        self.num_inference_steps = None
        self._step_index = None
        self._begin_index = None

    @classmethod
    def from_config(cls, config, **kwargs):
        base = dict(config) if config is not None else {}
        base.update(kwargs)
        return cls(**base)

    @property
    def init_noise_sigma(self):
        m = float(self.sigmas.max())
        if self.config.timestep_spacing in ("linspace", "trailing"):
            return m
        return (m ** 2 + 1) ** 0.5

    @property
    def step_index(self):
        return self._step_index

    def set_begin_index(self, begin_index: int = 0):
        self._begin_index = begin_index

    def set_timesteps(self, num_inference_steps: int, device=None):
        n = self.config.num_train_timesteps
        self.num_inference_steps = num_inference_steps
        sp = self.config.timestep_spacing
        if sp == "linspace":
            ts = np.linspace(0, n - 1, num_inference_steps, dtype=np.float32)[::-1].copy()
        elif sp == "leading":
            ratio = n // num_inference_steps
            ts = (np.arange(0, num_inference_steps) * ratio).round()[::-1].copy().astype(np.float32)
            ts += self.config.steps_offset
        elif sp == "trailing":
            ratio = n / num_inference_steps
            ts = (np.arange(n, 0, -ratio)).round().copy().astype(np.float32) - 1
        else:
            raise ValueError(sp)
        sig = np.interp(ts, np.arange(0, len(self._sigmas_train)), self._sigmas_train)
        sig = np.concatenate([sig, [0.0]]).astype(np.float32)
        self.sigmas = torch.from_numpy(sig)
        self.timesteps = torch.from_numpy(ts.astype(np.float32)).to(device)
        self._step_index = None
        self._begin_index = None

    def index_for_timestep(self, timestep, schedule_timesteps=None):
        st = self.timesteps if schedule_timesteps is None else schedule_timesteps
        idx = (st.cpu() == float(timestep)).nonzero()
        if len(idx) == 0:
            raise ValueError(f"timestep {float(timestep)} is not in the schedule")
        return int(idx[1 if len(idx) > 1 else 0])  # diffusers: the second match for img2img restarts

    def _init_step_index(self, timestep):
        self._step_index = self.index_for_timestep(timestep) if self._begin_index is None else self._begin_index

    def input_divisor(self, i: int) -> float:
        """scale_model_input's divisor at step i: (sigma_i^2 + 1) ** 0.5 in fp32 torch math."""
        s = self.sigmas[i]
        return float(sqrt32(s ** 2 + 1))

    def scale_model_input(self, sample, timestep):
        if self._step_index is None:
            self._init_step_index(timestep)
        return sample / self.input_divisor(self._step_index)

    def coefficients(self, i: int) -> torch.Tensor:
        """fp32 {sigma_i, sigma_{i+1}, sqrt(sigma_{i+1}^2 + 1), 0} for step index i (the last
        step's next-input divisor is that of sigma = 0, i.e. 1)."""
        s, sn = self.sigmas[i], self.sigmas[i + 1]
        return torch.stack([s, sn, sqrt32(sn ** 2 + 1), torch.zeros(())]).float()

    def coefficient_table(self, timesteps=None) -> torch.Tensor:
        """Rows for the given schedule timesteps (default: the whole schedule), indexed by
        the pipeline's device step counter; a timestep repeated past the schedule (the
        benchmark replays it) maps back onto its schedule position."""
        ts = self.timesteps if timesteps is None else torch.as_tensor(timesteps)
        pos = {float(t): i for i, t in enumerate(self.timesteps.cpu().tolist())}
        return torch.stack([self.coefficients(pos[float(t)]) for t in ts.cpu().tolist()])

    def step(self, model_output, timestep, sample, s_churn: float = 0.0, s_tmin: float = 0.0,
             s_tmax: float = float("inf"), s_noise: float = 1.0, generator=None, return_dict: bool = True):
        if self.num_inference_steps is None:
            raise ValueError("call set_timesteps() first")
        if s_churn != 0.0:
            raise NotImplementedError("s_churn > 0 (the reference pipeline runs s_churn = 0)")
        if not (model_output.is_cuda and sample.is_cuda):
            raise ValueError("EulerDiscreteScheduler.step runs the HIP kernel; tensors must be on the GPU")
        if self._step_index is None:
            self._init_step_index(timestep)
        coef = self.coefficients(self._step_index).to(sample.device)
        x = sample.float().contiguous().clone()
        eps = model_output.float().contiguous()
        x0 = torch.empty_like(x)
        flat = lambda t: t.view(1, 1, 1, 1, t.numel())  # noqa: E731  elementwise view
        ops.euler_cfg_step(eps.view(-1, 1), 1, 1.0, flat(x), coef, x0_out=flat(x0))
        self._step_index += 1
        prev = x.to(model_output.dtype)
        if not return_dict:
            return (prev,)
        return EulerDiscreteSchedulerOutput(prev_sample=prev, pred_original_sample=x0)

    def __len__(self):
        return self.config.num_train_timesteps

