"""Seeded synthetic weights and diffusers-format weight loading.

No checkpoints are reachable offline, so benchmarks and parity tests use:
torch.manual_seed(seed) CPU generator, every Linear/Conv weight and every bias
~ N(0, std^2); GroupNorm/LayerNorm gamma = 1 + N(0, std^2), beta ~ N(0, std^2);
all values rounded to bf16 once so the CPU oracle and the GPU path see
identical numbers.  `proj_out` is NOT zeroed (AnimateDiff's training init
would hide the motion path).
"""
from __future__ import annotations

from pathlib import Path

import torch
import torch.nn as nn


@torch.no_grad()
def init_synthetic_(model: nn.Module, seed: int = 0, std: float = 0.02, device="cpu") -> nn.Module:
    """device="cpu" is the reproducible reference stream (tests, fixtures);
    device="cuda" draws from the GPU generator (fast setup for benchmarks;
    different values, same distribution)."""
    g = torch.Generator(device=device).manual_seed(seed)
    norms = {id(m) for m in model.modules() if isinstance(m, (nn.GroupNorm, nn.LayerNorm))}
    owner = {}
    for m in model.modules():
        for n, p in m.named_parameters(recurse=False):
            owner[id(p)] = (m, n)
    for _, p in model.named_parameters():
        m, leaf = owner[id(p)]
        r = torch.randn(p.shape, generator=g, device=device) * std
        if id(m) in norms and leaf == "weight":
            r = r + 1.0
        p.copy_(r.to(torch.bfloat16).to(p.dtype))
    return model


def load_diffusers_state_dict(model: nn.Module, paths, strict: bool = True):
    """Load diffusers-keyed .safetensors files (UNet and/or motion adapter) into
    the model.  Keys are the diffusers parameter names the module tree mirrors."""
    from safetensors.torch import load_file

    sd = {}
    for p in ([paths] if isinstance(paths, (str, Path)) else paths):
        sd.update(load_file(str(p)))
    sd = {k: v for k, v in sd.items() if not k.endswith(".pos_embed.pe")}
    missing, unexpected = model.load_state_dict(sd, strict=False)
    missing = [k for k in missing if not k.endswith(".pos_embed.pe")]
    if strict and (missing or unexpected):
        raise KeyError(f"state dict mismatch: missing={missing[:8]} unexpected={unexpected[:8]}")
    if getattr(model, "_prepared", False):
        model.prepare()
    return missing, unexpected


def materialize_synthetic(config="full", device="cuda", dtype=torch.bfloat16, seed: int = 0):
    """Build a UNetMotionModel directly on `device` (meta -> to_empty -> buffers
    recomputed -> GPU-seeded synthetic weights): seconds for the 1.31B-param
    full config, no 5 GB fp32 CPU copy."""
    from .models import UNetMotionModel
    from .models.layers import SinusoidalPositionalEmbedding

    with torch.device("meta"):
        m = UNetMotionModel(config)
    m = m.to_empty(device=device)
    for mod in m.modules():
        if isinstance(mod, SinusoidalPositionalEmbedding):
            mod.reset_buffers()
    m = m.to(dtype=dtype)
    init_synthetic_(m, seed=seed, device=device)
    return m
