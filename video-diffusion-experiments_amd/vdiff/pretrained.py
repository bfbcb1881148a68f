"""Local diffusers-layout checkpoints: `MotionAdapter.from_pretrained` and
`AnimateDiffPipeline.from_pretrained` as the reference calls them
(experiments/05_grid_search_ablation.py:121-147, also 01:60-75, 02:17-30, 03:39-50):

    adapter = MotionAdapter.from_pretrained(<adapter dir>, torch_dtype=...)
    pipe = AnimateDiffPipeline.from_pretrained(<sd-1.5 dir>, motion_adapter=adapter, torch_dtype=...)
    pipe.scheduler = DDIMScheduler.from_config(pipe.scheduler.config, beta_schedule="linear", ...)

There is no network here, so the model names of the reference become local directory paths
with diffusers' own layout: `<adapter>/config.json` + `diffusion_pytorch_model[.<variant>].
safetensors` (or a `.safetensors.index.json` shard index); `<pipe>/unet/`, `<pipe>/vae/` (same
files) and `<pipe>/scheduler/scheduler_config.json`.  The UNet checkpoint holds the SD-1.5
UNet2DConditionModel keys and the adapter the `*.motion_modules.*` keys; diffusers'
UNetMotionModel.from_unet2d joins the two under exactly those names, which are the names of
vdiff.UNetMotionModel's parameters, so the join is a dict union.  The adapter's
`pos_embed.pe` buffers are recomputed (they are fixed sinusoids).  The VAE's encoder half
(`encoder.*`, `quant_conv.*`) is not on the text-to-video path and is skipped.  Weights are
stored in bf16 on the device: the kernels compute in bf16, whatever `torch_dtype` the caller
passes (the reference's float16 is recorded in `.torch_dtype`).
"""
from __future__ import annotations

import json
from pathlib import Path

import torch

from .config import get_config

WEIGHTS_NAME = "diffusion_pytorch_model"
_DOWN = {"CrossAttnDownBlock2D": "CrossAttnDownBlockMotion", "DownBlock2D": "DownBlockMotion",
         "CrossAttnDownBlockMotion": "CrossAttnDownBlockMotion", "DownBlockMotion": "DownBlockMotion"}
_UP = {"CrossAttnUpBlock2D": "CrossAttnUpBlockMotion", "UpBlock2D": "UpBlockMotion",
       "CrossAttnUpBlockMotion": "CrossAttnUpBlockMotion", "UpBlockMotion": "UpBlockMotion"}


def _local_dir(path, what: str) -> Path:
    p = Path(path)
    if not p.is_dir():
        raise FileNotFoundError(f"{what}: {path!r} is not a local directory (hub checkpoints are "
                                "unreachable offline: pass a diffusers-layout directory)")
    return p


def read_json(path: Path) -> dict:
    with open(path) as f:
        return json.load(f)


def load_weights(folder: Path, variant=None) -> dict:
    """All tensors of a diffusers model folder: `diffusion_pytorch_model[.variant].safetensors`
    or its sharded form (`….safetensors.index.json` naming the shard files)."""
    from safetensors.torch import load_file

    stem = WEIGHTS_NAME + (f".{variant}" if variant else "")
    single = folder / f"{stem}.safetensors"
    index = folder / f"{stem}.safetensors.index.json"
    if single.exists():
        return load_file(str(single))
    if index.exists():
        sd = {}
        for shard in sorted(set(read_json(index)["weight_map"].values())):
            sd.update(load_file(str(folder / shard)))
        return sd
    raise FileNotFoundError(f"no {stem}.safetensors (or its .index.json) in {folder}")


class MotionAdapter:
    """diffusers.MotionAdapter as the reference uses it: a config plus the motion-module weights
    (`down_blocks.i.motion_modules.j.*`, `up_blocks.i.motion_modules.j.*`,
    `mid_block.motion_modules.0.*`) that AnimateDiffPipeline.from_pretrained joins to the UNet."""

    def __init__(self, config: dict, state_dict: dict, torch_dtype=None):
        self.config = dict(config)
        self.torch_dtype = torch_dtype
        self._state = {k: v for k, v in state_dict.items() if not k.endswith(".pos_embed.pe")}
        bad = [k for k in self._state if ".motion_modules." not in k]
        if bad:
            raise KeyError(f"not motion-module keys: {bad[:4]}")

    @classmethod
    def from_pretrained(cls, path, torch_dtype=None, variant=None, **unused):
        d = _local_dir(path, "MotionAdapter.from_pretrained")
        return cls(read_json(d / "config.json"), load_weights(d, variant), torch_dtype)

    def state_dict(self) -> dict:
        return dict(self._state)


def motion_unet_config(unet_cfg: dict, adapter_cfg: dict) -> dict:
    """diffusers UNet2DConditionModel config.json + MotionAdapter config.json -> the
    vdiff.UNetMotionModel config (what UNetMotionModel.from_unet2d builds)."""
    boc = tuple(unet_cfg["block_out_channels"])
    heads = unet_cfg.get("num_attention_heads") or unet_cfg.get("attention_head_dim", 8)  # diffusers' legacy name
    if isinstance(heads, (list, tuple)):
        if len(set(heads)) != 1:
            raise NotImplementedError(f"per-block attention heads {heads}")
        heads = heads[0]
    lpb = unet_cfg.get("layers_per_block", 2)
    if isinstance(lpb, (list, tuple)):
        raise NotImplementedError("per-block layers_per_block")
    if tuple(adapter_cfg.get("block_out_channels", boc)) != boc:
        raise ValueError("motion adapter block_out_channels differ from the UNet's")
    if adapter_cfg.get("motion_layers_per_block", lpb) != lpb:
        raise NotImplementedError("motion_layers_per_block != the UNet's layers_per_block")
    if adapter_cfg.get("motion_norm_num_groups", unet_cfg.get("norm_num_groups", 32)) != unet_cfg.get("norm_num_groups", 32):
        raise NotImplementedError("motion_norm_num_groups != norm_num_groups")
    if adapter_cfg.get("conv_in_channels"):
        raise NotImplementedError("motion adapters with their own conv_in (PIA / SparseCtrl) are not on 05's path")
    cfg = get_config("full")
    cfg.update(
        in_channels=unet_cfg.get("in_channels", 4), out_channels=unet_cfg.get("out_channels", 4),
        sample_size=unet_cfg.get("sample_size", 64), block_out_channels=boc, layers_per_block=lpb,
        down_block_types=tuple(_DOWN[t] for t in unet_cfg["down_block_types"]),
        up_block_types=tuple(_UP[t] for t in unet_cfg["up_block_types"]),
        norm_num_groups=unet_cfg.get("norm_num_groups", 32), norm_eps=unet_cfg.get("norm_eps", 1e-5),
        cross_attention_dim=unet_cfg.get("cross_attention_dim", 768), num_attention_heads=heads,
        motion_num_attention_heads=adapter_cfg.get("motion_num_attention_heads", 8),
        motion_max_seq_length=adapter_cfg.get("motion_max_seq_length", 32),
        use_motion_mid_block=adapter_cfg.get("use_motion_mid_block", True),
    )
    return cfg


def vae_config(cfg: dict) -> dict:
    """diffusers AutoencoderKL config.json -> the vdiff.AutoencoderKL (decoder) config."""
    from .models.vae import VAE_FULL
    out = dict(VAE_FULL)
    for k in ("in_channels", "out_channels", "latent_channels", "layers_per_block", "norm_num_groups",
              "sample_size", "scaling_factor"):
        if cfg.get(k) is not None:
            out[k] = cfg[k]
    out["block_out_channels"] = tuple(cfg.get("block_out_channels", out["block_out_channels"]))
    return out


def _empty_on(cls, cfg, device):
    """Build on the meta device, then allocate on `device` (no fp32 CPU copy of 1.3B params)."""
    from .models.layers import SinusoidalPositionalEmbedding
    with torch.device("meta"):
        m = cls(cfg)
    m = m.to_empty(device=device)
    for mod in m.modules():
        if isinstance(mod, SinusoidalPositionalEmbedding):
            mod.reset_buffers()
    return m.to(dtype=torch.bfloat16)


@torch.no_grad()
def _assign(model, sd: dict, skip=lambda k: False, what="model"):
    own = model.state_dict()
    keep = {k: v for k, v in sd.items() if not skip(k) and not k.endswith(".pos_embed.pe")}
    missing = [k for k in own if k not in keep and not k.endswith(".pos_embed.pe")]
    unexpected = [k for k in keep if k not in own]
    if missing or unexpected:
        raise KeyError(f"{what}: state dict mismatch: missing={missing[:6]} unexpected={unexpected[:6]}")
    for k, v in keep.items():
        if tuple(own[k].shape) != tuple(v.shape):
            raise ValueError(f"{what}: {k} has shape {tuple(v.shape)}, the model {tuple(own[k].shape)}")
        own[k].copy_(v.to(own[k].dtype))
    return model


def load_unet_motion(unet_dir, adapter: MotionAdapter, device="cuda", variant=None):
    """UNetMotionModel.from_unet2d(unet, motion_adapter) over local files."""
    from .models import UNetMotionModel
    d = _local_dir(unet_dir, "unet")
    cfg = motion_unet_config(read_json(d / "config.json"), adapter.config)
    unet = _empty_on(UNetMotionModel, cfg, device)
    sd = load_weights(d, variant)
    clash = [k for k in adapter.state_dict() if k in sd]
    if clash:
        raise KeyError(f"UNet checkpoint already holds motion keys: {clash[:4]}")
    return _assign(unet, {**sd, **adapter.state_dict()}, what="UNetMotionModel")


def load_vae(vae_dir, device="cuda", variant=None):
    from .models.vae import AutoencoderKL
    d = _local_dir(vae_dir, "vae")
    vae = _empty_on(AutoencoderKL, vae_config(read_json(d / "config.json")), device)
    return _assign(vae, load_weights(d, variant), skip=lambda k: k.startswith(("encoder.", "quant_conv.")),
                   what="AutoencoderKL")


def load_scheduler(sched_dir):
    """The pipeline's scheduler from scheduler_config.json.  SD-1.5 ships PNDMScheduler, which the
    reference immediately replaces (05:136-141 DDIM, 01/03 Euler) from `pipe.scheduler.config`;
    DDIM / Euler configs build that class, anything else a DDIMScheduler holding the same config
    (its unknown keys are kept in `.config` so the reference's from_config(...) sees them)."""
    from .sched import DDIMScheduler, EulerDiscreteScheduler
    cfg = read_json(Path(sched_dir) / "scheduler_config.json")
    cls = EulerDiscreteScheduler if cfg.get("_class_name") == "EulerDiscreteScheduler" else DDIMScheduler
    s = cls.from_config({k: v for k, v in cfg.items() if not k.startswith("_")})
    s.source_config = cfg
    return s
