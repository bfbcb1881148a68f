"""UNetMotionModel configurations (diffusers-style config dicts).

FULL is SD-1.5 + `guoyww/animatediff-motion-adapter-v1-5-2`, the model the
reference loads at experiments/05_grid_search_ablation.py:124-134 (SURVEY.md
App. A.0).  TINY is the build-defined parity-gate instance of the same class
(BASELINE config 1).
"""
from __future__ import annotations

import copy

FULL = dict(
    in_channels=4,
    out_channels=4,
    sample_size=64,
    block_out_channels=(320, 640, 1280, 1280),
    layers_per_block=2,
    down_block_types=("CrossAttnDownBlockMotion",) * 3 + ("DownBlockMotion",),
    up_block_types=("UpBlockMotion",) + ("CrossAttnUpBlockMotion",) * 3,
    norm_num_groups=32,
    norm_eps=1e-5,
    cross_attention_dim=768,
    num_attention_heads=8,
    motion_num_attention_heads=8,
    motion_max_seq_length=32,
    use_motion_mid_block=True,
)

TINY = dict(
    in_channels=4,
    out_channels=4,
    sample_size=64,
    block_out_channels=(64, 128),
    layers_per_block=1,
    down_block_types=("CrossAttnDownBlockMotion", "DownBlockMotion"),
    up_block_types=("UpBlockMotion", "CrossAttnUpBlockMotion"),
    norm_num_groups=32,
    norm_eps=1e-5,
    cross_attention_dim=64,
    num_attention_heads=2,
    motion_num_attention_heads=2,
    motion_max_seq_length=32,
    use_motion_mid_block=True,
)

CONFIGS = {"full": FULL, "tiny": TINY}


def get_config(name_or_cfg) -> dict:
    if isinstance(name_or_cfg, dict):
        return copy.deepcopy(name_or_cfg)
    return copy.deepcopy(CONFIGS[name_or_cfg])


def up_block_plan(cfg: dict):
    """Per up block: (out_channels, [resnet in_channels...], has_attn, add_upsample).

    Mirrors UNetMotionModel.__init__'s up-block channel arithmetic
    (up0 2560x3, up1 2560,2560,1920, ...).
    """
    boc = list(cfg["block_out_channels"])
    rev = boc[::-1]
    n = len(rev)
    nl = cfg["layers_per_block"] + 1
    out_ch = rev[0]
    plan = []
    for i, bt in enumerate(cfg["up_block_types"]):
        prev = out_ch
        out_ch = rev[i]
        in_ch = rev[min(i + 1, n - 1)]
        ins = []
        for j in range(nl):
            skip = in_ch if j == nl - 1 else out_ch
            rin = prev if j == 0 else out_ch
            ins.append(rin + skip)
        plan.append((out_ch, ins, bt.startswith("CrossAttn"), i != n - 1))
    return plan


def down_block_plan(cfg: dict):
    """Per down block: (out_channels, [resnet in_channels...], has_attn, add_downsample)."""
    boc = list(cfg["block_out_channels"])
    n = len(boc)
    plan = []
    out_ch = boc[0]
    for i, bt in enumerate(cfg["down_block_types"]):
        in_ch = out_ch
        out_ch = boc[i]
        ins = [in_ch if j == 0 else out_ch for j in range(cfg["layers_per_block"])]
        plan.append((out_ch, ins, bt.startswith("CrossAttn"), i != n - 1))
    return plan
