"""Structural known-answers of the reference (CPU).

The reference publishes, for the SD-1.5 + motion-adapter-v1-5-2 UNet it loads
(experiments/02_architecture_inspection.py:38-60 -> docs/02_video_diffusion_
architecture.md:86-91): 1312.7M parameters (~860M SD-1.5 + ~450M motion), 639
"temporal-related" modules and 32 spatial Attention modules.  These pin the
module tree the HIP path and the oracle both follow.
"""
import torch

from vdiff.config import FULL, TINY, down_block_plan, up_block_plan
from vdiff.models import UNetMotionModel


def _meta(cfg):
    with torch.device("meta"):
        return UNetMotionModel(cfg)


def _inspection_counts(m):
    # the exact filters of experiments/02_architecture_inspection.py:51-60
    temporal, spatial = [], []
    for name, module in m.named_modules():
        t = type(module).__name__
        if "temporal" in name.lower() or "motion" in name.lower():
            temporal.append(name)
        elif "attn" in name.lower() and "temporal" not in name.lower():
            if t in ["Attention", "CrossAttention", "SelfAttention"]:
                spatial.append(name)
    return temporal, spatial


def test_full_param_count_matches_reference():
    m = _meta("full")
    total = sum(p.numel() for p in m.parameters())
    motion = sum(p.numel() for n, p in m.named_parameters() if "motion_modules" in n)
    assert total == 1_312_730_244          # "1312.7M" (docs/02:86)
    assert total - motion == 859_520_964   # SD-1.5 UNet ("~860M")
    assert motion == 453_209_280           # motion adapter ("~450M")


def test_full_module_counts_match_reference():
    temporal, spatial = _inspection_counts(_meta("full"))
    assert len(temporal) == 639
    assert len(spatial) == 32


def test_attention_naming_contract():
    # experiments/03_trace_forward_pass.py:134-139 classifies by these names
    m = _meta("full")
    att = [(n, mod) for n, mod in m.named_modules() if type(mod).__name__ == "Attention"]
    temporal = [n for n, _ in att if "motion_modules" in n]
    spatial = [n for n, _ in att if "attentions" in n]
    assert len(temporal) == 42 and len(spatial) == 32
    a = m.down_blocks[0].motion_modules[0].transformer_blocks[0].attn1
    assert a.heads == 8 and a.to_q.in_features == 320
    assert m.config.in_channels == 4 and m.config.sample_size == 64


def test_tiny_param_count():
    m = _meta("tiny")
    total = sum(p.numel() for p in m.parameters())
    motion = sum(p.numel() for n, p in m.named_parameters() if "motion_modules" in n)
    assert (total, total - motion, motion) == (4_879_556, 3_152_644, 1_726_912)


def test_channel_plans():
    # SURVEY.md App. A.1 up-block table
    assert [ins for _, ins, _, _ in up_block_plan(FULL)] == [
        [2560, 2560, 2560], [2560, 2560, 1920], [1920, 1280, 960], [960, 640, 640]]
    assert [ins for _, ins, _, _ in down_block_plan(FULL)] == [[320, 320], [320, 640], [640, 1280], [1280, 1280]]
    assert [ins for _, ins, _, _ in up_block_plan(TINY)] == [[256, 192], [192, 128]]


def test_state_dict_keys_are_diffusers_names():
    sd = _meta("full").state_dict()
    for k in ["conv_in.weight", "time_embedding.linear_1.weight",
              "down_blocks.0.resnets.0.norm1.weight", "down_blocks.0.resnets.0.time_emb_proj.bias",
              "down_blocks.0.attentions.0.transformer_blocks.0.attn2.to_k.weight",
              "down_blocks.0.attentions.0.transformer_blocks.0.ff.net.0.proj.weight",
              "down_blocks.0.motion_modules.0.transformer_blocks.0.pos_embed.pe",
              "down_blocks.0.downsamplers.0.conv.weight", "up_blocks.0.resnets.0.conv_shortcut.weight",
              "up_blocks.0.upsamplers.0.conv.weight", "mid_block.motion_modules.0.proj_out.bias",
              "conv_norm_out.weight", "conv_out.bias"]:
        assert k in sd, k
    assert "up_blocks.3.upsamplers.0.conv.weight" not in sd
    assert "down_blocks.3.downsamplers.0.conv.weight" not in sd


def test_vae_decoder_tree():
    """SD-1.5 AutoencoderKL decode side: the decoder + post_quant_conv
    of the public SD-1.5 vae/config.json.  49,490,199 = 83,653,863 (SD-1.5 VAE total, public)
    - 34,163,592 (encoder) - 72 (quant_conv); not a reference-published number, so a
    consistency check of the tree rather than a parity pin."""
    from vdiff.models.vae import AutoencoderKL
    with torch.device("meta"):
        m = AutoencoderKL("full")
    assert sum(p.numel() for p in m.parameters()) == 49_490_199
    keys = set(m.state_dict())
    for k in ("post_quant_conv.weight", "decoder.conv_in.weight",
              "decoder.mid_block.attentions.0.group_norm.weight", "decoder.mid_block.attentions.0.to_out.0.bias",
              "decoder.mid_block.resnets.1.conv2.weight", "decoder.up_blocks.0.upsamplers.0.conv.weight",
              "decoder.up_blocks.2.resnets.0.conv_shortcut.weight", "decoder.up_blocks.3.resnets.2.norm2.bias",
              "decoder.conv_norm_out.weight", "decoder.conv_out.bias"):
        assert k in keys, k
    assert not any(k.startswith("decoder.up_blocks.3.upsamplers") for k in keys)
    assert m.decoder.mid_block.attentions[0].heads == 1
