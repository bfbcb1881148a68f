"""Local diffusers-layout checkpoints through the reference's own loading calls
(experiments/05_grid_search_ablation.py:121-147): MotionAdapter.from_pretrained +
AnimateDiffPipeline.from_pretrained(path, motion_adapter=, torch_dtype=) + the DDIM swap.

No checkpoint is reachable offline, so the test writes one: synthetic weights of the tiny
config under diffusers' key names and file layout — the SD UNet's keys in unet/, the motion
modules (with their pos_embed.pe buffers) in the adapter folder, the VAE with an encoder half
that the decoder-only AutoencoderKL must skip, SD-1.5's PNDM scheduler_config.json — then loads
it and requires every parameter bit-identical to the model the weights came from."""
import json

import pytest
import torch

import vdiff
from vdiff import AnimateDiffPipeline, AutoencoderKL, DDIMScheduler, MotionAdapter, UNetMotionModel, init_synthetic_
from safetensors.torch import save_file

UNET_CFG = {  # diffusers UNet2DConditionModel config.json of the tiny config (SD-1.5's keys)
    "_class_name": "UNet2DConditionModel", "act_fn": "silu", "attention_head_dim": 2,
    "block_out_channels": [64, 128], "cross_attention_dim": 64, "center_input_sample": False,
    "down_block_types": ["CrossAttnDownBlock2D", "DownBlock2D"], "downsample_padding": 1,
    "flip_sin_to_cos": True, "freq_shift": 0, "in_channels": 4, "layers_per_block": 1,
    "mid_block_scale_factor": 1, "norm_eps": 1e-05, "norm_num_groups": 32, "out_channels": 4,
    "sample_size": 64, "up_block_types": ["UpBlock2D", "CrossAttnUpBlock2D"]}
ADAPTER_CFG = {"_class_name": "MotionAdapter", "block_out_channels": [64, 128], "motion_layers_per_block": 1,
               "motion_mid_block_layers_per_block": 1, "motion_num_attention_heads": 2,
               "motion_norm_num_groups": 32, "motion_max_seq_length": 32, "use_motion_mid_block": True,
               "conv_in_channels": None}
VAE_CFG = {"_class_name": "AutoencoderKL", "act_fn": "silu", "block_out_channels": [64, 64], "in_channels": 3,
           "latent_channels": 4, "layers_per_block": 1, "norm_num_groups": 32, "out_channels": 3,
           "sample_size": 32, "scaling_factor": 0.18215}
PNDM_CFG = {"_class_name": "PNDMScheduler", "beta_end": 0.012, "beta_schedule": "scaled_linear",
            "beta_start": 0.00085, "num_train_timesteps": 1000, "set_alpha_to_one": False,
            "skip_prk_steps": True, "steps_offset": 1, "trained_betas": None, "clip_sample": False}


def _write(folder, cfg, sd, name="config.json"):
    folder.mkdir(parents=True, exist_ok=True)
    (folder / name).write_text(json.dumps(cfg))
    if sd is not None:
        save_file({k: v.contiguous() for k, v in sd.items()}, str(folder / "diffusion_pytorch_model.safetensors"))


@pytest.fixture(scope="module")
def checkpoint(tmp_path_factory):
    root = tmp_path_factory.mktemp("ckpt")
    unet = init_synthetic_(UNetMotionModel("tiny"), seed=0)
    vae = init_synthetic_(AutoencoderKL("tiny"), seed=1)
    sd = {k: v.float() for k, v in unet.state_dict().items()}
    motion = {k: v for k, v in sd.items() if ".motion_modules." in k}
    assert any(k.endswith(".pos_embed.pe") for k in motion)   # diffusers keeps the PE buffers
    _write(root / "adapter", ADAPTER_CFG, motion)
    _write(root / "sd" / "unet", UNET_CFG, {k: v for k, v in sd.items() if k not in motion})
    vsd = {k: v.float() for k, v in vae.state_dict().items()}
    vsd["encoder.conv_in.weight"] = torch.randn(64, 3, 3, 3)  # the encoder half: skipped
    vsd["quant_conv.weight"] = torch.randn(8, 8, 1, 1)
    _write(root / "sd" / "vae", VAE_CFG, vsd)
    _write(root / "sd" / "scheduler", PNDM_CFG, None, "scheduler_config.json")
    return root, unet, vae


def load_pipeline(adapter_path, pipe_path, device):
    """experiments/05_grid_search_ablation.py:121-147 with the hub names replaced by paths."""
    adapter = MotionAdapter.from_pretrained(adapter_path, torch_dtype=torch.float16)
    pipe = AnimateDiffPipeline.from_pretrained(pipe_path, motion_adapter=adapter, torch_dtype=torch.float16,
                                               device=device)
    pipe.scheduler = DDIMScheduler.from_config(pipe.scheduler.config, beta_schedule="linear", steps_offset=1,
                                               clip_sample=False)
    pipe.enable_vae_slicing()
    pipe.enable_model_cpu_offload()
    return pipe


def _bit_identical(model, want):
    got, ref = model.state_dict(), want.state_dict()
    assert set(got) == set(ref)
    for k, v in ref.items():
        assert torch.equal(got[k].cpu(), v.to(got[k].dtype)), k


def test_load_pipeline_round_trip_cpu(checkpoint):
    root, unet, vae = checkpoint
    pipe = load_pipeline(root / "adapter", root / "sd", "cpu")
    _bit_identical(pipe.unet, unet.to(torch.bfloat16))
    _bit_identical(pipe.vae, vae.to(torch.bfloat16))
    assert pipe.unet.config["num_attention_heads"] == 2 and pipe.unet.config["layers_per_block"] == 1
    assert pipe.torch_dtype == torch.float16
    s = pipe.scheduler  # the swap read the PNDM config's betas (scaled_linear -> linear override)
    assert s.config.beta_start == 0.00085 and s.config.beta_schedule == "linear" and s.config.steps_offset == 1


def test_from_pretrained_refuses_hub_names_and_bad_checkpoints(checkpoint, tmp_path):
    root, _, _ = checkpoint
    with pytest.raises(FileNotFoundError, match="local directory"):
        MotionAdapter.from_pretrained("guoyww/animatediff-motion-adapter-v1-5-2")
    adapter = MotionAdapter.from_pretrained(root / "adapter")
    with pytest.raises(FileNotFoundError, match="local directory"):
        AnimateDiffPipeline.from_pretrained("runwayml/stable-diffusion-v1-5", motion_adapter=adapter)
    with pytest.raises(ValueError, match="motion_adapter"):
        AnimateDiffPipeline.from_pretrained(root / "sd", device="cpu")
    # a UNet checkpoint with a parameter missing is refused, not half-loaded
    from safetensors.torch import load_file
    sd = load_file(str(root / "sd" / "unet" / "diffusion_pytorch_model.safetensors"))
    sd.pop("conv_in.weight")
    _write(tmp_path / "bad" / "unet", UNET_CFG, sd)
    with pytest.raises(KeyError, match="conv_in.weight"):
        vdiff.pretrained.load_unet_motion(tmp_path / "bad" / "unet", adapter, device="cpu")


@pytest.mark.gpu
def test_load_pipeline_round_trip_gpu_forward(checkpoint):
    """On the device: the loaded pipeline's UNet gives bit-identical eps to the model the
    checkpoint was written from (same weights, same kernels)."""
    root, unet, _ = checkpoint
    pipe = load_pipeline(root / "adapter", root / "sd", "cuda")
    ref = init_synthetic_(UNetMotionModel("tiny"), seed=0).to("cuda", torch.bfloat16).prepare()
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 4, 4, 64, 64, generator=g).cuda()
    ehs = torch.randn(2, 77, 64, generator=g).cuda()
    a = pipe.unet(x, 500, encoder_hidden_states=ehs).sample
    b = ref(x, 500, encoder_hidden_states=ehs).sample
    assert torch.equal(a, b)


def test_load_diffusers_state_dict_into_existing_model(checkpoint):
    """vdiff.load_diffusers_state_dict (weights.py): the UNet + adapter safetensors loaded into an
    already-built model with other weights."""
    root, unet, _ = checkpoint
    m = init_synthetic_(UNetMotionModel("tiny"), seed=7).to(torch.bfloat16)
    missing, unexpected = vdiff.load_diffusers_state_dict(
        m, [root / "sd" / "unet" / "diffusion_pytorch_model.safetensors",
            root / "adapter" / "diffusion_pytorch_model.safetensors"])
    assert not missing and not unexpected
    _bit_identical(m, unet.to(torch.bfloat16))
    with pytest.raises(KeyError, match="mismatch"):
        vdiff.load_diffusers_state_dict(m, root / "adapter" / "diffusion_pytorch_model.safetensors")


@pytest.mark.gpu
def test_baseline_generation_caller_sequence(checkpoint, tmp_path):
    """experiments/01_baseline_generation.py:55-123 unchanged except for the hub names: MotionAdapter /
    AnimateDiffPipeline.from_pretrained with torch_dtype=float16, the Euler swap
    (timestep_spacing="linspace", beta_schedule="linear"), pipe.to("cuda"), enable_vae_slicing(), then
    pipe(prompt=, negative_prompt=, generator=torch.Generator("cuda").manual_seed(42), **DEFAULT_CONFIG)
    -> .frames[0] = 16 PIL frames saved as GIF + PNGs.  The initial noise is drawn on the CUDA
    generator in float16, as diffusers' randn_tensor does (01:103)."""
    from vdiff import EulerDiscreteScheduler
    from vdiff.utils import export_to_gif
    root, _, _ = checkpoint
    adapter = MotionAdapter.from_pretrained(root / "adapter", torch_dtype=torch.float16)
    pipe = AnimateDiffPipeline.from_pretrained(root / "sd", motion_adapter=adapter, torch_dtype=torch.float16)
    pipe.scheduler = EulerDiscreteScheduler.from_config(pipe.scheduler.config, timestep_spacing="linspace",
                                                        beta_schedule="linear")
    pipe.to("cuda")
    pipe.enable_vae_slicing()
    # the draw: exactly torch.randn on the CUDA generator, float16, scaled by init_noise_sigma
    pipe.scheduler.set_timesteps(25)
    x = pipe.prepare_latents(1, 16, 64, 64, generator=torch.Generator("cuda").manual_seed(42))
    want = torch.randn((1, 4, 16, 64, 64), generator=torch.Generator("cuda").manual_seed(42), device="cuda",
                       dtype=torch.float16)
    assert x.is_cuda and torch.equal(x, want.float() * pipe.scheduler.init_noise_sigma)
    config = {"num_frames": 16, "num_inference_steps": 25, "guidance_scale": 7.5, "width": 512, "height": 512}
    out = pipe(prompt="a corgi walking on the beach, sunset lighting, high quality",
               negative_prompt="bad quality, blurry, distorted, ugly, deformed",
               generator=torch.Generator("cuda").manual_seed(42), **config)
    frames = out.frames[0]
    assert len(frames) == 16 and frames[0].mode == "RGB"
    export_to_gif(frames, str(tmp_path / "corgi_beach.gif"))
    for i, frame in enumerate(frames):
        frame.save(tmp_path / f"frame_{i:03d}.png")
    assert (tmp_path / "corgi_beach.gif").stat().st_size > 0 and (tmp_path / "frame_015.png").exists()
    # same seed, same generator device -> the same video
    again = pipe(prompt="a corgi walking on the beach, sunset lighting, high quality",
                 negative_prompt="bad quality, blurry, distorted, ugly, deformed",
                 generator=torch.Generator("cuda").manual_seed(42), output_type="latent", **config).frames
    first = pipe(prompt="a corgi walking on the beach, sunset lighting, high quality",
                 negative_prompt="bad quality, blurry, distorted, ugly, deformed",
                 generator=torch.Generator("cuda").manual_seed(42), output_type="latent", **config).frames
    assert torch.equal(again, first) and torch.isfinite(first).all()
