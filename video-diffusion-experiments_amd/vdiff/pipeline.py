"""AnimateDiffPipeline-compatible denoising loop on MI355X.

Mirrors the `pipe(...)` surface the reference drives at
experiments/05_grid_search_ablation.py:121-169 (from_pretrained-like
construction, settable `.scheduler`, enable_vae_slicing()/
enable_model_cpu_offload() as no-ops, `pipe(prompt=, negative_prompt=,
num_frames=, guidance_scale=, num_inference_steps=, height=, width=,
generator=).frames[0]`) and the loop body of diffusers'
AnimateDiffPipeline.__call__:

    x_in = cat([x, x]); eps = unet(x_in, t, ehs).sample
    eps = eps_u + g (eps_c - eps_u); x = scheduler.step(eps, t, x).prev_sample

Here that body is ONE captured hipGraph (torch.cuda.CUDAGraph == hipGraph on
ROCm): time embedding from a device timestep table indexed by a device step
counter, the UNet on packed NHWC rows, the fused CFG+DDIM kernel that also
writes the next step's packed input, and the counter increment — replayed
num_inference_steps times with no host work in between.  The cross-attention
K/V of the (constant) prompt embeddings are projected once per video, outside
the graph.

Out of scope: CLIP text encoding (a deterministic stub encoder
stands in; real embeddings can be passed as prompt_embeds).  VAE decoding (§8f
rank 1) runs when the pipeline holds a `vdiff.AutoencoderKL` (from_config builds one
by default): output_type "pil" (diffusers' default: `.frames[0]` is the first video's
list of PIL images, which 05_grid_search_ablation.py:169-182 saves as PNG / GIF),
"pt" / "np" (diffusers' postprocessed video, (B, F, 3, H, W) tensor / (B, F, H, W, 3)
array in [0, 1]) or "latent" (the final latents).

prepare_latents follows diffusers' randn_tensor: x_T = torch.randn(shape, generator, dtype)
drawn on the generator's device — the CPU for 05:156's `torch.manual_seed(seed)`, the GPU
for 01:103's `torch.Generator("cuda").manual_seed(seed)` — in the pipeline's torch_dtype
(float16 in the reference, 05:35, 05:130-134), then moved to the GPU (kept in fp32 from
there on).
"""
from __future__ import annotations

import zlib
from collections import namedtuple

import torch

from . import ops
from .models.unet_motion import CIN_PAD, UNetMotionModel
from .models.vae import AutoencoderKL
from .sched.ddim import DDIMScheduler
from .weights import init_synthetic_

AnimateDiffPipelineOutput = namedtuple("AnimateDiffPipelineOutput", ["frames"])


class SyntheticTextEncoder:
    """Stand-in for CLIPTextModel (out of scope): prompt -> deterministic
    N(0,1) [77, dim] embedding seeded by crc32(prompt)."""

    def __init__(self, dim: int, seq_len: int = 77):
        self.dim, self.seq_len = dim, seq_len

    def __call__(self, prompt: str) -> torch.Tensor:
        g = torch.Generator().manual_seed(zlib.crc32(prompt.encode()))
        return torch.randn((self.seq_len, self.dim), generator=g)


class DenoiseLoop:
    """Preallocated device state + the captured graph of one denoising step."""

    def __init__(self, unet: UNetMotionModel, scheduler, latents: torch.Tensor,
                 prompt_embeds: torch.Tensor, guidance_scale: float, timesteps=None,
                 use_graph: bool = True, cfg_shard=None):
        """cfg_shard (vdiff.dist.CfgShard, CFG only): this rank runs the UNet on ONE half
        (cfg_shard.index: 0 uncond, 1 cond) and swaps eps rows with its pair before the
        fused CFG+scheduler update, which both ranks apply to their replicated latents
        (SURVEY.md §8e (ii)).  prompt_embeds still holds both halves, uncond first."""
        if not unet._prepared:
            unet.prepare()
        dev = unet.device
        self.unet = unet
        self.ncfg = 2 if guidance_scale > 1 else 1
        self.g = float(guidance_scale)
        self.lat = latents.to(dev, torch.float32).contiguous().clone()
        self.B, _, self.F, self.H, self.W = self.lat.shape
        self.Bt = self.ncfg * self.B
        self.cfg_shard = cfg_shard if self.ncfg == 2 else None
        ts = scheduler.timesteps if timesteps is None else timesteps
        self.n_steps = len(ts)
        self.ts = torch.as_tensor(ts).to(dev, torch.float32)
        self.coef = scheduler.coefficient_table(torch.as_tensor(ts).cpu()).to(dev)
        # the scheduler's fused CFG+update kernel; Euler's also applies the next step's
        # scale_model_input, and the first input is packed with step 0's divisor
        self.kind = getattr(scheduler, "kind", "ddim")
        self.sched_step = ops.SCHED_STEP[self.kind]
        self.in_div0 = 1.0
        if self.kind == "euler":
            self.in_div0 = scheduler.input_divisor(scheduler.index_for_timestep(float(torch.as_tensor(ts)[0])))
        self.step_idx = torch.zeros(1, device=dev, dtype=torch.int32)
        pe = prompt_embeds.to(dev, torch.bfloat16).contiguous()
        if pe.shape[0] != self.Bt:
            raise ValueError(f"prompt_embeds batch {pe.shape[0]} != {self.Bt} (uncond first when CFG)")
        self.L = pe.shape[1]
        # the UNet batch: both CFG halves, or this rank's half under cfg_shard
        self.Bu = self.Bt
        if self.cfg_shard is not None:
            h = self.cfg_shard.index
            pe = pe[h * self.B:(h + 1) * self.B].contiguous()
            self.Bu = self.B
        self.ehs_rows = pe.reshape(self.Bu * self.L, -1)
        # the CFG step kernel writes the next input for both halves; under cfg_shard the
        # UNet reads only the first copy (the latents are replicated over the pair)
        self.x_in2 = ops.pack_latents(self.lat, dup=self.ncfg, cpad=CIN_PAD, in_div=self.in_div0)
        self.x_in = self.x_in2[:self.Bu * self.F * self.H * self.W]
        self.kv_cache = {}
        # conv_in + down_blocks[0].resnets[0] once for both CFG halves (UNetMotionModel.forward_rows)
        self.cfg_dedup = True
        self.use_graph = use_graph
        self.graph = None
        self.graph_error = None
        self.issued = 0  # steps run since the last reset(): the device index into ts / coef

    def _claim(self, n):
        """Host-side bound on the device step counter: the timestep and coefficient tables
        hold n_steps rows; running past them without reset() is an error (the kernels also
        clamp the index, so a stray replay can never read past the tables)."""
        if n < 0 or self.issued + n > self.n_steps:
            raise RuntimeError(f"run({n}) after {self.issued} of {self.n_steps} scheduled steps: "
                               "call reset(latents) to start a new schedule")
        self.issued += n

    def step(self):
        u = self.unet
        te = ops.timestep_embed(self.ts, u.time_proj.num_channels, step_idx=self.step_idx, batch=self.Bu)
        ctx = u.make_ctx(te, self.ehs_rows, self.Bu, self.F, self.L, kv_cache=self.kv_cache)
        ctx.cfg_dup = self.cfg_dedup and self.Bu == self.Bt == 2 * self.B  # x_in = [lat; lat]
        eps = u.forward_rows(self.x_in, self.H, self.W, ctx)
        if self.cfg_shard is not None:
            eps = self.cfg_shard.gather_eps(eps)
        self.sched_step(eps, self.ncfg, self.g, self.lat, self.coef, step_idx=self.step_idx,
                        next_in=self.x_in2)
        ops.step_advance(self.step_idx)

    def reset(self, latents):
        self.lat.copy_(latents)
        self.step_idx.zero_()
        self.issued = 0
        ops.pack_latents(self.lat, dup=self.ncfg, cpad=CIN_PAD, out=self.x_in2, in_div=self.in_div0)

    def prime(self):
        """One eager step (loads kernels, fills the cross-attention K/V cache,
        initialises communicators), then restore the state; capture the graph."""
        saved = self.lat.clone()
        self.step()
        self.reset(saved)
        torch.cuda.synchronize()
        if self.use_graph and self.graph is None:
            try:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self.step()
                self.graph = g
            except Exception as e:  # capture unsupported (e.g. a collective): run eagerly
                self.graph_error = repr(e)
                self.graph = None
                torch.cuda.synchronize()
                self.reset(saved)
        return self

    def run(self, n=None):
        n = self.n_steps - self.issued if n is None else n
        self._claim(n)
        for _ in range(n):
            if self.graph is not None:
                self.graph.replay()
            else:
                self.step()
        return self.lat


def randn_tensor(shape, generator=None, device=None, dtype=None):
    """diffusers.utils.torch_utils.randn_tensor: N(0, 1) drawn on the generator's device (the
    target device when there is no generator), in `dtype`, then moved to `device`.  A list of
    generators draws one batch row each.  A CUDA generator for a CPU target is refused."""
    device = torch.device(device or "cpu")
    gens = generator if isinstance(generator, (list, tuple)) else None
    if gens is not None and len(gens) == 1:
        generator, gens = gens[0], None
    rand_device = device
    if generator is not None:
        gtype = (gens[0] if gens is not None else generator).device.type
        if gtype != device.type:
            if gtype != "cpu":
                raise ValueError(f"Cannot generate a {device} tensor from a generator of type {gtype}.")
            rand_device = torch.device("cpu")
    if gens is not None:
        if len(gens) != shape[0]:
            raise ValueError(f"{len(gens)} generators for a batch of {shape[0]}")
        one = (1,) + tuple(shape[1:])
        x = torch.cat([torch.randn(one, generator=gen, device=rand_device, dtype=dtype) for gen in gens])
    else:
        x = torch.randn(shape, generator=generator, device=rand_device, dtype=dtype)
    return x.to(device)


def numpy_to_pil(images):
    """diffusers' numpy_to_pil: (F, H, W, 3) floats in [0, 1] -> list of RGB PIL images."""
    from PIL import Image
    arr = (images * 255).round().astype("uint8")
    return [Image.fromarray(a) for a in arr]


def export_to_gif(frames, output_gif_path, fps: int = 10):
    """diffusers.utils.export_to_gif (05:28, :181): PIL frames -> an animated GIF."""
    frames[0].save(str(output_gif_path), save_all=True, append_images=list(frames[1:]), optimize=False,
                   duration=1000 // fps, loop=0)
    return str(output_gif_path)


class AnimateDiffPipeline:
    # dtype the initial noise is drawn in on the CPU generator: the reference loads the
    # pipeline with torch_dtype=torch.float16 (05:35, 05:130-134) and diffusers' randn_tensor
    # draws in that dtype
    latent_draw_dtype = torch.float16

    def __init__(self, unet: UNetMotionModel, scheduler=None, text_encoder=None, vae=None, dist=None):
        self.unet = unet
        self.scheduler = scheduler or DDIMScheduler()
        self.text_encoder = text_encoder or SyntheticTextEncoder(unet.config["cross_attention_dim"])
        self.vae = vae
        self.dist = dist
        self.unet.dist = dist
        # the dtype the initial noise is drawn in (diffusers: prompt_embeds.dtype, i.e. the
        # pipeline's torch_dtype, fp32 when none is given); from_config keeps the reference's fp16
        self.torch_dtype = None

    @classmethod
    def from_config(cls, config="full", device="cuda", seed=0, scheduler=None, dist=None, vae="auto"):
        """Synthetic-weight pipeline; vae "auto" (a synthetic AutoencoderKL of the UNet's config,
        so the default output_type "pil" works), "tiny"/"full", an AutoencoderKL instance, or
        None (latents only)."""
        if vae == "auto":
            vae = config if config in ("tiny", "full") else None
        unet = UNetMotionModel(config)
        init_synthetic_(unet, seed)
        unet = unet.to(device=device, dtype=torch.bfloat16)
        unet.prepare()
        sched = scheduler or DDIMScheduler.from_config(None, beta_schedule="linear", steps_offset=1,
                                                       clip_sample=False)
        if isinstance(vae, str):
            vae = init_synthetic_(AutoencoderKL(vae), seed).to(device=device, dtype=torch.bfloat16).prepare()
        pipe = cls(unet, sched, dist=dist, vae=vae)
        pipe.torch_dtype = cls.latent_draw_dtype  # the reference's torch_dtype=torch.float16 (05:35)
        return pipe

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path, motion_adapter=None, torch_dtype=None, variant=None,
                        device="cuda", dist=None, **unused):
        """diffusers AnimateDiffPipeline.from_pretrained(path, motion_adapter=, torch_dtype=) as
        05:130-134 calls it, over a LOCAL diffusers-layout directory (vdiff.pretrained): unet/
        joined with the MotionAdapter's motion modules, vae/ (decoder), scheduler/.  The text
        encoder stays the deterministic stub (CLIP is out of scope; pass prompt_embeds for real
        embeddings).  device="cpu" builds the modules without preparing device operands."""
        from . import pretrained as P
        root = P._local_dir(pretrained_model_name_or_path, "AnimateDiffPipeline.from_pretrained")
        if motion_adapter is None:
            raise ValueError("AnimateDiffPipeline needs motion_adapter=MotionAdapter.from_pretrained(...)")
        unet = P.load_unet_motion(root / "unet", motion_adapter, device=device, variant=variant)
        vae = P.load_vae(root / "vae", device=device, variant=variant) if (root / "vae").is_dir() else None
        sched = P.load_scheduler(root / "scheduler") if (root / "scheduler").is_dir() else None
        if torch.device(device).type == "cuda":
            unet.prepare()
            if vae is not None:
                vae.prepare()
        pipe = cls(unet, sched, dist=dist, vae=vae)
        pipe.torch_dtype = torch_dtype
        return pipe

    def enable_vae_slicing(self):
        pass  # decoding is always chunked (AutoencoderKL.frames_per_chunk)

    def enable_model_cpu_offload(self, *a, **k):
        pass  # 288 GB HBM: the 12 GB-GPU workaround is unnecessary

    def to(self, *a, **k):
        return self

    def encode_prompt(self, prompt, batch):
        if isinstance(prompt, str):
            prompt = [prompt] * batch
        return torch.stack([self.text_encoder(p) for p in prompt])

    @torch.no_grad()
    def decode_latents(self, latents):
        """diffusers AnimateDiffPipeline.decode_latents: latents / scaling_factor, frames
        batched frame-major through vae.decode, -> (B, 3, F, H, W) fp32 in about [-1, 1]."""
        if self.vae is None:
            raise ValueError("this pipeline has no VAE (pass vae=vdiff.AutoencoderKL(...).to(...))")
        B, Cc, Fr, h, w = latents.shape
        z = latents.float() / self.vae.config["scaling_factor"]
        z = z.permute(0, 2, 1, 3, 4).reshape(B * Fr, Cc, h, w)
        img = self.vae.decode(z).sample
        return img[None].reshape((B, Fr) + tuple(img.shape[1:])).permute(0, 2, 1, 3, 4).float()

    @staticmethod
    def postprocess_video(video, output_type):
        """diffusers VideoProcessor.postprocess_video for "pt" / "np" / "pil": per video, frames
        first, denormalised (x / 2 + 0.5).clamp(0, 1); "pil" -> a list (per video) of lists of
        PIL images."""
        v = (video / 2 + 0.5).clamp(0, 1).permute(0, 2, 1, 3, 4)      # (B, F, 3, H, W)
        if output_type == "pt":
            return v
        arr = v.permute(0, 1, 3, 4, 2).float().cpu().numpy()           # (B, F, H, W, 3)
        if output_type == "np":
            return arr
        return [numpy_to_pil(a) for a in arr]

    def prepare_latents(self, batch, num_frames, h, w, generator=None, latents=None):
        """diffusers AnimateDiffPipeline.prepare_latents -> fp32 on the GPU, x init_noise_sigma.
        The draw follows randn_tensor: on the generator's device (a CPU generator from 05:156's
        torch.manual_seed, a CUDA one from 01:103's torch.Generator("cuda")), in the pipeline's
        torch_dtype (float16 in the reference, 01:21 / 05:35; fp32 when the pipeline was loaded
        with torch_dtype=None, as diffusers draws in prompt_embeds.dtype), then moved."""
        if latents is None:
            shape = (batch, self.unet.config["in_channels"], num_frames, h, w)
            dtype = self.torch_dtype or torch.float32
            latents = randn_tensor(shape, generator=generator, device=self.unet.device, dtype=dtype)
        return latents.to(self.unet.device, torch.float32) * self.scheduler.init_noise_sigma

    @torch.no_grad()
    def __call__(self, prompt=None, num_frames=16, height=None, width=None, num_inference_steps=50,
                 guidance_scale=7.5, negative_prompt=None, num_videos_per_prompt=1, eta=0.0,
                 generator=None, latents=None, prompt_embeds=None, negative_prompt_embeds=None,
                 output_type="pil", return_dict=True, use_graph=True, **unused):
        if eta != 0.0:
            raise NotImplementedError("eta > 0")
        if output_type not in ("latent", "pt", "np", "pil"):
            raise NotImplementedError(f"output_type {output_type!r}: use 'pil', 'pt', 'np' or 'latent'")
        if output_type != "latent" and self.vae is None:
            raise ValueError(f"output_type {output_type!r} needs a VAE: AnimateDiffPipeline(..., vae=...)")
        dev = self.unet.device
        sample = self.unet.config["sample_size"]
        h = (height or sample * 8) // 8
        w = (width or sample * 8) // 8
        if prompt_embeds is None:
            if prompt is None:
                raise ValueError("prompt or prompt_embeds required")
            n = 1 if isinstance(prompt, str) else len(prompt)
            prompt_embeds = self.encode_prompt(prompt, n)
        B = prompt_embeds.shape[0] * num_videos_per_prompt
        prompt_embeds = prompt_embeds.repeat_interleave(num_videos_per_prompt, 0)
        do_cfg = guidance_scale > 1
        if do_cfg:
            if negative_prompt_embeds is None:
                negative_prompt_embeds = self.encode_prompt(negative_prompt or "", B)
            ehs = torch.cat([negative_prompt_embeds.to(prompt_embeds), prompt_embeds])
        else:
            ehs = prompt_embeds
        self.scheduler.set_timesteps(num_inference_steps)
        latents = self.prepare_latents(B, num_frames, h, w, generator=generator, latents=latents)
        local = latents
        if self.dist is not None:
            fl = self.dist.frames_local(num_frames)
            local = latents[:, :, self.dist.rank * fl:(self.dist.rank + 1) * fl]
        loop = DenoiseLoop(self.unet, self.scheduler, local, ehs, guidance_scale,
                           use_graph=use_graph).prime()
        out = loop.run()
        if self.dist is not None:
            out = self.dist.all_gather_frames(out)
        if output_type != "latent":
            out = self.postprocess_video(self.decode_latents(out), output_type)
        return AnimateDiffPipelineOutput(frames=out) if return_dict else (out,)
