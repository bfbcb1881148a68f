"""DiT-style video denoiser (BASELINE config 5: "DiT-style transformer
denoiser (patchified 3D latents) … 32 frames × 768×768").

The reference has no DiT — its denoiser is diffusers' UNetMotionModel — so the model is
build-defined (the public DiT / Latte recipe, restated op by op in oracle/dit_ref.py) and
exposes the same call surface as the UNet so the sampling loop drives either:
`forward(sample (B,C,F,H,W), timestep, encoder_hidden_states (B,L,Dt)).sample`.

MI355X layout: tokens are bf16 rows [(b, f, hp, wp)][D] (frame-major, channels contiguous),
so spatial attention reads each frame's Hp*Wp rows contiguously and temporal attention
walks frames at a fixed position with a row stride of Hp*Wp (vd_temporal_attention), with
no transposes.  Per block, on HIP kernels only:
  res_ln_mod (previous MLP's gated residual + LN + adaLN modulate, one HBM pass)
  -> GEMM to_qkv -> vd_rope_qk (in place on the q,k columns) -> flash attention
  -> GEMM to_out -> res_ln_mod (gated residual + plain LN)
  -> GEMM cross.to_q -> attention on the per-video text K/V (projected once per video)
  -> GEMM cross.to_out (+residual in the epilogue)
  -> res_ln_mod (modulate) -> GEMM fc1 (+GELU epilogue) -> GEMM fc2 (gated residual
     deferred into the next block's res_ln_mod).
All adaLN modulation vectors of all blocks come from ONE GEMM (M = batch) per forward.
"""
from __future__ import annotations

from collections import namedtuple

import torch

from .. import ops

DiTOutput = namedtuple("DiTOutput", ["sample"])

DIT_FULL = dict(  # BASELINE config 5: 32 frames x 768x768 (96x96 latents), Latte-XL width
    in_channels=4, out_channels=4, patch_size=2, hidden_size=1152, num_heads=18, depth=28,
    mlp_ratio=4, text_dim=768, num_frames=32, sample_size=96, rope_theta=10000.0, freq_dim=256,
)
DIT_TINY = dict(DIT_FULL, hidden_size=128, num_heads=2, depth=2, text_dim=64, num_frames=4,
                sample_size=16)
DIT_CONFIGS = {"full": DIT_FULL, "tiny": DIT_TINY}


def dit_param_shapes(cfg: dict) -> dict:
    D, p, Dt = cfg["hidden_size"], cfg["patch_size"], cfg["text_dim"]
    Hm = cfg["mlp_ratio"] * D
    s = {
        "patch_embed.weight": (D, cfg["in_channels"], 1, p, p), "patch_embed.bias": (D,),
        "t_embedder.linear_1.weight": (D, cfg["freq_dim"]), "t_embedder.linear_1.bias": (D,),
        "t_embedder.linear_2.weight": (D, D), "t_embedder.linear_2.bias": (D,),
    }
    for i in range(cfg["depth"]):
        pre = f"blocks.{i}."
        for name, (n, k) in {"adaLN_modulation": (6 * D, D), "attn.to_qkv": (3 * D, D),
                             "attn.to_out": (D, D), "cross.to_q": (D, D), "cross.to_kv": (2 * D, Dt),
                             "cross.to_out": (D, D), "mlp.fc1": (Hm, D), "mlp.fc2": (D, Hm)}.items():
            s[pre + name + ".weight"] = (n, k)
            s[pre + name + ".bias"] = (n,)
    s["final.adaLN_modulation.weight"] = (2 * D, D)
    s["final.adaLN_modulation.bias"] = (2 * D,)
    s["final.linear.weight"] = (p * p * cfg["out_channels"], D)
    s["final.linear.bias"] = (p * p * cfg["out_channels"],)
    return s


def init_dit_state_dict(cfg: dict, seed: int = 0, device="cpu", dtype=torch.float32) -> dict:
    """Synthetic weights (SURVEY.md §8d convention): every tensor ~ N(0, 0.02^2), rounded
    to bf16 once so the CPU oracle and the GPU see identical values.  No adaLN-Zero
    zeroing (it would hide every block behind a zero gate)."""
    g = torch.Generator(device=device).manual_seed(seed)
    sd = {}
    for k, shp in dit_param_shapes(cfg).items():
        sd[k] = (torch.randn(shp, generator=g, device=device) * 0.02).to(torch.bfloat16).to(dtype)
    return sd


class DiT3DModel:
    """Build-defined DiT video denoiser over HIP kernels (see module docstring)."""

    def __init__(self, cfg: dict, state_dict: dict, device="cuda", attn_fp8: bool = False):
        """attn_fp8: spatial self-attention on the block-scaled fp8 MFMA (vd_attention_fp8,
        d = 64, frames of a multiple of 64 tokens); text cross- and temporal attention stay bf16."""
        self.attn_fp8 = attn_fp8
        # RoPE inside the attention kernels' Q/K loads (fp8 quantization pass, 32-frame temporal
        # kernel); False runs the separate in-place rope_qk pass everywhere (A/B hook)
        self.fuse_rope = True
        self.config = dict(cfg)
        self.device = torch.device(device)
        self.dtype = torch.bfloat16
        D, p, Ci = cfg["hidden_size"], cfg["patch_size"], cfg["in_channels"]
        if D % cfg["num_heads"]:
            raise ValueError("hidden_size must be a multiple of num_heads")
        self.D, self.p, self.heads = D, p, cfg["num_heads"]
        self.d = D // self.heads
        self.kpad = (Ci * p * p + 7) // 8 * 8
        dev = self.device

        def w(key, kpad=None):
            t = state_dict[key].detach().reshape(state_dict[key].shape[0], -1)
            if kpad and kpad > t.shape[1]:
                t = torch.nn.functional.pad(t, (0, kpad - t.shape[1]))
            return t.to(dev, torch.bfloat16).contiguous()

        def b(key):
            return state_dict[key].detach().to(dev, torch.float32).contiguous()

        self.w_pe, self.b_pe = w("patch_embed.weight", self.kpad), b("patch_embed.bias")
        self.w_t1, self.b_t1 = w("t_embedder.linear_1.weight"), b("t_embedder.linear_1.bias")
        self.w_t2, self.b_t2 = w("t_embedder.linear_2.weight"), b("t_embedder.linear_2.bias")
        depth = cfg["depth"]
        ada = [f"blocks.{i}.adaLN_modulation" for i in range(depth)] + ["final.adaLN_modulation"]
        self.w_ada = torch.cat([w(k + ".weight") for k in ada]).contiguous()
        self.b_ada = torch.cat([b(k + ".bias") for k in ada]).contiguous()
        self.blocks = []
        for i in range(depth):
            pre = f"blocks.{i}."
            self.blocks.append({n: (w(pre + n + ".weight"), b(pre + n + ".bias")) for n in
                                ("attn.to_qkv", "attn.to_out", "cross.to_q", "cross.to_kv",
                                 "cross.to_out", "mlp.fc1", "mlp.fc2")})
        self.w_fin, self.b_fin = w("final.linear.weight"), b("final.linear.bias")

    # ------------------------------------------------------------------ pieces
    def modulation(self, te):
        """te: bf16 [B, freq_dim] sinusoidal embedding -> fp32 [B, depth*6D + 2D]."""
        h = ops.gemm(te, self.w_t1, bias=self.b_t1, act=ops.ACT_SILU)
        sc = ops.gemm(h, self.w_t2, bias=self.b_t2, act=ops.ACT_SILU)  # SiLU(c)
        return ops.gemm(sc, self.w_ada, bias=self.b_ada, out_f32=True)

    def text_kv(self, ehs_rows):
        """Per-block cross-attention K/V of the (constant) text rows [B*L, Dt]."""
        return [ops.gemm(ehs_rows, blk["cross.to_kv"][0], bias=blk["cross.to_kv"][1]) for blk in self.blocks]

    def _block(self, i, blk, x, y, gate, mod, B, F, P, rope, kv, L, rpb, spatial):
        """One block over rows (b, f, p) of F frames x P positions; the previous MLP's gated
        residual (y, gate) is folded into the first row pass.  Returns the new x and the
        block's own pending (y, gate)."""
        D, d, heads = self.D, self.d, self.heads
        base = 6 * D * i
        sh1, sc1, g1, sh2, sc2, g2 = (mod[:, base + j * D: base + (j + 1) * D] for j in range(6))
        h = ops.res_ln_mod(x, y=y, gate=gate, x_out=x if y is not None else None, shift=sh1, scale=sc1,
                           rows_per_b=rpb)
        qkv = ops.gemm(h, blk["attn.to_qkv"][0], bias=blk["attn.to_qkv"][1])
        q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
        theta = self.config["rope_theta"]
        fp8 = spatial and self.attn_fp8 and d == 64 and P % 64 == 0
        if fp8 and self.fuse_rope:
            # the spatial RoPE runs inside the fp8 quantization pass (q, k stay un-rotated)
            a = ops.attention_fp8(q, k, v, B * F, heads, P, P, d, rope=(rope[1], rope[2], theta))
        elif fp8:
            ops.rope_qk(qkv, 2 * D, d, 0, *rope, theta)
            a = ops.attention_fp8(q, k, v, B * F, heads, P, P, d)
        elif not spatial and self.fuse_rope and d == 64 and 17 <= F <= 32:
            # the temporal RoPE runs inside the 32-frame MFMA kernel's Q/K loads
            a = ops.temporal_attention(q, k, v, B, F, P, heads, d, rope_theta=theta)
        elif not spatial:
            ops.rope_qk(qkv, 2 * D, d, 1, *rope, theta)
            a = ops.temporal_attention(q, k, v, B, F, P, heads, d)
        else:
            ops.rope_qk(qkv, 2 * D, d, 0, *rope, theta)
            a = ops.attention(q, k, v, B * F, heads, P, P, d)
        y = ops.gemm(a, blk["attn.to_out"][0], bias=blk["attn.to_out"][1])
        h = ops.res_ln_mod(x, y=y, gate=g1, x_out=x, rows_per_b=rpb)
        qc = ops.gemm(h, blk["cross.to_q"][0], bias=blk["cross.to_q"][1])
        a = ops.attention(qc, kv[i][:, :D], kv[i][:, D:], B * F, heads, P, L, d, kv_div=F)
        x = ops.gemm(a, blk["cross.to_out"][0], bias=blk["cross.to_out"][1], res=x)
        h = ops.res_ln_mod(x, shift=sh2, scale=sc2, rows_per_b=rpb)
        m = ops.gemm(h, blk["mlp.fc1"][0], bias=blk["mlp.fc1"][1], act=ops.ACT_GELU)
        y = ops.gemm(m, blk["mlp.fc2"][0], bias=blk["mlp.fc2"][1])
        return x, y, g2

    def forward_rows(self, x_tok, B, F, Hp, Wp, mod, kv, L, dist=None):
        """x_tok: bf16 patch rows [B*F*Hp*Wp, kpad] -> fp32 token rows [.., p*p*C_out].

        dist (vdiff.dist.FrameShard): this rank holds F of the world*F frames (both CFG
        halves).  Spatial blocks are frame-local; each temporal block re-shards the residual
        stream frame -> position shards with one all-to-all, runs on all frames of
        Hp*Wp/world positions, and re-shards back (as the UNet's motion
        modules)."""
        D = self.D
        S = Hp * Wp
        rpb = F * S  # rows per video: the same in the frame and the position layout
        x = ops.gemm(x_tok, self.w_pe, bias=self.b_pe)
        y = gate = None
        for i, blk in enumerate(self.blocks):
            if i % 2 == 0:
                x, y, gate = self._block(i, blk, x, y, gate, mod, B, F, S, (F, Hp, Wp), kv, L, rpb, True)
            elif dist is None:
                x, y, gate = self._block(i, blk, x, y, gate, mod, B, F, S, (F, Hp, Wp), kv, L, rpb, False)
            else:
                W = dist.world
                if S % W:
                    raise ValueError(f"{S} positions do not shard over {W} ranks")
                if y is not None:  # finish the pending residual before the re-shard
                    ops.res_ln_mod(x, y=y, gate=gate, x_out=x, rows_per_b=rpb)
                xp = dist.to_position_shards(x, B, F, S, ops.block_transpose)
                Fg, Pl = F * W, S // W
                xp, y, gate = self._block(i, blk, xp, None, None, mod, B, Fg, Pl, (Fg, 1, Pl), kv, L, rpb, False)
                ops.res_ln_mod(xp, y=y, gate=gate, x_out=xp, rows_per_b=rpb)
                x = dist.to_frame_shards(xp, B, F, S, ops.block_transpose)
                y = gate = None
        base = 6 * D * len(self.blocks)
        shf, scf = mod[:, base:base + D], mod[:, base + D:base + 2 * D]
        h = ops.res_ln_mod(x, y=y, gate=gate, x_out=x if y is not None else None, shift=shf, scale=scf,
                           rows_per_b=rpb)
        return ops.gemm(h, self.w_fin, bias=self.b_fin, out_f32=True)

    # ------------------------------------------------------------------ call surface
    def forward(self, sample, timestep, encoder_hidden_states, return_dict=True, **unused):
        """Same surface as UNetMotionModel.forward: (B,C,F,H,W) fp32 -> .sample (B,C,F,H,W)."""
        B, Ci, F, H, W = sample.shape
        p = self.p
        x = sample.to(self.device, torch.float32).contiguous()
        t = torch.as_tensor(timestep, dtype=torch.float32).reshape(-1).expand(B).contiguous().to(self.device)
        te = ops.timestep_embed(t, self.config["freq_dim"])
        mod = self.modulation(te)
        ehs = encoder_hidden_states.to(self.device, torch.bfloat16).contiguous()
        L = ehs.shape[1]
        kv = self.text_kv(ehs.reshape(B * L, -1))
        tok = ops.patchify(x, p, self.kpad)
        out_tok = self.forward_rows(tok, B, F, H // p, W // p, mod, kv, L)
        Co = self.config["out_channels"]
        eps = ops.unpatchify(out_tok, B * F, H, W, p, Co)
        out = ops.unpack_nhwc(eps, B, Co, F, H, W)
        return DiTOutput(out) if return_dict else (out,)

    __call__ = forward


class DiTDenoiseLoop:
    """CFG denoising loop over the DiT, one captured hipGraph per step: timestep embedding
    from a device table + step counter, the modulation GEMM, the DiT on patch rows,
    unpatchify, the fused CFG + scheduler kernel, re-patchify of the new latents."""

    def __init__(self, model: DiT3DModel, scheduler, latents, prompt_embeds, guidance_scale,
                 use_graph=True, dist=None):
        """dist (vdiff.dist.FrameShard): latents hold this rank's frames only (the CFG
        update and patchify are per frame); temporal blocks re-shard (forward_rows)."""
        self.dist = dist
        dev = model.device
        self.m = model
        self.ncfg = 2 if guidance_scale > 1 else 1
        self.g = float(guidance_scale)
        self.lat = latents.to(dev, torch.float32).contiguous().clone()
        self.B, self.C, self.F, self.H, self.W = self.lat.shape
        self.Bt = self.ncfg * self.B
        ts = scheduler.timesteps
        self.n_steps = len(ts)
        self.ts = torch.as_tensor(ts).to(dev, torch.float32)
        self.coef = scheduler.coefficient_table(torch.as_tensor(ts).cpu()).to(dev)
        self.sched_step = ops.SCHED_STEP[getattr(scheduler, "kind", "ddim")]
        if getattr(scheduler, "kind", "ddim") != "ddim":
            raise ValueError("DiTDenoiseLoop drives the DDIM schedule (epsilon prediction)")
        self.step_idx = torch.zeros(1, device=dev, dtype=torch.int32)
        pe = prompt_embeds.to(dev, torch.bfloat16).contiguous()
        if pe.shape[0] != self.Bt:
            raise ValueError(f"prompt_embeds batch {pe.shape[0]} != {self.Bt}")
        self.L = pe.shape[1]
        self.kv = model.text_kv(pe.reshape(self.Bt * self.L, -1))
        p = model.p
        self.x_tok = ops.patchify(self.lat, p, model.kpad, dup=self.ncfg)
        self.use_graph = use_graph
        self.graph = None
        self.issued = 0  # steps run since the last reset() (the device index into ts / coef)

    def step(self):
        m = self.m
        te = ops.timestep_embed(self.ts, m.config["freq_dim"], step_idx=self.step_idx, batch=self.Bt)
        mod = m.modulation(te)
        p = m.p
        out = m.forward_rows(self.x_tok, self.Bt, self.F, self.H // p, self.W // p, mod, self.kv, self.L,
                             dist=self.dist)
        eps = ops.unpatchify(out, self.Bt * self.F, self.H, self.W, p, m.config["out_channels"])
        self.sched_step(eps, self.ncfg, self.g, self.lat, self.coef, step_idx=self.step_idx)
        ops.patchify(self.lat, p, m.kpad, dup=self.ncfg, out=self.x_tok)
        ops.step_advance(self.step_idx)

    def reset(self, latents):
        self.lat.copy_(latents)
        self.step_idx.zero_()
        self.issued = 0
        ops.patchify(self.lat, self.m.p, self.m.kpad, dup=self.ncfg, out=self.x_tok)

    def prime(self):
        saved = self.lat.clone()
        self.step()
        self.reset(saved)
        torch.cuda.synchronize()
        if self.use_graph and self.graph is None:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self.step()
            self.graph = g
        return self

    def run(self, n=None):
        n = self.n_steps - self.issued if n is None else n
        if n < 0 or self.issued + n > self.n_steps:
            raise RuntimeError(f"run({n}) after {self.issued} of {self.n_steps} scheduled steps: "
                               "call reset(latents) to start a new schedule")
        if self.graph is None and self.use_graph:
            self.prime()
        self.issued += n
        for _ in range(n):
            if self.graph is not None:
                self.graph.replay()
            else:
                self.step()
        return self.lat
