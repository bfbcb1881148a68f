"""A/B of a host-side policy on the full denoising step, in one process on one box (box-to-box
variance is ~3 %): python tools/ab_step.py MODE [frames] — alternates two captured-graph loops:
  gn   GroupNorm policy (two-launch image norms vs partial/finalize/apply everywhere)
  ln   LayerNorm fused into the residual GEMM's epilogue (ops.gemm_ln) vs GEMM + vd_layernorm
  v3p  persistent v3 GEMM vs one unit per workgroup (vd_gemm_select_path 0 vs 11)
  mq   motion-module Q/K/V projection fused into the temporal attention (L1) vs GEMM + attention
  mq2  the fused motion kernel of round 3 (register tokens, LDS-DMA weight ring) vs round 2's
  pf   v2/v6 GEMM fragment-read order: the default vs round 1's, k-step-pipelined and all-ahead
       (vd_gemm_select_path 0 / 12 / 13 / 14)
  v3e  v3 GEMM with the LDS-bias load-free epilogue vs gemm_epilogue (vd_gemm_select_path 0 vs 15)
  roll v5 GEMM with the rolling W-fragment window vs round 1's halves (vd_gemm_select_path 0 vs 16)
  mf   v2 in the 32x32x16 form on the short-K level-1 convs vs the automatic plan (16x16x32)
       (vd_gemm_select_path 19 vs 0)
  fd   v2 conv row setup with 32-bit shifts (the default) vs round 2's int64 divisions (0 vs 20)
  mqpw the fused motion kernel with two positions per wave (the default) vs one
       (vd_attention_select 42 vs 40)"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd")]
import torch  # noqa: E402

from vdiff import DDIMScheduler, DenoiseLoop, ops  # noqa: E402
from vdiff.weights import materialize_synthetic  # noqa: E402

frames = int(sys.argv[2]) if len(sys.argv) > 2 else 16
unet = materialize_synthetic("full", device="cuda", seed=0)
unet.prepare()
lat = torch.randn((1, 4, frames, 64, 64), generator=torch.Generator().manual_seed(42)).cuda()
ehs = torch.randn((2, 77, 768), generator=torch.Generator().manual_seed(1)).cuda()
sched = DDIMScheduler(beta_schedule="linear", steps_offset=1, clip_sample=False)
sched.set_timesteps(50)
mode = sys.argv[1] if len(sys.argv) > 1 else "gn"
loops = {}
if mode == "gn":
    orig = ops.group_norm

    def four_pass(*a, **k):
        k["two_pass"] = False
        return orig(*a, **k)

    for name, fn in (("two-launch", orig), ("four-launch", four_pass)):
        ops.group_norm = fn  # modules hold `ops`, so patching ops is enough
        loops[name] = DenoiseLoop(unet, sched, lat, ehs, 7.5).prime()
    ops.group_norm = orig
elif mode == "ln":
    orig = ops.gemm_ln

    def unfused(a, w, gamma, beta, *, eps=1e-5, pe=None, pe_div=1, pe_period=1, bias=None, res=None, **k):
        out = ops.gemm(a, w, bias=bias, res=res)
        return out, ops.layer_norm(out, gamma, beta, eps, pe=pe, pe_div=pe_div, pe_period=pe_period)

    for name, fn in (("ln-fused", orig), ("ln-separate", unfused)):
        ops.gemm_ln = fn
        loops[name] = DenoiseLoop(unet, sched, lat, ehs, 7.5).prime()
    ops.gemm_ln = orig
elif mode == "mqpw":
    from vdiff._lib import lib
    for name, sel in (("motion-pw2", 42), ("motion-pw1", 40)):
        lib().vd_attention_select(sel)  # the kernel choice is fixed at capture
        loops[name] = DenoiseLoop(unet, sched, lat, ehs, 7.5).prime()
    lib().vd_attention_select(42)
elif mode == "fd":
    from vdiff._lib import lib
    for name, path in (("div-shift", 0), ("div-int64", 20)):
        lib().vd_gemm_select_path(path)  # the plan is fixed at capture
        loops[name] = DenoiseLoop(unet, sched, lat, ehs, 7.5).prime()
    lib().vd_gemm_select_path(0)
elif mode == "mf":
    from vdiff._lib import lib
    for name, path in (("mf32-L1conv", 19), ("mf32-never", 0)):
        lib().vd_gemm_select_path(path)  # the plan is fixed at capture
        loops[name] = DenoiseLoop(unet, sched, lat, ehs, 7.5).prime()
    lib().vd_gemm_select_path(0)
elif mode == "v3p":
    from vdiff._lib import lib
    for name, path in (("v3-persistent", 0), ("v3-per-tile", 11)):
        lib().vd_gemm_select_path(path)  # the plan is fixed at capture
        loops[name] = DenoiseLoop(unet, sched, lat, ehs, 7.5).prime()
    lib().vd_gemm_select_path(0)
elif mode == "pf":
    from vdiff._lib import lib
    for name, path in (("frag-default", 0), ("frag-r1-order", 12), ("frag-pipelined", 13), ("frag-all-ahead", 14)):
        lib().vd_gemm_select_path(path)  # the launch choice is fixed at capture
        loops[name] = DenoiseLoop(unet, sched, lat, ehs, 7.5).prime()
    lib().vd_gemm_select_path(0)
elif mode == "v3e":
    from vdiff._lib import lib
    for name, path in (("v3-lds-bias", 0), ("v3-gemm-epi", 15)):
        lib().vd_gemm_select_path(path)
        loops[name] = DenoiseLoop(unet, sched, lat, ehs, 7.5).prime()
    lib().vd_gemm_select_path(0)
elif mode == "roll":
    from vdiff._lib import lib
    for name, path in (("v5-rolling-w", 0), ("v5-w-halves", 16)):
        lib().vd_gemm_select_path(path)
        loops[name] = DenoiseLoop(unet, sched, lat, ehs, 7.5).prime()
    lib().vd_gemm_select_path(0)
elif mode == "mq":
    from vdiff.models.blocks import BasicTransformerBlock
    blocks = [m for m in unet.modules() if isinstance(m, BasicTransformerBlock)]
    for name, on in (("qkv-attn-fused", True), ("qkv-gemm+attn", False)):
        for m in blocks:
            m.fuse_qkv_attention = on
        loops[name] = DenoiseLoop(unet, sched, lat, ehs, 7.5).prime()
    for m in blocks:
        m.fuse_qkv_attention = True
elif mode == "mq2":
    from vdiff._lib import lib
    for name, sel in (("motion-qkv v2", 32), ("motion-qkv v1", 31)):
        lib().vd_attention_select(sel)  # kernel version fixed at capture
        loops[name] = DenoiseLoop(unet, sched, lat, ehs, 7.5).prime()
    lib().vd_attention_select(32)
else:
    sys.exit(f"unknown mode {mode}")
res = {k: [] for k in loops}
for rep in range(4):
    for name, lp in loops.items():
        lp.reset(lat.to(lp.lat.device))  # 13 steps per round: restart the 50-step schedule
        lp.run(3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lp.run(10)
        torch.cuda.synchronize()
        res[name].append((time.perf_counter() - t0) / 10 * 1e3)
for k, v in res.items():
    print(f"{k:12s} frames={frames} ms/step: " + " ".join(f"{x:.2f}" for x in v) + f"  min {min(v):.2f}", flush=True)
