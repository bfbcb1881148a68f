"""Module- and model-level parity on the MI355X against the CPU oracle.

Module tests use random weights sharper than the §8d synthetic init (std 0.1,
attention q/k 0.3) so attention is far from uniform and the cross-attention /
time-embedding paths move the output well above bf16 noise — the whole-UNet
test alone cannot see them (with std 0.02 weights cond and uncond eps differ by
only 0.24%, below the bf16 storage noise of the network).

Tolerance: the device path stores bf16 activations; the whole tiny UNet is
compared by relative L2 error against the fp32 oracle with a bound of 1.8% (the
oracle itself with the device's bf16 storage emulated lands at 1.4%, committed in
tests/golden/tiny_unet.npz) and against that device-emulating oracle (act="dev":
bf16 at every store, the kernels' folded softmax scale and bf16 probabilities) at
1.8% (both measured 1.33-1.38% at t in {961, 500, 1}); the tight check is per block against
the device-emulating oracle at 0.25% (test_tiny_blocks_match_device_emulation).  Module tests
use 2.5% rel-L2 (a few bf16 roundings in sequence).
"""
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import ddim_ref, unet_ref
from vdiff import DDIMScheduler, DenoiseLoop, EulerDiscreteScheduler, UNetMotionModel, init_synthetic_, ops
from vdiff.config import TINY
from vdiff.models.blocks import AnimateDiffTransformer3D, Ctx, ResnetBlock2D, Transformer2DModel
from vdiff.models.layers import Act, prepare_tree

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"


def rel_l2(got, want):
    got, want = got.double().cpu(), want.double().cpu()
    return ((got - want).norm() / want.norm()).item()


def randomize_(mod, seed, std=0.1, attn_std=0.3):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for n, p in mod.named_parameters():
            s = attn_std if (".to_q" in n or ".to_k" in n) else std
            r = torch.randn(p.shape, generator=g) * s
            if ("norm" in n.split(".")[-2]) and n.endswith("weight"):
                r = r + 1.0
            p.copy_(r.to(torch.bfloat16).float())
    return mod


def sd_of(mod, prefix):
    return {f"{prefix}.{k}": v.detach().float().cpu() for k, v in mod.state_dict().items()}


def to_rows(x):  # (N, C, H, W) -> NHWC rows bf16 on GPU
    n, c, h, w = x.shape
    return x.permute(0, 2, 3, 1).reshape(n * h * w, c).to("cuda", torch.bfloat16).contiguous()


def from_rows(t, n, h, w):
    return t.float().cpu().reshape(n, h, w, -1).permute(0, 3, 1, 2)


def test_resnet_block_concat_shortcut(cuda):
    cin_x, cin_s, cout, tdim = 128, 64, 128, 256
    B, Fr, H, W = 2, 2, 16, 16
    r = randomize_(ResnetBlock2D(cin_x + cin_s, cout, tdim), 0)
    sd = sd_of(r, "r")
    r = r.to("cuda", torch.bfloat16)
    prepare_tree(r)
    x = torch.randn(B * Fr, cin_x, H, W).to(torch.bfloat16).float()
    s = torch.randn(B * Fr, cin_s, H, W).to(torch.bfloat16).float()
    temb = torch.randn(B, tdim).to(torch.bfloat16).float()
    temb_silu = torch.nn.functional.silu(temb).to(torch.bfloat16).float()
    temb_all = ops.gemm(temb_silu.to("cuda", torch.bfloat16), r.time_emb_proj.weight.to(torch.bfloat16),
                        bias=r.time_emb_proj.bias.float(), out_f32=True)
    ctx = Ctx(B, Fr, temb_all, None, 77)
    out = r.run(Act(to_rows(x), B * Fr, H, W), ctx, skip=Act(to_rows(s), B * Fr, H, W))
    want = unet_ref.resnet(sd, "r", torch.cat([x, s], 1), temb_silu.repeat_interleave(Fr, 0), 32)
    assert rel_l2(from_rows(out.t, B * Fr, H, W), want) < 0.025


def test_transformer2d_with_cross_attention(cuda):
    heads, C, L, D = 2, 64, 77, 64
    B, Fr, H, W = 2, 2, 16, 16
    t = randomize_(Transformer2DModel(heads, C // heads, C, D), 1)
    sd = sd_of(t, "t")
    t = t.to("cuda", torch.bfloat16)
    prepare_tree(t)
    x = torch.randn(B * Fr, C, H, W).to(torch.bfloat16).float()
    ehs = torch.randn(B, L, D).to(torch.bfloat16).float()
    ctx = Ctx(B, Fr, None, ehs.reshape(B * L, D).to("cuda", torch.bfloat16), L)
    out = t.run(Act(to_rows(x), B * Fr, H, W), ctx)
    want = unet_ref.transformer2d(sd, "t", x, ehs.repeat_interleave(Fr, 0), heads, 32)
    got = from_rows(out.t, B * Fr, H, W)
    assert rel_l2(got, want) < 0.025
    # the cross-attention path must matter at this weight scale
    ctx2 = Ctx(B, Fr, None, torch.zeros_like(ctx.ehs_rows), L)
    other = from_rows(t.run(Act(to_rows(x), B * Fr, H, W), ctx2).t, B * Fr, H, W)
    assert rel_l2(other, want) > 0.05


def test_motion_module(cuda):
    heads, C = 2, 64
    B, Fr, H, W = 2, 8, 8, 8
    m = randomize_(AnimateDiffTransformer3D(heads, C // heads, C), 2)
    sd = sd_of(m, "m")
    m = m.to("cuda", torch.bfloat16)
    prepare_tree(m)
    x = (torch.randn(B * Fr, C, H, W) + 0.5).to(torch.bfloat16).float()
    ctx = Ctx(B, Fr, None, None, 77)
    out = m.run(Act(to_rows(x), B * Fr, H, W), ctx)
    want = unet_ref.motion_module(sd, "m", x, Fr, heads, 32, 32)
    assert rel_l2(from_rows(out.t, B * Fr, H, W), want) < 0.025


@pytest.fixture(scope="module")
def tiny_unet(cuda):
    m = init_synthetic_(UNetMotionModel("tiny"), seed=0)
    return m.to("cuda", torch.bfloat16).prepare()


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD / "tiny_unet.npz")


@pytest.mark.parametrize("t", [961, 500, 1])
def test_tiny_unet_matches_oracle(tiny_unet, gold, t):
    lat = torch.from_numpy(gold["latents"]).cuda()
    ehs = torch.from_numpy(gold["ehs"]).cuda()
    out = tiny_unet(torch.cat([lat, lat]), t, encoder_hidden_states=ehs).sample
    assert out.shape == (2, 4, 4, 64, 64) and out.dtype == torch.float32
    want = torch.from_numpy(gold[f"eps_t{t}"])
    err = rel_l2(out, want)
    r_dev, m_dev = _errs(out, torch.from_numpy(gold[f"eps_t{t}_dev"]))
    print(f"tiny UNet t={t}: vs fp32 oracle rel-L2 {err:.5f}; vs device-emulating oracle rel-L2 "
          f"{r_dev:.5f} max|err|/max|want| {m_dev:.5f}")
    # end to end both oracles sit at the bf16 realisation floor (~1.3 %, test_oracle.py::
    # test_bf16_realisation_floor); the tight bound is per block, test_tiny_blocks_match_...
    assert err < 0.018, err      # measured 0.0137-0.0138 (1.3x headroom)
    assert r_dev < 0.018, r_dev  # measured 0.0133-0.0134


def test_tiny_blocks_match_device_emulation(tiny_unet, gold):
    """Per block, from the device's own input (tests/parity_blocks.py): every block of the
    tiny UNet against the device-emulating oracle within 0.25 % rel-L2 (a fraction of one bf16
    rounding: the residual is fp32 summation order flipping a few stores) and against the fp32
    oracle within 0.6 %; the table is printed."""
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    from parity_blocks import block_errors
    rows = block_errors(tiny_unet, torch.from_numpy(gold["latents"]), torch.from_numpy(gold["ehs"]), log=print)
    assert len(rows) >= 20
    worst_dev = max(r[2] for r in rows)
    worst_32 = max(r[1] for r in rows)
    print(f"worst block: vs dev {worst_dev:.5f}, vs fp32 {worst_32:.5f}")
    assert worst_dev < 0.0025, rows
    assert worst_32 < 0.006, rows


def test_scheduler_step_api_matches_oracle(tiny_unet, gold):
    lat = torch.from_numpy(gold["latents"]).cuda()
    ehs = torch.from_numpy(gold["ehs"]).cuda()
    s = DDIMScheduler.from_config(DDIMScheduler().config, beta_schedule="linear", steps_offset=1,
                                  clip_sample=False)
    s.set_timesteps(50)
    t = int(s.timesteps[0])
    eps = tiny_unet(torch.cat([lat, lat]), t, encoder_hidden_states=ehs).sample
    u, c = eps.chunk(2)
    out = s.step(u + 7.5 * (c - u), t, lat)
    assert rel_l2(out.prev_sample, torch.from_numpy(gold["ddim_step0_x"])) < 0.01
    # exact DDIM arithmetic on identical eps: the kernel rounds once per operation in
    # diffusers' order (no FMA contraction, correctly rounded division) -> bit-exact
    acp = ddim_ref.alphas_cumprod()
    e = (u + 7.5 * (c - u)).cpu()
    want, want0 = ddim_ref.ddim_step(e, t, lat.cpu(), 50, acp)
    assert torch.equal(out.prev_sample.cpu(), want)
    assert torch.equal(out.pred_original_sample.cpu(), want0)


@pytest.mark.parametrize("use_graph", [True, False])
def test_denoise_loop_graph_matches_oracle(tiny_unet, gold, use_graph):
    lat = torch.from_numpy(gold["latents"]).cuda()
    ehs = torch.from_numpy(gold["ehs"]).cuda()
    s = DDIMScheduler(beta_schedule="linear", steps_offset=1, clip_sample=False)
    s.set_timesteps(50)
    loop = DenoiseLoop(tiny_unet, s, lat, ehs, 7.5, use_graph=use_graph).prime()
    if use_graph:
        assert loop.graph is not None, loop.graph_error
    x = loop.run(3)
    assert int(loop.step_idx.item()) == 3
    assert rel_l2(x, torch.from_numpy(gold["loop3_x"])) < 0.01
    with pytest.raises(RuntimeError, match="scheduled steps"):
        loop.run(48)  # 3 + 48 > the 50-step schedule: refused before anything is enqueued
    assert int(loop.step_idx.item()) == 3


@pytest.mark.parametrize("model", ["tiny", "full2"])
def test_cfg_dedup_is_bit_exact(tiny_unet, model):
    """The CFG dedup (DenoiseLoop.cfg_dedup: conv_in, resnets[0] and attentions[0] up to its
    cross-attention on one guidance half, planned as the whole batch by ops.plan_scaled) changes
    no kernel choice and no bit: the hipGraph loop with and without it is identical (tiny model at
    4 frames; the full model at 2 frames, whose level-1 path runs v8 / flash40)."""
    if model == "tiny":
        unet, shape, cdim = tiny_unet, (1, 4, 4, 64, 64), tiny_unet.config["cross_attention_dim"]
    else:
        from vdiff.weights import materialize_synthetic
        unet = materialize_synthetic("full", device="cuda", seed=0).prepare()
        shape, cdim = (1, 4, 2, 64, 64), unet.config["cross_attention_dim"]
    g = torch.Generator(device="cuda").manual_seed(5)
    lat = torch.randn(*shape, device="cuda", generator=g)
    ehs = torch.randn(2, 77, cdim, device="cuda", generator=g)
    outs = []
    for dedup in (True, False):
        s = DDIMScheduler(beta_schedule="linear", steps_offset=1, clip_sample=False)
        s.set_timesteps(50)
        loop = DenoiseLoop(unet, s, lat.clone(), ehs, 7.5, use_graph=True)
        loop.cfg_dedup = dedup
        loop = loop.prime()
        assert loop.graph is not None, loop.graph_error
        outs.append(loop.run(2).clone())
    assert torch.equal(outs[0], outs[1]), f"rel {rel_l2(outs[0], outs[1]):.2e}"


def test_euler_scheduler_api_and_graph_loop_match_oracle(tiny_unet, gold):
    """EulerDiscreteScheduler (the reference's
    01_baseline_generation.py:76-80 configuration) behind the same surface: the
    scale_model_input -> unet -> CFG -> step API on the device, and the hipGraph loop
    with the fused Euler kernel, against the oracle's 3-step Euler loop (rel-L2 1%)."""
    from oracle import euler_ref
    eu = np.load(GOLD / "euler.npz")
    lat = torch.from_numpy(gold["latents"]).cuda()
    ehs = torch.from_numpy(gold["ehs"]).cuda()
    want = torch.from_numpy(eu["loop3_x"])

    s = EulerDiscreteScheduler.from_config(DDIMScheduler().config, timestep_spacing="linspace",
                                           beta_schedule="linear")
    s.set_timesteps(25)
    x = lat * s.init_noise_sigma
    for t in s.timesteps[:3]:
        xi = s.scale_model_input(torch.cat([x, x]), t)
        eps = tiny_unet(xi, t, encoder_hidden_states=ehs).sample
        u, c = eps.chunk(2)
        out = s.step(u + 7.5 * (c - u), t, x)
        if t == s.timesteps[0]:  # exact Euler arithmetic on identical eps
            e = (u + 7.5 * (c - u)).cpu()
            w1, w0 = euler_ref.euler_step(e, x.cpu(), s.sigmas[0], s.sigmas[1])
            torch.testing.assert_close(out.prev_sample.cpu(), w1, rtol=1e-6, atol=1e-5)
            torch.testing.assert_close(out.pred_original_sample.cpu(), w0, rtol=1e-6, atol=1e-5)
        x = out.prev_sample
    assert s.step_index == 3
    assert rel_l2(x, want) < 0.01

    s.set_timesteps(25)
    loop = DenoiseLoop(tiny_unet, s, lat * s.init_noise_sigma, ehs, 7.5, use_graph=True).prime()
    assert loop.graph is not None, loop.graph_error
    x = loop.run(3)
    assert rel_l2(x, want) < 0.01


def test_full_unet_two_frames_matches_oracle(cuda):
    """The FULL SD-1.5 + motion-adapter shapes (1.31B params; every level L1-L4, d = 40/80/160
    attention, the v2/v3/v5/v6 GEMM paths at their real shapes, split-K, concat skips) on a
    2-frame CFG batch at t = 500, against the fp32 oracle on the same bf16 weights
    (~10 s of host CPU).  Bound: rel-L2 2 % (measured 1.62 % on the MI355X; the value is printed)."""
    from vdiff.weights import materialize_synthetic
    torch.manual_seed(0)
    unet = materialize_synthetic("full", device="cuda", seed=0)
    unet.prepare()
    g = torch.Generator().manual_seed(42)
    lat = torch.randn((1, 4, 2, 64, 64), generator=g).to(torch.bfloat16).float()
    ehs = torch.randn((2, 77, 768), generator=torch.Generator().manual_seed(1)).to(torch.bfloat16).float()
    x = torch.cat([lat, lat])
    got = unet(x.cuda(), 500, encoder_hidden_states=ehs.cuda()).sample.cpu()
    sd = {k: v.detach().float().cpu() for k, v in unet.state_dict().items()}
    del unet
    torch.cuda.empty_cache()
    with torch.no_grad():
        want = unet_ref.unet_forward(sd, unet_ref_cfg("full"), x, 500, ehs)
    err = rel_l2(got, want)
    print(f"full UNet (2 frames) rel-L2 vs oracle: {err:.4f}")
    assert err < 0.02, err


def test_full_blocks_match_device_emulation(cuda):
    """the tight per-block bound on the FULL model's product plan.  Every
    block of the 1.31B-parameter UNet on a 2-frame CFG batch (4 images: the 8-way rank's
    shapes — v8 on the L1 K = 320 projections, QKV and GEGLU; v6 and split-K + reduce at L2-L4;
    flash40 at S = 4096, d = 40; flash_attn at d = 80 / 160; the temporal MFMA kernel; the
    concat-skip convs), run from the device's own input, against the device-emulating oracle
    within 0.3 % rel-L2 and the fp32 oracle within 0.6 %.  Measured on the MI355X (round 5,
    profiles/r05_full_blocks.txt): 64 of the 65 blocks within the tiny model's 0.25 %; the worst,
    down_blocks.2.motion_modules.0 (C 1280, 14 bf16 stores in sequence, split-K ff2 at M 1024),
    0.253-0.266 % vs the device emulation and 0.247 % vs fp32 — about two thirds of one bf16 ulp
    (0.39 %); resnets 0.03-0.11 %, spatial transformers 0.05-0.19 %.  The table is printed.
    Round 6 bisected the level-3 excess (test_full_motion_stages_match_device_emulation): every
    stage of those blocks matches its emulation within 1e-4 from its own input, and the whole
    block sits at the emulation's own bf16 realisation floor (0.222 % there), so 0.25 % is below
    what any faithful bf16 realisation of that block can meet; the tight bound is per stage."""
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    from parity_blocks import block_errors
    from vdiff.weights import materialize_synthetic
    unet = materialize_synthetic("full", device="cuda", seed=0)
    unet.prepare()
    g = torch.Generator().manual_seed(42)
    lat = torch.randn((1, 4, 2, 64, 64), generator=g).to(torch.bfloat16).float()
    ehs = torch.randn((2, 77, 768), generator=torch.Generator().manual_seed(1)).to(torch.bfloat16).float()
    with torch.no_grad():
        rows = block_errors(unet, lat, ehs, t=500, log=print)
    del unet
    torch.cuda.empty_cache()
    assert len(rows) >= 40
    worst_dev = max(r[2] for r in rows)
    worst_32 = max(r[1] for r in rows)
    print(f"full model, worst block: vs dev {worst_dev:.5f}, vs fp32 {worst_32:.5f}")
    assert worst_dev < 0.003, rows
    assert worst_32 < 0.006, rows


def test_full_motion_stages_match_device_emulation(cuda):
    """where the device-emulating oracle and the device part on the FULL model's
    motion modules (2-frame CFG batch, the 8-way rank's product plan).  Two checks per module
    (tests/parity_blocks.py, tools/motion_bisect.py; profiles/r06_motion_bisect.txt):
      * teacher-forced stages — GroupNorm, proj_in (+ norm1 + PE), the folded norm + PE QKV GEMM,
        the temporal attention, to_out + residual (+ the next norm), GEGLU (+ folded norm3),
        ff2 + residual, proj_out + residual — each from the device's own input to it, against
        fp64 of that stage rounded where the device stores: within 1.5e-4 rel-L2 (measured
        <= 1.0e-4, the attention core; 1e-4 is 1/40 of one bf16 ulp) and <= 5e-4 of the stored
        values one ulp off (measured <= 2.8e-4).  Every kernel does the emulated arithmetic.
      * the free-running block against the emulation, bounded by the emulation's own bf16
        realisation floor: the same oracle with 2e-4 of EVERY stage's stored values moved by one
        ulp (the device's per-stage flip rate) drifts 0.10-0.22 % from itself; the device sits
        within 1.75x of that (measured 1.14x at down_blocks.2.motion_modules.0, 0.253 % vs 0.222 %).
    The level-3 blocks' 0.25-0.27 % per block (test_full_blocks_match_device_emulation) is that
    floor: 14 stores in sequence amplify a 2e-4 flip rate until the roundings decorrelate."""
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    from parity_blocks import motion_floor, motion_stages, nchw, rel
    from vdiff.weights import materialize_synthetic
    unet = materialize_synthetic("full", device="cuda", seed=0)
    unet.prepare()
    names = ["down_blocks.0.motion_modules.0", "down_blocks.1.motion_modules.0",
             "down_blocks.2.motion_modules.0", "mid_block.motion_modules.0"]
    mods = dict(unet.named_modules())
    caps = {}
    for nm in names:
        def run(x, ctx, _nm=nm, _orig=mods[nm].run):
            caps[_nm] = (x, ctx)
            return _orig(x, ctx)
        mods[nm].run = run
    g = torch.Generator().manual_seed(42)
    lat = torch.randn((1, 4, 2, 64, 64), generator=g).to(torch.bfloat16).float()
    ehs = torch.randn((2, 77, 768), generator=torch.Generator().manual_seed(1)).to(torch.bfloat16).float()
    bad = []
    with torch.no_grad():
        unet(torch.cat([lat, lat]).cuda(), 500, encoder_hidden_states=ehs.cuda())
        for nm in names:
            del mods[nm].run
            x, ctx = caps[nm]
            print(f"== {nm}")
            for st, r_emu, r_ex, flips in motion_stages(mods[nm], x, ctx, log=print):
                if not (r_emu < 1.5e-4 and flips < 5e-4):
                    bad.append((nm, st, r_emu, flips))
            got = nchw(mods[nm].run(x, ctx))
            d0, d1, _ = motion_floor(unet, nm, x, ctx.frames)
            r, floor = rel(got, d0), rel(d1, d0)
            print(f"  block: device vs emulation {r:.5f}; emulation's realisation floor {floor:.5f} ({r / floor:.2f}x)")
            if not r < 1.75 * floor:
                bad.append((nm, "block", r, floor))
    del unet
    torch.cuda.empty_cache()
    assert not bad, bad


def unet_ref_cfg(name):
    from vdiff.config import get_config
    return get_config(name)


def _errs(got, want):
    got, want = got.double().cpu(), want.double().cpu()
    return rel_l2(got, want), ((got - want).abs().max() / want.abs().max()).item()


def test_full_unet_sixteen_frames_matches_oracle(cuda):
    """BASELINE config 3's workload shape, one CFG forward: the FULL model (CPU-seeded synthetic
    weights, as the committed fixture tests/golden/full_f16_t500.npz) on all 16 frames — every
    motion module attends over F = 16 — at t = 500, against the fp32 oracle and the oracle that
    emulates the device's bf16 storage and attention arithmetic (act="dev").  Printed: rel-L2
    and max|err|/max|want| against both.  Bounds: 2 % rel-L2 against the fp32 oracle (measured
    1.48 %) and 2.2 % against the device-emulating one (measured 1.76 %) — end to end any
    two bf16 realisations of the network sit ~1.3-1.5 % apart (the fixture's own dev-vs-fp32
    is 1.48 %; test_oracle.py::test_bf16_realisation_floor), so the tight check is per block
    (test_tiny_blocks_match_device_emulation)."""
    sys.path.insert(0, str(GOLD))
    from make_full_golden import T, full_inputs
    gold = np.load(GOLD / "full_f16_t500.npz")
    unet = init_synthetic_(UNetMotionModel("full"), seed=0).to("cuda", torch.bfloat16).prepare()
    lat, ehs = full_inputs()
    got = unet(torch.cat([lat, lat]).cuda(), T, encoder_hidden_states=ehs.cuda()).sample.cpu()
    del unet
    torch.cuda.empty_cache()
    assert got.shape == (2, 4, 16, 64, 64) and torch.isfinite(got).all()
    r32, m32 = _errs(got, torch.from_numpy(gold["eps"]))
    rdv, mdv = _errs(got, torch.from_numpy(gold["eps_dev"]))
    print(f"full UNet F=16 t={T}: vs fp32 oracle rel-L2 {r32:.5f} max {m32:.5f}; "
          f"vs device-emulating oracle rel-L2 {rdv:.5f} max {mdv:.5f}")
    assert r32 < 0.02, r32
    assert rdv < 0.022, rdv
