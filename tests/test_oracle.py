"""The CPU oracle against the pinned known-answers and the committed fixtures (CPU)."""
import math
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import ddim_ref, unet_ref
from vdiff.config import TINY
from vdiff.sched import DDIMScheduler

GOLD = Path(__file__).resolve().parent / "golden"


def test_alphas_cumprod_check_values():
    # SURVEY.md App. A.7 check values (fp32 cumprod of linspace(0.00085, 0.012, 1000))
    acp = ddim_ref.alphas_cumprod()
    for t, v in [(961, 0.00247833), (921, 0.00391383), (981, 0.00195883), (1, 0.99828953), (0, 0.99914998)]:
        assert abs(float(acp[t]) - v) < 5e-8, t


def test_leading_timesteps():
    assert list(ddim_ref.timesteps_leading(25)[:3]) == [961, 921, 881]
    assert ddim_ref.timesteps_leading(25)[-1] == 1
    assert list(ddim_ref.timesteps_leading(50)[:2]) == [981, 961]
    assert len(ddim_ref.timesteps_leading(15)) == 15


def test_product_scheduler_host_math_matches_oracle():
    # the reference's override idiom: from_config(base, beta_schedule="linear", ...)
    base = DDIMScheduler().config
    s = DDIMScheduler.from_config(base, beta_schedule="linear", steps_offset=1, clip_sample=False)
    tab = np.load(GOLD / "ddim_tables.npz")
    for n in (15, 25, 50):
        s.set_timesteps(n)
        assert s.timesteps.tolist() == tab[f"ts{n}"].tolist()
        np.testing.assert_array_equal(s.coefficient_table().numpy(), tab[f"coef{n}"])
    np.testing.assert_array_equal(s.alphas_cumprod.numpy(), tab["alphas_cumprod"])
    assert s.init_noise_sigma == 1.0 and s.order == 1
    x = torch.randn(3)
    assert s.scale_model_input(x, 5) is x


def test_scheduler_spacings_and_defaults():
    s = DDIMScheduler(beta_schedule="linear", timestep_spacing="trailing")
    s.set_timesteps(10)
    assert s.timesteps[0] == 999 and s.timesteps[-1] == 99
    s = DDIMScheduler(beta_schedule="linear", timestep_spacing="linspace")
    s.set_timesteps(10)
    assert s.timesteps[0] == 999 and s.timesteps[-1] == 0
    # SD-1.5 default schedule is scaled_linear
    assert DDIMScheduler().config.beta_schedule == "scaled_linear"


def test_timestep_embedding_closed_form():
    e = unet_ref.timestep_embedding(torch.tensor([0.0, 500.0]), 320)
    assert torch.allclose(e[0, :160], torch.ones(160)) and torch.allclose(e[0, 160:], torch.zeros(160))
    j = 7
    f = math.exp(-math.log(10000.0) * j / 160)
    assert abs(float(e[1, j]) - math.cos(500 * f)) < 1e-4  # fp32 argument
    assert abs(float(e[1, 160 + j]) - math.sin(500 * f)) < 1e-4


def test_sinusoidal_pe_closed_form():
    pe = unet_ref.sinusoidal_pe(32, 320)
    assert pe.shape == (1, 32, 320)
    assert float(pe[0, 3, 0]) == pytest.approx(math.sin(3.0), abs=1e-6)
    assert float(pe[0, 3, 1]) == pytest.approx(math.cos(3.0), abs=1e-6)
    assert float(pe[0, 5, 10]) == pytest.approx(math.sin(5 * math.exp(-10 * math.log(1e4) / 320)), abs=1e-6)


def test_oracle_blocks_match_torch_module_semantics():
    """Cross-check the functional oracle against torch.nn modules of the same math."""
    torch.manual_seed(0)
    C, heads = 64, 2
    sd = {}
    for n in ("to_q", "to_k", "to_v"):
        sd[f"a.{n}.weight"] = torch.randn(C, C) * 0.1
    sd["a.to_out.0.weight"] = torch.randn(C, C) * 0.1
    sd["a.to_out.0.bias"] = torch.randn(C) * 0.1
    x = torch.randn(3, 10, C)
    ref = torch.nn.MultiheadAttention(C, heads, bias=False, batch_first=True)
    with torch.no_grad():
        ref.in_proj_weight.copy_(torch.cat([sd["a.to_q.weight"], sd["a.to_k.weight"], sd["a.to_v.weight"]]))
        ref.out_proj.weight.copy_(sd["a.to_out.0.weight"])
    want = ref(x, x, x, need_weights=False)[0] + sd["a.to_out.0.bias"]
    got = unet_ref.attention(sd, "a", x, None, heads)
    assert torch.allclose(got, want, atol=1e-5)


@pytest.mark.slow
def test_oracle_reproduces_committed_fixture():
    """Regression pin: the oracle still produces the committed tiny-config eps."""
    import make_golden_path  # noqa: F401  (adds tests/golden to sys.path)
    from make_golden import tiny_inputs

    sd, lat, ehs = tiny_inputs()
    gold = np.load(GOLD / "tiny_unet.npz")
    np.testing.assert_array_equal(gold["latents"], lat.numpy())
    with torch.no_grad():
        eps = unet_ref.unet_forward(sd, TINY, torch.cat([lat, lat]), 961, ehs)
    np.testing.assert_allclose(eps.numpy(), gold["eps_t961"], rtol=1e-4, atol=1e-5)


# ---------------------------------------------------------------- Euler
def test_euler_sigma_tables_closed_form():
    """sigma_i = sqrt((1 - a_bar) / a_bar) interpolated at linspace(0, 999, n)[::-1];
    endpoints are exact training sigmas, the table ends in 0."""
    from oracle import euler_ref
    acp = ddim_ref.alphas_cumprod().double()
    sig_train = ((1 - acp) / acp) ** 0.5
    ts, sig = euler_ref.set_timesteps(25)
    assert ts[0] == 999.0 and ts[-1] == 0.0 and len(sig) == 26 and sig[-1] == 0.0
    assert abs(float(sig[0]) - float(sig_train[999])) < 1e-5 * float(sig_train[999])
    assert abs(float(sig[-2]) - float(sig_train[0])) < 1e-6
    # an interior, fractional timestep interpolates linearly between its neighbours
    t = float(ts[1])
    lo = int(math.floor(t))
    want = float(sig_train[lo]) + (t - lo) * float(sig_train[lo + 1] - sig_train[lo])
    assert abs(float(sig[1]) - want) < 1e-5 * want
    assert abs(euler_ref.init_noise_sigma(sig) - float(sig[0])) == 0  # linspace: max sigma, no sqrt(s^2+1)
    assert 25.0 < float(sig[0]) < 25.3  # linear betas (the reference override): sigma_max ~ 25.15


def test_euler_product_scheduler_matches_oracle_tables():
    """The product's host math (vdiff.EulerDiscreteScheduler built with the reference's
    override idiom) reproduces the committed oracle tables exactly."""
    from vdiff.sched import EulerDiscreteScheduler
    tab = np.load(GOLD / "euler.npz")
    s = EulerDiscreteScheduler.from_config(DDIMScheduler().config, timestep_spacing="linspace",
                                           beta_schedule="linear")
    for n in (15, 25, 50):
        s.set_timesteps(n)
        np.testing.assert_array_equal(s.timesteps.numpy(), tab[f"ts{n}"])
        np.testing.assert_array_equal(s.sigmas.numpy(), tab[f"sigmas{n}"])
        assert s.init_noise_sigma == float(tab[f"sigmas{n}"].max())
        coef = s.coefficient_table().numpy()
        np.testing.assert_array_equal(coef[:, 0], tab[f"sigmas{n}"][:-1])
        np.testing.assert_array_equal(coef[:, 1], tab[f"sigmas{n}"][1:])
        assert coef[-1, 2] == 1.0
    # step-index bookkeeping and scale_model_input (x / sqrt(sigma^2 + 1))
    s.set_timesteps(25)
    x = torch.randn(4, 8)
    y = s.scale_model_input(x, s.timesteps[0])
    assert s.step_index == 0
    torch.testing.assert_close(y, x / float(torch.sqrt((s.sigmas[0] ** 2 + 1).double()).float()), rtol=0, atol=0)
    assert s.index_for_timestep(s.timesteps[3]) == 3 and s.order == 1
    with pytest.raises(ValueError):
        s.index_for_timestep(123.456)


def test_euler_oracle_step_is_probability_flow_update():
    """The diffusers operation order reduces to x + (sigma_next - sigma) * eps up to fp32 rounding
    (docs/01_diffusion_fundamentals.md's Euler step in the sigma parameterisation)."""
    from oracle import euler_ref
    g = torch.Generator().manual_seed(3)
    x, e = torch.randn(1000, generator=g) * 14.0, torch.randn(1000, generator=g)
    got, x0 = euler_ref.euler_step(e, x, 14.6, 12.0)
    torch.testing.assert_close(got, x + (12.0 - 14.6) * e, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(x0, x - 14.6 * e, rtol=1e-6, atol=1e-5)


# ---------------------------------------------------------------- metrics
def test_metrics_oracle_pinned_to_reference_records():
    """oracle/metrics_ref.py on the committed frames of one reference experiment reproduces the
    reference's own outputs/06_grid_search_metrics record; the recorded sweep over all 78
    experiments (tests/golden/make_metrics_golden.py) stays within 1e-6 relative."""
    import json
    from oracle import metrics_ref
    d = GOLD / "metrics" / "portrait_cfg9.0_steps25"
    ref = json.loads((d / "metrics.json").read_text())
    frames = metrics_ref.load_frames_u8(d / "frames")
    assert frames.shape == (16, 512, 512, 3)
    got = metrics_ref.measure_frames(frames, lpips=[m["lpips"] for m in ref["frame_metrics"]])
    for k in ("mean_mse", "std_mse", "mean_psnr", "flicker_index", "temporal_consistency_score"):
        assert got[k] == pytest.approx(ref[k], rel=1e-6), k
    sweep = json.loads((GOLD / "metrics" / "oracle_vs_reference.json").read_text())
    assert sweep["experiments"] == 78
    exact = {k: v for k, v in sweep["max_relative_deviation"].items() if "flow" not in k and "warp" not in k}
    assert max(exact.values()) < 1e-6  # the flow / warp fields: tests/test_flow_oracle.py


def test_bf16_realisation_floor():
    """Why the whole-network bound is ~3 % and the tight parity check is per block: with bf16
    storage at every store (act="dev"), a 1e-5 relative nudge of ONE bias flips a few
    roundings, which propagate until the output has decorrelated to the full rounding-noise
    level (~1.3 % rel-L2 on the tiny UNet) — while the fp32 oracle moves by ~1e-6.  Any two bf16
    realisations (the device, the emulation, a sharded run) therefore differ end to end by
    about this floor, however exactly each op is emulated."""
    import numpy as np
    from vdiff.models import UNetMotionModel
    from vdiff.weights import init_synthetic_
    m = init_synthetic_(UNetMotionModel("tiny"), seed=0)
    sd = {k: v.float() for k, v in m.state_dict().items()}
    g = np.load(Path(__file__).resolve().parent / "golden" / "tiny_unet.npz")
    x = torch.cat([torch.from_numpy(g["latents"])] * 2)
    ehs = torch.from_numpy(g["ehs"])
    sd2 = dict(sd)
    k = "down_blocks.0.resnets.0.conv1.bias"
    sd2[k] = sd[k] * (1 + 1e-5)
    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()  # noqa: E731
    with torch.no_grad():
        d0 = torch.from_numpy(g["eps_t961_dev"])
        d1 = unet_ref.unet_forward(sd2, TINY, x, 961, ehs, act="dev")
        f0 = torch.from_numpy(g["eps_t961"])
        f1 = unet_ref.unet_forward(sd2, TINY, x, 961, ehs, act="fp32")
    floor, fp32 = rel(d1, d0), rel(f1, f0)
    print(f"bf16 realisation floor {floor:.4f}; fp32 sensitivity {fp32:.2e}")
    assert 0.005 < floor < 0.03 and fp32 < 1e-4


def test_euler_sigma_table_within_one_ulp_of_diffusers_pow_form():
    """the product tables take correctly rounded square roots (host-independent);
    diffusers computes ((1 - a) / a) ** 0.5 in torch fp32 on the host, which some hosts round
    one ulp off.  Bound the divergence from that form at 1 ulp on every training sigma."""
    import numpy as np
    import torch
    from vdiff.sched.euler import EulerDiscreteScheduler
    s = EulerDiscreteScheduler(beta_schedule="linear")
    ac = s.alphas_cumprod
    pow_form = (((1 - ac) / ac) ** 0.5).numpy().astype(np.float32)
    ours = s._sigmas_train.astype(np.float32)
    ulp = np.abs(ours.view(np.int32).astype(np.int64) - pow_form.view(np.int32).astype(np.int64))
    assert ulp.max() <= 1
    q32 = ((1 - ac) / ac).double().numpy()
    assert np.array_equal(ours, np.sqrt(q32).astype(np.float32))  # correctly rounded sqrt of the fp32 quotient
