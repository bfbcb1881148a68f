"""Host-side packing logic (CPU): the weight layouts the HIP kernels assume."""
import torch
import torch.nn.functional as F

from vdiff.dist import block_transpose_reference
from vdiff.models.layers import pack_conv3x3, pack_geglu
from vdiff.pipeline import SyntheticTextEncoder
from vdiff.weights import init_synthetic_
from vdiff.models import UNetMotionModel


def im2col_nhwc(x_nhwc, stride=1):
    """K index = tap*Cin + ci, tap = 3*dy + dx: the order csrc/gemm.hip gathers."""
    n, h, w, c = x_nhwc.shape
    xp = F.pad(x_nhwc, (0, 0, 1, 1, 1, 1))
    ho, wo = (h - 1) // stride + 1, (w - 1) // stride + 1
    cols = []
    for dy in range(3):
        for dx in range(3):
            cols.append(xp[:, dy:dy + stride * (ho - 1) + 1:stride, dx:dx + stride * (wo - 1) + 1:stride, :])
    return torch.cat(cols, -1).reshape(n * ho * wo, 9 * c), ho, wo


def test_conv_pack_matches_conv2d():
    torch.manual_seed(0)
    x = torch.randn(2, 16, 9, 7)
    w = torch.randn(24, 16, 3, 3)
    for stride in (1, 2):
        want = F.conv2d(x, w, stride=stride, padding=1)
        cols, ho, wo = im2col_nhwc(x.permute(0, 2, 3, 1), stride)
        got = (cols @ pack_conv3x3(w).float().T).reshape(2, ho, wo, 24).permute(0, 3, 1, 2)
        wb = w.to(torch.bfloat16).float()
        want = F.conv2d(x, wb, stride=stride, padding=1)
        assert torch.allclose(got, want, atol=1e-4)


def test_conv_pack_channel_padding():
    w = torch.randn(8, 4, 3, 3)
    p = pack_conv3x3(w, cin_pad=8).reshape(8, 9, 8)
    assert torch.all(p[:, :, 4:] == 0)
    assert torch.equal(p[:, :, :4].float(), w.permute(0, 2, 3, 1).reshape(8, 9, 4).to(torch.bfloat16).float())


def test_geglu_pack_interleave():
    w = torch.arange(64 * 3, dtype=torch.float32).reshape(64, 3)
    p = pack_geglu(w)
    h, g = w[:32], w[32:]
    assert torch.equal(p[0:16], h[0:16]) and torch.equal(p[16:32], g[0:16])
    assert torch.equal(p[32:48], h[16:32]) and torch.equal(p[48:64], g[16:32])


def test_block_transpose_reference():
    src = torch.arange(2 * 3 * 4).reshape(24, 1).float().repeat(1, 8)
    dst = block_transpose_reference(src, 2, 3, 4)
    # dst block (a, b) = src block (b, a)
    for a in range(3):
        for b in range(2):
            assert torch.equal(dst[(a * 2 + b) * 4:(a * 2 + b + 1) * 4], src[(b * 3 + a) * 4:(b * 3 + a + 1) * 4])


def test_synthetic_weights_deterministic_and_bf16_exact():
    m1 = init_synthetic_(UNetMotionModel("tiny"), seed=0)
    m2 = init_synthetic_(UNetMotionModel("tiny"), seed=0)
    for (n, a), (_, b) in zip(m1.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), n
    w = m1.down_blocks[0].resnets[0].conv1.weight
    assert torch.equal(w, w.to(torch.bfloat16).float())
    assert abs(float(m1.down_blocks[0].resnets[0].norm1.weight.mean()) - 1.0) < 0.02
    assert abs(float(w.std()) - 0.02) < 0.002


def test_text_encoder_stub_deterministic():
    e = SyntheticTextEncoder(64)
    assert torch.equal(e("a cat"), e("a cat")) and not torch.equal(e("a cat"), e("a dog"))
    assert e("").shape == (77, 64)


def test_prepare_latents_follows_randn_tensor_cpu_fp16():
    """SURVEY §8a a14 / VERDICT r1: the reference draws x_T with its CPU generator
    (05_grid_search_ablation.py:156 torch.manual_seed(42)) in the pipeline dtype float16
    (05:35, 05:130-134) through diffusers' randn_tensor (draw on the generator's device in
    that dtype, then move); the pipeline restates exactly that, then keeps fp32."""
    import torch
    from vdiff import AnimateDiffPipeline, UNetMotionModel
    with torch.device("meta"):
        unet = UNetMotionModel("tiny")
    pipe = AnimateDiffPipeline(unet.to_empty(device="cpu"))
    pipe.torch_dtype = torch.float16  # from_pretrained(..., torch_dtype=torch.float16), as 05:130-134
    x = pipe.prepare_latents(1, 16, 64, 64, generator=torch.manual_seed(42))
    want = torch.randn((1, 4, 16, 64, 64), generator=torch.manual_seed(42), dtype=torch.float16)
    assert x.dtype == torch.float32 and torch.equal(x, want.float())
    # torch_dtype=None: diffusers draws in prompt_embeds.dtype = fp32
    pipe.torch_dtype = None
    x = pipe.prepare_latents(1, 16, 64, 64, generator=torch.manual_seed(42))
    assert torch.equal(x, torch.randn((1, 4, 16, 64, 64), generator=torch.manual_seed(42)))


def test_randn_tensor_generator_devices():
    """diffusers randn_tensor semantics (AnimateDiffPipeline.prepare_latents): draw on the
    generator's device, a list of generators draws one batch row each, and a CUDA generator
    cannot feed a CPU target."""
    import torch
    from vdiff.utils import randn_tensor
    x = randn_tensor((2, 4, 3, 8, 8), generator=torch.Generator().manual_seed(7), device="cpu",
                     dtype=torch.float16)
    assert torch.equal(x, torch.randn((2, 4, 3, 8, 8), generator=torch.Generator().manual_seed(7),
                                      dtype=torch.float16))
    gens = [torch.Generator().manual_seed(s) for s in (1, 2)]
    y = randn_tensor((2, 4, 3, 8, 8), generator=gens, device="cpu", dtype=torch.float32)
    assert torch.equal(y[1:], torch.randn((1, 4, 3, 8, 8), generator=torch.Generator().manual_seed(2)))

    class FakeCudaGen:  # a CUDA generator object needs a GPU; only its .device is read first
        device = torch.device("cuda")
    import pytest
    with pytest.raises(ValueError, match="Cannot generate"):
        randn_tensor((1, 4), generator=FakeCudaGen(), device="cpu")
