"""The frame-sharded path on the real RCCL backend (world_size 1 on the 1-GPU box).

With one rank every collective is an identity, so the sharded denoise loop must
reproduce the unsharded one exactly — while exercising the real code path the
8-GPU run takes: GroupNorm partials all-gathered through RCCL, the motion-module
re-shard (vd_block_transpose + all_to_all_single), the final frame all-gather,
and all of it captured into the step's hipGraph.  The multi-rank decomposition
itself is checked on CPU (tests/test_dist.py, gloo, world_size 2).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist

from vdiff import DDIMScheduler, DenoiseLoop, UNetMotionModel, init_synthetic_
from vdiff.dist import FrameShard

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def pg(cuda):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


def test_sharded_loop_world1_matches_unsharded(pg):
    torch.manual_seed(0)
    unet = init_synthetic_(UNetMotionModel("tiny"), seed=3).to("cuda", torch.bfloat16).prepare()
    lat = torch.randn(1, 4, 4, 64, 64, device="cuda")
    ehs = torch.randn(2, 77, 64, device="cuda")
    s = DDIMScheduler(beta_schedule="linear", steps_offset=1, clip_sample=False)
    s.set_timesteps(50)
    ref = DenoiseLoop(unet, s, lat, ehs, 7.5, use_graph=True).prime().run(2).clone()
    fs = FrameShard()
    unet.dist = fs
    try:
        loop = DenoiseLoop(unet, s, lat, ehs, 7.5, use_graph=True).prime()
        assert loop.graph is not None, f"graph capture with RCCL collectives failed: {loop.graph_error}"
        got = loop.run(2)
        out = fs.all_gather_frames(got)
    finally:
        unet.dist = None
    assert torch.equal(out, ref)


@pytest.mark.parametrize("kw", [dict(overlap_chunks=2), dict(window="kv-gather")])
def test_overlapped_window_world1_rccl_graph(pg, kw):
    """FrameShard(overlap_chunks=2) on the real RCCL backend: the chunked motion blocks run on a
    side stream joined by events, all captured into the step's hipGraph; FrameShard(window=
    "kv-gather"): the K/V all-gathers (RCCL all_gather_into_tensor) captured likewise.  At world
    size 1 every collective is an identity, so the loop must equal the unsharded one bit for bit
    (kv-gather splits the QKV GEMM into Q and KV GEMMs: same products, same fp32 sums)."""
    torch.manual_seed(0)
    unet = init_synthetic_(UNetMotionModel("tiny"), seed=3).to("cuda", torch.bfloat16).prepare()
    lat = torch.randn(1, 4, 4, 64, 64, device="cuda")
    ehs = torch.randn(2, 77, 64, device="cuda")
    s = DDIMScheduler(beta_schedule="linear", steps_offset=1, clip_sample=False)
    s.set_timesteps(50)
    ref = DenoiseLoop(unet, s, lat, ehs, 7.5, use_graph=True).prime().run(2).clone()
    fs = FrameShard(**kw)
    unet.dist = fs
    try:
        loop = DenoiseLoop(unet, s, lat, ehs, 7.5, use_graph=True).prime()
        assert loop.graph is not None, f"graph capture of the overlapped all-to-alls failed: {loop.graph_error}"
        got = loop.run(2)
        out = fs.all_gather_frames(got)
    finally:
        unet.dist = None
    assert torch.equal(out, ref)


def test_dit_sharded_loop_world1_matches_unsharded(pg):
    """The DiT's frame-sharded path (an all-to-all re-shard around every temporal block,
    tools/dit_bench.py's multi-GPU mode) on RCCL, captured into the step's hipGraph."""
    from vdiff.models.dit import DIT_TINY, DiT3DModel, DiTDenoiseLoop, init_dit_state_dict
    torch.manual_seed(0)
    m = DiT3DModel(DIT_TINY, init_dit_state_dict(DIT_TINY, seed=3), device="cuda")
    lat = torch.randn(1, 4, 4, 16, 16, device="cuda")
    ehs = torch.randn(2, 77, 64, device="cuda")
    s = DDIMScheduler(beta_schedule="linear", steps_offset=1, clip_sample=False)
    s.set_timesteps(50)
    ref = DiTDenoiseLoop(m, s, lat, ehs, 7.5, use_graph=True).prime().run(2).clone()
    loop = DiTDenoiseLoop(m, s, lat, ehs, 7.5, use_graph=True, dist=FrameShard()).prime()
    assert loop.graph is not None
    assert torch.equal(loop.run(2), ref)


def test_halo_conv3d_world1_rccl_graph(pg):
    """The kt = 3 temporal conv's frame halo (FrameShard.halo_frames: one RCCL all-gather of the
    boundary frames, no point-to-point request, no host wait) captured into a hipGraph with the
    halo'd conv (frames_in = F + 2, t_off = 1) and replayed: at world size 1 the halo is the
    video's zero padding, so the graph's output equals the unsharded 3-D conv bit for bit."""
    from vdiff import ops
    from vdiff.models.layers import pack_conv3d
    fs = FrameShard()
    B, F, h, w, ci, co = 2, 4, 16, 16, 64, 64
    g = torch.Generator(device="cuda").manual_seed(5)
    x = (torch.randn(B * F * h * w, ci, device="cuda", generator=g)).to(torch.bfloat16)
    wt = (torch.randn(co, ci, 3, 3, 3, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    wp = pack_conv3d(wt)
    full, _, _ = ops.conv3d(x, B, F, h, w, wp, kt=3, ks=3)
    out = torch.empty_like(full)

    def step():
        halo = fs.halo_frames(x, B, F, h * w)
        ops.conv3d(halo, B, F + 2, h, w, wp, kt=3, ks=3, frames_out=F, t_off=1, out=out)

    step()  # eager: communicator set-up
    torch.cuda.synchronize()
    out.zero_()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step()
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, full)
