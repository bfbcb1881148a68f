"""Frame-sharded DiT (SURVEY.md §8e applied to the §8f rank 3 denoiser) on ONE MI355X:
2 and 4 processes share cuda:0, each holds 4/world of the 4 frames of both CFG halves and runs
the product path (HIP kernels; every temporal block re-shards frame -> position shards with
vd_block_transpose + an all-to-all and back), with the all-to-alls staged through gloo on the
host (RCCL refuses two ranks on one device).  The gathered latents after 2 CFG DDIM steps must
match the unsharded loop (rel-L2 < 1e-2: the GEMM plans differ with the per-rank row count).
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
FRAMES = 4
FRAMES_LONG = 20  # 2 ranks x 10 frames: the temporal blocks see 20 frames (fused-RoPE 32-frame kernel)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(frames=FRAMES):
    g = torch.Generator().manual_seed(0)
    size = 16 if frames == FRAMES else 8
    return torch.randn(1, 4, frames, size, size, generator=g), torch.randn(2, 77, 64, generator=g)


def _model(frames=FRAMES):
    from vdiff.models.dit import DIT_TINY, DiT3DModel, init_dit_state_dict
    cfg = DIT_TINY if frames == FRAMES else dict(DIT_TINY, num_frames=frames, sample_size=8)
    return DiT3DModel(cfg, init_dit_state_dict(cfg, seed=3), device="cuda")


def _sched():
    from vdiff import DDIMScheduler
    s = DDIMScheduler(beta_schedule="linear", steps_offset=1, clip_sample=False)
    s.set_timesteps(50)
    return s


def _worker(rank, world, port, out_path, frames=FRAMES):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vdiff.dist import FrameShard
    from vdiff.models.dit import DiTDenoiseLoop

    class HostStagedShard(FrameShard):
        def _a2a(self, x):
            return super()._a2a(x.cpu()).to(x.device)

    try:
        lat, ehs = _inputs(frames)
        fl = frames // world
        local = lat[:, :, rank * fl:(rank + 1) * fl].cuda()
        loop = DiTDenoiseLoop(_model(frames), _sched(), local, ehs.cuda(), 7.5, use_graph=False,
                              dist=HostStagedShard()).prime()
        mine = loop.run(2).cpu()
        parts = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine)
        if rank == 0:
            torch.save(torch.cat(parts, dim=2), out_path)
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def unsharded_ref(cuda):
    from vdiff.models.dit import DiTDenoiseLoop
    lat, ehs = _inputs()
    return DiTDenoiseLoop(_model(), _sched(), lat.cuda(), ehs.cuda(), 7.5, use_graph=False).prime().run(2).cpu()


@pytest.mark.parametrize("world", [2, 4])
def test_dit_ranks_on_one_gpu_match_unsharded(unsharded_ref, world):
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "out.pt")
        mp.start_processes(_worker, args=(world, _port(), path), nprocs=world, join=True, start_method="spawn")
        got = torch.load(path, weights_only=True)
    assert got.shape == unsharded_ref.shape
    err = ((got.double() - unsharded_ref.double()).norm() / unsharded_ref.double().norm()).item()
    assert err < 1e-2, err


def test_dit_20_frames_two_ranks_match_unsharded(cuda):
    """the sharded DiT whose temporal blocks see >= 17 frames (frames = world x
    F_local = 2 x 10) routes through the fused-RoPE 32-frame kernel on the global frame index."""
    from vdiff.models.dit import DiTDenoiseLoop
    lat, ehs = _inputs(FRAMES_LONG)
    ref = DiTDenoiseLoop(_model(FRAMES_LONG), _sched(), lat.cuda(), ehs.cuda(), 7.5,
                         use_graph=False).prime().run(2).cpu()
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "out.pt")
        mp.start_processes(_worker, args=(2, _port(), path, FRAMES_LONG), nprocs=2, join=True,
                           start_method="spawn")
        got = torch.load(path, weights_only=True)
    err = ((got.double() - ref.double()).norm() / ref.double().norm()).item()
    assert err < 1e-2, err
