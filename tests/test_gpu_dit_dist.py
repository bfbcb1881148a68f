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


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs():
    g = torch.Generator().manual_seed(0)
    return torch.randn(1, 4, FRAMES, 16, 16, generator=g), torch.randn(2, 77, 64, generator=g)


def _model():
    from vdiff.models.dit import DIT_TINY, DiT3DModel, init_dit_state_dict
    return DiT3DModel(DIT_TINY, init_dit_state_dict(DIT_TINY, seed=3), device="cuda")


def _sched():
    from vdiff import DDIMScheduler
    s = DDIMScheduler(beta_schedule="linear", steps_offset=1, clip_sample=False)
    s.set_timesteps(50)
    return s


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vdiff.dist import FrameShard
    from vdiff.models.dit import DiTDenoiseLoop

    class HostStagedShard(FrameShard):
        def _a2a(self, x):
            return super()._a2a(x.cpu()).to(x.device)

    try:
        lat, ehs = _inputs()
        fl = FRAMES // world
        local = lat[:, :, rank * fl:(rank + 1) * fl].cuda()
        loop = DiTDenoiseLoop(_model(), _sched(), local, ehs.cuda(), 7.5, use_graph=False,
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
