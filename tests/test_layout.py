"""Node layouts of the CFG batch and the frames (vdiff.dist.layout) on CPU
with gloo: rank placement, group membership and the eps exchange order of a CFG pair."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vdiff.dist import NodeLayout


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, errq):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        lay = NodeLayout("cfg-frame", 16, world=world, rank=rank)
        fr = world // 2
        assert lay.half == rank // fr and lay.frame_index == rank % fr
        assert lay.frames_local == 16 // fr
        assert (lay.frame_shard is None) == (fr == 1)
        if lay.frame_shard is not None:
            assert lay.frame_shard.world == fr and lay.frame_shard.rank == rank % fr
        assert lay.cfg_shard.index == lay.half
        # eps rows tagged by (half, frame slice): the pair gathers uncond first
        eps = torch.full((6, 4), float(100 * lay.half + lay.frame_index))
        got = lay.cfg_shard.gather_eps(eps)
        want = torch.cat([torch.full((6, 4), float(lay.frame_index)),
                          torch.full((6, 4), float(100 + lay.frame_index))])
        assert torch.equal(got, want), (rank, got[:, 0])
        # the frame group sums over exactly this half's ranks
        if lay.frame_shard is not None:
            t = torch.tensor([float(rank)])
            dist.all_reduce(t, group=lay.frame_shard.group)
            assert t.item() == sum(range(lay.half * fr, (lay.half + 1) * fr))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        errq.put(f"rank {rank}: {e!r}")
        raise


@pytest.mark.parametrize("world", [2, 4])
def test_cfg_frame_layout_gloo(world):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    mp.start_processes(_worker, args=(world, _port(), errq), nprocs=world, join=True, start_method="spawn")
    assert errq.empty()


def test_auto_layout_choice():
    r = NodeLayout.resolve
    assert r("auto", 1) == "frame"
    assert r("auto", 2) == "cfg-frame"          # one CFG half per GPU: no motion-module collective
    assert r("auto", 2, cfg=False) == "frame"
    assert r("auto", 4) == r("auto", 8) == "frame"
    with pytest.raises(ValueError):
        r("cfg-frame", 2, cfg=False)
    with pytest.raises(ValueError):
        r("cfg-frame", 3)
    with pytest.raises(ValueError):
        r("bogus", 2)
    lay = NodeLayout("frame", 16, world=1, rank=0)
    assert lay.frame_shard is None and lay.cfg_shard is None and lay.describe() == "single-GPU"
