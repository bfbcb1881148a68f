"""Frame sharding on CPU with gloo, world_size 2.

Checks the decomposition the product path uses around every motion module —
GroupNorm partial statistics all-gathered across ranks, and the all-to-all
re-shard frame-sharded <-> position-sharded — by running a sharded motion
module built from oracle primitives through vdiff.dist.FrameShard and
comparing it with the unsharded oracle motion module.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import unet_ref
from vdiff.dist import FrameShard, block_transpose_reference as bt, rev3_reference


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gn_partial(rows, B, pix):
    """[B, 1, C, 4] {n, mean, M2, 0} per channel over `pix` rows per video (the vd_gn_partial record)."""
    x = rows.reshape(B, pix, -1).double()
    mean = x.mean(1)
    m2 = ((x - mean[:, None]) ** 2).sum(1)
    n = torch.full_like(mean, pix)
    return torch.stack([n, mean, m2, torch.zeros_like(mean)], -1)[:, None].float()


def _gn_finalize(ws, groups, eps, gamma, beta):
    """Chan-combine records over splits and channels of a group -> (a, b) per (inst, channel)."""
    inst, S, C, _ = ws.shape
    ws = ws.double()
    cpg = C // groups
    r = ws.permute(0, 2, 1, 3).reshape(inst, groups, cpg * S, 4)
    n = r[..., 0].sum(-1)
    mean = (r[..., 0] * r[..., 1]).sum(-1) / n
    m2 = r[..., 2].sum(-1) + (r[..., 0] * (r[..., 1] - mean[..., None]) ** 2).sum(-1)
    rstd = (m2 / n + eps).rsqrt()
    a = rstd.repeat_interleave(cpg, 1) * gamma
    b = beta - mean.repeat_interleave(cpg, 1) * a
    return a.float(), b.float()


def sharded_motion_rows(sd, p, local, B, Fl, HW, heads, groups, fs):
    C = local.shape[1]
    ws = fs.gather_gn_partials(_gn_partial(local, B, Fl * HW))
    a, b = _gn_finalize(ws, groups, 1e-6, sd[p + ".norm.weight"].double(), sd[p + ".norm.bias"].double())
    x3 = local.reshape(B, Fl * HW, C)
    hn = (x3 * a[:, None] + b[:, None]).reshape(-1, C)
    h = unet_ref.linear(sd, p + ".proj_in", hn)
    hp = fs.to_position_shards(h, B, Fl, HW, bt)                  # (b, f, p_loc)
    Ftot, Pl = Fl * fs.world, HW // fs.world
    tok = hp.reshape(B, Ftot, Pl, C).permute(0, 2, 1, 3).reshape(B * Pl, Ftot, C)
    pe = unet_ref.sinusoidal_pe(32, C)
    tok = unet_ref.basic_transformer_block(sd, p + ".transformer_blocks.0", tok, None, heads, pe=pe,
                                           double_self=True)
    hp = tok.reshape(B, Pl, Ftot, C).permute(0, 2, 1, 3).reshape(-1, C)
    h = fs.to_frame_shards(hp, B, Fl, HW, bt)
    return unet_ref.linear(sd, p + ".proj_out", h) + local


def sharded_motion_rows_fused(sd, p, local, B, Fl, HW, heads, groups, fs):
    """The product's fused re-shard (round 5, FrameShard.send_perm / return_perm): the norm's rows
    go out in send order, the block runs on the received (frame, video, position) rows with one
    video of B*pl positions, and proj_out maps the returned rows into the rank's layout."""
    C = local.shape[1]
    ws = fs.gather_gn_partials(_gn_partial(local, B, Fl * HW))
    a, b = _gn_finalize(ws, groups, 1e-6, sd[p + ".norm.weight"].double(), sd[p + ".norm.bias"].double())
    hn = (local.reshape(B, Fl * HW, C) * a[:, None] + b[:, None]).reshape(-1, C)
    recv = fs.exchange(rev3_reference(hn, *fs.send_perm(B, Fl, HW)))   # rows (f, b, j)
    h = unet_ref.linear(sd, p + ".proj_in", recv)
    Ftot, Pl = Fl * fs.world, HW // fs.world
    tok = h.reshape(Ftot, B * Pl, C).permute(1, 0, 2)                   # (b*pl + j, f, C)
    tok = unet_ref.basic_transformer_block(sd, p + ".transformer_blocks.0", tok, None, heads,
                                           pe=unet_ref.sinusoidal_pe(32, C), double_self=True)
    back = fs.exchange(tok.permute(1, 0, 2).reshape(-1, C))             # rows (r', f_loc, b, j)
    y = unet_ref.linear(sd, p + ".proj_out", back)
    return rev3_reference(y, *fs.return_perm(B, Fl, HW)) + local


def _worker(rank, world, port, errq):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.manual_seed(0)
        fs = FrameShard()
        B, F, H, W, C = 2, 4, 4, 4, 64
        HW, Fl = H * W, F // world
        # ---- 1. re-shard round trip and content
        full = torch.arange(B * F * HW, dtype=torch.float32)[:, None].repeat(1, 8)   # rows (b, f, p)
        loc = full.reshape(B, F, HW, 8)[:, rank * Fl:(rank + 1) * Fl].reshape(-1, 8)
        hp = fs.to_position_shards(loc, B, Fl, HW, bt)
        Pl = HW // world
        want = full.reshape(B, F, HW, 8)[:, :, rank * Pl:(rank + 1) * Pl].reshape(-1, 8)
        assert torch.equal(hp, want), "to_position_shards content"
        assert torch.equal(fs.to_frame_shards(hp, B, Fl, HW, bt), loc), "round trip"
        # ---- 1b. the chunked, overlapped temporal window (FrameShard(overlap_chunks=2)) ==
        # the plain one, with a block that mixes every frame of each position
        def mix(rows, b_, f_, p_):
            r4 = rows.reshape(b_, f_, p_, -1)
            w = torch.arange(1, f_ + 1, dtype=rows.dtype).reshape(1, f_, 1, 1)
            return (r4 * w + r4.sum(1, keepdim=True)).reshape(-1, rows.shape[1])
        HW2 = 16
        base = torch.randn(B * F * HW2, 8)
        loc2 = base.reshape(B, F, HW2, 8)[:, rank * Fl:(rank + 1) * Fl].reshape(-1, 8).contiguous()
        plain = fs.temporal_window(loc2, B, Fl, HW2, bt, mix)
        over = FrameShard(overlap_chunks=2).temporal_window(loc2, B, Fl, HW2, bt, mix)
        assert torch.equal(plain, over), "overlapped temporal window"
        full_mix = mix(base, B, F, HW2).reshape(B, F, HW2, 8)[:, rank * Fl:(rank + 1) * Fl].reshape(-1, 8)
        assert torch.allclose(plain, full_mix, atol=1e-5), "temporal window content"
        # ---- 1c. the K/V all-gather window (FrameShard(window="kv-gather")): every rank ends
        # with the rows (b, f, p) of ALL frames, in the unsharded order
        kvfs = FrameShard(window="kv-gather")
        assert torch.equal(kvfs.gather_kv_frames(loc2, B, Fl, HW2, bt), base), "gather_kv_frames content"
        # ---- 2. sharded motion module == unsharded oracle
        sd = {}
        p = "m"
        sd[p + ".norm.weight"] = 1 + 0.1 * torch.randn(C)
        sd[p + ".norm.bias"] = 0.1 * torch.randn(C)
        for lin in ("proj_in", "proj_out"):
            sd[f"{p}.{lin}.weight"] = 0.1 * torch.randn(C, C)
            sd[f"{p}.{lin}.bias"] = 0.1 * torch.randn(C)
        tb = p + ".transformer_blocks.0"
        for nrm in ("norm1", "norm2", "norm3"):
            sd[f"{tb}.{nrm}.weight"] = 1 + 0.1 * torch.randn(C)
            sd[f"{tb}.{nrm}.bias"] = 0.1 * torch.randn(C)
        for at in ("attn1", "attn2"):
            for n in ("to_q", "to_k", "to_v"):
                sd[f"{tb}.{at}.{n}.weight"] = 0.3 * torch.randn(C, C)
            sd[f"{tb}.{at}.to_out.0.weight"] = 0.1 * torch.randn(C, C)
            sd[f"{tb}.{at}.to_out.0.bias"] = 0.1 * torch.randn(C)
        sd[f"{tb}.ff.net.0.proj.weight"] = 0.1 * torch.randn(8 * C, C)
        sd[f"{tb}.ff.net.0.proj.bias"] = 0.1 * torch.randn(8 * C)
        sd[f"{tb}.ff.net.2.weight"] = 0.1 * torch.randn(C, 4 * C)
        sd[f"{tb}.ff.net.2.bias"] = 0.1 * torch.randn(C)
        x = torch.randn(B * F, C, H, W) + 0.5
        ref = unet_ref.motion_module(sd, p, x, F, heads=2, groups=32, max_len=32)
        rows = x.reshape(B, F, C, HW).permute(0, 1, 3, 2)                    # (b, f, p, c)
        local = rows[:, rank * Fl:(rank + 1) * Fl].reshape(-1, C).contiguous()
        got = sharded_motion_rows(sd, p, local, B, Fl, HW, 2, 32, fs)
        want = ref.reshape(B, F, C, HW).permute(0, 1, 3, 2)[:, rank * Fl:(rank + 1) * Fl].reshape(-1, C)
        err = (got - want).abs().max().item()
        assert err < 1e-4, f"sharded motion module max err {err}"
        assert fs.fused_ok(B, Fl, HW)
        got = sharded_motion_rows_fused(sd, p, local, B, Fl, HW, 2, 32, fs)
        err = (got - want).abs().max().item()
        assert err < 1e-4, f"fused re-shard motion module max err {err}"
        # the two row maps are inverse to the old transposes' composition: send order = what
        # to_position_shards' first transpose + a frame/video swap would send
        rows = torch.arange(B * Fl * HW, dtype=torch.float32)[:, None]
        snd = rev3_reference(rows, *fs.send_perm(B, Fl, HW)).reshape(world, Fl, B, HW // world)
        src = rows.reshape(B, Fl, world, HW // world)
        assert torch.equal(snd, src.permute(2, 1, 0, 3)), "send_perm"
        # ---- 3. kt = 3 temporal conv under frame sharding: one-frame halo (all-gather) + a conv
        # over the halo'd frames with no temporal padding == the unsharded 3-D conv's frames
        Cc, Co = 8, 16
        vid = torch.randn(B, Cc, F, H, W)
        wt = torch.randn(Co, Cc, 3, 3, 3) * 0.2
        full = torch.nn.functional.conv3d(vid, wt, padding=1)                  # (B, Co, F, H, W)
        rows = vid.permute(0, 2, 3, 4, 1)[:, rank * Fl:(rank + 1) * Fl].reshape(-1, Cc).contiguous()
        halo = fs.halo_frames(rows, B, Fl, HW)                                # (b, Fl + 2, p) rows
        hv = halo.reshape(B, Fl + 2, H, W, Cc).permute(0, 4, 1, 2, 3)
        got = torch.nn.functional.conv3d(hv, wt, padding=(0, 1, 1))
        err = (got - full[:, :, rank * Fl:(rank + 1) * Fl]).abs().max().item()
        assert err < 1e-4, f"halo'd temporal conv max err {err}"
        # ---- 3b. the GroupNorm records rank-major (round 6: FrameShard.gather_gn_records, what
        # vd_gn_finalize_g_ranks merges) hold exactly gather_gn_partials' records, split order kept
        recs = torch.randn(B, 3, 32, 4) + rank
        rm = fs.gather_gn_records(recs)
        assert rm.shape == (world, B, 3, 32, 4)
        assert torch.equal(rm.transpose(0, 1).reshape(B, world * 3, 32, 4), fs.gather_gn_partials(recs))
        # ---- 4. latent all-gather over frames
        lat = torch.full((1, 4, Fl, 2, 2), float(rank))
        g = fs.all_gather_frames(lat)
        assert g.shape == (1, 4, F, 2, 2) and torch.equal(g[0, 0, :, 0, 0], torch.tensor([0., 0., 1., 1.]))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        errq.put(f"rank {rank}: {e}\n{traceback.format_exc()}")
        raise


def test_frame_shard_world2_gloo():
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, errq)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_frames_must_divide():
    class Fake(FrameShard):
        def __init__(self):
            self.world, self.rank, self.group = 3, 0, None

    with pytest.raises(ValueError):
        Fake().frames_local(16)


def _halo_worker(rank, world, port, errq):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        fs = FrameShard()
        B, F, H, W, Cc, Co = 2, 6, 4, 3, 8, 16
        Fl, HW = F // world, H * W
        g = torch.Generator().manual_seed(7)
        vid = torch.randn(B, Cc, F, H, W, generator=g)
        wt = torch.randn(Co, Cc, 3, 3, 3, generator=g) * 0.2
        full = torch.nn.functional.conv3d(vid, wt, padding=1)
        rows = vid.permute(0, 2, 3, 4, 1)[:, rank * Fl:(rank + 1) * Fl].reshape(-1, Cc).contiguous()
        halo = fs.halo_frames(rows, B, Fl, HW)
        hv = halo.reshape(B, Fl + 2, H, W, Cc).permute(0, 4, 1, 2, 3)
        # the halo frames are exactly the neighbours' boundary frames (zeros at the ends)
        for side, f in ((0, rank * Fl - 1), (Fl + 1, (rank + 1) * Fl)):
            want = vid[:, :, f] if 0 <= f < F else torch.zeros_like(vid[:, :, 0])
            assert torch.equal(hv[:, :, side], want), (rank, side)
        got = torch.nn.functional.conv3d(hv, wt, padding=(0, 1, 1))
        err = (got - full[:, :, rank * Fl:(rank + 1) * Fl]).abs().max().item()
        assert err < 1e-4, f"rank {rank}: halo'd temporal conv max err {err}"
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        errq.put(f"rank {rank}: {e}\n{traceback.format_exc()}")
        raise


def test_halo_frames_world3_gloo():
    """FrameShard.halo_frames' all-gather form with a middle rank (both neighbours present)
    and both video ends (zero halo): the halo'd per-rank temporal conv equals the full 3-D conv."""
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_halo_worker, args=(r, 3, port, errq)) for r in range(3)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
