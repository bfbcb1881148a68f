"""Frame sharding of the denoising step across the GPUs of one node.

SURVEY.md §8e: every op of the UNet is independent per frame except the 21
motion modules.  Each rank holds F/world frames of BOTH CFG halves (so the CFG
combine and the DDIM update stay local).  A motion module needs:

  1. GroupNorm statistics over all frames of a video: every rank computes its
     partial {n, mean, M2} records and they are all-gathered (tiny, latency
     bound); the finalize kernel Chan-combines world x splits records.
  2. The temporal window: rows are re-sharded frame-sharded -> position-sharded
     with an all-to-all (Ulysses-style), the whole transformer block runs
     locally over all F frames of HW/world positions, and an all-to-all brings
     the rows back.  Volume per module per rank: 2 x (world-1)/world x the
     local activation — 1/world of an all-gather of K and V,
     which is why this build uses all-to-all rather than the K/V all-gather.

Collectives go through torch.distributed (backend "nccl" = RCCL over xGMI on
MI355X, "gloo" in the CPU tests) and every one of them — the GroupNorm-record and K/V
all-gathers, the all-to-all re-shards, the conv halo's all-gather — is issued from the
capturing stream: ProcessGroupNCCL joins its internal stream to the current stream with
events, which capture as graph edges, and nothing waits on the host, so they are captured
into the step's hipGraph (tests/test_gpu_dist.py captures all three windows at world 1).
The chunked overlap issues its compute, never a collective, on the side stream.  The row permutations around the all-to-alls are
`transpose(src, nb, na, nc)` — the HIP kernel vd_block_transpose in the product
path, injected so the decomposition itself is testable on CPU.

`FrameShard(overlap_chunks=c)` (c > 1) splits each rank's positions into c chunks and
pipelines the temporal window: each chunk's transformer block runs on a second stream
(captured into the same graph through event edges) while the capturing stream carries the
neighbouring chunks' all-to-alls.  Same arithmetic, same result.
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist


class FrameShard:
    WINDOWS = ("a2a", "kv-gather")

    def __init__(self, group=None, overlap_chunks: int = 1, window: str = "a2a"):
        """window: how a motion module sees all frames — "a2a" re-shards rows frame ->
        position shards and back (two all-to-alls per transformer block, the default), or
        "kv-gather" keeps the rows frame-sharded and all-gathers every temporal attention's
        K/V over the frame shards (SURVEY §8e's north-star collective: each rank's queries
        against all frames' keys; 2 all-gathers per block, ≈ 8x the a2a bytes at N = 8)."""
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if overlap_chunks < 1:
            raise ValueError("overlap_chunks must be >= 1")
        if window not in self.WINDOWS:
            raise ValueError(f"window must be one of {self.WINDOWS}")
        self.chunks = overlap_chunks
        self.window = window
        self.fused = True  # the fused re-shard where it applies (fused_ok); False: the transposes (A/B)
        self._side = {}  # device -> compute stream of the overlapped temporal window

    def frames_local(self, frames: int) -> int:
        if frames % self.world:
            raise ValueError(f"{frames} frames do not shard over {self.world} ranks")
        return frames // self.world

    # -- GroupNorm statistics -------------------------------------------------
    def gather_gn_partials(self, ws: torch.Tensor) -> torch.Tensor:
        """[inst, splits, C, 4] per rank -> [inst, world*splits, C, 4] on every rank."""
        out = torch.empty(self.world * ws.numel(), device=ws.device, dtype=ws.dtype)
        dist.all_gather_into_tensor(out, ws.contiguous().reshape(-1), group=self.group)
        return out.reshape((self.world,) + tuple(ws.shape)).transpose(0, 1).reshape(ws.shape[0], self.world * ws.shape[1], *ws.shape[2:]).contiguous()

    def gather_gn_records(self, ws: torch.Tensor) -> torch.Tensor:
        """[inst, splits, G, 4] per rank -> rank-major [world, inst, splits, G, 4] on every rank: the
        all-gather's output as it lands, a view (vdiff.ops.gn_finalize_g merges it in
        gather_gn_partials' split order through vd_gn_finalize_g_ranks, so the result is the same
        bits without the transpose copy — round 6)."""
        out = torch.empty(self.world * ws.numel(), device=ws.device, dtype=ws.dtype)
        dist.all_gather_into_tensor(out, ws.contiguous().reshape(-1), group=self.group)
        return out.reshape((self.world,) + tuple(ws.shape))

    # -- temporal window re-shard ---------------------------------------------
    def _a2a(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        out = torch.empty_like(x) if out is None else out
        dist.all_to_all_single(out, x, group=self.group)
        return out

    def _all_gather(self, x: torch.Tensor) -> torch.Tensor:
        """[R, w] per rank -> [world*R, w], rank-major (RCCL all-gather over xGMI)."""
        out = torch.empty((self.world * x.shape[0],) + tuple(x.shape[1:]), device=x.device, dtype=x.dtype)
        dist.all_gather_into_tensor(out, x.contiguous(), group=self.group)
        return out

    def gather_kv_frames(self, kv, batch, frames_local, hw, transpose):
        """rows (b, f_loc, p) of this rank's frames -> rows (b, f, p) of ALL frames (the
        temporal K/V window of the "kv-gather" layout)."""
        allr = self._all_gather(kv)                                  # (r, b, f_loc, p)
        return transpose(allr, self.world, batch, frames_local * hw)  # (b, r, f_loc, p) = (b, f, p)

    def to_position_shards(self, h, batch, frames_local, hw, transpose):
        """rows (b, f_loc, p) of this rank's frames -> rows (b, f, p_loc) of this rank's
        hw/world positions, f over ALL frames."""
        W = self.world
        if hw % W:
            raise ValueError(f"{hw} positions do not shard over {W} ranks")
        pl = hw // W
        send = transpose(h, batch * frames_local, W, pl)           # (r', b, f_loc, pl)
        recv = self._a2a(send)                                      # (r,  b, f_loc, pl)
        return transpose(recv, W, batch, frames_local * pl)         # (b, r, f_loc, pl) = (b, f, pl)

    def to_frame_shards(self, hp, batch, frames_local, hw, transpose):
        """Inverse of to_position_shards."""
        W = self.world
        pl = hw // W
        send = transpose(hp, batch, W, frames_local * pl)           # (r', b, f_loc, pl)
        recv = self._a2a(send)                                      # (r,  b, f_loc, pl)  r = position chunk
        return transpose(recv, W, batch * frames_local, pl)         # (b, f_loc, r, pl) = (b, f_loc, p)

    # -- the fused re-shard (round 5): no transposes around the all-to-alls ---------------
    # The frame-sharded rows of a rank are (b, f_loc, p) with p = (r', j), r' the position chunk
    # rank r' takes, j < pl = hw / world.  The motion norm writes them straight into the send
    # order (r', f_loc, b, j) (vd_gn_apply_rev3 with send_perm), so what a rank receives is
    # (r, f_loc, b, j) = (f, b, j): frame-major rows of ALL frames of its pl positions of both
    # videos — the temporal attention's layout with one "video" and b*pl + j as the position
    # (frame stride batch*pl), so the transformer block runs on the received rows as they are.
    # Its output rows (f, b, j) are already in the returning all-to-all's send order (chunk r =
    # rank r's frames), and the rows that come back, (r', f_loc, b, j), are mapped into the
    # rank's (b, f_loc, r', j) layout by proj_out's epilogue (vd_gemm_desc.rmap_*, return_perm),
    # which also reads the residual there.  Four vd_block_transpose launches per motion module
    # fewer than to_position_shards / to_frame_shards, the same bytes on the wire.
    def fused_ok(self, batch: int, frames_local: int, hw: int) -> bool:
        """The fused re-shard applies: a2a window, no chunked overlap, power-of-two axes (the
        rev3 row maps are shifts)."""
        def p2(v):
            return v > 0 and v & (v - 1) == 0
        return (getattr(self, "fused", True) and self.window == "a2a" and self.chunks == 1 and hw % self.world == 0
                and all(p2(v) for v in (hw // self.world, self.world, batch, frames_local)))

    def send_perm(self, batch: int, frames_local: int, hw: int):
        """rev3 (n1, n2, inner) taking rows (b, f_loc, r', j) to the send order (r', f_loc, b, j)."""
        return (frames_local, self.world, hw // self.world)

    def return_perm(self, batch: int, frames_local: int, hw: int):
        """rev3 (n1, n2, inner) taking the returned rows (r', f_loc, b, j) to (b, f_loc, r', j)."""
        return (frames_local, batch, hw // self.world)

    def exchange(self, x: torch.Tensor) -> torch.Tensor:
        """One all-to-all of equal row chunks (chunk r to rank r), on the current stream."""
        return self._a2a(x)

    def _side_stream(self, device):
        if device not in self._side:
            self._side[device] = torch.cuda.Stream(device=device)
        return self._side[device]

    def temporal_window(self, h, batch, frames_local, hw, transpose, block):
        """rows (b, f_loc, p) of this rank's frames -> block over ALL frames of this rank's
        positions -> rows (b, f_loc, p) again.  `block(rows, batch, frames, positions)` is the
        motion module's transformer block on rows (b, f, p).  With overlap_chunks == 1 this is
        to_position_shards / block / to_frame_shards.  With c > 1 the positions are cut into c
        chunks; chunk k's block runs on a side stream while the capturing stream carries chunk
        k+1's incoming and chunk k-1's outgoing all-to-all.  (RCCL collectives must stay on the
        capturing stream: issued from a forked stream, hipGraph capture of them segfaults —
        tools/capture_probe.py; a forked COMPUTE stream captures and replays correctly.)
        The block is per position, so which positions a rank takes per chunk is free: chunk c
        sends positions (c*W + r)*pc + j to rank r, making every chunk's buffers contiguous."""
        from .. import ops  # the plan controls only (no launch)
        W, C = self.world, self.chunks
        if hw % W:
            raise ValueError(f"{hw} positions do not shard over {W} ranks")
        pl = hw // W
        if C == 1 or pl % C:
            hp = self.to_position_shards(h, batch, frames_local, hw, transpose)
            hp = block(hp, batch, frames_local * W, pl)
            return self.to_frame_shards(hp, batch, frames_local, hw, transpose)
        pc, BF, cols = pl // C, batch * frames_local, h.shape[1]
        send = transpose(h, BF, C * W, pc).view(C, W * BF * pc, cols)  # (c, r, bf, j)
        cuda = h.is_cuda
        if cuda:
            main = torch.cuda.current_stream(h.device)
            side = self._side_stream(h.device)
        recv = [self._a2a(send[0])]                                     # (s, b, f_loc, j)
        back_recv = torch.empty_like(send)                              # (c, s', bf, j)
        for c in range(C):
            if cuda:
                ev = torch.cuda.Event()
                ev.record(main)
                side.wait_event(ev)
                ctx = torch.cuda.stream(side)
            else:
                ctx = contextlib.nullcontext()
            with ctx:
                hp = transpose(recv[c], W, batch, frames_local * pc)      # (b, s, f_loc, j) = (b, f, j)
                with ops.plan_scaled(C):  # the chunk planned as the whole block: same kernels / folds
                    hp = block(hp, batch, frames_local * W, pc)
                back = transpose(hp, batch, W, frames_local * pc)        # (s, b, f_loc, j)
                if cuda:
                    done = torch.cuda.Event()
                    done.record(side)
            if cuda:
                back.record_stream(main)  # made on the side stream, read by main's all-to-all
            if c + 1 < C:
                recv.append(self._a2a(send[c + 1]))                     # overlaps chunk c's block
            if cuda:
                main.wait_event(done)
            self._a2a(back.view(W * BF * pc, cols), back_recv[c])       # (s', b, f_loc, j)
        # rows (c, s', bf, j) -> (bf, c, s', j) = (b, f_loc, p)
        return transpose(back_recv.view(C * W * BF * pc, cols), C * W, BF, pc)

    # -- temporal conv halo ------------------------------------------------------
    def halo_frames(self, x: torch.Tensor, batch: int, frames_local: int, hw: int) -> torch.Tensor:
        """rows (b, f_loc, p) -> rows (b, f_loc + 2, p): every video's local frames between the
        last frame of the previous rank and the first frame of the next (zeros at the video's
        ends = the conv's temporal zero padding) — the one-frame halo a kt = 3 temporal conv
        (ops.conv3d with frames_in = f_loc + 2, t_off = 1) needs under frame sharding.
        One all-gather of every rank's first and last frame per video (2 frames x world per
        video, ~MBs), issued on the current stream like the module's other collectives — no
        point-to-point requests and no host-side wait, so the halo is captured into the step's
        hipGraph as it is (round 3 used batch_isend_irecv + req.wait())."""
        C = x.shape[1]
        W, r = self.world, self.rank
        v = x.view(batch, frames_local, hw, C)
        ends = torch.stack([v[:, 0], v[:, -1]], 1).contiguous()                 # (b, 2, p, C)
        allr = self._all_gather(ends.view(-1, C)).view(W, batch, 2, hw, C)     # (r, b, {first, last}, p, C)
        left = allr[r - 1, :, 1] if r > 0 else torch.zeros_like(v[:, 0])     # previous rank's last frame
        right = allr[r + 1, :, 0] if r < W - 1 else torch.zeros_like(v[:, 0])  # next rank's first frame
        return torch.cat([left[:, None], v, right[:, None]], 1).reshape(-1, C)

    def all_gather_frames(self, x: torch.Tensor) -> torch.Tensor:
        """(B, C, F_loc, H, W) latents of every rank -> (B, C, F, H, W)."""
        parts = torch.empty(self.world * x.numel(), device=x.device, dtype=x.dtype)
        dist.all_gather_into_tensor(parts, x.contiguous().reshape(-1), group=self.group)
        return torch.cat(list(parts.reshape((self.world,) + tuple(x.shape)).unbind(0)), dim=2)


def rev3_reference(src: torch.Tensor, n1: int, n2: int, inner: int) -> torch.Tensor:
    """torch statement of the rev3 row map (vd_gn_apply_rev3, vd_gemm_desc.rmap_*): input row
    ((i0*n1 + i1)*n2 + i2)*inner + j goes to output row ((i2*n1 + i1)*n0 + i0)*inner + j."""
    w = src.shape[1]
    n0 = src.shape[0] // (n1 * n2 * inner)
    return src.reshape(n0, n1, n2, inner, w).permute(2, 1, 0, 3, 4).reshape(-1, w).contiguous()


def block_transpose_reference(src: torch.Tensor, nb: int, na: int, nc: int) -> torch.Tensor:
    """torch statement of vd_block_transpose (for CPU tests of the decomposition):
    dst[(a*nb + b)*nc + c] = src[(b*na + a)*nc + c]."""
    w = src.shape[1]
    return src.reshape(nb, na, nc, w).transpose(0, 1).reshape(nb * na * nc, w).contiguous()
