"""Same-process A/B of one model-side switch over the whole captured denoising step.

    python tools/ab_step.py --switch ln_fold [--world 1|2|4|8] [--frames 16] [--rounds 6] [--steps 10]

Both arms are captured on ONE model in one process (each its own hipGraph), then replayed in
alternating rounds, so box-to-box clock differences cancel (MI355X_MICROARCH.md rule of same-box
A/Bs).  --world N > 1 runs rank 0 of an N-way frame-sharded step with the collectives replaced by
same-size device copies (tools/rank_emulate.py's EmulatedShard).

Switches:
  ln_fold    LayerNorm folded into its consuming v8 GEMM (BasicTransformerBlock._fold; round 5)
             against the unfolded norm -> GEMM;
  cfg_dedup  conv_in + down_blocks[0].resnets[0] once for both CFG halves (DenoiseLoop.cfg_dedup);
  mfold      the motion block's norm1 / norm2 + PE folded into the fused QKV attention (_mfold);
  pfold      the same norms + PE folded into the levels-2-4 QKV GEMM, PE as a row bias (_pfold);
  fold_v6    the folds the plan runs on v6 (a rank's levels 2-4) against the unfolded form there;
  gn_apply   vd_gn_apply_g's blocks per instance (ops.gn_apply_blocks) as GN_APPLY_SPEC="T,R" (about
             T blocks in all, at least R rows each) against the product choice;
  gn_grec    the motion norm on per-group records (vd_gn_partial_g + vd_gn_finalize_g) against
             per-channel ones (vd_gn_partial + vd_gn_finalize);
  gn_mframe  the motion norm's records per frame (ops.gn_splits_per_frame) capped at GN_MFRAME_CAP
             (default 64) against the product choice;
  gn_small   the one-launch small-image GroupNorm (vd_gn_small) against the two-launch form there;
  fold_force_v6  LayerNorm folds on a forced unsplit v6 wherever the automatic plan would not fold
             (M <= 4096: a rank's level-2 QKV; with FOLD_V6_GEGLU=1 also the GEGLU) against the
             unfolded norm -> v2 there;
  skinny     the time-embedding GEMMs (M = 2) on v9 against v1 (forced path 1);
  gn_split   vd_gn_partial_g's records per image (ops.gn_image_splits) capped at GN_SPLIT_CAP
             (default 64) and at least GN_SPLIT_ROWS (default 16) rows each."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "video-diffusion-experiments_amd"), str(ROOT / "tools")]

import torch  # noqa: E402

from vdiff import DDIMScheduler, DenoiseLoop  # noqa: E402
from vdiff.models.blocks import BasicTransformerBlock  # noqa: E402
from vdiff.weights import materialize_synthetic  # noqa: E402


def set_ln_fold(unet, on, saved):
    for m in unet.modules():
        if isinstance(m, BasicTransformerBlock):
            if id(m) not in saved:
                saved[id(m)] = getattr(m, "_fold", {})
            m._fold = saved[id(m)] if on else {}


def set_cfg_dedup(unet, on, saved):  # a hook on the loop before its capture
    def hook(lp):
        lp.cfg_dedup = on
    return hook


def set_mfold(unet, on, saved):
    for m in unet.modules():
        if isinstance(m, BasicTransformerBlock):
            key = ("m", id(m))
            if key not in saved:
                saved[key] = getattr(m, "_mfold", {})
            m._mfold = saved[key] if on else {}


def set_pfold(unet, on, saved):
    for m in unet.modules():
        if isinstance(m, BasicTransformerBlock):
            key = ("p", id(m))
            if key not in saved:
                saved[key] = getattr(m, "_pfold", {})
            m._pfold = saved[key] if on else {}


def set_fold_v6(unet, on, saved):  # folds the plan runs on v6 (levels 2-4 of a rank) vs none there
    from vdiff import ops
    orig = saved.setdefault("ln_fold_runs", ops.ln_fold_runs)

    def runs(M, w, s, *, act=0, rowbias=False):
        if not orig(M, w, s, act=act, rowbias=rowbias):
            return False
        N, K = w.shape
        d = ops.GemmDesc(a0=256, lda0=K, k0=K, a_mode=0, w=w.data_ptr(), ldw=K, M=M, N=N, K=K, bias=256, act=act,
                         out=256, ldc=N // 2 if act == ops.ACT_GEGLU else N, ln_fold_s=s.data_ptr(), ln_fold_eps=1e-5)
        if rowbias:
            d.rowbias, d.ld_rb, d.rb_div = 256, N, 1
        return on or ops.gemm_plan_of(d)[0] != 6
    ops.ln_fold_runs = runs


def set_gn_apply(unet, on, saved):
    import math

    from vdiff import ops
    orig = saved.setdefault("gn_apply_blocks", ops.gn_apply_blocks)
    t, r = (int(v) for v in os.environ.get("GN_APPLY_SPEC", "512,1").split(","))

    def blocks(n_inst, pix, C):
        return max(1, min(max(1, pix // r), math.ceil(t / n_inst)))
    ops.gn_apply_blocks = blocks if on else orig


def set_gn_split(unet, on, saved):
    from vdiff import ops
    orig = saved.setdefault("gn_image_splits", ops.gn_image_splits)
    cap, rows = int(os.environ.get("GN_SPLIT_CAP", "64")), int(os.environ.get("GN_SPLIT_ROWS", "16"))

    def splits(pix):
        return max(1, min(pix // rows, cap))
    ops.gn_image_splits = splits if on else orig


def set_skinny(unet, on, saved):
    from vdiff import ops
    orig = saved.setdefault("make_ctx", unet.make_ctx)

    def make_ctx_v1(*a, **k):
        with ops.gemm_plan(path=1):
            return orig(*a, **k)
    unet.make_ctx = orig if on else make_ctx_v1


def set_gn_grec(unet, on, saved):
    from vdiff import ops
    orig = saved.setdefault("group_norm", ops.group_norm)

    def per_channel(x, n_inst, pix, groups, eps, gamma, beta, silu=False, x1=None, gather=None, two_pass=True,
                    n_split=None, rev3=None):
        if two_pass and gather is None and rev3 is None:
            return orig(x, n_inst, pix, groups, eps, gamma, beta, silu=silu, x1=x1, n_split=n_split)
        C = x.shape[1] + (x1.shape[1] if x1 is not None else 0)
        ws = ops.gn_partial(x, C, n_inst, pix, n_split or ops.gn_splits(n_inst, pix), x1=x1)
        if gather is not None:
            ws = gather(ws)
        ss = ops.gn_finalize(ws, groups, eps, gamma, beta)
        return ops.gn_apply(x, ss, pix, silu, x1=x1, rev3=rev3)
    ops.group_norm = orig if on else per_channel


def set_gn_mframe(unet, on, saved):
    from vdiff import ops
    orig = saved.setdefault("gn_splits_per_frame", ops.gn_splits_per_frame)
    cap = int(os.environ.get("GN_MFRAME_CAP", "64"))

    def per_frame(hw):
        return max(1, min(hw // 16, cap))
    ops.gn_splits_per_frame = per_frame if on else orig


def set_gn_small(unet, on, saved):  # GN_SMALL_OFF_MAXPIX=P: the off arm keeps vd_gn_small for pix <= P
    from vdiff import ops
    orig = saved.setdefault("gn_small_chunk", ops.gn_small_chunk)
    pmax = int(os.environ.get("GN_SMALL_OFF_MAXPIX", "0"))
    ops.gn_small_chunk = orig if on else (lambda pix, C, groups: orig(pix, C, groups) if pix <= pmax else 0)


def set_fold_force_v6(unet, on, saved):
    from vdiff import ops
    from vdiff.models.layers import LnFold
    orig_runs = saved.setdefault("ln_fold_runs", ops.ln_fold_runs)
    orig_gemm = saved.setdefault("lnfold_gemm", LnFold.gemm)
    geglu = os.environ.get("FOLD_V6_GEGLU", "0") == "1"

    def forced(M, act):
        return M <= 4096 and (geglu or act != ops.ACT_GEGLU)

    def runs(M, w, s, *, act=0, rowbias=False):
        if orig_runs(M, w, s, act=act, rowbias=rowbias):
            return True
        if not forced(M, act):
            return False
        with ops.gemm_plan(path=6):
            return orig_runs(M, w, s, act=act, rowbias=rowbias)

    def gemm(self, x, act=0, pe_div=1, pe_period=1, pe_off=0):
        if orig_runs(x.shape[0], self.w, self.s, act=act, rowbias=self.pe_b is not None) or not forced(x.shape[0], act):
            return orig_gemm(self, x, act, pe_div, pe_period, pe_off)
        with ops.gemm_plan(path=6):
            return orig_gemm(self, x, act, pe_div, pe_period, pe_off)
    ops.ln_fold_runs = runs if on else orig_runs
    LnFold.gemm = gemm if on else orig_gemm


SWITCHES = {"ln_fold": set_ln_fold, "cfg_dedup": set_cfg_dedup, "mfold": set_mfold, "pfold": set_pfold,
            "fold_v6": set_fold_v6, "gn_apply": set_gn_apply, "gn_split": set_gn_split, "skinny": set_skinny, "gn_grec": set_gn_grec, "gn_mframe": set_gn_mframe, "gn_small": set_gn_small, "fold_force_v6": set_fold_force_v6}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--switch", default="ln_fold", choices=sorted(SWITCHES))
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--swap", action="store_true", help="capture and replay the off arm first (order-bias check)")
    args = ap.parse_args()
    unet = materialize_synthetic("full", device="cuda", seed=0)
    if args.world > 1:
        from rank_emulate import EmulatedShard
        unet.dist = EmulatedShard(args.world, 1, "copy")
    unet.prepare()
    fl = args.frames // args.world
    lat = torch.randn(1, 4, fl, 64, 64, device="cuda")
    ehs = torch.randn(2, 77, unet.config["cross_attention_dim"], device="cuda")
    s = DDIMScheduler(beta_schedule="linear", steps_offset=1, clip_sample=False)
    s.set_timesteps(50)
    ts = s.timesteps.repeat(1 + (args.rounds * args.steps + 10) // 50)
    saved, loops = {}, {}
    for arm in (("off", "on") if args.swap else ("on", "off")):
        hook = SWITCHES[args.switch](unet, arm == "on", saved)
        lp = DenoiseLoop(unet, s, lat.clone(), ehs, 7.5, timesteps=ts, use_graph=True)
        if callable(hook):
            hook(lp)
        loops[arm] = lp.prime()
        assert loops[arm].graph is not None, loops[arm].graph_error
        loops[arm].run(3)
    SWITCHES[args.switch](unet, True, saved)
    res = {a: [] for a in loops}
    for _ in range(args.rounds):
        for arm, lp in loops.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            lp.run(args.steps)
            torch.cuda.synchronize()
            res[arm].append(1e3 * (time.perf_counter() - t0) / args.steps)
    for arm, v in res.items():
        v = sorted(v)
        print(f"{args.switch} {arm}: world {args.world} frames/rank {fl}: median {v[len(v) // 2]:.3f} ms/step, "
              f"min {v[0]:.3f} (rounds {len(v)})", flush=True)
    print(json.dumps({"switch": args.switch, "world": args.world, "frames_local": fl,
                      "ms_per_step": {a: sorted(round(x, 3) for x in v) for a, v in res.items()}}))


if __name__ == "__main__":
    main()
