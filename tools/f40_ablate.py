"""What bounds flash40 (the roofline kernel): timing-only ABLATIONS of its loop (DIAGNOSTIC builds,
wrong results, never the product library), spliced into a copy of csrc/attention.hip at build time
and timed against the product library on the level-1 shape (32 images x 8 heads, S = 4096, d = 40,
bench.py's `synthetic` inputs), arms interleaved in one process:

  noexp   the V phase's 64 v_exp_f32 per wave-tile removed (P = bf16(s - mu) instead of exp2):
          what the exp issue costs;
  pv1half half of the PV d-block-1 MFMAs skipped (4 of the 28 per wave-tile): what a 16x16x32 PV for
          d 32..47 (the d = 40 -> 48 pad instead of -> 64) would save in matrix-pipe time, before
          the 16 permlane16_swap per wave-tile that form needs to re-lay P;
  qk2     one of QK^T's three k-steps per key block skipped (12 -> 8 MFMAs): the QK share;
  novphase / nomphase  one phase's work removed (V: decide, softmax, V reads; M: its MFMAs and
          reads): each phase alone, behind the same barriers and DMA;
  vread_early  the V phase's V^T fragment reads issued before its exps (their LDS latency under
          the exps instead of after them) — a schedule variant with the same arithmetic;
  dma_v   group 1's LDS-DMA pieces issued at the start of its V phase (the round-5 schedule) instead
          of its M phase (as group 0's; adopted in round 6 after the dma_m arm of this tool measured
          -1.6 %) — a schedule variant with the same arithmetic;
  ord_qpq / ord_qqp  the M phase as PV(d0) QK(k0) PV(d1) QK(k1) / PV(d0) QK QK PV(d1) instead of
          PV(d0) PV(d1) QK QK — schedule variants with the same arithmetic (F40_VARIANTS=... selects).

    python tools/f40_ablate.py --build    # here (CPU): tools/diag_f40/libvdiff_f40_*.so
    python tools/f40_ablate.py            # GPU box
"""
from __future__ import annotations

import argparse
import ctypes as C
import math
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "video-diffusion-experiments_amd"
OUT = ROOT / "tools" / "diag_f40"  # git-ignored; not gpurun-ignored (the box loads these libs)

EXP_F4 = ("  auto softmax = [&]() {  // V(t): S(t) -> P(t), exp2 and bf16 packs only",
          "f[j] = (__bf16)__builtin_amdgcn_exp2f(UNITC ? s[kb][qb][8 * s2 + j] : s[kb][qb][8 * s2 + j] * c);",
          "f[j] = (__bf16)(UNITC ? s[kb][qb][8 * s2 + j] : s[kb][qb][8 * s2 + j] * c);")
PV_OLD = """  auto pv = [&](int db) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
          oacc[db][qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vfr[db][kb][s2], pf[kb][s2][qb], oacc[db][qb], 0, 0, 0);
  };"""
PV_HALF = """  auto pv = [&](int db) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
          if (db == 0 || s2 == 0)
            oacc[db][qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vfr[db][kb][s2], pf[kb][s2][qb], oacc[db][qb], 0, 0, 0);
  };"""
M_OLD = """    v1_join();
    if (more) read_k(t + 1, 1);
    __builtin_amdgcn_sched_barrier(0);
    pv(1);
    __builtin_amdgcn_sched_barrier(0);
    if (more) {
      qk(0);
      qk(1);
    }
"""
M_QPQ = """    v1_join();
    if (more) read_k(t + 1, 1);
    __builtin_amdgcn_sched_barrier(0);
    if (more) qk(0);
    __builtin_amdgcn_sched_barrier(0);
    pv(1);
    __builtin_amdgcn_sched_barrier(0);
    if (more) qk(1);
"""
M_QQP = """    v1_join();
    if (more) read_k(t + 1, 1);
    __builtin_amdgcn_sched_barrier(0);
    if (more) {
      qk(0);
      qk(1);
    }
    __builtin_amdgcn_sched_barrier(0);
    pv(1);
"""
QK_OLD = """  auto qk = [&](int kb) {  // S(kb) = K'.Q'^T from the fragments read_k left
#pragma unroll
    for (int ks = 0; ks < 3; ++ks)"""
QK_2 = """  auto qk = [&](int kb) {  // S(kb) = K'.Q'^T from the fragments read_k left
#pragma unroll
    for (int ks = 0; ks < 3; ks += 2)"""


SOFTMAX_CALL = """    if (t > 0) decide(t);
    softmax();
    __builtin_amdgcn_sched_barrier(0);
    read_v(t, 0);
"""
MPHASE_CALL = """    mphase(t);
"""


def instrument(text: str, name: str) -> str:
    i0 = text.index("// ============================================================ flash40")
    i1 = text.index("// kernel (per call, test hook")
    body = text[i0:i1]
    if name == "noexp":
        anchor, old, new = EXP_F4
        j = body.index(anchor)
        k = body.index(old, j)
        body = body[:k] + new + body[k + len(old):]
    elif name == "pv1half":
        assert body.count(PV_OLD) == 1
        body = body.replace(PV_OLD, PV_HALF)
    elif name in ("ord_qpq", "ord_qqp"):  # schedule variants with the product's arithmetic (same bits)
        assert body.count(M_OLD) == 1
        body = body.replace(M_OLD, M_QPQ if name == "ord_qpq" else M_QQP)
    elif name == "vread_early":  # schedule variant (same bits): tile t's V^T reads before the exps
        assert body.count(SOFTMAX_CALL) == 1
        body = body.replace(SOFTMAX_CALL, """    read_v(t, 0);
    __builtin_amdgcn_sched_barrier(0);
    if (t > 0) decide(t);
    softmax();
    __builtin_amdgcn_sched_barrier(0);
""")
    elif name == "dma_v":  # schedule variant (same bits): group 1's DMA back in its V phase (the
        # round-5 schedule; the product adopted dma_m — group 1 issues in its M phase — in round 6)
        top = "  for (int t = 0; t < T; ++t) {\n"
        assert body.count(top) == 1 and body.count("    issue(t + 3);\n    mphase(t);\n") == 1
        body = body.replace(top, top + "    if (!g0) issue(t + 3);\n")
        body = body.replace("    issue(t + 3);\n    mphase(t);\n", "    if (g0) issue(t + 3);\n    mphase(t);\n")
    elif name == "novphase":  # the V phase's work removed (decide, softmax, V reads): M phase alone
        assert body.count(SOFTMAX_CALL) == 1
        body = body.replace(SOFTMAX_CALL, "")
        assert body.count("    bad |= __any(over);") == 1  # garbage P: never flag the block (no fix-up pass)
        body = body.replace("    bad |= __any(over);", "")
    elif name == "nomphase":  # the M phase's MFMAs and reads removed: V phase alone
        assert body.count(MPHASE_CALL) == 1
        body = body.replace(MPHASE_CALL, "")
    elif name == "qk2":
        assert body.count(QK_OLD) == 1
        body = body.replace(QK_OLD, QK_2)
    out = text[:i0] + body + text[i1:]
    if name in ("novphase", "nomphase"):  # their outputs are garbage / NaN: keep the exact fix-up pass out
        flag = "    return out_f32 ? __builtin_isnan(((const float*)o)[f]) : ((o[f] & 0x7FFF) > 0x7F80);"
        assert out.count(flag) == 1
        out = out.replace(flag, "    return false;")
    return out


VARIANTS = tuple(os.environ.get("F40_VARIANTS", "noexp,pv1half,qk2").split(","))


def build():
    sys.path.insert(0, str(PKG))
    import build_ext as B
    OUT.mkdir(exist_ok=True)
    for name in VARIANTS:
        src_dir = OUT / f"src_f40_{name}"
        src_dir.mkdir(exist_ok=True)
        (src_dir / "attention.hip").write_text(instrument((B.CSRC / "attention.hip").read_text(), name))
        defs = ['-DVD_BUILD_HASH="diag"', f'-DVD_BUILD_ARCH="{B.ARCH}"', f"-I{B.CSRC}", f"-I{ROOT / 'include'}"]
        obj = OUT / f"attention_{name}.o"
        subprocess.run([B.HIPCC, *B.CFLAGS, *defs, "-c", str(src_dir / "attention.hip"), "-o", str(obj)], check=True)
        objs = [str(obj)] + [str(p) for p in sorted(B.BUILD.glob("*.o")) if p.stem != "attention"]
        lib = OUT / f"libvdiff_f40_{name}.so"
        subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(lib), *objs,
                        "-L/opt/rocm/lib", "-lrccl"], check=True)
        print("built", lib)


def run(rounds: int):
    import torch
    sys.path.insert(0, str(PKG))
    from vdiff._lib import SIGNATURES, lib as product_lib
    libs = {"product": product_lib()}
    for name in VARIANTS:
        lb = C.CDLL(str(OUT / f"libvdiff_f40_{name}.so"), mode=os.RTLD_NOW | os.RTLD_LOCAL)
        argt, rest = SIGNATURES["vd_attention_ex"]
        lb.vd_attention_ex.argtypes, lb.vd_attention_ex.restype = argt, rest
        libs[name] = lb
    imgs, heads, S, d = 32, 8, 4096, 40
    Cc = heads * d
    g = torch.Generator(device="cuda").manual_seed(0)
    q = (torch.randn(imgs * S, Cc, device="cuda", generator=g) * 1.5 * d ** -0.5 * math.log2(math.e)).to(torch.bfloat16)
    k = (torch.randn(imgs * S, Cc, device="cuda", generator=g) * 1.5).to(torch.bfloat16)
    v = (torch.randn(imgs * S, Cc, device="cuda", generator=g) * 1.5).to(torch.bfloat16)
    out = torch.empty(imgs * S, Cc, device="cuda", dtype=torch.bfloat16)
    stream = torch.cuda.current_stream().cuda_stream
    sc = 1.0 / math.log2(math.e)

    def call(lb):
        rc = lb.vd_attention_ex(q.data_ptr(), Cc, k.data_ptr(), Cc, v.data_ptr(), Cc, out.data_ptr(), Cc, imgs, heads,
                                S, S, d, 1, sc, 0, 3, C.c_void_p(stream))
        assert rc == 0, rc

    fl = 4.0 * S * S * d * heads * imgs
    res = {a: [] for a in libs}
    for r in range(rounds + 1):
        for a, lb in libs.items():
            for _ in range(3):
                call(lb)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                call(lb)
            e1.record()
            torch.cuda.synchronize()
            if r:
                res[a].append(e0.elapsed_time(e1) * 100.0)
    base = sorted(res["product"])[len(res["product"]) // 2]
    for a, t in res.items():
        t = sorted(t)
        med = t[len(t) // 2]
        print(f"{a:8s} median {med:7.1f} us ({med / base - 1:+6.1%})  min {t[0]:.1f} max {t[-1]:.1f}  "
              f"(product-FLOP rate {fl / med / 1e6:6.1f} TF/s)", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--rounds", type=int, default=9)
    args = ap.parse_args()
    build() if args.build else run(args.rounds)
