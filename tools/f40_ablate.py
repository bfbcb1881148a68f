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
    elif name == "stamps":  # s_memtime stamps at the phase boundaries (shares, not the run time)
        assert body.count(LOOP_OLD) == 1
        body = body.replace(LOOP_OLD, LOOP_STAMPED)
        ret = "  return bad;\n}\n"
        assert body.count(ret) == 1
        body = body.replace(ret, STAMP_STORE + ret)
    elif name == "dec1":  # schedule variant (same bits): decide(t > 1) with the partner exchange up
        # front (the round-5 form; the product adopted dec2 in round 6)
        assert body.count(DEC_NEW_PRODUCT) == 1
        body = body.replace(DEC_NEW_PRODUCT, DEC_OLD)
    elif name == "dma_gap":  # schedule variant (same bits)
        if True:
            assert body.count(GAP_OLD) == 1 and body.count("    issue(t + 3);\n    mphase(t);\n") == 1
            body = body.replace(GAP_OLD, GAP_NEW)
            body = body.replace("    issue(t + 3);\n    mphase(t);\n", "    mphase(t);\n")
            anchor = "template <bool UNITC>\n__device__ __forceinline__ bool f4_loop("
            assert body.count(anchor) == 1
            body = body.replace(anchor, ISSUE_ONE + anchor)
    elif name == "qk2":
        assert body.count(QK_OLD) == 1
        body = body.replace(QK_OLD, QK_2)
    # round 6, session 3: rebalancing the two sides of a phase (the V side: decide at its head and the
    # V^T read latency drained before its barrier; the M side: the DMA issue at its head)
    if name in ("dec_even", "dec_even_vnw", "dec_even_vnw_dmav"):  # row-sum check on even tiles only
        assert body.count("    if (t > 0) decide(t);\n") == 1
        body = body.replace("    if (t > 0) decide(t);\n", "    if (t > 0 && (t & 1) == 0) decide(t);\n")
    if name in ("vnowait", "dec_even_vnw", "dec_even_vnw_dmav", "vnw_dmav"):
        # the V-end barrier without lgkmcnt(0) (V^T(t)'s slot is next overwritten two phases later; the
        # M-end barrier still drains), and no pin on the V^T fragments: their wait moves to PV's first MFMA
        old = """    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        f4_pin(vfr[0][kb][s2]);
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) f4_pin(pf[kb][s2][qb]);
      }
    if (g0) wait_tile(t + 1);
    bar();
"""
        new = """    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) f4_pin(pf[kb][s2][qb]);
      }
    if (g0) wait_tile(t + 1);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
"""
        assert body.count(old) == 1
        body = body.replace(old, new)
    if name in ("dec_even_vnw_dmav", "vnw_dmav"):  # group 1's DMA in its V phase (as dma_v)
        top = "  for (int t = 0; t < T; ++t) {\n"
        assert body.count(top) == 1 and body.count("    issue(t + 3);\n    mphase(t);\n") == 1
        body = body.replace(top, top + "    if (!g0) issue(t + 3);\n")
        body = body.replace("    issue(t + 3);\n    mphase(t);\n", "    if (g0) issue(t + 3);\n    mphase(t);\n")
    if name == "stamps":
        anchor = "  // prologue: tiles 0 and 1 in flight, tile 0 landed everywhere\n"
        assert body.count(anchor) == 1
        body = body.replace(anchor, "  unsigned long long st_[8] = {0, 0, 0, 0, 0, 0, 0, 0};\n" + anchor)
        top = "  for (int t = 0; t < T; ++t) {\n"
        assert body.count(top) == 1
        body = body.replace(top, "  unsigned long long tp_ = f4_stamp();\n" + top)
        body = STAMP_DEFS + body
    out = text[:i0] + body + text[i1:]
    if name in ("novphase", "nomphase"):  # their outputs are garbage / NaN: keep the exact fix-up pass out
        flag = "    return out_f32 ? __builtin_isnan(((const float*)o)[f]) : ((o[f] & 0x7FFF) > 0x7F80);"
        assert out.count(flag) == 1
        out = out.replace(flag, "    return false;")
    return out


LOOP_OLD = """    if (t > 0) decide(t);
    softmax();
    __builtin_amdgcn_sched_barrier(0);
    read_v(t, 0);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        f4_pin(vfr[0][kb][s2]);
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) f4_pin(pf[kb][s2][qb]);
      }
    if (g0) wait_tile(t + 1);
    bar();
    issue(t + 3);
    mphase(t);
    if (!g0) wait_tile(t + 2);
    bar();
  }
"""
LOOP_STAMPED = """    if (t > 0) decide(t);
    F4ST(0);
    softmax();
    __builtin_amdgcn_sched_barrier(0);
    F4ST(1);
    read_v(t, 0);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        f4_pin(vfr[0][kb][s2]);
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) f4_pin(pf[kb][s2][qb]);
      }
    if (g0) wait_tile(t + 1);
    F4ST(2);
    bar();
    F4ST(3);
    issue(t + 3);
    F4ST(4);
    mphase(t);
    F4ST(5);
    if (!g0) wait_tile(t + 2);
    F4ST(6);
    bar();
    F4ST(7);
  }
"""
# the stamp (MI355X guide idiom: s_memtime + lgkmcnt(0) in one statement, sched barriers around it),
# the per-wave scalar sums, and their store after the loop (lane 0 of each wave, a buffer of its own)
STAMP_DEFS = """
__device__ unsigned long long f4_stamp_buf[256][8][9];
__device__ __forceinline__ unsigned long long f4_stamp() {
  unsigned long long x;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\\n\\ts_waitcnt lgkmcnt(0)" : "=s"(x) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return x;
}
#define F4ST(i) do { const unsigned long long a_ = f4_stamp(); st_[i] += a_ - tp_; tp_ = a_; } while (0)
extern "C" int f4_stamp_read(void* dst) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(f4_stamp_buf), sizeof(f4_stamp_buf));
}
"""
STAMP_STORE = """  {
    const int w_ = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (blockIdx.x < 256 && (threadIdx.x & 63) == 0) {
      for (int i = 0; i < 8; ++i) f4_stamp_buf[blockIdx.x][w_][i] = st_[i];
      f4_stamp_buf[blockIdx.x][w_][8] = (unsigned long long)T;
    }
  }
"""

# decide(t > 1) without the partner exchange: the wave-wide any() over the lanes that hold a row
# sum (half L_H) is the same decision; the exchange moves into the (rare) rescale branch
DEC_OLD = """      float lq[QB];
      bool resc = false, over = false;
#pragma unroll
      for (int qb = 0; qb < QB; ++qb) {
        const float lown = oacc[C::L_DB][qb][C::L_I];
        const float lp = partner32(lown);
        lq[qb] = hh == C::L_H ? lown : lp;
        resc |= lq[qb] > RESCALE;
        over |= !(lq[qb] < BAD);
      }
      if (__any(over)) {
        bad = true;
      } else if (__any(resc)) {
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) {"""
DEC_NEW = """      bool resc = false, over = false;
      const bool own = hh == C::L_H;
#pragma unroll
      for (int qb = 0; qb < QB; ++qb) {
        const float lown = oacc[C::L_DB][qb][C::L_I];
        resc |= own && lown > RESCALE;
        over |= own && !(lown < BAD);
      }
      if (__any(over)) {
        bad = true;
      } else if (__any(resc)) {
        float lq[QB];
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) {
          const float lown = oacc[C::L_DB][qb][C::L_I];
          const float lp = partner32(lown);
          lq[qb] = own ? lown : lp;
        }
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) {"""
DEC_NEW_PRODUCT = DEC_NEW.replace(
    "      bool resc = false, over = false;\n      const bool own = hh == C::L_H;",
    "      // the wave-wide any() over the lanes that hold a row sum (half L_H) is the decision; the\n"
    "      // partner exchange is needed only for a rescale (round 6: -0.7 %, profiles/r06_flash40_ablations.txt)\n"
    "      bool resc = false, over = false;\n      const bool own = hh == C::L_H;")
# the M phase's two DMA pieces in PV(d-block 0)'s empty MFMA gaps 6 and 7 instead of before its first MFMA
GAP_OLD = """        if (r < 8) read_v1_piece(t, r);
        else if (r < 11 && more) read_k0_piece(t + 1, r - 8);
      }
"""
GAP_NEW = """        if (r < 8) read_v1_piece(t, r);
        else if (r < 11 && more) read_k0_piece(t + 1, r - 8);
      }
      if (i >= 6 && issuer && t + 3 < T) f4_issue_one(dma, lds0, t + 3, skv, i - 6);
"""
ISSUE_ONE = """__device__ __forceinline__ void f4_issue_one(const F4Dma& m, uint32_t lds0, int t, int64_t skv, int i) {
  const uint32_t key0 = (uint32_t)t * KT;
  const uint32_t slot = lds0 + (uint32_t)(t % F4_RING) * F4_SLOT;
  const uint32_t off = m.step[i] ? m.voff[i] + key0 * m.step[i] : ((int64_t)(key0 + m.row[i]) < skv ? 0u : 16u);
  f4_dma(m.rs[i], slot + m.lds[i], off);
}

"""

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
    call(libs["product"])
    ref = out.clone()
    for a, lb in libs.items():
        if a != "product":
            out.zero_()
            call(lb)
            torch.cuda.synchronize()
            print(f"{a:8s} output {'bit-identical to' if torch.equal(out, ref) else 'DIFFERS from'} the product's", flush=True)
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
    if "stamps" in libs:
        import numpy as np
        buf = np.zeros((256, 8, 9), dtype=np.uint64)
        lb = libs["stamps"]
        lb.f4_stamp_read.argtypes, lb.f4_stamp_read.restype = [C.c_void_p], C.c_int
        torch.cuda.synchronize()
        assert lb.f4_stamp_read(buf.ctypes.data) == 0
        segs = ["decide", "softmax", "vtail+wait", "bar(V end)", "dma issue", "mphase", "wait(g1)", "bar(M end)"]
        per = buf[:, :, :8].astype(np.float64) / np.maximum(buf[:, :, 8:9].astype(np.float64), 1)
        print("stamps: cycles per loop iteration (s_memtime ticks), mean over the first 256 workgroups of the "
              "last stamped launch; each stamp itself costs ~40", flush=True)
        for gname, ws in (("group 0 (waves 0-3)", slice(0, 4)), ("group 1 (waves 4-7)", slice(4, 8))):
            m = per[:, ws, :].mean(axis=(0, 1))
            print(f"  {gname}: " + "  ".join(f"{s} {v:6.0f}" for s, v in zip(segs, m)) + f"  | total {m.sum():6.0f}",
                  flush=True)
        for w in range(8):
            m = per[:, w, :].mean(axis=0)
            print(f"    wave {w}: " + " ".join(f"{v:6.0f}" for v in m), flush=True)
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
