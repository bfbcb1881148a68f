"""What bounds flash80 (the level-2 d = 80 self-attention): timing-only ABLATIONS of its loop
(DIAGNOSTIC builds, wrong results, never the product library), spliced into a copy of
csrc/attention.hip and timed against the product library on the level-2 shape (32 images x 8 heads,
S = 1024, d = 80, unit scale), arms interleaved in one process (tools/f40_ablate.py's method).

  nodma     no LDS-DMA issued or waited in the loop (the ring keeps tile 0-2's bytes)
  novphase  the V phase's softmax and V^T reads removed (P = 0)
  nomphase  the M phase's MFMAs and reads removed
  noprio    (same arithmetic) the M phase without s_setprio 1
  dma_m     (same arithmetic) both groups' DMA at the head of their M phase (the first form; the product
            moved group 1's to the head of its V phase: -2.6 %; group 0's cannot move, its V(t) runs
            beside group 1's M(t - 1), which still reads the slot tile t + 3 takes)

    F80_VARIANTS=nodma,novphase,nomphase python tools/f80_ablate.py --build    # here (CPU)
    F80_VARIANTS=... python tools/f80_ablate.py                                # GPU box
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
OUT = ROOT / "tools" / "diag_f80"  # git-ignored; not gpurun-ignored (the box loads these libs)
VARIANTS = tuple(os.environ.get("F80_VARIANTS", "nodma,novphase,nomphase,dma_m").split(","))

LOOP = """    vphase(t);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) read_v(t, 0, kb, s2);
"""


def instrument(text: str, name: str) -> str:
    i0 = text.index("// ============================================================ flash80")
    i1 = text.index("// kernel (per call, test hook")
    body = text[i0:i1]
    if name == "nodma":
        for old in ("    if (g0) issue(t + 3);\n", "    if (!g0) issue(t + 3);\n"):
            assert body.count(old) == 1
            body = body.replace(old, "")
        for w in ("    if (g0) wait_tile(t + 1);\n", "    if (!g0) wait_tile(t + 2);\n"):
            assert body.count(w) == 1
            body = body.replace(w, "")
    elif name == "novphase":
        assert body.count(LOOP) == 1
        body = body.replace(LOOP, "    if (t == 0) vphase(t);\n")
    elif name == "noprio":
        assert body.count("    __builtin_amdgcn_s_setprio(1);\n") == 1
        body = body.replace("    __builtin_amdgcn_s_setprio(1);\n", "")
    elif name == "dma_m":  # (same arithmetic) both groups' DMA in their M phase (the first form)
        for old, new in (("    if (!g0) issue(t + 3);\n", ""), ("    if (g0) issue(t + 3);\n", "    issue(t + 3);\n")):
            assert body.count(old) == 1
            body = body.replace(old, new)
    elif name == "nomphase":
        assert body.count("    mphase(t);\n") == 1
        body = body.replace("    mphase(t);\n", "")
    return text[:i0] + body + text[i1:]


def build():
    sys.path.insert(0, str(PKG))
    import build_ext as B
    OUT.mkdir(exist_ok=True)
    for name in VARIANTS:
        src_dir = OUT / f"src_{name}"
        src_dir.mkdir(exist_ok=True)
        (src_dir / "attention.hip").write_text(instrument((B.CSRC / "attention.hip").read_text(), name))
        defs = ['-DVD_BUILD_HASH="diag"', f'-DVD_BUILD_ARCH="{B.ARCH}"', f"-I{B.CSRC}", f"-I{ROOT / 'include'}"]
        obj = OUT / f"attention_{name}.o"
        subprocess.run([B.HIPCC, *B.CFLAGS, *defs, "-c", str(src_dir / "attention.hip"), "-o", str(obj)], check=True)
        objs = [str(obj)] + [str(p) for p in sorted(B.BUILD.glob("*.o")) if p.stem != "attention"]
        lib = OUT / f"libvdiff_f80_{name}.so"
        subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(lib), *objs,
                        "-L/opt/rocm/lib", "-lrccl"], check=True)
        print("built", lib)


def run(rounds: int):
    import torch
    sys.path.insert(0, str(PKG))
    from vdiff._lib import SIGNATURES, lib as product_lib
    libs = {"product": product_lib()}
    for name in VARIANTS:
        lb = C.CDLL(str(OUT / f"libvdiff_f80_{name}.so"), mode=os.RTLD_NOW | os.RTLD_LOCAL)
        argt, rest = SIGNATURES["vd_attention_ex"]
        lb.vd_attention_ex.argtypes, lb.vd_attention_ex.restype = argt, rest
        libs[name] = lb
    imgs, heads, S, d = 32, 8, 1024, 80
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
    torch.cuda.synchronize()
    ref = out.clone()
    for a, lb in libs.items():
        if a != "product":
            out.zero_()
            call(lb)
            torch.cuda.synchronize()
            print(f"{a:9s} output {'bit-identical to' if torch.equal(out, ref) else 'DIFFERS from'} the product's", flush=True)
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
        print(f"{a:9s} median {med:7.1f} us ({med / base - 1:+6.1%})  min {t[0]:.1f} max {t[-1]:.1f}  "
              f"(product-FLOP rate {fl / med / 1e6:6.1f} TF/s)", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--rounds", type=int, default=9)
    args = ap.parse_args()
    build() if args.build else run(args.rounds)
