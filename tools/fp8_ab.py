"""Same-process A/B of the fp8 DiT attention (vd_attention_fp8) against earlier forms of its source:
each arm is a DIAGNOSTIC library built from a saved copy of csrc/attention_fp8.hip (plus the
product's other objects), loaded RTLD_LOCAL beside the product library, fed the same quantized
operands (DiT shape: S = 2304, d = 64, 64 images x 18 heads, the folded form ops.attention_fp8
uses), timed interleaved with HIP events, outputs compared bit for bit.

    python tools/fp8_ab.py --save NAME [--rev REV]   # here: tools/diag_fp8/src_NAME/ from git REV (default HEAD)
    python tools/fp8_ab.py --build                   # here (CPU): tools/diag_fp8/libvdiff_fp8_NAME.so per saved source
    python tools/fp8_ab.py [--rounds 9]              # GPU box
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "video-diffusion-experiments_amd"
OUT = ROOT / "tools" / "diag_fp8"  # git-ignored; not gpurun-ignored (the box loads these libs)
REL = "video-diffusion-experiments_amd/csrc/attention_fp8.hip"


def save(name: str, rev: str):
    d = OUT / f"src_{name}"
    d.mkdir(parents=True, exist_ok=True)
    src = subprocess.run(["git", "-C", str(ROOT), "show", f"{rev}:{REL}"], check=True, capture_output=True, text=True).stdout
    (d / "attention_fp8.hip").write_text(src)
    print("saved", d / "attention_fp8.hip", "from", rev)


def arms():
    return sorted(p.name[4:] for p in OUT.glob("src_*") if (p / "attention_fp8.hip").exists())


def build():
    sys.path.insert(0, str(PKG))
    import build_ext as B
    for name in arms():
        src = OUT / f"src_{name}" / "attention_fp8.hip"
        defs = ['-DVD_BUILD_HASH="diag"', f'-DVD_BUILD_ARCH="{B.ARCH}"', f"-I{B.CSRC}", f"-I{ROOT / 'include'}"]
        obj = OUT / f"attention_fp8_{name}.o"
        subprocess.run([B.HIPCC, *B.CFLAGS, *defs, "-c", str(src), "-o", str(obj)], check=True)
        objs = [str(obj)] + [str(p) for p in sorted(B.BUILD.glob("*.o")) if p.stem != "attention_fp8"]
        lib = OUT / f"libvdiff_fp8_{name}.so"
        subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(lib), *objs,
                        "-L/opt/rocm/lib", "-lrccl"], check=True)
        print("built", lib)


def run(rounds: int):
    sys.path[:0] = [str(ROOT), str(PKG)]
    import torch
    from vdiff import ops
    from vdiff._lib import SIGNATURES, lib as product_lib
    libs = {"product": product_lib()}
    for name in arms():
        lb = C.CDLL(str(OUT / f"libvdiff_fp8_{name}.so"), mode=os.RTLD_NOW | os.RTLD_LOCAL)
        argt, rest = SIGNATURES["vd_attention_fp8"]
        lb.vd_attention_fp8.argtypes, lb.vd_attention_fp8.restype = argt, rest
        libs[name] = lb
    n, heads, S, d = 64, 18, 2304, 64
    D = heads * d
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(n * S, 3 * D, device="cuda", generator=g).to(torch.bfloat16)
    q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
    out = torch.empty(n * S, D, device="cuda", dtype=torch.bfloat16)
    ws = ops.attention_fp8_quant(q, k, v, n, heads, S, S, d, q_scale=d ** -0.5 * ops.LOG2E)
    stream = torch.cuda.current_stream().cuda_stream
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731

    def call(lb):
        rc = lb.vd_attention_fp8(p(ws["q8"]), p(ws["k8"]), ws["ld8"], p(ws["qs"]), p(ws["ks"]), p(ws["vt8"]),
                                 p(ws["vs"]), p(out), out.stride(0), n, heads, S, S, d, 1.0 / ops.LOG2E,
                                 C.c_void_p(stream))
        assert rc == 0, rc

    call(libs["product"])
    torch.cuda.synchronize()
    ref = out.clone()
    for a, lb in libs.items():
        if a != "product":
            out.zero_()
            call(lb)
            torch.cuda.synchronize()
            print(f"{a:10s} output {'bit-identical to' if torch.equal(out, ref) else 'DIFFERS from'} the product's",
                  flush=True)
    fl = 4.0 * n * heads * S * S * d
    res = {a: [] for a in libs}
    for r in range(rounds + 1):
        for a, lb in libs.items():
            for _ in range(2):
                call(lb)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                call(lb)
            e1.record()
            torch.cuda.synchronize()
            if r:
                res[a].append(e0.elapsed_time(e1) / 10.0)
    base = sorted(res["product"])[len(res["product"]) // 2]
    for a, t in res.items():
        t = sorted(t)
        med = t[len(t) // 2]
        print(f"{a:10s} median {med:.4f} ms ({med / base - 1:+6.1%})  min {t[0]:.4f} max {t[-1]:.4f}  "
              f"{fl / med / 1e9:7.1f} TF/s = {fl / med / 1e9 / 5000.0:.3f} of the 5 PF fp8 dense peak", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--save")
    ap.add_argument("--rev", default="HEAD")
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--rounds", type=int, default=9)
    a = ap.parse_args()
    if a.save:
        save(a.save, a.rev)
    elif a.build:
        build()
    else:
        run(a.rounds)
