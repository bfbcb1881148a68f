"""Same-process A/B of the GEMM / implicit-GEMM conv library code (csrc/gemm.hip) against earlier
forms of its source: each arm is a DIAGNOSTIC library built from a saved copy of gemm.hip (plus the
product's other objects), loaded RTLD_LOCAL beside the product library.  Every case runs through
the real vdiff.ops API with the arm's library swapped in as vdiff._lib's handle (same plan, same
descriptors), arms interleaved, outputs compared bit for bit against the product's.

Cases: the UNet's 3x3 convs at the 16-frame CFG batch (32 images) — stride 1 at every level,
the channel-concat convs of the up blocks, a stride-2 downsample, a nearest-x2 upsample — and a
(2+1)D temporal conv (kt = 3, ks = 1); GEMM_AB_CASES=geglu: the four GEGLU projections instead.

    python tools/gemm_ab.py --save NAME [--rev REV]   # here: tools/diag_gemm/src_NAME/ from git REV (default HEAD)
    python tools/gemm_ab.py --build                   # here (CPU): tools/diag_gemm/libvdiff_gemm_NAME.so
    python tools/gemm_ab.py [--rounds 7]              # GPU box
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
OUT = ROOT / "tools" / "diag_gemm"  # git-ignored; not gpurun-ignored (the box loads these libs)
REL = "video-diffusion-experiments_amd/csrc/gemm.hip"


def save(name: str, rev: str):
    d = OUT / f"src_{name}"
    d.mkdir(parents=True, exist_ok=True)
    src = subprocess.run(["git", "-C", str(ROOT), "show", f"{rev}:{REL}"], check=True, capture_output=True, text=True).stdout
    (d / "gemm.hip").write_text(src)
    print("saved", d / "gemm.hip", "from", rev)


def arms():
    return sorted(p.name[4:] for p in OUT.glob("src_*") if (p / "gemm.hip").exists())


def build():
    sys.path.insert(0, str(PKG))
    import build_ext as B
    for name in arms():
        src = OUT / f"src_{name}" / "gemm.hip"
        defs = ['-DVD_BUILD_HASH="diag"', f'-DVD_BUILD_ARCH="{B.ARCH}"', f"-I{B.CSRC}", f"-I{ROOT / 'include'}"]
        obj = OUT / f"gemm_{name}.o"
        subprocess.run([B.HIPCC, *B.CFLAGS, *defs, "-c", str(src), "-o", str(obj)], check=True)
        objs = [str(obj)] + [str(p) for p in sorted(B.BUILD.glob("*.o")) if p.stem != "gemm"]
        lib = OUT / f"libvdiff_gemm_{name}.so"
        subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(lib), *objs,
                        "-L/opt/rocm/lib", "-lrccl"], check=True)
        print("built", lib)


def run(rounds: int):
    sys.path[:0] = [str(ROOT), str(PKG)]
    import torch
    import vdiff._lib as L
    from vdiff import ops
    libs = {"product": L.lib()}
    for name in arms():
        h = C.CDLL(str(OUT / f"libvdiff_gemm_{name}.so"), mode=os.RTLD_NOW | os.RTLD_LOCAL)
        for fn, (argt, rest) in L.SIGNATURES.items():
            f = getattr(h, fn)
            f.argtypes, f.restype = argt, rest
        libs[name] = h

    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*s, scale=1.0):
        return (torch.randn(*s, device=dev, generator=g) * scale).to(torch.bfloat16)

    n = 32
    cases = []

    def conv(name, h, w, c0, cout, c1=0, stride=1, upsample=False):
        x = rnd(n * h * w, c0)
        x1 = rnd(n * h * w, c1) if c1 else None
        wt = rnd(cout, 9 * (c0 + c1), scale=(9 * (c0 + c1)) ** -0.5)
        b = torch.randn(cout, device=dev, generator=g)
        fl = 2.0 * n * (2 * h if upsample else (h - 1) // stride + 1) * (2 * w if upsample else (w - 1) // stride + 1) \
            * cout * 9 * (c0 + c1)
        cases.append((name, lambda: ops.conv3x3(x, n, h, w, wt, x1=x1, stride=stride, upsample=upsample, bias=b)[0],
                      fl))

    def geglu(name, M, N, K):  # GEGLU projection (hidden | gate interleaved, 2N rows of W) with its GELU epilogue
        a = rnd(M, K)
        wt = rnd(2 * N, K, scale=K ** -0.5)
        b = torch.randn(2 * N, device=dev, generator=g)
        cases.append((name, lambda: ops.gemm(a, wt, bias=b, act=ops.ACT_GEGLU), 2.0 * M * 2 * N * K))

    if os.environ.get("GEMM_AB_CASES") == "geglu":
        geglu("L1 GEGLU 320->2x1280", n * 64 * 64, 1280, 320)
        geglu("L2 GEGLU 640->2x2560", n * 32 * 32, 2560, 640)
        geglu("L3 GEGLU 1280->2x5120", n * 16 * 16, 5120, 1280)
        geglu("L4 GEGLU 1280->2x5120", n * 8 * 8, 5120, 1280)
    else:
        conv("L1 conv 320->320", 64, 64, 320, 320)
        conv("L2 conv 640->640", 32, 32, 640, 640)
        conv("L3 conv 1280->1280", 16, 16, 1280, 1280)
        conv("L4 conv 1280->1280", 8, 8, 1280, 1280)
        conv("L1 up concat 320+320", 64, 64, 320, 320, c1=320)
        conv("L2 up concat 640+320", 32, 32, 640, 640, c1=320)
        conv("L1 down stride 2", 64, 64, 320, 320, stride=2)
        conv("L2 upsample x2", 16, 16, 640, 640, upsample=True)
        # (2+1)D temporal half: kt = 3, ks = 1 over 2 videos x 16 frames at level 2
        xt = rnd(n * 32 * 32, 640)
        wtt = rnd(640, 3 * 640, scale=(3 * 640) ** -0.5)
        cases.append(("L2 temporal kt3", lambda: ops.conv3d(xt, 2, 16, 32, 32, wtt, kt=3, ks=1)[0],
                      2.0 * n * 32 * 32 * 640 * 3 * 640))

    def with_lib(h, fn):
        saved = L._lib
        L._lib = h
        try:
            return fn()
        finally:
            L._lib = saved

    for name, fn, fl in cases:
        ref = with_lib(libs["product"], fn)
        torch.cuda.synchronize()
        ref = ref.clone()
        same = {}
        for a, h in libs.items():
            if a != "product":
                o = with_lib(h, fn)
                torch.cuda.synchronize()
                same[a] = torch.equal(o, ref)
        res = {a: [] for a in libs}
        for r in range(rounds + 1):
            for a, h in libs.items():
                with_lib(h, fn)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    with_lib(h, fn)
                e1.record()
                torch.cuda.synchronize()
                if r:
                    res[a].append(e0.elapsed_time(e1) * 100.0)  # us per call
        med = {a: sorted(v)[len(v) // 2] for a, v in res.items()}
        line = "  ".join(f"{a} {m:7.1f} us ({fl / m / 1e6:5.0f} TF/s{'' if a == 'product' else ', ' + ('bit-identical' if same[a] else 'DIFFERS')})"
                         for a, m in med.items())
        print(f"{name:22s} {line}", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--save")
    ap.add_argument("--rev", default="HEAD")
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    if a.save:
        save(a.save, a.rev)
    elif a.build:
        build()
    else:
        run(a.rounds)
