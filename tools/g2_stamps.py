"""Where the v2 GEMM's k-tile loop spends its cycles: a DIAGNOSTIC build of the library with
s_memtime stamps in gemm2_kernel (cdna_hip_programming.md "In-kernel stamps"), never the product
library: the stamps live HERE (STAMPS below) and are spliced into a copy of csrc/gemm.hip at build
time, so the shipping kernel carries no diagnostic code.  Read the SHARES, not the run time (the stamps' lgkmcnt(0) fences
forbid overlaps the real kernel has).

    python tools/g2_stamps.py --build          # here (CPU): tools/diag_build/libvdiff_diag.so
    python tools/g2_stamps.py                  # GPU box: per-shape segment shares

Segments per k-tile and wave: ring wait (the counted vmcnt for this k-tile's LDS-DMA), barrier,
fragment reads + MFMA issue, epilogue + next DMA issue."""
from __future__ import annotations

import argparse
import ctypes as C
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "video-diffusion-experiments_amd"
OUT = ROOT / "tools" / "diag_build"
LIB = OUT / "libvdiff_diag.so"


# The stamps: (anchor inside gemm2_kernel, text inserted before it / after it).  Each anchor
# must occur exactly once in the kernel's body; instrument() fails loudly when the kernel changes.
PRELUDE = r"""
__device__ unsigned long long g2_diag[4096 * 8 * 6];
#define G2_STAMP(t)                                                                      \
  do {                                                                                   \
    __builtin_amdgcn_sched_barrier(0);                                                   \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");            \
    __builtin_amdgcn_sched_barrier(0);                                                   \
  } while (0)
"""
EPILOGUE = r"""
extern "C" int vd_diag_g2_read(void* host, int64_t n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g2_diag), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
}
extern "C" int vd_diag_g2_clear() {
  static unsigned long long z[4096 * 8 * 6];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g2_diag), z, sizeof(z), 0, hipMemcpyHostToDevice);
}
"""
STAMPS = [  # (anchor, before, after)
    ("  int stage = 0;\n", "",
     "  unsigned long long st0, st1, st2, st3, st4, sw = 0, sb = 0, sm = 0, stl = 0, tbeg;\n  G2_STAMP(tbeg);\n"),
    ("  for (int it = 0; it < n_it; ++it) {\n", "", "    G2_STAMP(st0);\n"),
    ('    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");\n    __builtin_amdgcn_s_barrier();',
     "    G2_STAMP(st1);\n", "\n    G2_STAMP(st2);"),
    ("    if (++ckt == ckt1) {", "    G2_STAMP(st3);\n", ""),
    ("    stage = stage == 2 ? 0 : stage + 1;\n", "",
     "    G2_STAMP(st4);\n    sw += st1 - st0; sb += st2 - st1; sm += st3 - st2; stl += st4 - st3;\n"),
]
TAIL = """  unsigned long long tend;
  G2_STAMP(tend);
  if (lane == 0 && blockIdx.x < 4096) {
    unsigned long long* o = g2_diag + ((size_t)blockIdx.x * 8 + wid) * 6;
    o[0] = sw; o[1] = sb; o[2] = sm; o[3] = stl; o[4] = tend - tbeg; o[5] = (unsigned long long)n_it;
  }
"""


def instrument(text: str) -> str:
    """gemm.hip with the stamps spliced into gemm2_kernel (a diagnostic copy under diag_build/src)."""
    sig = "template <int BN, int MODE>\n__global__ __launch_bounds__(G2_NT, 1) void gemm2_kernel("
    i0 = text.index(sig)
    i1 = text.index("\n}\n", i0) + 1  # the kernel's closing brace (column 0)
    body = text[i0:i1]
    for anchor, before, after in STAMPS:
        if body.count(anchor) != 1:
            raise RuntimeError(f"stamp anchor not unique in gemm2_kernel: {anchor!r}")
        body = body.replace(anchor, before + anchor + after)
    body = body + TAIL
    return text[:i0] + PRELUDE + body + text[i1:] + EPILOGUE


def build():
    sys.path.insert(0, str(PKG))
    import build_ext as B
    OUT.mkdir(exist_ok=True)
    src_dir = OUT / "src"
    src_dir.mkdir(exist_ok=True)
    for f in B.CSRC.iterdir():
        if f.suffix in (".hip", ".h"):
            text = f.read_text()
            (src_dir / f.name).write_text(instrument(text) if f.name == "gemm.hip" else text)
    defs = ['-DVD_BUILD_HASH="diag"', f'-DVD_BUILD_ARCH="{B.ARCH}"', f"-I{B.CSRC}", f"-I{ROOT / 'include'}"]
    objs = []
    for src in sorted(src_dir.glob("*.hip")):
        obj = OUT / (src.stem + ".o")
        subprocess.run([B.HIPCC, *B.CFLAGS, *defs, "-c", str(src), "-o", str(obj)], check=True)
        objs.append(str(obj))
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(LIB), *objs,
                    "-L/opt/rocm/lib", "-lrccl"], check=True)
    print("built", LIB)


def run(reps):
    import torch
    sys.path.insert(0, str(PKG))
    from vdiff._lib import GemmDesc  # the struct only; the product library is not loaded
    lib = C.CDLL(str(LIB), mode=os.RTLD_LOCAL)
    lib.vd_gemm.argtypes = [C.c_void_p, C.c_void_p]
    lib.vd_gemm_ws_bytes.argtypes = [C.c_void_p]
    lib.vd_gemm_ws_bytes.restype = C.c_int64
    lib.vd_diag_g2_read.argtypes = [C.c_void_p, C.c_int64]
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    cases = [  # name, conv?, (n_img, h, w) or M, N, K
        ("L1 conv 320->320 (32 img)", True, (32, 64, 64), 320, 2880),
        ("L2 conv 640->640 (32 img)", True, (32, 32, 32), 640, 5760),
        ("L3 conv 1280->1280 (32 img)", True, (32, 16, 16), 1280, 11520),
        ("L1 ff2 dense +res", False, 131072, 320, 1280),
        ("L2 ff2 dense +res", False, 32768, 640, 2560),
        ("L2 proj dense +res", False, 32768, 640, 640),
    ]
    stream = torch.cuda.current_stream().cuda_stream
    for (name, conv, shp, N, K), variant in [(c, 0) for c in cases]:
        if conv:
            n, h, w = shp
            M = n * h * w
            a = (torch.randn(M, K // 9, device=dev, generator=g)).to(torch.bfloat16)
        else:
            M = shp
            a = (torch.randn(M, K, device=dev, generator=g)).to(torch.bfloat16)
        wt = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
        bias = torch.randn(N, device=dev, generator=g)
        res = None if conv else torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        d = GemmDesc(a0=a.data_ptr(), lda0=a.shape[1], k0=a.shape[1], a_mode=int(conv), w=wt.data_ptr(), ldw=K,
                     M=M, N=N, K=K, bias=bias.data_ptr(), out=out.data_ptr(), ldc=N, path=2,
                     res=res.data_ptr() if res is not None else None, ld_res=N if res is not None else 0)
        if conv:
            d.n_img, d.h_in, d.w_in, d.h_out, d.w_out, d.stride = n, h, w, h, w, 1
        nb = lib.vd_gemm_ws_bytes(C.byref(d))
        ws = torch.empty(max(nb, 4) // 4, device=dev) if nb else None
        if ws is not None:
            d.ws, d.ws_bytes = ws.data_ptr(), nb
        for _ in range(reps):
            assert lib.vd_gemm(C.byref(d), C.c_void_p(stream)) == 0
        torch.cuda.synchronize()
        lib.vd_diag_g2_clear()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        assert lib.vd_gemm(C.byref(d), C.c_void_p(stream)) == 0
        e1.record()
        torch.cuda.synchronize()
        buf = (C.c_ulonglong * (4096 * 8 * 6))()
        assert lib.vd_diag_g2_read(buf, 4096 * 8 * 6) == 0
        rows = [buf[i * 6:(i + 1) * 6] for i in range(4096 * 8) if buf[i * 6 + 5]]
        tot = [sum(r[k] for r in rows) for k in range(6)]
        seg = tot[0] + tot[1] + tot[2] + tot[3]
        per_kt = seg / max(tot[5], 1)
        print(f"{name + (' SPLIT' if variant else ''):36s} {e0.elapsed_time(e1) * 1e3:7.1f} us (stamped)  waves {len(rows)}  "
              f"k-tiles/wave {tot[5] / len(rows):.1f}  cycles/k-tile {per_kt:6.0f} = "
              f"wait {tot[0] / seg:5.1%}  barrier {tot[1] / seg:5.1%}  reads+MFMA issue {tot[2] / seg:5.1%}  "
              f"epilogue+DMA issue {tot[3] / seg:5.1%}  (loop / kernel-life {seg / tot[4]:5.1%})", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    build() if args.build else run(args.reps)
