"""What bounds the v2 implicit-GEMM conv: timing-only ABLATIONS of gemm2_kernel's operand traffic
(DIAGNOSTIC builds, wrong results, never the product library).  Each variant is spliced into a
copy of csrc/gemm.hip at build time:

  a6   the A (activation) pieces of a k-tile cut from 32 to 6 (waves 0-5 issue one piece each):
       the traffic a halo-tiled conv would move per tap (a 6 x 66-pixel, 64-channel patch = 49.5
       KiB serves all 9 taps, ~5.5 KiB per tap against 32 KiB);
  w1   the W (weight) pieces cut to one per k-tile (wave 0);
  gn   (a pricing build) the landed A tile GroupNorm-applied and SiLU'd in
       place in LDS once per k-tile (one FMA + SiLU per element, a row mask for the conv padding)
       behind a second barrier: what Conv + GroupNorm + SiLU fused into the conv costs.

The counted ring waits follow each wave's actual piece count.  Compared against the product
library on the UNet's stride-1 conv shapes (path 2 forced, 32 images):

    python tools/g2_ablate.py --build      # here (CPU): tools/diag_build/libvdiff_{a6,gn,w1}.so
    python tools/g2_ablate.py              # GPU box
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
OUT = ROOT / "tools" / "diag_build"

WAIT_OLD = """      if (nbw == C::NBMAX) wait_vm<C::NA + C::NBMAX>();
      else wait_vm<C::NA + C::NBMAX - 1>();"""
WAIT_NEW = """      switch (G2X_NA + nbw) {  // ablation: this wave's actual pieces per k-tile
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
      }"""
ADMA_OLD = """#pragma unroll
      for (int j = 0; j < C::NA; ++j)
        dma16(s0 ? ra0 : ra1, la + (wid * 4 + j) * 1024, (s0 ? aoff0[j] : aoff1[j]) + coff);"""
BDMA_OLD = """#pragma unroll
    for (int j = 0; j < C::NBMAX; ++j)
      if (j < nbw) dma16(rw, lb + (j * 8 + wid) * 1024, boff[j] + (uint32_t)kb * 2);"""
NBW_OLD = "  const int nbw = (C::NBI - wid + 7) / 8;  // this wave's B DMA instructions per K-tile"

SBASE_OLD = "    const char* sbase = smem + stage * C::STAGE;\n"
# the Conv+GroupNorm+SiLU form VERDICT r05 item 5 asked to price: the landed A tile normalised and
# SiLU'd once, in place in LDS, by the whole workgroup (thread: one 16-B channel chunk of 4 rows;
# its 8 channels' (a, b) from LDS — a stand-in for the tile's per-(image, channel) table; a row
# mask so a conv tap outside the image stays zero), then a second barrier before the fragment reads
GN_PASS = SBASE_OLD + """    if constexpr (MODE == VD_A_CONV3X3) {
      char* sa = smem + stage * C::STAGE;
      const int c8 = tid & 7, r0 = tid >> 3;
      const float4* abp = (const float4*)(sa + C::A_BYTES + c8 * 64);
      const float4 a0 = abp[0], a1 = abp[1], b0 = abp[2], b1 = abp[3];
      const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = r0 + 64 * j;
        uint4* pp = (uint4*)(sa + r * 128 + ((c8 ^ (r & 7)) << 4));
        float f[8];
        unpack8(*pp, f);
        const bool ok = ((r + it) & 63) != 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float y = fmaf(f[e], av[e], bv[e]);
          f[e] = ok ? silu_f(y) : 0.f;
        }
        *pp = pack8(f);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
"""

VARIANTS = {
    "a6": {
        "na": "(wid < 6 ? 1 : 0)",
        ADMA_OLD: """      if (wid < 6) dma16(s0 ? ra0 : ra1, la + (wid * 4) * 1024, (s0 ? aoff0[0] : aoff1[0]) + coff);""",
    },
    "gn": {
        "na": "C::NA",
        SBASE_OLD: GN_PASS,
    },
    "w1": {
        "na": "C::NA",
        NBW_OLD: "  const int nbw = wid == 0 ? 1 : 0;  // ablation: one W piece per k-tile",
        BDMA_OLD: """    if (nbw) dma16(rw, lb + wid * 1024, boff[0] + (uint32_t)kb * 2);""",
    },
}


def instrument(text: str, var: dict) -> str:
    sig = "template <int BN, int MODE>\n__global__ __launch_bounds__(G2_NT, 1) void gemm2_kernel("
    i0 = text.index(sig)
    i1 = text.index("\n}\n", i0) + 1
    body = text[i0:i1]
    reps = {WAIT_OLD: WAIT_NEW.replace("G2X_NA", var["na"])}
    reps.update({k: v for k, v in var.items() if k != "na"})
    for old, new in reps.items():
        if body.count(old) != 1:
            raise RuntimeError(f"ablation anchor not unique in gemm2_kernel: {old[:60]!r}")
        body = body.replace(old, new)
    return text[:i0] + body + text[i1:]


def build():
    sys.path.insert(0, str(PKG))
    import build_ext as B
    OUT.mkdir(exist_ok=True)
    for name, var in VARIANTS.items():
        src_dir = OUT / f"src_{name}"
        src_dir.mkdir(exist_ok=True)
        (src_dir / "gemm.hip").write_text(instrument((B.CSRC / "gemm.hip").read_text(), var))
        defs = ['-DVD_BUILD_HASH="diag"', f'-DVD_BUILD_ARCH="{B.ARCH}"', f"-I{B.CSRC}", f"-I{ROOT / 'include'}"]
        obj = OUT / f"gemm_{name}.o"
        subprocess.run([B.HIPCC, *B.CFLAGS, *defs, "-c", str(src_dir / "gemm.hip"), "-o", str(obj)], check=True)
        objs = [str(obj)] + [str(p) for p in sorted(B.BUILD.glob("*.o")) if p.stem != "gemm"]
        lib = OUT / f"libvdiff_{name}.so"
        subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(lib), *objs,
                        "-L/opt/rocm/lib", "-lrccl"], check=True)
        print("built", lib)


def run(reps: int):
    import torch
    sys.path.insert(0, str(PKG))
    from vdiff._lib import GemmDesc, lib as product_lib
    libs = {"product": product_lib()}
    for name in VARIANTS:
        lb = C.CDLL(str(OUT / f"libvdiff_{name}.so"), mode=os.RTLD_NOW | os.RTLD_LOCAL)
        lb.vd_gemm.argtypes = [C.c_void_p, C.c_void_p]
        lb.vd_gemm_ws_bytes.argtypes = [C.c_void_p]
        lb.vd_gemm_ws_bytes.restype = C.c_int64
        libs[name] = lb
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    cases = [("L1 conv 320->320", (32, 64, 64), 320, 2880), ("L2 conv 640->640", (32, 32, 32), 640, 5760),
             ("L3 conv 1280->1280", (32, 16, 16), 1280, 11520)]
    stream = torch.cuda.current_stream().cuda_stream
    for name, (n, h, w), N, K in cases:
        M = n * h * w
        a = torch.randn(M, K // 9, device=dev, generator=g).to(torch.bfloat16)
        wt = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
        bias = torch.randn(N, device=dev, generator=g)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        d = GemmDesc(a0=a.data_ptr(), lda0=a.shape[1], k0=a.shape[1], a_mode=1, w=wt.data_ptr(), ldw=K,
                     M=M, N=N, K=K, bias=bias.data_ptr(), out=out.data_ptr(), ldc=N, path=2)
        d.n_img, d.h_in, d.w_in, d.h_out, d.w_out, d.stride = n, h, w, h, w, 1
        nb = libs["product"].vd_gemm_ws_bytes(C.byref(d))
        ws = torch.empty(max(nb, 4) // 4, device=dev) if nb else None
        if ws is not None:
            d.ws, d.ws_bytes = ws.data_ptr(), nb
        res = {k: [] for k in libs}
        for rnd in range(reps):
            for k, lb in libs.items():
                for _ in range(3):
                    assert lb.vd_gemm(C.byref(d), C.c_void_p(stream)) == 0
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    assert lb.vd_gemm(C.byref(d), C.c_void_p(stream)) == 0
                e1.record()
                torch.cuda.synchronize()
                res[k].append(e0.elapsed_time(e1) * 100.0)  # us per launch
        fl = 2.0 * M * N * K
        line = "  ".join(f"{k} {sorted(v)[len(v) // 2]:7.1f} us ({fl / sorted(v)[len(v) // 2] / 1e6:6.0f} TF/s)"
                         for k, v in res.items())
        print(f"{name:22s} {line}", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    build() if args.build else run(args.reps)
