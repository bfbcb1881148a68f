// fp8 (OCP e4m3) spatial self-attention for d = 64 on the block-scaled MFMA
// v_mfma_scale_f32_32x32x64_f8f6f4 (2x the bf16 MFMA rate on gfx950): the "fp8 MFMA
// QK^T/PV" of BASELINE config 5 (the DiT's spatial blocks).
//
// Operand map (lane l, r = l & 31, h = l >> 5; checked with exact integer data by
// tools/mb/fp8_probe.py): A row r / B column r, 32 bytes per lane = k-slots (h, j),
// j < 32; C/D as every 32x32 MFMA: column r, row (i & 3) + 8 (i >> 2) + 4 h for
// accumulator register i.  The E8M0 scale a lane passes applies to its 32 k-slots.
//
//   S^T = K . Q^T   A = K rows (key r), B = Q^T (query r), k-slot (h, j) = d 32h + j:
//                   both are plain 32-byte slices of the fp8 rows, scaled per token
//                   (the lane's own key / query scale).
//   O^T = V^T . P^T B = P^T: the two S^T accumulators of a 64-key tile, converted to fp8
//                   in register order, ARE the operand: k-slot (h, j) = key
//                   32 (j >> 4) + (j & 3) + 8 ((j & 15) >> 2) + 4 h.  A = V^T rows (d r)
//                   must hold the same keys in the same slots: the pre-pass writes V^T
//                   with the keys of every 64-key tile permuted that way, so a lane's
//                   32 bytes are contiguous.  V's scale is one E8M0 per (image, head, tile).
//
// Pre-pass (attn_fp8_quant_*): per (token, head) power-of-two scale 2^ceil(log2(amax/448))
// for Q and K; V per 64-key tile.  Softmax: fp32 scores * (d^-1/2 log2 e), running max per
// query (lanes r and r+32 share a query: one permlane32 swap), P = exp2(s - m) <= 1 in
// fp8 with unit scale, row sum in fp32 (halves summed at the end), lazy O rescale when a
// query's max grows.  Block = 4 waves x 32 queries sharing double-buffered LDS tiles.
#include "common.h"

namespace {

constexpr int NT = 256;
constexpr int FD = 64;        // head dim
constexpr int KT8 = 64;       // keys per tile
constexpr int KROW = 80;      // LDS bytes per K row (64 + 16 pad: conflict-light b128 reads)
constexpr int VROW = 80;      // LDS bytes per V^T row
constexpr int STAGE8 = KT8 * KROW + FD * VROW + KT8;  // K, V^T, K scales

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

__device__ __forceinline__ float partner32f(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}

__device__ __forceinline__ int e8m0_for(float amax) {
  // smallest e with amax / 2^e <= 448 (OCP e4m3 max); zero rows get 2^0
  if (!(amax > 0.f)) return 127;
  int e = (int)ceilf(log2f(amax * (1.0f / 448.0f)));
  e = e < -126 ? -126 : (e > 127 ? 127 : e);
  return e + 127;
}
__device__ __forceinline__ float e8m0_inv(int b) { return exp2f((float)(127 - b)); }

__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d) {
  const float L = 448.f;
  a = __builtin_amdgcn_fmed3f(a, L, -L); b = __builtin_amdgcn_fmed3f(b, L, -L);
  c = __builtin_amdgcn_fmed3f(c, L, -L); d = __builtin_amdgcn_fmed3f(d, L, -L);
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}

// Q or K rows: one thread per (row, head): 64 bf16 -> 64 fp8 + one E8M0 byte.
__global__ void quant_rows_kernel(const bf16_t* __restrict__ x, int64_t ldx, int64_t rows, int heads,
                                  uint8_t* __restrict__ x8, int64_t ld8, uint8_t* __restrict__ sc, float mul) {
  const int64_t total = rows * heads;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int64_t r = i / heads;
    const int h = (int)(i % heads);
    const bf16_t* src = x + r * ldx + h * FD;
    float v[FD];
    float amax = 0.f;
#pragma unroll
    for (int c = 0; c < FD / 8; ++c) {
      unpack8(*(const uint4*)(src + 8 * c), v + 8 * c);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[8 * c + j] *= mul;
        amax = fmaxf(amax, fabsf(v[8 * c + j]));
      }
    }
    const int e = e8m0_for(amax);
    const float inv = e8m0_inv(e);
    uint8_t* dst = x8 + r * ld8 + h * FD;
#pragma unroll
    for (int c = 0; c < FD / 16; ++c) {
      const float* s = v + 16 * c;
      *(uint4*)(dst + 16 * c) =
          make_uint4(pack4_fp8(s[0] * inv, s[1] * inv, s[2] * inv, s[3] * inv),
                     pack4_fp8(s[4] * inv, s[5] * inv, s[6] * inv, s[7] * inv),
                     pack4_fp8(s[8] * inv, s[9] * inv, s[10] * inv, s[11] * inv),
                     pack4_fp8(s[12] * inv, s[13] * inv, s[14] * inv, s[15] * inv));
    }
    sc[r * heads + h] = (uint8_t)e;
  }
}

// Q or K rows with the DiT's spatial 2-D RoPE fused (vd_attention_fp8_quant_rope): eight
// lanes per (row, head), lane c owns elements [8c, 8c + 8) and also loads its rotate-half
// partner chunk c ^ 2 (same 32-wide section), so loads stay coalesced 16-byte chunks and
// every lane evaluates only 8 angles; the head's amax is reduced over the 8 lanes with
// xor shuffles.  Section 0 (chunks 0-3) rotates by h = (r / Wp) % Hp, section 1 by
// w = r % Wp; pair (i, i + 16) of a section at angle pos * theta^(-2i/32) (dit.hip
// rope_kernel mode 0).  Rotation in fp32, never rounded to bf16.
__global__ __launch_bounds__(NT) void quant_rows_rope_kernel(const bf16_t* __restrict__ x, int64_t ldx,
                                                             int64_t rows, int heads, uint8_t* __restrict__ x8,
                                                             int64_t ld8, uint8_t* __restrict__ sc, int64_t Hp,
                                                             int64_t Wp, float log2_theta, float mul) {
  // 32-bit index math (the host checks rows * heads * 8 < 2^31): 64-bit divisions by heads,
  // Wp and Hp would dominate this HBM pass.  total is a multiple of 8, so a lane group never
  // straddles the grid stride.
  const uint32_t total = (uint32_t)(rows * heads * 8);
  const uint32_t uh = (uint32_t)heads, uw = (uint32_t)Wp, uhp = (uint32_t)Hp;
  for (uint32_t i = blockIdx.x * NT + threadIdx.x; i < total; i += gridDim.x * NT) {
    const int c = (int)(i & 7);
    const uint32_t rh = i >> 3;
    const uint32_t r = rh / uh;
    const int h = (int)(rh - r * uh);
    const bf16_t* src = x + (int64_t)r * ldx + h * FD;
    float own[8], par[8];
    unpack8(*(const uint4*)(src + 8 * c), own);
    unpack8(*(const uint4*)(src + 8 * (c ^ 2)), par);
    const uint32_t rw = r / uw;
    const float pos = (float)(c < 4 ? rw % uhp : r - rw * uw);
    const bool lo = (c & 2) == 0;  // holds the first half of its pairs
    const int j0 = 8 * (c & 1);
    float v[8];
    float amax = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float inv_freq = exp2f(-log2_theta * (float)(2 * (j0 + j)) * (1.0f / (FD / 2)));
      float sn, cs;
      __sincosf(pos * inv_freq, &sn, &cs);
      v[j] = (lo ? own[j] * cs - par[j] * sn : own[j] * cs + par[j] * sn) * mul;
      amax = fmaxf(amax, fabsf(v[j]));
    }
    amax = fmaxf(amax, __shfl_xor(amax, 1, 8));
    amax = fmaxf(amax, __shfl_xor(amax, 2, 8));
    amax = fmaxf(amax, __shfl_xor(amax, 4, 8));
    const int e = e8m0_for(amax);
    const float inv = e8m0_inv(e);
    *(uint2*)(x8 + (int64_t)r * ld8 + h * FD + 8 * c) =
        make_uint2(pack4_fp8(v[0] * inv, v[1] * inv, v[2] * inv, v[3] * inv),
                   pack4_fp8(v[4] * inv, v[5] * inv, v[6] * inv, v[7] * inv));
    if (c == 0) sc[rh] = (uint8_t)e;
  }
}

// slot p = 32h + j of a 64-key tile holds key 32 (j >> 4) + (j & 3) + 8 ((j & 15) >> 2) + 4h
__device__ __forceinline__ int slot_key(int p) {
  const int h = p >> 5, j = p & 31;
  return 32 * (j >> 4) + (j & 3) + 8 * ((j & 15) >> 2) + 4 * h;
}

// V -> V^T fp8, keys permuted per tile; one workgroup per (image, head, 64-key tile).
__global__ __launch_bounds__(NT) void quant_vt_kernel(const bf16_t* __restrict__ v, int64_t ldv, int heads,
                                                     int64_t skv, uint8_t* __restrict__ vt8,
                                                     uint8_t* __restrict__ vs) {
  __shared__ float tile[KT8][FD + 1];
  __shared__ float red[NT / 64];
  const int64_t ntiles = skv / KT8;
  const int64_t t = blockIdx.x % ntiles;
  const int64_t bh = blockIdx.x / ntiles;
  const int h = (int)(bh % heads);
  const int64_t b = bh / heads;
  const int tid = threadIdx.x;
  // 64 keys x 64 d bf16 = 512 chunks of 8: two per thread
  float amax = 0.f;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = tid + u * NT;
    const int key = c >> 3, dc = (c & 7) * 8;
    float f[8];
    unpack8(*(const uint4*)(v + (b * skv + t * KT8 + key) * ldv + h * FD + dc), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      tile[key][dc + j] = f[j];
      amax = fmaxf(amax, fabsf(f[j]));
    }
  }
  amax = wave_max(amax);
  if ((tid & 63) == 0) red[tid >> 6] = amax;
  __syncthreads();
  amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const int e = e8m0_for(amax);
  const float inv = e8m0_inv(e);
  // write V^T: row d (64 bytes per tile), 16 slots per thread
  const int d = tid >> 2, q = (tid & 3) * 16;
  uint32_t w[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int p = q + 4 * g;
    w[g] = pack4_fp8(tile[slot_key(p)][d] * inv, tile[slot_key(p + 1)][d] * inv, tile[slot_key(p + 2)][d] * inv,
                     tile[slot_key(p + 3)][d] * inv);
  }
  *(uint4*)(vt8 + (bh * FD + d) * skv + t * KT8 + q) = make_uint4(w[0], w[1], w[2], w[3]);
  if (tid == 0) vs[bh * ntiles + t] = (uint8_t)e;
}

__global__ __launch_bounds__(NT, 2) void flash_fp8_kernel(
    const uint8_t* __restrict__ q8, const uint8_t* __restrict__ k8, int64_t ld8,
    const uint8_t* __restrict__ qs, const uint8_t* __restrict__ ks, const uint8_t* __restrict__ vt8,
    const uint8_t* __restrict__ vs, bf16_t* __restrict__ o, int64_t ldo, int heads, int64_t sq, int64_t skv,
    float c, int unit_scale) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * STAGE8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = (int)((sq + 127) / 128);
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int qblk = lid % nqb;
  const int h = (lid / nqb) % heads;
  const int64_t b = lid / (nqb * heads);
  const int64_t bh = b * heads + h;
  const int64_t q0 = (int64_t)qblk * 128 + wave * 32;
  const bool qvalid = q0 < sq;
  const int64_t qrow = b * sq + (qvalid ? q0 + r : 0);
  // Q^T fragment: d = 32 hh + j of this lane's query, and its scale
  const i32x8 qf = *(const i32x8*)(q8 + qrow * ld8 + h * FD + 32 * hh);
  const int qsc = qs[qrow * heads + h];
  const int64_t ntiles = skv / KT8;
  const uint8_t* kbase = k8 + b * skv * ld8 + h * FD;
  const uint8_t* vbase = vt8 + bh * FD * skv;
  // cooperative tile load: K 64 rows x 64 B (256 x 16 B), V^T 64 rows x 64 B (256 x 16 B)
  const int lr = tid >> 2, lc = (tid & 3) * 16;
  uint4 kreg, vreg;
  uint8_t sreg = 0;
  auto gload = [&](int64_t t) {
    kreg = *(const uint4*)(kbase + (t * KT8 + lr) * ld8 + lc);
    vreg = *(const uint4*)(vbase + (int64_t)lr * skv + t * KT8 + lc);
    if (tid < KT8) sreg = ks[(b * skv + t * KT8 + tid) * heads + h];
  };
  auto sstore = [&](int buf) {
    uint8_t* st = lds + buf * STAGE8;
    *(uint4*)(st + lr * KROW + lc) = kreg;
    *(uint4*)(st + KT8 * KROW + lr * VROW + lc) = vreg;
    if (tid < KT8) st[KT8 * KROW + FD * VROW + tid] = sreg;
  };
  f32x16 ot[2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int i = 0; i < 16; ++i) ot[a][i] = 0.f;
  float m = -INFINITY, l = 0.f;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int64_t t = 0; t < ntiles; ++t) {
    const int buf = (int)(t & 1);
    if (t + 1 < ntiles) gload(t + 1);
    const uint8_t* st = lds + buf * STAGE8;
    // ---- S^T for the two 32-key blocks
    f32x16 s[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const uint8_t* kr = st + (32 * kb + r) * KROW + 32 * hh;
      const uint4 k0 = *(const uint4*)kr, k1 = *(const uint4*)(kr + 16);
      const i32x8 kf = {(int)k0.x, (int)k0.y, (int)k0.z, (int)k0.w, (int)k1.x, (int)k1.y, (int)k1.z, (int)k1.w};
      const int ksc = st[KT8 * KROW + FD * VROW + 32 * kb + r];
      f32x16 z;
#pragma unroll
      for (int i = 0; i < 16; ++i) z[i] = 0.f;
      s[kb] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(kf, qf, z, 0, 0, 0, ksc, 0, qsc);
    }
    // V^T fragments (d rows r and 32 + r, this lane's 32 slots)
    i32x8 vf[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const uint8_t* vr = st + KT8 * KROW + (32 * a + r) * VROW + 32 * hh;
      const uint4 v0 = *(const uint4*)vr, v1 = *(const uint4*)(vr + 16);
      vf[a] = i32x8{(int)v0.x, (int)v0.y, (int)v0.z, (int)v0.w, (int)v1.x, (int)v1.y, (int)v1.z, (int)v1.w};
    }
    const int vsc = vs[bh * ntiles + t];
    // ---- online softmax over this lane's 32 scores (its query; the other half in lane ^ 32)
    float mt = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) mt = fmaxf(mt, s[kb][i]);
    mt = fmaxf(mt, partner32f(mt)) * c;
    if (mt > m) {
      const float alpha = exp2f(m - mt);
      l *= alpha;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int i = 0; i < 16; ++i) ot[a][i] *= alpha;
      m = mt;
    }
    uint32_t pw[8];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float p0 = __builtin_amdgcn_exp2f(fmaf(s[kb][4 * g + 0], c, -m));
        const float p1 = __builtin_amdgcn_exp2f(fmaf(s[kb][4 * g + 1], c, -m));
        const float p2 = __builtin_amdgcn_exp2f(fmaf(s[kb][4 * g + 2], c, -m));
        const float p3 = __builtin_amdgcn_exp2f(fmaf(s[kb][4 * g + 3], c, -m));
        l += (p0 + p1) + (p2 + p3);
        pw[4 * kb + g] = pack4_fp8(p0, p1, p2, p3);
      }
    const i32x8 pf = {(int)pw[0], (int)pw[1], (int)pw[2], (int)pw[3], (int)pw[4], (int)pw[5], (int)pw[6], (int)pw[7]};
#pragma unroll
    for (int a = 0; a < 2; ++a)
      ot[a] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(vf[a], pf, ot[a], 0, 0, 0, vsc, 0, unit_scale);
    if (t + 1 < ntiles) {
      sstore(buf ^ 1);
    }
    __syncthreads();
  }
  const float lt = l + partner32f(l);
  const float inv = 1.0f / lt;
  if (qvalid) {
    bf16_t* orow = o + (b * sq + q0 + r) * ldo + h * FD;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int dd = 32 * a + 8 * g + 4 * hh;
        *(uint2*)(orow + dd) = make_uint2(pack2(ot[a][4 * g] * inv, ot[a][4 * g + 1] * inv),
                                          pack2(ot[a][4 * g + 2] * inv, ot[a][4 * g + 3] * inv));
      }
  }
}

// ---------------------------------------------------------------- v2 (round 3)
// flash_fp8_kernel's arithmetic re-staged.  v1 loaded each 64-key tile into registers one
// tile ahead, wrote it to LDS and synchronised per tile (an L2 round trip exposed every tile),
// rescaled O whenever a row max grew, clamped every P to the e4m3 range and summed P on the
// VALU.  v2: K, V^T and the K scales reach a 6-stage LDS ring by LDS-DMA (9 pieces per tile:
// K and V^T rows of 64 B XOR-swizzled on the source chunk, conflict-free b128 reads; the 64
// per-key scale bytes by one buffer_load_ubyte ... lds, one dword each), five tiles in flight behind counted
// vmcnt waits; the running offset m moves only when a row max passes it by 8 (P <= 2^8 < 448:
// no clamp; cdna_hip_programming.md T13), and the row sum is an fp32 VALU sum of the unrounded P.
// Measured forms (DiT shape, rel-L2 vs fp32 SDPA at S = 2304, profiles/r03l_fp8_variants.txt):
// v1 1.580 ms / 8.60 %; lazy + row sum on the MFMA (an all-ones e4m3 A operand against P)
// 1.389 ms / 8.93 %; lazy + fp32 VALU row sum (this kernel) 1.426 ms / 8.78 %; eager offset +
// VALU sum 1.520 ms / 8.60 %.  The MFMA row sum is faster but sums the e4m3-rounded P, which
// costs accuracy.  v1 (flash_fp8_kernel) stays as the path for shapes whose ring offsets do not
// fit 32 bits.
constexpr int F8S = 6;  // ring stages
constexpr int F8_K = 0, F8_V = 4096, F8_KS = 8192, F8_STAGE = 8192 + 256;

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4f;

__device__ __forceinline__ u32x4f f8_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  u32x4f r;
  r[0] = __builtin_amdgcn_readfirstlane((uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) & 0xffffu;  // stride 0
  r[2] = __builtin_amdgcn_readfirstlane(bytes);                          // num_records: range check
  r[3] = 0x00020000u;
  return r;
}
// LDS-DMA: lane l's 16 bytes (x4) at voff land at LDS lds + 16 l; a ubyte load lands zero-extended
// in the dword at lds + 4 l;
// inline asm so hipcc neither counts them in vmcnt nor drains them before the LDS reads
__device__ __forceinline__ void f8_dma16(u32x4f rs, uint32_t lds, uint32_t voff) {
  uint32_t keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
               "buffer_load_dwordx4 %2, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(voff), "s"(rs) : "memory");
}
__device__ __forceinline__ void f8_dma1(u32x4f rs, uint32_t lds, uint32_t voff) {
  uint32_t keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
               "buffer_load_ubyte %2, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(voff), "s"(rs) : "memory");
}
__device__ __forceinline__ void f8_wait(int n) {  // s_waitcnt vmcnt(n), n in {0, 2, 3, 4, 6, 8, 9, 12}
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
  }
}
// physical 16-byte chunk of logical chunk c in a 64-byte row r of a K / V^T tile image
__device__ __forceinline__ uint32_t f8_chunk(uint32_t r, uint32_t c) { return c ^ ((r >> 2) & 3); }

// FOLDED (round 5): the softmax scale x log2 e is folded into q8 by the quantization
// (vd_attention_fp8_quant's q_scale) and the running offset into the S MFMA's accumulator input
// (C = -m), so the MFMA emits the exp2 argument itself: no scale FMA per score.  The row sum is a
// fifth MFMA, an all-ones e4m3 A operand against P^T (the sum of the rounded P the numerator uses),
// instead of 32 VALU adds; the V scales of all tiles are read once (a per-tile global load made
// hipcc drain the whole LDS-DMA ring with vmcnt(0) before every PV MFMA); the fp8 packs write
// over the previous tile's registers (no zeroing moves).  The tile is VALU-issue bound (32 exp,
// 16 packs, the max pass against 5 MFMAs), so every VALU instruction removed is time.
template <bool FOLDED>
__global__ __launch_bounds__(NT, 2) void flash_fp8_v2_kernel(
    const uint8_t* __restrict__ q8, const uint8_t* __restrict__ k8, int64_t ld8,
    const uint8_t* __restrict__ qs, const uint8_t* __restrict__ ks, const uint8_t* __restrict__ vt8,
    const uint8_t* __restrict__ vs, bf16_t* __restrict__ o, int64_t ldo, int heads, int64_t sq, int64_t skv,
    float c) {
  __shared__ __attribute__((aligned(1024))) uint8_t lds[F8S * F8_STAGE];
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)lds;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = (int)((sq + 127) / 128);
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int qblk = lid % nqb;
  const int h = (lid / nqb) % heads;
  const int64_t b = lid / (nqb * heads);
  const int64_t bh = b * heads + h;
  const int64_t q0 = (int64_t)qblk * 128 + wave * 32;
  const bool qvalid = q0 < sq;
  const int64_t qrow = b * sq + (qvalid ? q0 + r : 0);
  const int ntiles = (int)(skv / KT8);

  // Q^T fragment (d = 32 hh + j of this lane's query), its scale, and the V scales of the first
  // 64 tiles — all landed before the first ring DMA goes out (a plain load waited for later
  // would drain the ring: vmcnt counts the DMAs too)
  const i32x8 qf = *(const i32x8*)(q8 + qrow * ld8 + h * FD + 32 * hh);
  const int qsc = qs[qrow * heads + h];
  int vsr = lane < ntiles ? vs[bh * ntiles + lane] : 127;
  asm volatile("" ::"v"(qf[0]), "v"(qf[7]), "v"(qsc), "v"(vsr));

  // ---- ring: wave w moves K rows and V^T rows 16w .. 16w + 15 of each tile, wave 0 the scales
  const u32x4f rk = f8_rsrc(k8 + b * skv * ld8 + h * FD, (uint32_t)((skv - 1) * ld8 + FD));
  const u32x4f rv = f8_rsrc(vt8 + bh * FD * skv, (uint32_t)(FD * skv));
  const u32x4f rks = f8_rsrc(ks + b * skv * heads + h, (uint32_t)((skv - 1) * heads + 1));
  const uint32_t prow = (uint32_t)(16 * wave) + ((uint32_t)lane >> 2);       // row of this lane's 16 bytes
  const uint32_t pchk = f8_chunk(prow, (uint32_t)lane & 3);                  // the source chunk they hold
  const uint32_t kdo = prow * (uint32_t)ld8 + 16u * pchk, vdo = prow * (uint32_t)skv + 16u * pchk;
  const uint32_t sdo = (uint32_t)lane * (uint32_t)heads;
  const int npc = wave == 0 ? 3 : 2;  // this wave's DMA instructions per tile
  auto issue = [&](int t) {
    const uint32_t slot = lds0 + (uint32_t)(t % F8S) * F8_STAGE;
    f8_dma16(rk, slot + F8_K + 1024u * wave, kdo + (uint32_t)t * KT8 * (uint32_t)ld8);
    f8_dma16(rv, slot + F8_V + 1024u * wave, vdo + (uint32_t)t * KT8);
    if (wave == 0) f8_dma1(rks, slot + F8_KS, sdo + (uint32_t)t * KT8 * (uint32_t)heads);
  };
  for (int t = 0; t < F8S - 1 && t < ntiles; ++t) issue(t);

  // per-lane LDS read offsets: K row 32 kb + r and V^T row 32 a + r, logical chunks 2 hh, 2 hh + 1
  uint32_t kro[2][2], vro[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint32_t row = (uint32_t)(32 * x + r);
      kro[x][j] = F8_K + row * 64 + 16u * f8_chunk(row, (uint32_t)(2 * hh + j));
      vro[x][j] = F8_V + row * 64 + 16u * f8_chunk(row, (uint32_t)(2 * hh + j));
    }
  const i32x8 ones = {0x38383838, 0x38383838, 0x38383838, 0x38383838,   // e4m3 1.0 in every k-slot
                      0x38383838, 0x38383838, 0x38383838, 0x38383838};

  f32x16 ot[2], ls, nm;  // O^T, the row sums (every register of a lane holds its query's sum), -m
#pragma unroll
  for (int i = 0; i < 16; ++i) { ot[0][i] = 0.f; ot[1][i] = 0.f; ls[i] = 0.f; nm[i] = 0.f; }
  float m = FOLDED ? 0.f : -INFINITY;
  uint32_t pw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int t = 0; t < ntiles; ++t) {
    const int ahead = (ntiles - 1 - t) < (F8S - 2) ? (ntiles - 1 - t) : (F8S - 2);
    // this wave's pieces of tile t landed; the steady state as two constant waits (round 6: a
    // runtime count became a ~50-instruction branch tree of s_waitcnt immediates per tile)
    if (ahead == F8S - 2) {
      if (wave == 0) f8_wait(3 * (F8S - 2));
      else f8_wait(2 * (F8S - 2));
    } else {
      f8_wait(ahead * npc);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                       // everyone's; stage (t-1) % S free
    asm volatile("" ::: "memory");
    if (t + F8S - 1 < ntiles) issue(t + F8S - 1);
    const uint8_t* st = lds + (t % F8S) * F8_STAGE;
    f32x16 s[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const uint4 k0 = *(const uint4*)(st + kro[kb][0]), k1 = *(const uint4*)(st + kro[kb][1]);
      const i32x8 kf = {(int)k0.x, (int)k0.y, (int)k0.z, (int)k0.w, (int)k1.x, (int)k1.y, (int)k1.z, (int)k1.w};
      const int ksc = st[F8_KS + 4 * (32 * kb + r)];  // sub-dword LDS-DMA writes one dword per lane
      if constexpr (FOLDED) {
        s[kb] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(kf, qf, nm, 0, 0, 0, ksc, 0, qsc);  // = s' - m
      } else {
        f32x16 z;
#pragma unroll
        for (int i = 0; i < 16; ++i) z[i] = 0.f;
        s[kb] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(kf, qf, z, 0, 0, 0, ksc, 0, qsc);
      }
    }
    i32x8 vf[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const uint4 v0 = *(const uint4*)(st + vro[a][0]), v1 = *(const uint4*)(st + vro[a][1]);
      vf[a] = i32x8{(int)v0.x, (int)v0.y, (int)v0.z, (int)v0.w, (int)v1.x, (int)v1.y, (int)v1.z, (int)v1.w};
    }
    if (t > 0 && (t & 63) == 0) vsr = t + lane < ntiles ? vs[bh * ntiles + t + lane] : 127;
    const int vsc = __builtin_amdgcn_readlane(vsr, t & 63);
    // ---- softmax against the lazily moved offset m (P <= 2^8); always moved on the first tile
    float mt = s[0][0];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) mt = fmaxf(mt, s[kb][i]);
    // the offset test on each lane's own half-row max: x -> fl(x + m) (or x c) is monotone, so the
    // any() over lanes equals the any() over the row maxes; the partner exchange only when it moves
    if (t == 0 || __any((FOLDED ? mt + m : mt * c) > m + 8.f)) {  // wave-uniform
      mt = fmaxf(mt, partner32f(mt));
      const float mab = FOLDED ? mt + m : mt * c;  // the tile's row max, log2 units
      const float mn = t == 0 ? mab : fmaxf(m, mab);
      const float alpha = t == 0 ? 0.f : __builtin_amdgcn_exp2f(m - mn);
      if constexpr (FOLDED) {
        const float dl = mn - m;
#pragma unroll
        for (int i = 0; i < 16; ++i) { s[0][i] -= dl; s[1][i] -= dl; nm[i] = -mn; }
      }
      m = mn;
#pragma unroll
      for (int i = 0; i < 16; ++i) { ot[0][i] *= alpha; ot[1][i] *= alpha; ls[i] *= alpha; }
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float p[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          p[e] = __builtin_amdgcn_exp2f(FOLDED ? s[kb][4 * g + e] : fmaf(s[kb][4 * g + e], c, -m));
        const int w = __builtin_amdgcn_cvt_pk_fp8_f32(p[0], p[1], (int)pw[4 * kb + g], false);
        pw[4 * kb + g] = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(p[2], p[3], w, true);
      }
    const i32x8 pf = {(int)pw[0], (int)pw[1], (int)pw[2], (int)pw[3], (int)pw[4], (int)pw[5], (int)pw[6], (int)pw[7]};
#pragma unroll
    for (int a = 0; a < 2; ++a)
      ot[a] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(vf[a], pf, ot[a], 0, 0, 0, vsc, 0, 127);
    ls = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(ones, pf, ls, 0, 0, 0, 127, 0, 127);
  }
  const float inv = 1.0f / ls[0];
  if (qvalid) {
    bf16_t* orow = o + (b * sq + q0 + r) * ldo + h * FD;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int dd = 32 * a + 8 * g + 4 * hh;
        *(uint2*)(orow + dd) = make_uint2(pack2(ot[a][4 * g] * inv, ot[a][4 * g + 1] * inv),
                                          pack2(ot[a][4 * g + 2] * inv, ot[a][4 * g + 3] * inv));
      }
  }
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

int quant_operands(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                   int64_t batch, int32_t heads, int64_t sq, int64_t skv, int32_t d, bool rope, int64_t Hp,
                   int64_t Wp, float theta, void* q8, void* k8, int64_t ld8, void* vt8, void* qs, void* ks,
                   void* vs, float q_scale, vd_stream_t stream) {
  VD_CHECK_ARG(d == FD && heads > 0 && batch > 0 && sq > 0 && skv > 0 && skv % KT8 == 0);
  VD_CHECK_ARG(q && k && v && q8 && k8 && vt8 && qs && ks && vs && al16(q) && al16(k) && al16(v));
  VD_CHECK_ARG(al16(q8) && al16(k8) && al16(vt8) && ld8 % 16 == 0 && ld8 >= (int64_t)heads * FD);
  VD_CHECK_ARG(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && q_scale > 0.f);
  if (rope) {
    VD_CHECK_ARG(Hp > 0 && Wp > 0 && sq == Hp * Wp && skv == sq && theta > 1.f);
    VD_CHECK_ARG(batch * sq * heads * 8 < 0x7fffffff);
  }
  hipStream_t s = (hipStream_t)stream;
  auto grid = [](int64_t n) { const int64_t b = (n + NT - 1) / NT; return (unsigned)(b < 16384 ? b : 16384); };
  if (rope) {
    const float l2t = log2f(theta);
    hipLaunchKernelGGL(quant_rows_rope_kernel, dim3(grid(batch * sq * heads * 8)), dim3(NT), 0, s,
                       (const bf16_t*)q, ldq, batch * sq, (int)heads, (uint8_t*)q8, ld8, (uint8_t*)qs, Hp, Wp, l2t,
                       q_scale);
    hipLaunchKernelGGL(quant_rows_rope_kernel, dim3(grid(batch * skv * heads * 8)), dim3(NT), 0, s,
                       (const bf16_t*)k, ldk, batch * skv, (int)heads, (uint8_t*)k8, ld8, (uint8_t*)ks, Hp, Wp, l2t,
                       1.0f);
  } else {
    hipLaunchKernelGGL(quant_rows_kernel, dim3(grid(batch * sq * heads)), dim3(NT), 0, s, (const bf16_t*)q, ldq,
                       batch * sq, (int)heads, (uint8_t*)q8, ld8, (uint8_t*)qs, q_scale);
    hipLaunchKernelGGL(quant_rows_kernel, dim3(grid(batch * skv * heads)), dim3(NT), 0, s, (const bf16_t*)k, ldk,
                       batch * skv, (int)heads, (uint8_t*)k8, ld8, (uint8_t*)ks, 1.0f);
  }
  const int64_t nblk = batch * heads * (skv / KT8);
  VD_CHECK_ARG(nblk < 0x7fffffff);
  hipLaunchKernelGGL(quant_vt_kernel, dim3((unsigned)nblk), dim3(NT), 0, s, (const bf16_t*)v, ldv, (int)heads, skv,
                     (uint8_t*)vt8, (uint8_t*)vs);
  return vd_launch_status();
}

}  // namespace

extern "C" int vd_attention_fp8_quant(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v,
                                      int64_t ldv, int64_t batch, int32_t heads, int64_t sq, int64_t skv,
                                      int32_t d, void* q8, void* k8, int64_t ld8, void* vt8, void* qs,
                                      void* ks, void* vs, float q_scale, vd_stream_t stream) {
  return quant_operands(q, ldq, k, ldk, v, ldv, batch, heads, sq, skv, d, false, 0, 0, 0.f, q8, k8, ld8, vt8,
                        qs, ks, vs, q_scale, stream);
}

extern "C" int vd_attention_fp8_quant_rope(const void* q, int64_t ldq, const void* k, int64_t ldk,
                                           const void* v, int64_t ldv, int64_t batch, int32_t heads,
                                           int64_t s, int32_t d, int64_t Hp, int64_t Wp, float theta, void* q8,
                                           void* k8, int64_t ld8, void* vt8, void* qs, void* ks, void* vs,
                                           float q_scale, vd_stream_t stream) {
  return quant_operands(q, ldq, k, ldk, v, ldv, batch, heads, s, s, d, true, Hp, Wp, theta, q8, k8, ld8, vt8, qs,
                        ks, vs, q_scale, stream);
}

extern "C" int vd_attention_fp8(const void* q8, const void* k8, int64_t ld8, const void* qs, const void* ks,
                                const void* vt8, const void* vs, void* o, int64_t ldo, int64_t batch,
                                int32_t heads, int64_t sq, int64_t skv, int32_t d, float scale,
                                vd_stream_t stream) {
  VD_CHECK_ARG(d == FD && heads > 0 && batch > 0 && sq > 0 && sq % 32 == 0 && skv > 0 && skv % KT8 == 0);
  VD_CHECK_ARG(q8 && k8 && qs && ks && vt8 && vs && o && al16(q8) && al16(k8) && al16(vt8));
  VD_CHECK_ARG(ld8 % 16 == 0 && ld8 >= (int64_t)heads * FD && ldo % 4 == 0 && ((uintptr_t)o & 7) == 0);
  const int64_t nblk = (sq + 127) / 128 * heads * batch;
  VD_CHECK_ARG(nblk < 0x7fffffff);
  const float c = scale * 1.4426950408889634f;
  const bool folded = fabsf(c - 1.0f) < 1e-6f;  // vd_attention_fp8_quant folded scale x log2 e into q8
  const bool v2ok = skv * ld8 < 0x7fffffff && skv * FD < 0x7fffffff && skv * heads < 0x7fffffff;
  if (v2ok && folded)
    hipLaunchKernelGGL(flash_fp8_v2_kernel<true>, dim3((unsigned)nblk), dim3(NT), 0, (hipStream_t)stream,
                       (const uint8_t*)q8, (const uint8_t*)k8, ld8, (const uint8_t*)qs, (const uint8_t*)ks,
                       (const uint8_t*)vt8, (const uint8_t*)vs, (bf16_t*)o, ldo, (int)heads, sq, skv, 1.0f);
  else if (v2ok)
    hipLaunchKernelGGL(flash_fp8_v2_kernel<false>, dim3((unsigned)nblk), dim3(NT), 0, (hipStream_t)stream,
                       (const uint8_t*)q8, (const uint8_t*)k8, ld8, (const uint8_t*)qs, (const uint8_t*)ks,
                       (const uint8_t*)vt8, (const uint8_t*)vs, (bf16_t*)o, ldo, (int)heads, sq, skv, c);
  else
    hipLaunchKernelGGL(flash_fp8_kernel, dim3((unsigned)nblk), dim3(NT), 0, (hipStream_t)stream, (const uint8_t*)q8,
                       (const uint8_t*)k8, ld8, (const uint8_t*)qs, (const uint8_t*)ks, (const uint8_t*)vt8,
                       (const uint8_t*)vs, (bf16_t*)o, ldo, (int)heads, sq, skv, c, 127);
  return vd_launch_status();
}
