// flash512_kernel — the VAE mid-block self-attention (diffusers Attention with heads = 1,
// dim_head = 512 over the 64x64 = 4096 latent pixels of a frame; SURVEY.md §8f rank 1, the
// decode the reference runs after the loop at experiments/05_grid_search_ablation.py:143).
// Round 3: replaces the per-frame GEMM -> 64 MB fp32 score matrix -> softmax_rows -> GEMM
// chain with one flash pass over all frames.
//
// Per score this head does 4 * 512 FLOPs of MFMA work and one exp2, so unlike the d = 40
// spatial attention the softmax VALU is negligible; what bounds it is operand traffic.  The
// design therefore maximises reuse of every LDS byte:
//   * one wave per SIMD (4 waves, 128 queries per workgroup, ~450 registers per lane):
//     each wave owns 32 queries with their Q' fragments (128 VGPRs) and the whole O^T
//     accumulator (16 x 32x32 tiles = 256 registers) in registers;
//   * S^T = K.Q^T on v_mfma_f32_32x32x16_bf16 (A = K rows from LDS by ds_read_b128, B = Q^T
//     from registers): 32 MFMAs per 32-key tile, one accumulator;
//   * the S^T accumulator packed to bf16 IS P's B operand (cdna_hip_programming.md §3
//     "accumulator as the next operand"), V^T comes out of LDS by ds_read_b64_tr_b16 in that
//     permuted key order: O^T += V^T.P, 32 more MFMAs per tile;
//   * K/V tiles of 32 keys (32 KiB each) by LDS-DMA (buffer_load ... lds, one 1 KiB row per
//     wave-instruction), double-buffered: tile t+1 streams in under tile t's 64 MFMAs per wave;
//     XOR swizzles on the source chunk make the K row reads and the V transposed reads
//     bank-conflict free;
//   * softmax in log2 units (the softmax scale * log2 e is folded into W_q by the caller, as
//     for the UNet's attention: scale argument c = 1 then) against a FIXED per-query offset,
//     the first key tile's row max, so O is never rescaled; a block in which a later row max
//     passes it by > 32 (P > 2^32) reruns exactly (QK-only sweep for the true max, then the
//     flash sweep); row sums as lane-partial f32 adds.
// Work per frame: 4 * S^2 * 512 FLOP (34.4 GFLOP at S = 4096); bytes: Q, K, V read and O
// written once per frame from HBM (K/V re-read from L2 by the frame's 32 workgroups, which
// the XCD-aware block order keeps on one XCD).
#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int A5_D = 512, A5_NT = 256, A5_QW = 32, A5_QWG = 4 * A5_QW, A5_KT = 32;
constexpr int A5_ROW = A5_D * 2;            // bytes per K / V row
constexpr int A5_TILE = A5_KT * A5_ROW;     // 32 KiB
constexpr int A5_BUF = 2 * A5_TILE;         // K tile + V tile
constexpr int A5_LDS = 5 * A5_TILE;         // K ring of 3 + V ring of 2 slots: 160 KiB

// XOR swizzles of the 16-byte chunk index inside each 256-byte group of a 1 KiB row.
// K: rows r = 0..15 of a b128 lane group read the same chunk -> spread by r & 15.
// V: the transposed read takes 4 consecutive rows x 64 B -> spread rows over 64-B sections.
__device__ __forceinline__ uint32_t a5_kswz(uint32_t r) { return r & 15u; }
__device__ __forceinline__ uint32_t a5_vswz(uint32_t r) { return ((r & 3u) << 2) | ((r >> 2) & 3u); }

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_5;

__device__ __forceinline__ u32x4_5 a5_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  u32x4_5 r;
  r[0] = __builtin_amdgcn_readfirstlane((uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) & 0xffffu;  // stride 0
  r[2] = __builtin_amdgcn_readfirstlane(bytes);                          // num_records: range check
  r[3] = 0x00020000u;
  return r;
}

// One 1 KiB LDS-DMA row: lane l's 16 bytes at voff land at LDS byte lds + 16 l.  Inline asm so
// hipcc neither counts it in vmcnt nor drains it before the LDS reads of the other buffer; the
// loop waits for it explicitly (vmcnt(0) before the tile's barrier).
__device__ __forceinline__ void a5_dma(u32x4_5 rs_, uint32_t lds, uint32_t voff) {
  u32x4_5 rs;  // wave-uniform by construction; readfirstlane keeps the quad in SGPRs at every call site
#pragma unroll
  for (int i = 0; i < 4; ++i) rs[i] = __builtin_amdgcn_readfirstlane(rs_[i]);
  uint32_t keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
               "buffer_load_dwordx4 %2, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(voff), "s"(rs) : "memory");
}

__device__ __forceinline__ float a5_partner(float x) {  // the value of lane l ^ 32
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}

// PD: LDS fragment reads issued PD MFMAs ahead.  K and V stream one tile ahead in 2 + 2 slots (a
// 3-slot K ring two tiles ahead measured 15 % slower, 608 vs 529 us at 16 x 4096; a no-DMA
// ablation ran 439 us — the LDS-DMA issue, ~60 cycles per 1 KiB piece and 16 pieces per wave
// per tile, is the kernel's largest non-MFMA cost; profiles/r03h_flash512_dma_ab.txt)
template <bool RAGGED, int PD>
__global__ __launch_bounds__(A5_NT, 1) void flash512_kernel(const bf16_t* __restrict__ q, int64_t ldq,
                                                            const bf16_t* __restrict__ k, int64_t ldk,
                                                            const bf16_t* __restrict__ v, int64_t ldv,
                                                            bf16_t* __restrict__ o, int64_t ldo, int heads,
                                                            int64_t sq, int64_t skv, int64_t kv_div, float c,
                                                            int out_f32) {
  __shared__ __attribute__((aligned(1024))) char smem[A5_LDS];
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int nqb = (int)((sq + A5_QWG - 1) / A5_QWG);
  const int lid = xcd_remap(blockIdx.x, gridDim.x);  // a frame's blocks consecutive: one XCD's L2
  const int qblk = lid % nqb;
  const int h = (lid / nqb) % heads;
  const int64_t b = (lid / nqb) / heads;
  const int64_t q0 = (int64_t)qblk * A5_QWG + wave * A5_QW;
  const int64_t bkv = b / kv_div;
  const bf16_t* qb_ptr = q + b * sq * ldq + (int64_t)h * A5_D;
  const bf16_t* kb_ptr = k + bkv * skv * ldk + (int64_t)h * A5_D;
  const bf16_t* vb_ptr = v + bkv * skv * ldv + (int64_t)h * A5_D;

  // ---- K / V DMA: wave w moves rows 8w..8w+7 of both tiles; lane l of a row's instruction
  // writes LDS chunk l, i.e. source chunk l ^ swz(row) (the swizzle only flips bits 0-3)
  const uint32_t ldkb = (uint32_t)ldk * 2, ldvb = (uint32_t)ldv * 2;
  const u32x4_5 rk = a5_rsrc(kb_ptr, (uint32_t)(skv - 1) * ldkb + A5_ROW);
  const u32x4_5 rv = a5_rsrc(vb_ptr, (uint32_t)(skv - 1) * ldvb + A5_ROW);
  // LDS slots of 32 KiB: K(t) in slot t & 1, V(t) in slot 2 + (t & 1)
  auto ks_off = [&](int t) -> uint32_t { return (uint32_t)(t & 1) * A5_TILE; };
  auto vs_off = [&](int t) -> uint32_t { return (uint32_t)(2 + (t & 1)) * A5_TILE; };
  auto issue_k = [&](int t) {  // rows past skv: every byte out of the buffer's range -> zeros
    const uint32_t key0 = (uint32_t)t * A5_KT, kl = lds0 + ks_off(t);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t r = (uint32_t)(8 * wave + j);
      a5_dma(rk, kl + r * A5_ROW, (key0 + r) * ldkb + 16u * ((uint32_t)lane ^ a5_kswz(r)));
    }
  };
  auto issue_v = [&](int t) {
    const uint32_t key0 = (uint32_t)t * A5_KT, vl = lds0 + vs_off(t);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t r = (uint32_t)(8 * wave + j);
      a5_dma(rv, vl + r * A5_ROW, (key0 + r) * ldvb + 16u * ((uint32_t)lane ^ a5_vswz(r)));
    }
  };
  auto kslot = [&](int t) { return (const char*)smem + ks_off(t); };
  auto vslot = [&](int t) { return (const char*)smem + vs_off(t); };

  // ---- Q'^T fragments (B operand of S^T = K.Q^T): lane holds Q[q0 + r32][16 ks + 8 hh .. +7]
  const int64_t qi = q0 + r32;
  bf16x8 qf[32];
#pragma unroll
  for (int ks = 0; ks < 32; ++ks) {
    uint4 u = make_uint4(0, 0, 0, 0);
    if (qi < sq) u = *(const uint4*)(qb_ptr + qi * ldq + 16 * ks + 8 * hh);
    qf[ks] = __builtin_bit_cast(bf16x8, u);
  }

  // per-lane LDS read offsets inside a K / V tile
  //   K' fragment ks: row r32, chunk 2 ks + hh (swizzled); ks = j + 8 u -> koff[j] + 256 u
  uint32_t koff[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
    koff[j] = (uint32_t)r32 * A5_ROW + 16u * (((uint32_t)(2 * j + hh)) ^ a5_kswz((uint32_t)r32));
  //   V^T fragment (db, s2, half): lane 4qq + pp of 16-lane group g reads key
  //   16 s2 + 8 half + 4 hh + qq, d 32 db + 16 (g & 1) + 4 pp .. +3
  //   = chunk 4 db + 2 (g & 1) + (pp >> 1), byte 8 (pp & 1); db = j + 4 u -> voff[half][j] + 256 u
  const int g16 = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
  uint32_t voff[2][4];
#pragma unroll
  for (int half = 0; half < 2; ++half)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t kr = (uint32_t)(8 * half + 4 * hh + qq);  // + 16 s2 (does not change the swizzle)
      const uint32_t ch = (uint32_t)(4 * j + 2 * (g16 & 1) + (pp >> 1));
      voff[half][j] = kr * A5_ROW + 16u * (ch ^ a5_vswz(kr)) + 8u * (uint32_t)(pp & 1);
    }

  const int T = (int)((skv + A5_KT - 1) / A5_KT);
  // one barrier per step: this wave's DMAs of the previous step landed (vmcnt(0)), every
  // wave's LDS reads of the step before retired (lgkmcnt(0)) — the slots they read are free
  auto sync = [&](bool keep8 = false) {  // keep8: the youngest 8 DMAs (one K tile) stay in flight
    if (keep8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // S^T = K'.Q'^T of tile t: 32 MFMAs, K' fragments two ahead; keys past skv -> -inf
  auto qk = [&](const char* kl, int t, int) {
    f32x16 s;
#pragma unroll
    for (int i = 0; i < 16; ++i) s[i] = 0.f;
    auto kfrag = [&](int ks) { return *(const bf16x8*)(kl + koff[ks & 7] + 256 * (ks >> 3)); };
    bf16x8 kw[PD];  // rolling window: fragment ks sits in kw[ks % PD], read PD MFMAs ahead
#pragma unroll
    for (int i = 0; i < PD; ++i) kw[i] = kfrag(i);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < 32; ++ks) {
      const bf16x8 kc = kw[ks % PD];
      if (ks + PD < 32) kw[ks % PD] = kfrag(ks + PD);
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kc, qf[ks], s, 0, 0, 0);
    }
#pragma unroll
    for (int ks = 0; ks < 32; ++ks) {
      if (ks + PD < 32) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    }
    if (RAGGED && t == T - 1) {
      const int64_t kbase = (int64_t)t * A5_KT + 4 * hh;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (kbase + 8 * (i >> 2) + (i & 3) >= skv) s[i] = -INFINITY;
    }
    return s;
  };
  auto row_max = [&](const f32x16& s) {  // over the tile's 32 keys of this lane's query
    float tm = s[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) tm = fmaxf(tm, s[i]);
    return fmaxf(tm, a5_partner(tm)) * c;
  };

  f32x16 oacc[16];
  float m = 0.f, lsum = 0.f;
  bool bad = false;
  // P(t) = bf16(2^(S(t) - m)), the row sum over the unrounded values; FAST: m = the first
  // tile's row max, later tiles flag `bad` when their max passes m + 32
  auto softmax = [&](const f32x16& s, bool fast, bool first, bf16x8 (&pf)[2]) {
    if (fast) {
      const float tm = row_max(s);
      if (first) m = tm;
      else bad |= tm > m + 32.f;
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bf16x8 f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float p = __builtin_amdgcn_exp2f(fmaf(s[8 * s2 + j], c, -m));
        lsum += p;
        f[j] = (__bf16)p;
      }
      pf[s2] = f;
    }
  };
  // O^T += V^T.P: 32 MFMAs, V^T fragments (two tr reads each) PD MFMAs ahead
  auto pv = [&](const char* vl, const bf16x8 (&pf)[2]) {
    auto vfrag = [&](int i) {  // i = 2 db + s2
      const int db = i >> 1, s2 = i & 1;
      const char* p0 = vl + voff[0][db & 3] + 256 * (db >> 2) + 16 * A5_ROW * s2;
      const char* p1 = vl + voff[1][db & 3] + 256 * (db >> 2) + 16 * A5_ROW * s2;
      const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((bf16x4 __attribute__((address_space(3)))*)(p0));
      const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((bf16x4 __attribute__((address_space(3)))*)(p1));
      return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    };
    bf16x8 vw[PD];
#pragma unroll
    for (int i = 0; i < PD; ++i) vw[i] = vfrag(i);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const bf16x8 vc = vw[i % PD];
      if (i + PD < 32) vw[i % PD] = vfrag(i + PD);
      oacc[i >> 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vc, pf[i & 1], oacc[i >> 1], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      if (i + PD < 32) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    }
  };
  // One flash sweep over all key tiles with a FIXED offset m per query (no O rescale — a pass
  // over the 256 accumulators would need them in VGPRs: the kernel spilled).  FAST: m = the
  // first tile's row max, and the sweep reports whether a later tile's max passed m + 32
  // (P > 2^32 would then have entered O); otherwise m is the exact row max from a QK sweep.
  // Step t: wait for K(t)/V(t), one barrier, DMA K(t+1)/V(t+1) into the other slots, QK^T(t),
  // softmax(t), PV(t).
  auto sweep = [&](bool fast) {
#pragma unroll
    for (int db = 0; db < 16; ++db)
#pragma unroll
      for (int i = 0; i < 16; ++i) oacc[db][i] = 0.f;
    lsum = 0.f;
    sync();  // (the exact rerun's max sweep may still be reading K slot 0 in other waves)
    issue_k(0);
    issue_v(0);
    for (int t = 0; t < T; ++t) {
      sync();
      if (t + 1 < T) {
        issue_k(t + 1);
        issue_v(t + 1);
      }
      const f32x16 s = qk(kslot(t), t, -1);
      bf16x8 pf[2];
      softmax(s, fast, t == 0, pf);
      pv(vslot(t), pf);
    }
  };

  sweep(true);
  // the block-wide OR of `bad` through LDS (__syncthreads_or takes 256 B of LDS of its own, and
  // the rings use all 160 KiB): every wave is past its last LDS read after the first barrier
  sync();
  if (lane == 0) *(volatile uint32_t*)(smem + 4 * wave) = __any(bad) ? 1u : 0u;
  sync();
  const bool any_bad = (*(volatile const uint32_t*)(smem) | *(volatile const uint32_t*)(smem + 4) |
                        *(volatile const uint32_t*)(smem + 8) | *(volatile const uint32_t*)(smem + 12)) != 0;
  if (any_bad) {
    // rare: a row max jumped > 32 (log2) past the first tile's somewhere in the block.  The
    // block reruns exactly: a QK-only sweep for the exact row max, then the flash sweep.
    m = -INFINITY;
    sync();
    issue_k(0);
    for (int t = 0; t < T; ++t) {
      sync();
      if (t + 1 < T) issue_k(t + 1);
      m = fmaxf(m, row_max(qk(kslot(t), t, -1)));
    }
    sweep(false);
  }

  // ---- epilogue: O[q][d] = O^T[d][q] / l; lane (q, hh) holds d = 32 db + 8 (i >> 2) + 4 hh + (i & 3)
  const float l = lsum + a5_partner(lsum);
  const float inv = __builtin_amdgcn_rcpf(l);
  if (qi >= sq) return;  // lanes l and l ^ 32 share a query: no cross-lane op follows
  if (out_f32) {
    float* frow = (float*)o + (b * sq + qi) * ldo + (int64_t)h * A5_D;
#pragma unroll
    for (int db = 0; db < 16; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x16& a = oacc[db];
        *(float4*)(frow + 32 * db + 8 * g + 4 * hh) =
            make_float4(a[4 * g] * inv, a[4 * g + 1] * inv, a[4 * g + 2] * inv, a[4 * g + 3] * inv);
      }
    return;
  }
  bf16_t* orow = o + (b * sq + qi) * ldo + (int64_t)h * A5_D;
#pragma unroll
  for (int db = 0; db < 16; ++db)
#pragma unroll
    for (int mm = 0; mm < 2; ++mm) {
      const f32x16& a = oacc[db];
      const uint32_t x0 = pack2(a[8 * mm + 0] * inv, a[8 * mm + 1] * inv), x1 = pack2(a[8 * mm + 2] * inv, a[8 * mm + 3] * inv);
      const uint32_t y0 = pack2(a[8 * mm + 4] * inv, a[8 * mm + 5] * inv), y1 = pack2(a[8 * mm + 6] * inv, a[8 * mm + 7] * inv);
      const auto s0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
      const auto s1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
      *(uint4*)(orow + 32 * db + 16 * mm + 8 * hh) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
    }
}

}  // namespace

// d = 512 (the VAE mid-block attention) for attention_entry (attention.hip).
int launch_flash512(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv, void* o,
                    int64_t ldo, int64_t batch, int heads, int64_t sq, int64_t skv, int64_t kv_div, float scale,
                    hipStream_t s, int out_f32) {
  // 16-byte rows for the DMA pieces and the epilogue's 16-byte stores
  if (((uintptr_t)o & 15) != 0 || ldo % (out_f32 ? 4 : 8) != 0) return VD_EINVAL;
  if ((uint64_t)(skv - 1) * (uint64_t)ldk * 2 + A5_ROW >= 0x80000000ull ||
      (uint64_t)(skv - 1) * (uint64_t)ldv * 2 + A5_ROW >= 0x80000000ull)
    return VD_EINVAL;
  const int64_t nblk = (sq + A5_QWG - 1) / A5_QWG * heads * batch;
  if (nblk > 0x7fffffff) return VD_EINVAL;
  const float c = scale * 1.4426950408889634f;
  const dim3 grid((unsigned)nblk);
#define A5_LAUNCH(R)                                                                                          \
  hipLaunchKernelGGL((flash512_kernel<R, 3>), grid, dim3(A5_NT), 0, s, (const bf16_t*)q, ldq, (const bf16_t*)k,  \
                     ldk, (const bf16_t*)v, ldv, (bf16_t*)o, ldo, heads, sq, skv, kv_div, c, out_f32)
  if (skv % A5_KT != 0) A5_LAUNCH(true);
  else A5_LAUNCH(false);
#undef A5_LAUNCH
  return vd_launch_status();
}
