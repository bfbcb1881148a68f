// Attention kernels for gfx950.
//
// flash_attn_kernel — spatial self-attention and text cross-attention of
// diffusers Attention/AttnProcessor2_0 (F.scaled_dot_product_attention,
// SURVEY.md §8a a6/a7), bf16 MFMA with fp32 online softmax.
//
//   S^T = K . Q^T   (v_mfma_f32_16x16x32_bf16, A = K rows from LDS, B = Q^T
//                    from registers): the accumulator leaves each lane with 4
//                    keys of ONE query, so the row max needs 2 lane swaps and
//                    the row sum stays lane-local until the end.
//   O^T += V^T . P^T: the S^T accumulators of key blocks (2s, 2s+1), packed to
//                    bf16, ARE the P^T B-operand of k-step s (k order permuted;
//                    cdna_hip_programming.md §3 "accumulator as next operand"),
//                    and V^T comes out of LDS with ds_read_b64_tr_b16 (T10) in
//                    the same permuted key order.  No LDS round trip for P.
// Softmax VALU per score kept minimal: the scale is folded into the exp2
// argument (one FMA), the row max crosses lanes with v_permlane32/16_swap, the
// O rescale is skipped when no row max moved (wave-uniform), only a ragged
// last key tile is masked, and when PV is padded (d = 40 -> 48) column d of V
// holds 1.0 so the PV MFMA also produces the softmax row sum.
// Workgroup: 4 waves x 16*QBLK queries (QBLK = 4 for long sequences); K/V
// tiles of 64 keys double-buffered in LDS with the next tile's global loads
// issued before the current tile's MFMAs (T14).  Row strides are padded so
// 16-B K-row reads and the transposed V reads are bank-conflict free (§2/T10).
//
// temporal_attn_kernel — the motion-module attention over F <= 32 frames
// (a9).  Tiny per item (16x16 scores), so VALU with one wave per (position,
// head) and K/V staged in LDS; tokens are read in place from the NHWC rows.
#include "common.h"

namespace {

constexpr int NT = 256;
constexpr int KT = 64;   // keys per tile

template <int D>
struct AttnCfg {
  static constexpr int DQK = (D + 31) / 32 * 32;          // QK^T contraction, padded
  static constexpr int DV = (D + 15) / 16 * 16;           // PV output columns, padded
  static constexpr int KS = DQK + 16;                     // K LDS row (elements): +32 B pad, conflict-free
                                                          // b128 fragment reads (tools/lds_banks.py)
  static constexpr int VS = ((DV * 2 + 31) / 64 * 64 + 32) / 2;  // V LDS row: 32B * odd
  static constexpr int KCH = DQK / 8;                     // K 16-byte chunks per row
  static constexpr int VCH = DV / 8;
  static constexpr int DCH = D / 8;                       // valid 16-byte chunks per K/V row
  static constexpr int LREG = (KT * DCH + NT - 1) / NT;   // staged K (and V) chunks per thread
};

// Cross-lane max over the 4 lanes holding one query (l, l^16, l^32, l^48):
// v_permlane32_swap / v_permlane16_swap + max, no LDS traffic (T12).
__device__ __forceinline__ float max_over_query_lanes(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  auto t = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(t[0]), __uint_as_float(t[1]));
}

// K/V tile staging: the in-flight tile lives in one ext_vector register block
// (4 dwords per 16-byte chunk) with compile-time element indices — arrays of
// uint4 passed around were left as a scratch stack object by the compiler.
template <int L>
using stage_t = __attribute__((ext_vector_type(8 * L))) uint32_t;  // K chunks then V chunks

template <int L>
__device__ __forceinline__ stage_t<L> kv_load(const bf16_t* kb_ptr, const bf16_t* vb_ptr, int ldk,
                                              int ldv, int t, int64_t skv, const int (&krow)[L],
                                              const uint32_t (&kcol)[L]) {
  const int64_t key0 = (int64_t)t * KT;
  const bf16_t* kp = kb_ptr + key0 * ldk;
  const bf16_t* vp = vb_ptr + key0 * ldv;
  const int kmax = (int)(skv - 1 - key0);  // >= KT-1 except on a ragged last tile
  stage_t<L> st;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int r = krow[i] < kmax ? krow[i] : kmax;
    const uint4 a = *(const uint4*)(kp + (uint32_t)(r * ldk) + kcol[i]);
    const uint4 b = *(const uint4*)(vp + (uint32_t)(r * ldv) + kcol[i]);
    st[4 * i + 0] = a.x; st[4 * i + 1] = a.y; st[4 * i + 2] = a.z; st[4 * i + 3] = a.w;
    st[4 * L + 4 * i + 0] = b.x; st[4 * L + 4 * i + 1] = b.y;
    st[4 * L + 4 * i + 2] = b.z; st[4 * L + 4 * i + 3] = b.w;
  }
  return st;
}
template <int L>
__device__ __forceinline__ void kv_store(const stage_t<L>& st, bf16_t* kl, bf16_t* vl,
                                         const uint32_t (&ldsk)[L], const uint32_t (&ldsv)[L]) {
#pragma unroll
  for (int i = 0; i < L; ++i) {
    *(uint4*)(kl + ldsk[i]) = make_uint4(st[4 * i], st[4 * i + 1], st[4 * i + 2], st[4 * i + 3]);
    *(uint4*)(vl + ldsv[i]) = make_uint4(st[4 * L + 4 * i], st[4 * L + 4 * i + 1], st[4 * L + 4 * i + 2],
                                         st[4 * L + 4 * i + 3]);
  }
}

template <int D, int QBLK>
__global__ __launch_bounds__(NT, 2) void flash_attn_kernel(
    const bf16_t* __restrict__ q, int64_t ldq, const bf16_t* __restrict__ k, int64_t ldk,
    const bf16_t* __restrict__ v, int64_t ldv, bf16_t* __restrict__ o, int64_t ldo, int heads,
    int64_t sq, int64_t skv, int64_t kv_div, float c, int out_f32 = 0) {
  using C = AttnCfg<D>;
  // When PV is padded (DV > D) column D of V is set to 1.0, so the PV MFMA also
  // produces the softmax row sum (no per-score adds).
  constexpr bool ONES = C::DV > D;
  constexpr int QWV = 16 * QBLK;  // queries per wave
  __shared__ __attribute__((aligned(16))) bf16_t ks_lds[2][KT * C::KS];
  __shared__ __attribute__((aligned(16))) bf16_t vs_lds[2][KT * C::VS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = blockIdx.y;
  const int64_t b = blockIdx.z;
  const int64_t q0 = (int64_t)blockIdx.x * (4 * QWV) + wave * QWV;
  const int64_t bkv = b / kv_div;
  const bf16_t* qb_ptr = q + b * sq * ldq + (int64_t)h * D;
  const bf16_t* kb_ptr = k + bkv * skv * ldk + (int64_t)h * D;
  const bf16_t* vb_ptr = v + bkv * skv * ldv + (int64_t)h * D;
  const int fr = lane & 15, fg = lane >> 4;

  // Q^T fragments (B operand): lane holds Q[q0 + qb*16 + fr][dc*32 + 8*fg .. +7].
  bf16x8 qf[QBLK][C::DQK / 32];
#pragma unroll
  for (int qb = 0; qb < QBLK; ++qb) {
    const int64_t qi = q0 + qb * 16 + fr;
#pragma unroll
    for (int dc = 0; dc < C::DQK / 32; ++dc) {
      const int dd = dc * 32 + 8 * fg;
      uint4 u = make_uint4(0, 0, 0, 0);
      if (qi < sq && dd < D) u = *(const uint4*)(qb_ptr + qi * ldq + dd);
      qf[qb][dc] = __builtin_bit_cast(bf16x8, u);
    }
  }

  // K/V tile staging: only the D/8 valid chunks of each row are loaded; the
  // padding columns of both LDS buffers (zeros for K and V, and the 1.0 column
  // of V when ONES) are written once here and never overwritten.  Per-thread
  // (row, chunk) slots and their offsets are fixed for the whole kernel, so the
  // per-tile cost is one add per load; bounds are checked only on a ragged last tile.
  for (int idx = tid; idx < 2 * KT; idx += NT) {
    const int buf = idx / KT, r = idx % KT;
    for (int cc = C::DCH; cc < C::KCH; ++cc)
      *(uint4*)(&ks_lds[buf][r * C::KS + cc * 8]) = make_uint4(0, 0, 0, 0);
    for (int cc = C::DCH; cc < C::VCH; ++cc)
      *(uint4*)(&vs_lds[buf][r * C::VS + cc * 8]) = make_uint4(ONES && cc == C::DCH ? 0x3F80u : 0u, 0, 0, 0);
  }
  // Branch-free staging: every thread loads LREG (row, chunk) slots per tile;
  // slots past the tile's valid chunk count duplicate a valid one (same bytes to
  // the same LDS address), and rows past the last key are clamped to it (their
  // scores are masked to -inf, so P = 0 multiplies finite V).
  int krow[C::LREG];
  uint32_t kcol[C::LREG], ldsk[C::LREG], ldsv[C::LREG];
#pragma unroll
  for (int i = 0; i < C::LREG; ++i) {
    const int idx = (tid + i * NT) % (KT * C::DCH);
    const int r = idx / C::DCH, cc = idx % C::DCH;
    krow[i] = r;
    kcol[i] = (uint32_t)(cc * 8);
    ldsk[i] = (uint32_t)(r * C::KS + cc * 8);
    ldsv[i] = (uint32_t)(r * C::VS + cc * 8);
  }
  const int ldk32 = (int)ldk, ldv32 = (int)ldv;
  stage_t<C::LREG> kvst;

  f32x4 oacc[C::DV / 16][QBLK];
#pragma unroll
  for (int a = 0; a < C::DV / 16; ++a)
#pragma unroll
    for (int qb = 0; qb < QBLK; ++qb) oacc[a][qb] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrow[QBLK], lrow[QBLK];  // running max (scaled, log2 units) / lane-partial row sum
#pragma unroll
  for (int qb = 0; qb < QBLK; ++qb) { mrow[qb] = -INFINITY; lrow[qb] = 0.f; }

  const int ntiles = (int)((skv + KT - 1) / KT);
  const bool ragged = (skv % KT) != 0;
  kvst = kv_load<C::LREG>(kb_ptr, vb_ptr, ldk32, ldv32, 0, skv, krow, kcol);
  kv_store<C::LREG>(kvst, ks_lds[0], vs_lds[0], ldsk, ldsv);
  __syncthreads();
  const int qq = fr >> 2, pp = fr & 3;  // tr-read geometry: lane 4*qq+pp -> row qq, cols 4*pp..

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) kvst = kv_load<C::LREG>(kb_ptr, vb_ptr, ldk32, ldv32, t + 1, skv, krow, kcol);
    const bf16_t* kl = ks_lds[buf];
    const bf16_t* vl = vs_lds[buf];

    // ---- S^T = K . Q^T
    f32x4 s[4][QBLK];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int qb = 0; qb < QBLK; ++qb) s[kb][qb] = f32x4{0.f, 0.f, 0.f, 0.f};
    {  // K fragments two ahead in a rolling window (round 2): hipcc otherwise read each one right
       // before its QBLK MFMAs behind an lgkmcnt(0) — an exposed LDS latency per fragment
      constexpr int NK = C::DQK / 32 * 4;  // fragment i = (dc, kb) = (i / 4, i % 4)
      auto kfrag = [&](int i) { return *(const bf16x8*)(kl + ((i % 4) * 16 + fr) * C::KS + (i / 4) * 32 + 8 * fg); };
      bf16x8 k0 = kfrag(0), k1 = kfrag(1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < NK; ++i) {
        bf16x8 kn = k1;
        if (i + 2 < NK) kn = kfrag(i + 2);
#pragma unroll
        for (int qb = 0; qb < QBLK; ++qb)
          s[i % 4][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k0, qf[qb][i / 4], s[i % 4][qb], 0, 0, 0);
        k0 = k1;
        k1 = kn;
      }
#pragma unroll
      for (int i = 0; i < NK; ++i) {
        if (i + 2 < NK) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, QBLK, 0);
      }
    }
    if (ragged && t == ntiles - 1) {  // only the last tile of a ragged key range is masked
      const int64_t kbase = (int64_t)t * KT + 4 * fg;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (kbase + kb * 16 + j >= skv) {
#pragma unroll
            for (int qb = 0; qb < QBLK; ++qb) s[kb][qb][j] = -INFINITY;
          }
    }
    // ---- online softmax in log2 units: p = exp2(s*c - m)
    bf16x8 pf[2][QBLK];
    bool any_rescale = false;
    float alpha[QBLK];
#pragma unroll
    for (int qb = 0; qb < QBLK; ++qb) {
      float mx = s[0][qb][0];
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int j = 0; j < 4; ++j) mx = fmaxf(mx, s[kb][qb][j]);
      mx = max_over_query_lanes(mx) * c;
      const float mnew = fmaxf(mrow[qb], mx);
      alpha[qb] = __builtin_amdgcn_exp2f(mrow[qb] - mnew);
      any_rescale |= mnew != mrow[qb];
      mrow[qb] = mnew;
      float ls = 0.f;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float p = __builtin_amdgcn_exp2f(fmaf(s[kb][qb][j], c, -mnew));
          s[kb][qb][j] = p;
          if (!ONES) ls += p;
        }
      if (!ONES) lrow[qb] = lrow[qb] * alpha[qb] + ls;
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        bf16x8 f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f[j] = (__bf16)s[2 * st][qb][j];
          f[4 + j] = (__bf16)s[2 * st + 1][qb][j];
        }
        pf[st][qb] = f;
      }
    }
    if (__any(any_rescale)) {  // wave-uniform: skip the O-wide multiply when no max moved
#pragma unroll
      for (int a = 0; a < C::DV / 16; ++a)
#pragma unroll
        for (int qb = 0; qb < QBLK; ++qb)
#pragma unroll
          for (int j = 0; j < 4; ++j) oacc[a][qb][j] *= alpha[qb];
    }
    // ---- O^T += V^T . P^T
    {  // V^T fragments two ahead in a rolling window, as K above (fragment j = (a, st) = (j / 2, j % 2))
      constexpr int NV = C::DV / 16 * 2;
      auto vfrag = [&](int j) {
        const bf16_t* p0 = vl + (32 * (j % 2) + 4 * fg + qq) * C::VS + (j / 2) * 16 + 4 * pp;
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((bf16x4 __attribute__((address_space(3)))*)(p0));
        const bf16x4 hi =
            __builtin_amdgcn_ds_read_tr16_b64_v4bf16((bf16x4 __attribute__((address_space(3)))*)(p0 + 16 * C::VS));
        return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      };
      bf16x8 v0 = vfrag(0), v1 = vfrag(1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        bf16x8 vn = v1;
        if (j + 2 < NV) vn = vfrag(j + 2);
#pragma unroll
        for (int qb = 0; qb < QBLK; ++qb)
          oacc[j / 2][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(v0, pf[j % 2][qb], oacc[j / 2][qb], 0, 0, 0);
        v0 = v1;
        v1 = vn;
      }
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        if (j + 2 < NV) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, QBLK, 0);
      }
    }
    if (t + 1 < ntiles) kv_store<C::LREG>(kvst, ks_lds[buf ^ 1], vs_lds[buf ^ 1], ldsk, ldsv);
    __syncthreads();
  }

  // ---- epilogue: O[q][d] = O^T[d][q] / l
#pragma unroll
  for (int qb = 0; qb < QBLK; ++qb) {
    float l;
    if constexpr (ONES) {
      constexpr int a1 = D / 16, r1 = D % 16;
      l = __shfl(oacc[a1][qb][r1 % 4], (r1 / 4) * 16 + fr, 64);
    } else {
      l = lrow[qb];
      l += __shfl_xor(l, 16, 64);
      l += __shfl_xor(l, 32, 64);
    }
    const float inv = 1.0f / l;
    const int64_t qi = q0 + qb * 16 + fr;
    if (qi >= sq) continue;
    bf16_t* orow = o + (b * sq + qi) * ldo + (int64_t)h * D;
    float* frow = (float*)o + (b * sq + qi) * ldo + (int64_t)h * D;  // out_f32: O in fp32 (tests)
#pragma unroll
    for (int a = 0; a < C::DV / 16; ++a) {
      const int dd = a * 16 + 4 * fg;
      if (dd < D) {
        if (out_f32)
          *(float4*)(frow + dd) = make_float4(oacc[a][qb][0] * inv, oacc[a][qb][1] * inv, oacc[a][qb][2] * inv,
                                              oacc[a][qb][3] * inv);
        else
          *(uint2*)(orow + dd) = make_uint2(pack2(oacc[a][qb][0] * inv, oacc[a][qb][1] * inv),
                                            pack2(oacc[a][qb][2] * inv, oacc[a][qb][3] * inv));
      }
    }
  }
}

// ============================================================ flash32
// Small-head flash attention on v_mfma_f32_32x32x16_bf16 (d = 40: SD-1.5's
// level-1 spatial self-attention, the hottest attention of the step).
//
//   S^T = K'.Q'^T   A = K rows (32 keys x 16 d, ds_read_b128), B = Q'^T from
//                   registers; contraction over d padded to DK = 48 (3 MFMAs
//                   per 32x32 tile instead of 4 with 16x16x32 at 64).  Column D
//                   of K' holds 1.0 and column D of Q' holds -mu (mu = this
//                   query's running max, bf16-representable), so the MFMA emits
//                   x = s - mu directly.  When the caller folded the softmax
//                   scale and log2(e) into its Q projection (c == 1, the model
//                   path: vdiff Attention.prepare) p = exp2(x) needs no per-score
//                   FMA; otherwise p = exp2(c*x) (one multiply).
//   O^T += V^T.P^T  the S^T accumulator, packed to bf16, IS the P^T B operand
//                   (cdna_hip_programming.md §3 "accumulator tile as the next
//                   MFMA's operand"; permuted key order within each 16-key
//                   step), V^T comes from ds_read_b64_tr_b16 in that order; V's
//                   column D holds 1.0 so the same MFMA yields the row sum.
// Deferred max (T13): while every u of the tile is <= THR, p = exp2(u) (one
// v_exp + 1/2 v_max3 + 1/2 v_cvt_pk per score); otherwise (first tile, or a
// row max that grew by > THR) mu is raised for those rows, the tile's u and
// the O rows are rescaled and Q''s -mu entry is rewritten — the decision covers
// the whole tile before any of its P is formed, so nothing is half-scaled.
// P <= 2^THR stays exact in the fp32 O/l accumulators; P's bf16 rounding is
// relative, so the normalised result does not depend on THR.
// Layout: 4 waves x 64 queries (2 query blocks of 32); K/V tiles of 64 keys
// double-buffered in ONE LDS array (K rows padded to 56 elements, V as
// [2][64 keys][32 d] images): both the K b128 reads and the V transposed reads
// are bank-conflict free (tools/lds_banks.py).  Register staging (T14): the
// next tile's global loads issue before this tile's MFMAs, their LDS writes
// after the PV, one barrier per tile.  Epilogue: permlane32_swap pairs give
// 16-byte stores of 8 consecutive output channels.
typedef __attribute__((ext_vector_type(16))) float f32x16;

template <int D>
struct F32Cfg {
  static_assert(D % 8 == 0 && D <= 48, "flash32: d must be a multiple of 8, <= 48");
  static constexpr int DK = (D + 1 + 15) / 16 * 16;   // contraction incl. the -mu column
  static constexpr int KSTEPS = DK / 16;
  static constexpr int DVP = (D + 1 + 31) / 32 * 32;  // PV rows incl. the ones column
  static constexpr int NDB = DVP / 32;
  static constexpr int KS = DK + 8;                   // K LDS row (elements), conflict-free
  static constexpr int DCH = D / 8;                   // 16-B chunks per K/V row
  static constexpr int K_ELEMS = KT * KS;
  static constexpr int V_ELEMS = NDB * KT * 32;
  static constexpr int STAGE = K_ELEMS + V_ELEMS;     // elements per buffer
  static constexpr int LREG = (KT * DCH + NT - 1) / NT;
  // position of d = D in the Q'^T fragment (k-step, lane half, element)
  static constexpr int MU_KS = D / 16, MU_H = (D % 16) / 8, MU_J = D % 8;
  // position of the ones column in the O^T accumulator (d-block, lane half, register)
  static constexpr int L_DB = D / 32, L_H = ((D % 32) / 4) & 1, L_I = (D % 4) + 4 * ((D % 32) / 8);
};

constexpr float F32_THR = 6.0f;  // deferred-max threshold (log2 units): P <= 64

__device__ __forceinline__ float vmax3(float a, float b, float c) {
  // plain v_max3_f32: fmaxf would add IEEE canonicalising maxes on MFMA results
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float vmax2(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// max over the 32 scores a lane holds for its query in one 64-key tile
__device__ __forceinline__ float tile_max(const f32x16& a, const f32x16& b) {
  float m0 = vmax3(a[0], a[1], a[2]), m1 = vmax3(a[3], a[4], a[5]), m2 = vmax3(a[6], a[7], a[8]);
  float m3 = vmax3(a[9], a[10], a[11]), m4 = vmax3(a[12], a[13], a[14]), m5 = vmax3(a[15], b[0], b[1]);
  float m6 = vmax3(b[2], b[3], b[4]), m7 = vmax3(b[5], b[6], b[7]), m8 = vmax3(b[8], b[9], b[10]);
  float m9 = vmax3(b[11], b[12], b[13]), m10 = vmax2(b[14], b[15]);
  m0 = vmax3(m0, m1, m2);
  m3 = vmax3(m3, m4, m5);
  m6 = vmax3(m6, m7, m8);
  m9 = vmax2(m9, m10);
  return vmax2(vmax3(m0, m3, m6), m9);
}
// value of lane l ^ 32 (v_permlane32_swap)
__device__ __forceinline__ float partner32(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  // r[0] = new vdst (lanes 32-63 <- src of lanes 0-31), r[1] = new src (lanes 0-31 <- vdst of lanes 32-63)
  return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}

// One pass of flash32's key loop (prologue tile load included).  EXACT tracks the
// running max of every tile (deferred, THR); the fast pass computes it for the
// first tile only and afterwards lets P grow up to 2^32 before raising mu by
// log2(row sum) — the row sum comes free from the PV MFMA's ones column, so the
// common tile has no max reduction at all (-40 VALU ops per 64 keys).  mu stays
// >= the running max (l >= 2^(max - mu)), so nothing underflows that matters;
// a row sum >= 2^100 (or non-finite) means a score jumped past the fp32/bf16
// range and the pass reports `bad` so the block reruns EXACT.
template <int D, bool UNITC, bool EXACT, int QB = 2>
__device__ __forceinline__ bool f32_loop(bf16_t* lds, const bf16_t* kb_ptr, const bf16_t* vb_ptr, int ldk32,
                                         int ldv32, int64_t skv, const int (&krow)[F32Cfg<D>::LREG],
                                         const uint32_t (&kcol)[F32Cfg<D>::LREG],
                                         const uint32_t (&ldsk)[F32Cfg<D>::LREG],
                                         const uint32_t (&ldsv)[F32Cfg<D>::LREG],
                                         bf16x8 (&qf)[QB][F32Cfg<D>::KSTEPS], f32x16 (&oacc)[F32Cfg<D>::NDB][QB],
                                         int r32, int hh, int vtr, float c) {
  using C = F32Cfg<D>;
  constexpr float RESCALE = 4294967296.0f;        // 2^32
  constexpr float BAD = 1.2676506002282294e30f;   // 2^100
#pragma unroll
  for (int db = 0; db < C::NDB; ++db)
#pragma unroll
    for (int qb = 0; qb < QB; ++qb)
#pragma unroll
      for (int i = 0; i < 16; ++i) oacc[db][qb][i] = 0.f;
  float mu[QB];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) mu[qb] = 0.f;
  bool bad = false;

  const int ntiles = (int)((skv + KT - 1) / KT);
  const bool ragged = (skv % KT) != 0;
  stage_t<C::LREG> kvst = kv_load<C::LREG>(kb_ptr, vb_ptr, ldk32, ldv32, 0, skv, krow, kcol);
#pragma unroll
  for (int i = 0; i < C::LREG; ++i) {
    *(uint4*)(lds + ldsk[i]) = make_uint4(kvst[4 * i], kvst[4 * i + 1], kvst[4 * i + 2], kvst[4 * i + 3]);
    *(uint4*)(lds + ldsv[i]) = make_uint4(kvst[4 * C::LREG + 4 * i], kvst[4 * C::LREG + 4 * i + 1],
                                          kvst[4 * C::LREG + 4 * i + 2], kvst[4 * C::LREG + 4 * i + 3]);
  }
  __syncthreads();

  // one K/V tile: the general form (tile max on tile 0 / every tile of the exact pass,
  // ragged-key masking, rescale one tile late)
  auto tile_generic = [&](int t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) kvst = kv_load<C::LREG>(kb_ptr, vb_ptr, ldk32, ldv32, t + 1, skv, krow, kcol);
    const bf16_t* kl = lds + buf * C::STAGE;
    const bf16_t* vl = kl + C::K_ELEMS;
    // ---- x^T = K'.Q'^T  (= s - mu)
    f32x16 s[2][QB];
    bf16x8 kfr[2][C::KSTEPS];  // all K fragments of the tile first: one LDS latency, not six
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int ks = 0; ks < C::KSTEPS; ++ks)
        kfr[kb][ks] = *(const bf16x8*)(kl + (kb * 32 + r32) * C::KS + ks * 16 + 8 * hh);
    __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead (the scheduler sinks them to their MFMAs)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int ks = 0; ks < C::KSTEPS; ++ks) {
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) {
          if (ks == 0) {
            f32x16 z;
#pragma unroll
            for (int i = 0; i < 16; ++i) z[i] = 0.f;
            s[kb][qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kfr[kb][ks], qf[qb][ks], z, 0, 0, 0);
          } else {
            s[kb][qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kfr[kb][ks], qf[qb][ks], s[kb][qb], 0, 0, 0);
          }
        }
      }
    }
    if (ragged && t == ntiles - 1) {  // keys past skv: x = -inf (rows are clamped duplicates)
      const int kvalid = (int)(skv - (int64_t)t * KT);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = kb * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
          if (key >= kvalid) {
#pragma unroll
            for (int qb = 0; qb < QB; ++qb) s[kb][qb][i] = -INFINITY;
          }
        }
    }
    // V^T fragments for this tile's PV, issued now so their LDS latency hides
    // under the softmax VALU work (key order of each step: 16*s2 + 8*(j>>2) + 4*hh + (j&3))
    bf16x8 vfr[C::NDB][2][2];
#pragma unroll
    for (int db = 0; db < C::NDB; ++db)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16_t* p0 = vl + (db * KT + kb * 32 + 16 * s2) * 32 + vtr;
          const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (bf16x4 __attribute__((address_space(3)))*)(p0));
          const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (bf16x4 __attribute__((address_space(3)))*)(p0 + 8 * 32));
          vfr[db][kb][s2] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
    __builtin_amdgcn_sched_barrier(0);
    if (EXACT || t == 0) {  // ---- tile max (deferred, THR): every tile on the exact pass, tile 0 on the fast one
      float tm[QB];
      bool need = t == 0;
#pragma unroll
      for (int qb = 0; qb < QB; ++qb) {
        const float m = tile_max(s[0][qb], s[1][qb]);
        tm[qb] = vmax2(m, partner32(m));
        need |= (UNITC ? tm[qb] : tm[qb] * c) > F32_THR;
      }
      if (__any(need)) {  // wave-uniform: first tile or a row max moved by > THR
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) {
          const bool up = t == 0 || (UNITC ? tm[qb] : tm[qb] * c) > F32_THR;
          const float nmu = up ? (float)(__bf16)(mu[qb] + tm[qb]) : mu[qb];
          const float delta = nmu - mu[qb];  // exact: both bf16 values
          const float alpha = __builtin_amdgcn_exp2f(UNITC ? -delta : -delta * c);
          mu[qb] = nmu;
#pragma unroll
          for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int i = 0; i < 16; ++i) s[kb][qb][i] -= delta;
#pragma unroll
          for (int db = 0; db < C::NDB; ++db)
#pragma unroll
            for (int i = 0; i < 16; ++i) oacc[db][qb][i] *= alpha;
          if (hh == C::MU_H) qf[qb][C::MU_KS][C::MU_J] = (__bf16)(-nmu);
        }
      }
    }
    if (!EXACT && t > 1) {
      // ---- fast pass: rescale from the row sum of tiles 0..t-1 when it outgrows 2^32.
      // Checked one tile late, after this tile's QK^T MFMAs are issued, so reading the PV
      // accumulator does not drain the MFMA pipe right behind the PV chain; this tile's
      // scores (formed with the old mu) take the same shift as the exact path's.
      float lq[QB];
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
        for (int qb = 0; qb < QB; ++qb) {
          const float step = lq[qb] > RESCALE ? __builtin_amdgcn_logf(lq[qb]) : 0.f;  // log2(l)
          const float nmu = (float)(__bf16)(mu[qb] + (UNITC ? step : step / c));
          const float delta = nmu - mu[qb];
          const float alpha = __builtin_amdgcn_exp2f(UNITC ? -delta : -delta * c);
          mu[qb] = nmu;
#pragma unroll
          for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int i = 0; i < 16; ++i) s[kb][qb][i] -= delta;
#pragma unroll
          for (int db = 0; db < C::NDB; ++db)
#pragma unroll
            for (int i = 0; i < 16; ++i) oacc[db][qb][i] *= alpha;
          if (hh == C::MU_H) qf[qb][C::MU_KS][C::MU_J] = (__bf16)(-nmu);
        }
      }
    }
    // ---- P = exp2(x), packed: registers 8*s2 .. 8*s2+7 of tile kb = k-step (kb, s2)
    bf16x8 pf[2][2][QB];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int qb = 0; qb < QB; ++qb)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          bf16x8 f;
#pragma unroll
          for (int j = 0; j < 8; ++j)
            f[j] = (__bf16)__builtin_amdgcn_exp2f(UNITC ? s[kb][qb][8 * s2 + j] : s[kb][qb][8 * s2 + j] * c);
          pf[kb][s2][qb] = f;
        }
    // ---- O^T += V^T.P^T
#pragma unroll
    for (int db = 0; db < C::NDB; ++db)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int qb = 0; qb < QB; ++qb)
            oacc[db][qb] =
                __builtin_amdgcn_mfma_f32_32x32x16_bf16(vfr[db][kb][s2], pf[kb][s2][qb], oacc[db][qb], 0, 0, 0);
    if (t + 1 < ntiles) {
      bf16_t* nb = lds + (buf ^ 1) * C::STAGE;
#pragma unroll
      for (int i = 0; i < C::LREG; ++i) {
        *(uint4*)(nb + ldsk[i]) = make_uint4(kvst[4 * i], kvst[4 * i + 1], kvst[4 * i + 2], kvst[4 * i + 3]);
        *(uint4*)(nb + ldsv[i]) = make_uint4(kvst[4 * C::LREG + 4 * i], kvst[4 * C::LREG + 4 * i + 1],
                                             kvst[4 * C::LREG + 4 * i + 2], kvst[4 * C::LREG + 4 * i + 3]);
      }
    }
    __syncthreads();
  };
  for (int t = 0; t < ntiles; ++t) tile_generic(t);
  if (!EXACT) {  // the last tiles' row sums were not checked in the loop
    bool over = false;
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
      const float lown = oacc[C::L_DB][qb][C::L_I];
      const float lp = partner32(lown);  // every lane takes part in the swap
      over |= !((hh == C::L_H ? lown : lp) < BAD);
    }
    bad |= __any(over);
  }
  return bad;
}

// QB = 32-query blocks per wave: 2 (256 VGPRs, two waves per SIMD; one block per wave with three
// waves per SIMD measured slower, 1010 vs 878 us: profiles/r02_attn_occupancy_ab.txt).
// FIX: flash40's exact fix-up pass — a block whose first output element is a NaN flag (flash40
// found a score jump past its fast pass's range there) recomputes its 256 queries with the exact
// pass.  Round 6: one workgroup per F32_FIXW blocks (fix_blocks in all), whose first F32_FIXW
// lanes read those blocks' flags at once (one load latency) and which then recomputes the flagged
// ones in turn — the launch that follows every flash40 call was one workgroup per block, 4096 at
// the level-1 self-attention, ~8 us with nothing flagged.  The fix-up runs QB = 1 (128-query
// blocks, two per flagged quarter; a query's exact-pass arithmetic does not depend on QB): the
// block loop at QB = 2's 256 VGPRs spilled.  Both halves of a quarter sit in one workgroup
// (F32_FIXW even) and every flag is read before any block overwrites one.
constexpr int F32_FIXW = 16;
template <int D, bool UNITC, bool FIX = false, int QB = 2>
__global__ __launch_bounds__(NT, 2) void flash32_kernel(
    const bf16_t* __restrict__ q, int64_t ldq, const bf16_t* __restrict__ k, int64_t ldk,
    const bf16_t* __restrict__ v, int64_t ldv, bf16_t* __restrict__ o, int64_t ldo, int heads,
    int64_t sq, int64_t skv, int64_t kv_div, float c, int out_f32 = 0, int64_t fix_blocks = 0) {
  using C = F32Cfg<D>;
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * C::STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, hh = lane >> 5;
  // 1-D grid, XCD-aware (T1): the query blocks of one (image, head) get
  // consecutive logical ids and xcd_remap keeps consecutive ids on one XCD, so
  // that head's K/V is fetched into one L2 instead of eight.
  const int nqb = (int)((sq + 4 * 32 * QB - 1) / (4 * 32 * QB));
  auto flag_of = [&](int64_t lid) {  // the block's flag: a NaN in the first output element of its
    const int qblk = (int)(lid % nqb);  // flash40 256-query quarter
    const int h = (int)((lid / nqb) % heads);
    const int64_t b = (lid / nqb) / heads;
    const int64_t f = (b * sq + (((int64_t)qblk * (4 * 32 * QB)) & ~(int64_t)255)) * ldo + (int64_t)h * D;
    return out_f32 ? __builtin_isnan(((const float*)o)[f]) : ((o[f] & 0x7FFF) > 0x7F80);
  };
  auto block = [&](int lid) {
  const int qblk = lid % nqb;
  const int h = (lid / nqb) % heads;
  const int64_t b = (lid / nqb) / heads;
  const int64_t q0 = (int64_t)qblk * (4 * 32 * QB) + wave * (32 * QB);
  const int64_t bkv = b / kv_div;
  const bf16_t* qb_ptr = q + b * sq * ldq + (int64_t)h * D;
  const bf16_t* kb_ptr = k + bkv * skv * ldk + (int64_t)h * D;
  const bf16_t* vb_ptr = v + bkv * skv * ldv + (int64_t)h * D;

  // Q'^T fragments: lane holds Q'[q0 + qb*32 + r32][16*ks + 8*hh .. +7].  Q is
  // used as given (no bf16 prescale: that second rounding costs ~0.4% in P); with
  // UNITC the caller folded c into its Q projection (c == 1 exactly) and mu lives
  // in log2 units, otherwise mu is in raw score units and p = exp2(c * x).
  bf16x8 qf[QB][C::KSTEPS];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    const int64_t qi = q0 + qb * 32 + r32;
#pragma unroll
    for (int ks = 0; ks < C::KSTEPS; ++ks) {
      const int dd = ks * 16 + 8 * hh;
      uint4 u = make_uint4(0, 0, 0, 0);
      if (qi < sq && dd < D) u = *(const uint4*)(qb_ptr + qi * ldq + dd);
      qf[qb][ks] = __builtin_bit_cast(bf16x8, u);  // d = D entry starts at 0 (mu = 0)
    }
  }

  // LDS padding, written once: K' column D = 1.0 (the -mu column), V column D =
  // 1.0 (the row-sum column), every other padding element 0.
  for (int idx = tid; idx < 2 * KT; idx += NT) {
    const int buf = idx / KT, r = idx % KT;
    bf16_t* kl = lds + buf * C::STAGE;
    bf16_t* vl = kl + C::K_ELEMS;
    for (int cc = C::DCH; cc < C::DK / 8; ++cc)
      *(uint4*)(kl + r * C::KS + cc * 8) = make_uint4(cc == C::DCH ? 0x3F80u : 0u, 0, 0, 0);
    for (int cc = C::DCH; cc < C::DVP / 8; ++cc)
      *(uint4*)(vl + ((cc >> 2) * KT + r) * 32 + (cc & 3) * 8) = make_uint4(cc == C::DCH ? 0x3F80u : 0u, 0, 0, 0);
  }
  // staging slots (row, chunk) per thread, fixed for the kernel
  int krow[C::LREG];
  uint32_t kcol[C::LREG], ldsk[C::LREG], ldsv[C::LREG];
#pragma unroll
  for (int i = 0; i < C::LREG; ++i) {
    const int idx = (tid + i * NT) % (KT * C::DCH);
    const int r = idx / C::DCH, cc = idx % C::DCH;
    krow[i] = r;
    kcol[i] = (uint32_t)(cc * 8);
    ldsk[i] = (uint32_t)(r * C::KS + cc * 8);
    ldsv[i] = (uint32_t)(C::K_ELEMS + ((cc >> 2) * KT + r) * 32 + (cc & 3) * 8);
  }
  const int ldk32 = (int)ldk, ldv32 = (int)ldv;

  const int g16 = lane >> 4, i16 = lane & 15;
  // V^T tr-read lane offset inside a [32 d] image row block (elements)
  const int vtr = ((4 * hh + (i16 >> 2)) * 32) + 16 * (g16 & 1) + 4 * (i16 & 3);
  f32x16 oacc[C::NDB][QB];
  const bool bad = FIX || f32_loop<D, UNITC, false, QB>(lds, kb_ptr, vb_ptr, ldk32, ldv32, skv, krow, kcol, ldsk,
                                                           ldsv, qf, oacc, r32, hh, vtr, c);
  if (__syncthreads_or(bad)) {  // a score jumped > ~100 (log2) past mu somewhere: exact pass
#pragma unroll
    for (int qb = 0; qb < QB; ++qb)
      if (hh == C::MU_H) qf[qb][C::MU_KS][C::MU_J] = (__bf16)0.0f;
    f32_loop<D, UNITC, true, QB>(lds, kb_ptr, vb_ptr, ldk32, ldv32, skv, krow, kcol, ldsk, ldsv, qf, oacc, r32, hh,
                             vtr, c);
  }

  // ---- epilogue: O[q][d] = O^T[d][q] / l; register i of d-block db holds
  // d = 32*db + 8*(i>>2) + 4*hh + (i&3); swap 4-channel groups across lane halves
  // so each lane stores 8 consecutive channels (16 B).
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    const float lown = oacc[C::L_DB][qb][C::L_I];
    const float lp = partner32(lown);
    const float l = hh == C::L_H ? lown : lp;
    const float inv = __builtin_amdgcn_rcpf(l);
    const int64_t qi = q0 + qb * 32 + r32;
    if (out_f32) {  // tests: O in fp32; register i of d-block db holds d = 32 db + 8 (i >> 2) + 4 hh + (i & 3)
      float* frow = (float*)o + (b * sq + qi) * ldo + (int64_t)h * D;
#pragma unroll
      for (int db = 0; db < C::NDB; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d0 = 32 * db + 8 * g + 4 * hh;
          const f32x16& a = oacc[db][qb];
          if (qi < sq && d0 + 4 <= D)
            *(float4*)(frow + d0) = make_float4(a[4 * g] * inv, a[4 * g + 1] * inv, a[4 * g + 2] * inv, a[4 * g + 3] * inv);
        }
      continue;
    }
    bf16_t* orow = o + (b * sq + (qi < sq ? qi : 0)) * ldo + (int64_t)h * D;
#pragma unroll
    for (int db = 0; db < C::NDB; ++db) {
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const f32x16& a = oacc[db][qb];
        uint32_t x0 = pack2(a[8 * m + 0] * inv, a[8 * m + 1] * inv), x1 = pack2(a[8 * m + 2] * inv, a[8 * m + 3] * inv);
        uint32_t y0 = pack2(a[8 * m + 4] * inv, a[8 * m + 5] * inv), y1 = pack2(a[8 * m + 6] * inv, a[8 * m + 7] * inv);
        auto s0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
        auto s1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
        // lanes < 32: (x, y) = channels 16m + 0..7; lanes >= 32: channels 16m + 8..15
        const int dd = 32 * db + 16 * m + 8 * hh;
        if (qi < sq && dd + 8 <= D) *(uint4*)(orow + dd) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
      }
    }
  }
  };
  if constexpr (FIX) {
    __shared__ unsigned long long fmask;
    if (wave == 0) {
      const int64_t j = (int64_t)blockIdx.x * F32_FIXW + lane;
      const unsigned long long m = __ballot(lane < F32_FIXW && j < fix_blocks && flag_of(j));
      if (lane == 0) fmask = m;
    }
    __syncthreads();
    // workgroup-uniform: kept in SGPRs (a VGPR copy live across the exact pass spilled)
    const unsigned long long fm = fmask;
    unsigned long long m = ((unsigned long long)__builtin_amdgcn_readfirstlane((uint32_t)(fm >> 32)) << 32) |
                           __builtin_amdgcn_readfirstlane((uint32_t)fm);
    while (m) {
      const int bit = __builtin_ctzll(m);
      m &= m - 1;
      block((int)((int64_t)blockIdx.x * F32_FIXW + bit));
      __syncthreads();  // the next block rewrites the LDS tiles and padding
    }
  } else {
    block(xcd_remap(blockIdx.x, gridDim.x));
  }
}

// ============================================================ flash40
// The d = 40 spatial self-attention (SD-1.5 level 1, the roofline kernel) as a two-group
// ping-pong over an LDS-DMA ring (round 3).  flash32's arithmetic, tile for tile: S^T =
// K'.Q'^T on v_mfma_f32_32x32x16_bf16 with the running offset -mu folded into Q' (K' column 40
// = 1), P = exp2 packed to bf16 straight from the accumulator as the PV B operand, V's column
// 40 = 1 yields the row sum, mu from tile 0's max (every tile on the exact rerun), the fast
// pass's row-sum rescale past 2^32 and its exact rerun past 2^100 — results equal flash32's.
//
// What changes is the schedule.  Each wave's work per 64-key tile t splits into
//     V(t): the softmax of S(t) -> P(t)                    VALU only (64 exp2 + 32 packs)
//     M(t): PV(t) then QK^T(t+1) -> S(t+1)                  MFMA only (16 + 12 x 32x32x16)
// and the workgroup's 8 waves form two groups one barrier apart (waves w and w+4 share a
// SIMD): while group 0 runs M, group 1 runs V and vice versa, so on every SIMD the matrix
// pipe and the VALU work side by side (MI355X_MICROARCH.md "Two waves per SIMD").  One
// s_barrier per phase; 512 queries per workgroup (8 waves x 64) share every K/V tile.
//
// K/V tiles arrive by LDS-DMA (buffer_load ... lds: 12 x 1 KiB per tile, two per wave on
// waves 0-5, issued two tiles ahead) into a 4-slot ring: no register staging, no ds_write in
// the loop.  LDS image of a slot (12 KiB): K as [chunk c 0..5][key] 16-B rows, chunk 5 = K'
// column 40 ({1, 0 x 7}); V as [key][d 0..31], [key][d 32..39] and [key][{1, 0 x 7}] (V column
// 40 and the zero columns, by per-lane tr-read addresses).  The K'/V ones chunks are DMA'd from
// a 16-byte constant like the data, so a key past skv — every K/V byte of its row out of the
// buffer's range — reads all zeros: score 0, P = 1, V row and ones column 0, i.e. no
// contribution, with no masking code.  The K' ds_read_b128 of 32 keys is 512 contiguous bytes
// and the V tr-read of 4 keys x 32 d 256 contiguous bytes: conflict-free.  Tile u is issued at
// phase 2u-4 (group 0) / 2u-3 (group 1) and waited for (counted vmcnt; the DMA is inline asm so hipcc neither counts it nor
// drains it before the LDS reads) before the barrier that ends phase 2u-1; the slot it
// overwrites (tile u-4) was last read in phase 2u-6.
constexpr int F4_NW = 8, F4_NT = 512, F4_QB = 2, F4_QWG = F4_NW * 32 * F4_QB;
constexpr int F4_RING = 4;
constexpr int F4_K = 0, F4_V0 = 6 * 1024, F4_V1 = F4_V0 + 4096, F4_VONE = F4_V1 + 1024, F4_SLOT = F4_VONE + 1024;
constexpr int F4_LDS = F4_RING * F4_SLOT;

__device__ const uint32_t f4_ones[4] = {0x3F80u, 0u, 0u, 0u};  // bf16 {1, 0 x 7}: the ones chunks

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

__device__ __forceinline__ u32x4 f4_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  u32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) & 0xffffu;  // stride 0
  r[2] = __builtin_amdgcn_readfirstlane(bytes);                          // num_records: range check
  r[3] = 0x00020000u;
  return r;
}

// One 1 KiB LDS-DMA piece: lane l's 16 bytes at voff land at LDS byte lds + 16 l.  Inline asm:
// M0 written in the statement that reads it, and hipcc does not count it in vmcnt (f4_wait_vm).
__device__ __forceinline__ void f4_dma(u32x4 rs, uint32_t lds, uint32_t voff) {
  uint32_t keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
               "buffer_load_dwordx4 %2, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "s"(lds), "v"(voff), "s"(rs) : "memory");
}

// This wave's two pieces of every tile (waves 0-5; piece p = 2 wave + i): 0-4 = K chunk p of
// the 64 keys (lane = key), 5 = the K' ones chunk, 6-9 = V d 0..31 of keys 16 (p-6) + lane/4
// (lane % 4 = chunk), 10 = V d 32..39, 11 = the V ones chunk.
struct F4Dma {  // the issuing wave's two pieces (placements over other waves / phases measured
                // slower, profiles/r03h_flash40_dma_issuers_ab.txt, r03p_flash40_dma_interval_ab.txt)
  u32x4 rs[2];
  uint32_t voff[2];   // lane part of the byte offset (row r, column chunk), or 0 for a ones chunk
  uint32_t step[2];   // bytes per key (0 for a ones chunk)
  uint32_t row[2];    // the lane's key inside the tile
  uint32_t lds[2];    // byte offset of the piece inside a slot
};

template <int NP>
__device__ __forceinline__ void f4_issue(const F4Dma& m, uint32_t lds0, int t, int64_t skv) {
  const uint32_t key0 = (uint32_t)t * KT;
  const uint32_t slot = lds0 + (uint32_t)(t % F4_RING) * F4_SLOT;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    // data: (key0 + row) * ld + col, past skv out of range -> zeros; ones chunk: offset 0, or 16
    // (out of its 16-byte range -> zeros) for a key past skv
    const uint32_t off = m.step[i] ? m.voff[i] + key0 * m.step[i] : ((int64_t)(key0 + m.row[i]) < skv ? 0u : 16u);
    f4_dma(m.rs[i], slot + m.lds[i], off);
  }
}

// Pin a value at this point of the instruction stream: hipcc's sinking passes otherwise move
// the V phase's exp2/packs (pure register work) past the s_barrier into the M phase, next to
// the MFMAs that use them, which undoes the ping-pong.  Never pin an MFMA result: hipcc pads no
// wait states for an asm reader, and after the asm it takes the register as the asm's output, so
// the later VALU readers lose their MFMA hazard padding (a race with the still-running MFMA).
template <typename T>
__device__ __forceinline__ void f4_pin(T& x) {
  asm volatile("" : "+v"(x));
}

template <int N>
__device__ __forceinline__ void f4_wait_vm() {
  if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void f4_bar() {  // this wave's LDS reads drained, DMA left in flight
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <bool UNITC>
__device__ __forceinline__ bool f4_loop(const char* smem, uint32_t lds0, const F4Dma& dma, bool issuer,
                                        bool g0, int64_t skv, bf16x8 (&qf)[F4_QB][3], f32x16 (&oacc)[2][F4_QB],
                                        uint32_t kl0, uint32_t v0l, uint32_t v1l, int hh, float c) {
  auto bar = [&]() { f4_bar(); };
  using C = F32Cfg<40>;
  constexpr int QB = F4_QB;
  constexpr float RESCALE = 4294967296.0f;        // 2^32
  constexpr float BAD = 1.2676506002282294e30f;   // 2^100
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int qb = 0; qb < QB; ++qb)
#pragma unroll
      for (int i = 0; i < 16; ++i) oacc[db][qb][i] = 0.f;
  float mu[QB];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) mu[qb] = 0.f;
  bool bad = false;
  const int T = (int)((skv + KT - 1) / KT);  // >= 2 (launch condition)

  f32x16 s[2][QB];
  bf16x8 pf[2][2][QB];
  bf16x8 vfr[2][2][2];
  bf16x8 kfr[2][3];

  // V^T fragments of tile t (PV's A operand, key order as flash32): d-block 0 in the V phase,
  // d-block 1 at the start of the M phase (its 8 MFMAs of d-block 0 cover the latency)
  auto read_v = [&](int t, int db) {
    const uint32_t sb = (uint32_t)((t % F4_RING) * F4_SLOT);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const uint32_t R = (uint32_t)(kb * 32 + 16 * s2);
        const uint32_t a = db == 0 ? sb + v0l + R * 64 : sb + v1l + R * 16;
        const uint32_t ah = a + (db == 0 ? 512 : 128);
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((bf16x4 __attribute__((address_space(3)))*)(smem + a));
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((bf16x4 __attribute__((address_space(3)))*)(smem + ah));
        vfr[db][kb][s2] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
  };
  auto read_k = [&](int t, int kb) {  // K' fragments of tile t, key block kb: chunk 2 ks + hh
    const uint32_t sb = (uint32_t)((t % F4_RING) * F4_SLOT) + kl0 + 512 * kb;
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) kfr[kb][ks] = *(const bf16x8*)(smem + sb + 2048 * ks);
  };
  // piecewise forms of read_v(t, 1) and read_k(t, 0) (round 4): one LDS read per call, so the
  // M phase can place them between PV(d-block 0)'s MFMAs
  bf16x4 v1lo[2][2], v1hi[2][2];
  auto read_v1_piece = [&](int t, int i) {  // i = 0..7: (kb, s2, half)
    const int kb = i >> 2, s2 = (i >> 1) & 1, h = i & 1;
    const uint32_t sb = (uint32_t)((t % F4_RING) * F4_SLOT);
    const uint32_t R = (uint32_t)(kb * 32 + 16 * s2);
    const uint32_t a = sb + v1l + R * 16 + (h ? 128 : 0);
    const bf16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((bf16x4 __attribute__((address_space(3)))*)(smem + a));
    if (h) v1hi[kb][s2] = x; else v1lo[kb][s2] = x;
  };
  auto v1_join = [&]() {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x4 lo = v1lo[kb][s2], hi = v1hi[kb][s2];
        vfr[1][kb][s2] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
  };
  auto read_k0_piece = [&](int t, int ks) {
    const uint32_t sb = (uint32_t)((t % F4_RING) * F4_SLOT) + kl0;
    kfr[0][ks] = *(const bf16x8*)(smem + sb + 2048 * ks);
  };
  auto pv0_mfma = [&](int i) {  // i = 0..7: (kb, s2, qb) in pv(0)'s order
    const int kb = i >> 2, s2 = (i >> 1) & 1, qb = i & 1;
    oacc[0][qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vfr[0][kb][s2], pf[kb][s2][qb], oacc[0][qb], 0, 0, 0);
  };
  auto qk = [&](int kb) {  // S(kb) = K'.Q'^T from the fragments read_k left
#pragma unroll
    for (int ks = 0; ks < 3; ++ks)
#pragma unroll
      for (int qb = 0; qb < QB; ++qb) {
        if (ks == 0) {
          f32x16 z;
#pragma unroll
          for (int i = 0; i < 16; ++i) z[i] = 0.f;
          s[kb][qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kfr[kb][ks], qf[qb][ks], z, 0, 0, 0);
        } else {
          s[kb][qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kfr[kb][ks], qf[qb][ks], s[kb][qb], 0, 0, 0);
        }
      }
  };
  auto pv = [&](int db) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
          oacc[db][qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vfr[db][kb][s2], pf[kb][s2][qb], oacc[db][qb], 0, 0, 0);
  };
  auto rescale = [&](int qb, float nmu) {
    const float delta = nmu - mu[qb];  // exact: both bf16 values
    const float alpha = __builtin_amdgcn_exp2f(UNITC ? -delta : -delta * c);
    mu[qb] = nmu;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) s[kb][qb][i] -= delta;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int i = 0; i < 16; ++i) oacc[db][qb][i] *= alpha;
    if (hh == C::MU_H) qf[qb][C::MU_KS][C::MU_J] = (__bf16)(-nmu);
  };
  // flash32 tile_generic's decisions for tile t, taken after QK^T(t) and before softmax(t) (at the
  // start of tile t's V phase; the prologue's QK^T(0) for tile 0): the tile max on tile 0
  // (every tile on the exact pass), else the fast pass's row-sum check over tiles 0..t-1 (PV(t-1)
  // ran earlier in this phase) — the same values at the same point of the tile order as flash32
  auto decide = [&](int t) {
    if (t == 0) {
      // the tile-0 max with compiler-visible maxes (once per workgroup, so their canonicalising
      // cost does not matter): hipcc sees the MFMA results being read and inserts the hazard
      // wait states itself.  (The inline-asm v_max3 of tile_max hides that read from it; a
      // hand-counted s_nop pad before it raced the MFMAs when the schedule moved, round 3.)
      float tm[QB];
#pragma unroll
      for (int qb = 0; qb < QB; ++qb) {
        float m = s[0][qb][0];
#pragma unroll
        for (int i = 1; i < 16; ++i) m = __builtin_fmaxf(m, s[0][qb][i]);
#pragma unroll
        for (int i = 0; i < 16; ++i) m = __builtin_fmaxf(m, s[1][qb][i]);
        tm[qb] = __builtin_fmaxf(m, partner32(m));
      }
      {  // tile 0 always sets mu (flash32's t == 0 branch)
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) {
          rescale(qb, (float)(__bf16)(mu[qb] + tm[qb]));
        }
      }
    } else if (t > 1) {
      // the wave-wide any() over the lanes that hold a row sum (half L_H) is the decision; the
      // partner exchange is needed only for a rescale (round 6: -0.7 %, profiles/r06_flash40_ablations.txt)
      bool resc = false, over = false;
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
        for (int qb = 0; qb < QB; ++qb) {
          const float step = lq[qb] > RESCALE ? __builtin_amdgcn_logf(lq[qb]) : 0.f;
          rescale(qb, (float)(__bf16)(mu[qb] + (UNITC ? step : step / c)));
        }
      }
    }
  };
  auto softmax = [&]() {  // V(t): S(t) -> P(t), exp2 and bf16 packs only
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int qb = 0; qb < QB; ++qb)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          bf16x8 f;
#pragma unroll
          for (int j = 0; j < 8; ++j)
            f[j] = (__bf16)__builtin_amdgcn_exp2f(UNITC ? s[kb][qb][8 * s2 + j] : s[kb][qb][8 * s2 + j] * c);
          pf[kb][s2][qb] = f;
        }
  };
  // M(t) = PV(t) then QK^T(t+1): d-block 1's V reads and key block 0's K' reads go out first,
  // key block 1's under d-block 0's MFMAs
  auto mphase = [&](int t) {
    const bool more = t + 1 < T;
    // the M wave takes issue priority for its phase: its MFMAs go out every 32 cycles and the
    // partner's V-phase exp2/packs fill the slots between them (without it the older wave's
    // VALU stream held the issue port and the two phases ran one after the other: stamps, ~1.6k
    // cycles per M phase against 896 of MFMA)
    __builtin_amdgcn_s_setprio(1);
    // PV(d-block 0) needs nothing new (its V^T and P came from the V phase): the d-block-1 V reads
    // and key block 0's K' reads go out two per MFMA gap between its 8 MFMAs (round 4; they were
    // issued as one block before the first MFMA)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      pv0_mfma(i);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 2 * i; r < 2 * i + 2; ++r) {
        if (r < 8) read_v1_piece(t, r);
        else if (r < 11 && more) read_k0_piece(t + 1, r - 8);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    v1_join();
    if (more) read_k(t + 1, 1);
    __builtin_amdgcn_sched_barrier(0);
    pv(1);
    __builtin_amdgcn_sched_barrier(0);
    if (more) {
      qk(0);
      qk(1);
    }
    __builtin_amdgcn_s_setprio(0);
  };
  // tile u's DMA: issued at phase 2u-4 (group 0) / 2u-3 (group 1) (u >= 3), waited for at the end of phase 2u-1
  auto issue = [&](int u) {
    if (issuer && u < T) f4_issue<2>(dma, lds0, u, skv);
  };
  auto wait_tile = [&](int u) {
    if (issuer && u < T) {
      if (u + 1 < T) f4_wait_vm<2>();
      else f4_wait_vm<0>();
    }
  };
  // prologue: tiles 0 and 1 in flight, tile 0 landed everywhere
  issue(0);
  issue(1);
  wait_tile(0);
  bar();
  // one instruction stream for both groups; group 1 (waves 4-7) runs one phase behind:
  //   group 0: ph 0 [DMA 2, QK(0)] | ph 2t+1 [V(t), wait t+1] | ph 2t+2 [DMA t+3, M(t)] | ph 2T+1 []
  //   group 1: ph 0 [DMA 2] | ph 1 [QK(0), wait 1] | ph 2t+2 [V(t)] | ph 2t+3 [DMA t+3, M(t), wait t+2]
  // (round 6: group 1's DMA moved from its V phase to its M phase, like group 0's — the V phase is the
  // longer one, 609 vs 406 us of the L1 launch with the other phase's work removed; -1.6 % per launch,
  // profiles/r06_flash40_ablations.txt)
  issue(2);
  if (!g0) bar();
  read_k(0, 0);
  read_k(0, 1);
  qk(0);
  qk(1);
  decide(0);
  if (!g0) wait_tile(1);
  bar();
  for (int t = 0; t < T; ++t) {
    // tile t's decisions open its V phase (round 4; they closed the M phase that computed S(t)):
    // the same data at the same point of the tile order — after QK^T(t), before softmax(t),
    // PV(t) and QK^T(t+1) — but the M wave now reaches the barrier straight after its last MFMA
    // issue instead of waiting out the MFMA latency and the VALU checks (stamps: 268 + 116 of the
    // M phase's 2208 cycles), and the V wave has the slack (it waited 454-596 at the barrier)
    if (t > 0) decide(t);
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
  if (g0) bar();
  {  // the last tiles' row sums were not checked in the loop
    bool over = false;
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) over |= hh == C::L_H && !(oacc[C::L_DB][qb][C::L_I] < BAD);
    bad |= __any(over);
  }
  return bad;
}

// One workgroup's whole block: Q' load, DMA setup, the fast pass, the epilogue.  When a score
// jumped > ~100 (log2) past mu somewhere in the block it stores NaN flags instead, and flash32's
// exact pass (flash32_kernel<..., FIX>, launched right after) recomputes the flagged quarters —
// the exact loop inlined here as well would double the kernel's register pressure.
template <bool UNITC>
__device__ __forceinline__ bool f4_block(char* smem, const bf16_t* __restrict__ q, int64_t ldq,
                                         const bf16_t* __restrict__ k, int64_t ldk, const bf16_t* __restrict__ v,
                                         int64_t ldv, bf16_t* __restrict__ o, int64_t ldo, int heads, int64_t sq,
                                         int64_t skv, int64_t kv_div, float c, int out_f32) {
  constexpr int D = 40, QB = F4_QB;
  using C = F32Cfg<D>;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool g0 = wave < 4;
  const int r32 = lane & 31, hh = lane >> 5;
  const int nqb = (int)((sq + F4_QWG - 1) / F4_QWG);
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int qblk = lid % nqb;
  const int h = (lid / nqb) % heads;
  const int64_t b = (lid / nqb) / heads;
  const int64_t q0 = (int64_t)qblk * F4_QWG + wave * (32 * QB);
  const int64_t bkv = b / kv_div;
  const bf16_t* qb_ptr = q + b * sq * ldq + (int64_t)h * D;
  const bf16_t* kb_ptr = k + bkv * skv * ldk + (int64_t)h * D;
  const bf16_t* vb_ptr = v + bkv * skv * ldv + (int64_t)h * D;

  bf16x8 qf[QB][3];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    const int64_t qi = q0 + qb * 32 + r32;
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
      const int dd = ks * 16 + 8 * hh;
      uint4 u = make_uint4(0, 0, 0, 0);
      if (qi < sq && dd < D) u = *(const uint4*)(qb_ptr + qi * ldq + dd);
      qf[qb][ks] = __builtin_bit_cast(bf16x8, u);  // d = 40 entry starts at 0 (mu = 0)
    }
  }

  // LDS-DMA pieces (waves 0-5)
  F4Dma dma;
  // LDS-DMA issuers: waves 0-5, two pieces each
  const bool issuer = wave < 6;
  {
    const uint32_t ldkb = (uint32_t)ldk * 2, ldvb = (uint32_t)ldv * 2;
    const u32x4 rk = f4_rsrc(kb_ptr, (uint32_t)(skv - 1) * ldkb + 2 * D);
    const u32x4 rv = f4_rsrc(vb_ptr, (uint32_t)(skv - 1) * ldvb + 2 * D);
    const u32x4 r1 = f4_rsrc(f4_ones, 16);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int p = 2 * wave + i;
      uint32_t row = lane, col = 0, step = 0, lds = 0;
      u32x4 rs = r1;
      if (p < 5) {
        rs = rk; col = 16 * p; step = ldkb; lds = F4_K + 1024 * p;
      } else if (p == 5) {
        lds = F4_K + 1024 * 5;
      } else if (p < 10) {
        rs = rv; row = 16 * (p - 6) + (lane >> 2); col = 16 * (lane & 3); step = ldvb; lds = F4_V0 + 1024 * (p - 6);
      } else if (p == 10) {
        rs = rv; col = 64; step = ldvb; lds = F4_V1;
      } else {
        lds = F4_VONE;
      }
      dma.rs[i] = rs; dma.row[i] = row; dma.step[i] = step; dma.lds[i] = lds;
      dma.voff[i] = row * step + col;
    }
  }
  // per-lane LDS read offsets (inside a slot)
  const uint32_t kl0 = F4_K + hh * 1024 + r32 * 16;   // + 2048 ks + 512 kb: chunk 2 ks + hh
  const int g16 = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
  const uint32_t v0l = F4_V0 + (uint32_t)(((4 * hh + qq) * 32 + 16 * (g16 & 1) + 4 * pp) * 2);
  // d-block 1 (d 32..63): columns 32..39 from V d 32..39, column 40 = the ones chunk's 1, the
  // rest its zero half
  const uint32_t v1l = ((g16 & 1) == 0 && pp < 2 ? F4_V1 + 8 * pp : F4_VONE + ((g16 & 1) == 0 && pp == 2 ? 0 : 8)) +
                       (uint32_t)((4 * hh + qq) * 16);

  f32x16 oacc[2][QB];
  if (__syncthreads_or(f4_loop<UNITC>(smem, lds0, dma, issuer, g0, skv, qf, oacc, kl0, v0l, v1l, hh, c))) {
    // a score jumped > ~100 (log2) past mu somewhere in the block: no output here; a NaN in
    // element (first query, d 0) of each 256-query quarter tells flash32's exact fix-up pass,
    // launched right after, to recompute that quarter
    if (tid == 0)
      for (int64_t qs = (int64_t)qblk * F4_QWG; qs < (int64_t)(qblk + 1) * F4_QWG && qs < sq; qs += 256) {
        if (out_f32) ((float*)o)[(b * sq + qs) * ldo + (int64_t)h * D] = __builtin_nanf("");
        else o[(b * sq + qs) * ldo + (int64_t)h * D] = 0x7FC0;
      }
    return true;
  }

  // epilogue as flash32: O[q][d] = O^T[d][q] / l
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    const float lown = oacc[C::L_DB][qb][C::L_I];
    const float lp = partner32(lown);
    const float l = hh == C::L_H ? lown : lp;
    const float inv = __builtin_amdgcn_rcpf(l);
    const int64_t qi = q0 + qb * 32 + r32;
    if (out_f32) {
      float* frow = (float*)o + (b * sq + qi) * ldo + (int64_t)h * D;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d0 = 32 * db + 8 * g + 4 * hh;
          const f32x16& a = oacc[db][qb];
          if (qi < sq && d0 + 4 <= D)
            *(float4*)(frow + d0) = make_float4(a[4 * g] * inv, a[4 * g + 1] * inv, a[4 * g + 2] * inv, a[4 * g + 3] * inv);
        }
      continue;
    }
    bf16_t* orow = o + (b * sq + (qi < sq ? qi : 0)) * ldo + (int64_t)h * D;
#pragma unroll
    for (int db = 0; db < 2; ++db) {
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const f32x16& a = oacc[db][qb];
        uint32_t x0 = pack2(a[8 * m + 0] * inv, a[8 * m + 1] * inv), x1 = pack2(a[8 * m + 2] * inv, a[8 * m + 3] * inv);
        uint32_t y0 = pack2(a[8 * m + 4] * inv, a[8 * m + 5] * inv), y1 = pack2(a[8 * m + 6] * inv, a[8 * m + 7] * inv);
        auto s0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
        auto s1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
        const int dd = 32 * db + 16 * m + 8 * hh;
        if (qi < sq && dd + 8 <= D) *(uint4*)(orow + dd) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
      }
    }
  }
  return false;
}

template <bool UNITC>
__global__ __launch_bounds__(F4_NT, 1) void flash40_kernel(
    const bf16_t* __restrict__ q, int64_t ldq, const bf16_t* __restrict__ k, int64_t ldk,
    const bf16_t* __restrict__ v, int64_t ldv, bf16_t* __restrict__ o, int64_t ldo, int heads,
    int64_t sq, int64_t skv, int64_t kv_div, float c, int out_f32) {
  __shared__ __attribute__((aligned(1024))) char smem[F4_LDS];
  f4_block<UNITC>(smem, q, ldq, k, ldk, v, ldv, o, ldo, heads, sq, skv, kv_div, c, out_f32);
}

// ============================================================ flash80
// The d = 80 spatial self-attention (SD-1.5 level 2: S = 1024, 8 heads) on flash40's schedule
// (round 6): 8 waves in two groups one barrier apart, per 64-key tile V(t) = the softmax of S(t)
// (VALU) and M(t) = PV(t) then QK^T(t+1) (24 x 32x32x16: 12 + 12), K/V by LDS-DMA into a 4-slot ring
// issued three tiles ahead.  One 32-query block per wave (256 queries per workgroup): d = 80's
// fragments (Q' 6 k-steps, K' 12 per tile, V^T 12) leave no room for a second.  QK^T's contraction is
// padded 81 -> 96 (K' chunk 10 = the -mu column's ones, chunk 11 zeros), PV's rows 81 -> 96 (d-block 2
// = V d 64..79 | the ones column | zeros): 20 of every 24 MFMAs are algorithmic, against flash40's
// 20 of 28, so the tile is matrix-bound where flash40's is issue-bound.
// Softmax: flash32's exact deferred max, without its per-score maxes on the MFMA results — the
// decision reads P = exp2(S) (VALU results: plain v_max3, no canonicalising maxes): a row whose P
// passes 2^THR (a score THR past mu) raises mu to the bf16 of its exact tile max (taken, with P, in
// that rare branch), O and the row sum rescale, P is recomputed.  So P <= 2^THR always: no
// overflow, no flags, no fix-up launch (flash40 needs flash32's exact pass; d = 80 has none).
// Row sum = V's ones column (d = 80: d-block 2, accumulator row 16 = register 8 of lanes 0-31).
constexpr int F8K_QWG = F4_NW * 32;                     // queries per workgroup
constexpr int F8K_K = 0, F8K_VA = 12 * 1024, F8K_VB = F8K_VA + 4096, F8K_VC0 = F8K_VB + 4096,
              F8K_VC1 = F8K_VC0 + 1024, F8K_VONE = F8K_VC1 + 1024, F8K_SLOT = F8K_VONE + 1024;
constexpr int F8K_LDS = F4_RING * F8K_SLOT;             // 92 KiB
constexpr int F8K_NP = 3;                               // LDS-DMA pieces per wave and tile (wave 7: 2)

struct F80Dma {  // this wave's pieces of every tile (piece p = 3 wave + i, see f80_dma_setup)
  u32x4 rs[F8K_NP];
  uint32_t voff[F8K_NP], step[F8K_NP], row[F8K_NP], lds[F8K_NP];
};

// pieces per tile (23): 0-9 = K chunk p (d 8p .. 8p + 7) of the 64 keys (lane = key), 10 = K' ones chunk
// (the -mu column), 11 = K' zero chunk (d 88..95: the constant read past its 16 bytes), 12-15 = V
// d 0..31 of keys 16 (p - 12) + lane / 4 (lane % 4 = chunk), 16-19 = V d 32..63 likewise, 20 / 21 =
// V d 64..71 / 72..79 (lane = key), 22 = V's ones chunk.  Keys past skv read zeros (range check).
__device__ __forceinline__ void f80_dma_setup(F80Dma& dma, int wave, int lane, const bf16_t* kb_ptr, int64_t ldk,
                                              const bf16_t* vb_ptr, int64_t ldv, int64_t skv) {
  constexpr int D = 80;
  const uint32_t ldkb = (uint32_t)ldk * 2, ldvb = (uint32_t)ldv * 2;
  const u32x4 rk = f4_rsrc(kb_ptr, (uint32_t)(skv - 1) * ldkb + 2 * D);
  const u32x4 rv = f4_rsrc(vb_ptr, (uint32_t)(skv - 1) * ldvb + 2 * D);
  const u32x4 r1 = f4_rsrc(f4_ones, 16);
#pragma unroll
  for (int i = 0; i < F8K_NP; ++i) {
    const int p = F8K_NP * wave + i;
    uint32_t row = lane, col = 0, step = 0, lds = 0;
    u32x4 rs = r1;
    if (p < 10) {
      rs = rk; col = 16 * p; step = ldkb; lds = F8K_K + 1024 * p;
    } else if (p == 10) {
      lds = F8K_K + 1024 * 10;
    } else if (p == 11) {
      row = 1u << 30; lds = F8K_K + 1024 * 11;  // never a valid key: the zero half of the constant's range
    } else if (p < 20) {
      const int q = p < 16 ? p - 12 : p - 16;
      rs = rv; row = 16 * q + (lane >> 2); col = (p < 16 ? 0 : 64) + 16 * (lane & 3); step = ldvb;
      lds = (p < 16 ? F8K_VA : F8K_VB) + 1024 * q;
    } else if (p < 22) {
      rs = rv; col = p == 20 ? 128 : 144; step = ldvb; lds = p == 20 ? F8K_VC0 : F8K_VC1;
    } else {
      lds = F8K_VONE;
    }
    dma.rs[i] = rs; dma.row[i] = row; dma.step[i] = step; dma.lds[i] = lds;
    dma.voff[i] = step ? row * step + col : 0u;
  }
}

template <int NP>
__device__ __forceinline__ void f80_issue(const F80Dma& m, uint32_t lds0, int t, int64_t skv) {
  const uint32_t key0 = (uint32_t)t * KT;
  const uint32_t slot = lds0 + (uint32_t)(t % F4_RING) * F8K_SLOT;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const uint32_t off = m.step[i] ? m.voff[i] + key0 * m.step[i] : ((int64_t)(key0 + m.row[i]) < skv ? 0u : 16u);
    f4_dma(m.rs[i], slot + m.lds[i], off);
  }
}

template <bool UNITC>
__device__ __forceinline__ void f80_loop(const char* smem, uint32_t lds0, const F80Dma& dma, int wave, bool g0,
                                         int64_t skv, bf16x8 (&qf)[6], f32x16 (&oacc)[3], uint32_t kl0,
                                         uint32_t vl0, uint32_t vl2, int hh, float c) {
  constexpr int MU_KS = 5, MU_H = 0, MU_J = 0;  // d = 80 in the Q' fragments
#pragma unroll
  for (int db = 0; db < 3; ++db)
#pragma unroll
    for (int i = 0; i < 16; ++i) oacc[db][i] = 0.f;
  float mu = 0.f;
  const int T = (int)((skv + KT - 1) / KT);  // >= 4 (launch condition)
  constexpr float PTHR = 64.0f;  // 2^F32_THR: a P above it = a score THR past mu

  f32x16 s[2];
  bf16x8 pf[2][2];
  bf16x8 vfr[3][2][2];
  bf16x8 kfr[2][6];

  auto tr = [&](uint32_t a) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((bf16x4 __attribute__((address_space(3)))*)(smem + a));
  };
  // V^T fragment (d-block db, key block kb, k-step s2) of tile t: flash32's key order, lo keys
  // 16 s2 + 4 hh + 0..3, hi + 8; d-blocks 0-1 from the 64-B rows of V d 0..31 / 32..63, d-block 2
  // from the 16-B rows of V d 64..71 / 72..79 / the ones chunk
  auto read_v = [&](int t, int db, int kb, int s2) {
    const uint32_t sb = (uint32_t)((t % F4_RING) * F8K_SLOT);
    const uint32_t R = (uint32_t)(kb * 32 + 16 * s2);
    const uint32_t a = db < 2 ? sb + vl0 + (db == 1 ? 4096u : 0u) + R * 64 : sb + vl2 + R * 16;
    const uint32_t ah = a + (db < 2 ? 512 : 128);
    const bf16x4 lo = tr(a), hi = tr(ah);
    vfr[db][kb][s2] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  auto read_k = [&](int t, int kb, int ks) {
    kfr[kb][ks] = *(const bf16x8*)(smem + (t % F4_RING) * F8K_SLOT + kl0 + 512 * kb + 2048 * ks);
  };
  auto qk = [&](int kb) {
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) {
      if (ks == 0) {
        f32x16 z;
#pragma unroll
        for (int i = 0; i < 16; ++i) z[i] = 0.f;
        s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kfr[kb][ks], qf[ks], z, 0, 0, 0);
      } else {
        s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kfr[kb][ks], qf[ks], s[kb], 0, 0, 0);
      }
    }
  };
  auto pv = [&](int db, int kb, int s2) {
    oacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vfr[db][kb][s2], pf[kb][s2], oacc[db], 0, 0, 0);
  };
  f32x16 pe[2];       // P = exp2(S), fp32
  auto exps = [&]() {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) pe[kb][i] = __builtin_amdgcn_exp2f(UNITC ? s[kb][i] : s[kb][i] * c);
  };
  // V(t): P = exp2(S(t)); a row whose P passes 2^THR (or the first tile) moves mu to the bf16 of its
  // exact tile max and P is recomputed; then the bf16 packs.  The maxes over P are compiler-visible
  // (VALU results: hipcc adds no canonicalising max and pads the exp -> max hazards itself)
  auto vphase = [&](int t) {
    exps();
    float pm0 = pe[0][0], pm1 = pe[1][0];
#pragma unroll
    for (int i = 1; i < 16; ++i) {
      pm0 = __builtin_fmaxf(pm0, pe[0][i]);
      pm1 = __builtin_fmaxf(pm1, pe[1][i]);
    }
    const float pm = __builtin_fmaxf(pm0, pm1);
    if (t == 0 || __any(!(pm <= PTHR))) {  // wave-uniform; !(<=): an inf / NaN P takes the branch too
      float tm = s[0][0];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) tm = __builtin_fmaxf(tm, s[kb][i]);
      tm = __builtin_fmaxf(tm, partner32(tm));
      const float tmc = UNITC ? tm : tm * c;
      const bool up = t == 0 || tmc > F32_THR;
      const float nmu = up ? (float)(__bf16)(mu + tm) : mu;
      const float delta = nmu - mu;  // exact: both bf16 values
      const float alpha = __builtin_amdgcn_exp2f(UNITC ? -delta : -delta * c);
      mu = nmu;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) s[kb][i] -= delta;
#pragma unroll
      for (int db = 0; db < 3; ++db)
#pragma unroll
        for (int i = 0; i < 16; ++i) oacc[db][i] *= alpha;
      if (hh == MU_H) qf[MU_KS][MU_J] = (__bf16)(-nmu);
      exps();
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 f;
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = (__bf16)pe[kb][8 * s2 + j];
        pf[kb][s2] = f;
      }
  };
  // M(t) = PV(t) (d-blocks 0, 1, 2) then QK^T(t+1); the next d-block's V^T reads and then K'(t+1)'s
  // reads go out between the MFMAs
  auto mphase = [&](int t) {
    const bool more = t + 1 < T;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int db = 0; db < 3; ++db) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pv(db, i >> 1, i & 1);
        __builtin_amdgcn_sched_barrier(0);
        if (db < 2) {
          read_v(t, db + 1, i >> 1, i & 1);
        } else if (more) {
          read_k(t + 1, 0, i);
          if (i < 2) read_k(t + 1, 0, 4 + i);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (more) {
#pragma unroll
      for (int ks = 0; ks < 6; ++ks) read_k(t + 1, 1, ks);
      __builtin_amdgcn_sched_barrier(0);
      qk(0);
      qk(1);
    }
    __builtin_amdgcn_s_setprio(0);
  };
  const bool issuer7 = wave == 7;  // wave 7 moves two pieces (21, 22), the others three
  auto issue = [&](int u) {
    if (u < T) {
      if (issuer7) f80_issue<2>(dma, lds0, u, skv);
      else f80_issue<3>(dma, lds0, u, skv);
    }
  };
  auto wait_tile = [&](int u) {
    if (u < T) {
      if (u + 1 < T) {
        if (issuer7) f4_wait_vm<2>();
        else f4_wait_vm<3>();
      } else {
        f4_wait_vm<0>();
      }
    }
  };
  auto bar = [&]() { f4_bar(); };
  // flash40's prologue and phase order
  issue(0);
  issue(1);
  wait_tile(0);
  bar();
  issue(2);
  if (!g0) bar();
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) read_k(0, kb, ks);
  qk(0);
  qk(1);
  if (!g0) wait_tile(1);
  bar();
  for (int t = 0; t < T; ++t) {
    // group 1 issues its pieces of tile t + 3 at the head of its V phase, group 0 in its M phase (group 0's
    // V(t) runs beside group 1's M(t - 1), which still reads the slot tile t + 3 takes): -2.6 % against
    // both in M (profiles/r06_flash80.txt)
    if (!g0) issue(t + 3);
    vphase(t);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) read_v(t, 0, kb, s2);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        f4_pin(vfr[0][kb][s2]);
        f4_pin(pf[kb][s2]);
      }
    if (g0) wait_tile(t + 1);
    bar();
    if (g0) issue(t + 3);
    mphase(t);
    if (!g0) wait_tile(t + 2);
    bar();
  }
  if (g0) bar();
}

template <bool UNITC>
__global__ __launch_bounds__(F4_NT, 1) void flash80_kernel(
    const bf16_t* __restrict__ q, int64_t ldq, const bf16_t* __restrict__ k, int64_t ldk,
    const bf16_t* __restrict__ v, int64_t ldv, bf16_t* __restrict__ o, int64_t ldo, int heads,
    int64_t sq, int64_t skv, int64_t kv_div, float c, int out_f32) {
  __shared__ __attribute__((aligned(1024))) char smem[F8K_LDS];
  constexpr int D = 80;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool g0 = wave < 4;
  const int r32 = lane & 31, hh = lane >> 5;
  const int nqb = (int)((sq + F8K_QWG - 1) / F8K_QWG);
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int qblk = lid % nqb;
  const int h = (lid / nqb) % heads;
  const int64_t b = (lid / nqb) / heads;
  const int64_t q0 = (int64_t)qblk * F8K_QWG + wave * 32;
  const int64_t bkv = b / kv_div;
  const bf16_t* qb_ptr = q + b * sq * ldq + (int64_t)h * D;

  bf16x8 qf[6];  // Q'^T (B operand): k-step ks, lane half hh = d 16 ks + 8 hh .. +7; d = 80 (-mu) starts at 0
  {
    const int64_t qi = q0 + r32;
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) {
      const int dd = ks * 16 + 8 * hh;
      uint4 u = make_uint4(0, 0, 0, 0);
      if (qi < sq && dd < D) u = *(const uint4*)(qb_ptr + qi * ldq + dd);
      qf[ks] = __builtin_bit_cast(bf16x8, u);
    }
  }
  F80Dma dma;
  f80_dma_setup(dma, wave, lane, k + bkv * skv * ldk + (int64_t)h * D, ldk, v + bkv * skv * ldv + (int64_t)h * D,
                ldv, skv);
  const uint32_t kl0 = F8K_K + hh * 1024 + r32 * 16;  // + 2048 ks + 512 kb: chunk 2 ks + hh, key 32 kb + r32
  const int g16 = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
  const uint32_t vl0 = F8K_VA + (uint32_t)(((4 * hh + qq) * 32 + 16 * (g16 & 1) + 4 * pp) * 2);
  // d-block 2: columns 64..79 (lanes of the even 16-lane groups) from V d 64..71 / 72..79, column 80
  // = the ones chunk's 1, the rest its zero half
  const uint32_t vl2 = ((g16 & 1) == 0 ? (pp < 2 ? F8K_VC0 + 8 * pp : F8K_VC1 + 8 * (pp - 2))
                                       : F8K_VONE + (pp == 0 ? 0 : 8)) +
                       (uint32_t)((4 * hh + qq) * 16);

  f32x16 oacc[3];
  f80_loop<UNITC>(smem, lds0, dma, wave, g0, skv, qf, oacc, kl0, vl0, vl2, hh, c);

  // epilogue: O[q][d] = O^T[d][q] / l, the row sum in d-block 2, register 8 of lanes 0-31
  const float lown = oacc[2][8];
  const float lp = partner32(lown);
  const float l = hh == 0 ? lown : lp;
  const float inv = __builtin_amdgcn_rcpf(l);
  const int64_t qi = q0 + r32;
  if (out_f32) {
    if (qi >= sq) return;
    float* frow = (float*)o + (b * sq + qi) * ldo + (int64_t)h * D;
#pragma unroll
    for (int db = 0; db < 3; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d0 = 32 * db + 8 * g + 4 * hh;
        const f32x16& a = oacc[db];
        if (d0 + 4 <= D)
          *(float4*)(frow + d0) = make_float4(a[4 * g] * inv, a[4 * g + 1] * inv, a[4 * g + 2] * inv, a[4 * g + 3] * inv);
      }
    return;
  }
  bf16_t* orow = o + (b * sq + (qi < sq ? qi : 0)) * ldo + (int64_t)h * D;  // every lane takes part in the swaps
#pragma unroll
  for (int db = 0; db < 3; ++db) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const f32x16& a = oacc[db];
      uint32_t x0 = pack2(a[8 * m + 0] * inv, a[8 * m + 1] * inv), x1 = pack2(a[8 * m + 2] * inv, a[8 * m + 3] * inv);
      uint32_t y0 = pack2(a[8 * m + 4] * inv, a[8 * m + 5] * inv), y1 = pack2(a[8 * m + 6] * inv, a[8 * m + 7] * inv);
      auto s0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
      auto s1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
      const int dd = 32 * db + 16 * m + 8 * hh;
      if (qi < sq && dd + 8 <= D) *(uint4*)(orow + dd) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
    }
  }
}

// kernel (per call, test hook; 0 everywhere in the product): 0 = automatic — d = 40: flash40 from
// 4 key tiles, flash32 below (and for its text cross-attention), other d: flash_attn_kernel;
// 1 = flash_attn_kernel (16x16x32) for any d; 2 = flash32 (d = 40); 3 = flash40 wherever it
// applies (d = 40, >= 2 key tiles).  A kernel that does not take the shape falls through to
// the next one down.
template <int D>
int launch_flash(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                 void* o, int64_t ldo, int64_t batch, int heads, int64_t sq, int64_t skv,
                 int64_t kv_div, float scale, hipStream_t s, int out_f32, int kernel) {
  const float c = scale * 1.4426950408889634f;
  if constexpr (D == 40) {
    const bool oal = ((uintptr_t)o & 15) == 0 && ldo % (out_f32 ? 4 : 8) == 0;
    // flash40 (ping-pong, LDS-DMA ring): the default for the long self-attention
    if ((kernel == 3 || (kernel == 0 && skv >= 256)) && skv >= 2 * KT && oal) {
      const int64_t nblk = (sq + F4_QWG - 1) / F4_QWG * heads * batch;
      if (nblk > 0x7fffffff) return VD_EINVAL;
      const dim3 grid((unsigned)nblk);
      const int64_t nfix = (sq + 127) / 128 * heads * batch;  // 128-query blocks of the exact pass (QB = 1)
      const dim3 fix((unsigned)((nfix + F32_FIXW - 1) / F32_FIXW));
      if (c == 1.0f) {
        hipLaunchKernelGGL((flash40_kernel<true>), grid, dim3(F4_NT), 0, s, (const bf16_t*)q, ldq, (const bf16_t*)k,
                           ldk, (const bf16_t*)v, ldv, (bf16_t*)o, ldo, heads, sq, skv, kv_div, c, out_f32);
        hipLaunchKernelGGL((flash32_kernel<D, true, true, 1>), fix, dim3(NT), 0, s, (const bf16_t*)q, ldq,
                           (const bf16_t*)k, ldk, (const bf16_t*)v, ldv, (bf16_t*)o, ldo, heads, sq, skv, kv_div, c, out_f32,
                           nfix);
      } else {
        hipLaunchKernelGGL((flash40_kernel<false>), grid, dim3(F4_NT), 0, s, (const bf16_t*)q, ldq, (const bf16_t*)k,
                           ldk, (const bf16_t*)v, ldv, (bf16_t*)o, ldo, heads, sq, skv, kv_div, c, out_f32);
        hipLaunchKernelGGL((flash32_kernel<D, false, true, 1>), fix, dim3(NT), 0, s, (const bf16_t*)q, ldq,
                           (const bf16_t*)k, ldk, (const bf16_t*)v, ldv, (bf16_t*)o, ldo, heads, sq, skv, kv_div, c, out_f32,
                           nfix);
      }
      return vd_launch_status();
    }
    if (kernel != 1 && oal) {  // flash32
      const int64_t nblk = (sq + 255) / 256 * heads * batch;
      if (nblk > 0x7fffffff) return VD_EINVAL;
      const dim3 grid((unsigned)nblk);
      if (c == 1.0f)
        hipLaunchKernelGGL((flash32_kernel<D, true>), grid, dim3(NT), 0, s, (const bf16_t*)q, ldq,
                           (const bf16_t*)k, ldk, (const bf16_t*)v, ldv, (bf16_t*)o, ldo, heads, sq, skv, kv_div, c, out_f32);
      else
        hipLaunchKernelGGL((flash32_kernel<D, false>), grid, dim3(NT), 0, s, (const bf16_t*)q, ldq,
                           (const bf16_t*)k, ldk, (const bf16_t*)v, ldv, (bf16_t*)o, ldo, heads, sq, skv, kv_div, c, out_f32);
      return vd_launch_status();
    }
  }
  // (QBLK 4 only for D <= 40: wider heads' QBLK-4 instances spill 94-280 VGPRs, so they are
  // not instantiated at all)
  if constexpr (D == 80) {
    // flash80 (round 6): the level-2 self-attention, from 4 key tiles (kernel 3 forces it from 2)
    const bool oal = ((uintptr_t)o & 15) == 0 && ldo % (out_f32 ? 4 : 8) == 0;
    if ((kernel == 3 || (kernel == 0 && skv >= 4 * KT)) && skv >= 2 * KT && oal) {
      const int64_t nblk = (sq + F8K_QWG - 1) / F8K_QWG * heads * batch;
      if (nblk > 0x7fffffff) return VD_EINVAL;
      if (c == 1.0f)
        hipLaunchKernelGGL((flash80_kernel<true>), dim3((unsigned)nblk), dim3(F4_NT), 0, s, (const bf16_t*)q, ldq,
                           (const bf16_t*)k, ldk, (const bf16_t*)v, ldv, (bf16_t*)o, ldo, heads, sq, skv, kv_div, c,
                           out_f32);
      else
        hipLaunchKernelGGL((flash80_kernel<false>), dim3((unsigned)nblk), dim3(F4_NT), 0, s, (const bf16_t*)q, ldq,
                           (const bf16_t*)k, ldk, (const bf16_t*)v, ldv, (bf16_t*)o, ldo, heads, sq, skv, kv_div, c,
                           out_f32);
      return vd_launch_status();
    }
  }
  if constexpr (D <= 40) {
    if (sq >= 1024) {
      const dim3 grid((unsigned)((sq + 255) / 256), (unsigned)heads, (unsigned)batch);
      hipLaunchKernelGGL((flash_attn_kernel<D, 4>), grid, dim3(NT), 0, s, (const bf16_t*)q, ldq,
                         (const bf16_t*)k, ldk, (const bf16_t*)v, ldv, (bf16_t*)o, ldo, heads, sq, skv,
                         kv_div, c, out_f32);
      return vd_launch_status();
    }
  }
  {
    const dim3 grid((unsigned)((sq + 127) / 128), (unsigned)heads, (unsigned)batch);
    hipLaunchKernelGGL((flash_attn_kernel<D, 2>), grid, dim3(NT), 0, s, (const bf16_t*)q, ldq,
                       (const bf16_t*)k, ldk, (const bf16_t*)v, ldv, (bf16_t*)o, ldo, heads, sq, skv,
                       kv_div, c, out_f32);
  }
  return vd_launch_status();
}

// ---------------------------------------------------------------- temporal
// One wave per (b, p, h) item; lane = (query f = lane / LPQ, part = lane % LPQ);
// 16-byte dim chunks c of the head are owned by part c % LPQ.
template <int FMAX>
__global__ __launch_bounds__(NT) void temporal_attn_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    int64_t ld, bf16_t* __restrict__ o, int64_t ldo, int64_t batch, int frames, int64_t positions,
    int heads, int d, float scale_log2) {
  constexpr int LPQ = 64 / FMAX;
  __shared__ __attribute__((aligned(16))) bf16_t kv_lds[4][2][FMAX * 160];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t item = (int64_t)blockIdx.x * 4 + wave;
  const int64_t nitems = batch * positions * heads;
  if (item >= nitems) return;
  const int h = (int)(item % heads);
  const int64_t bp = item / heads;
  const int64_t p = bp % positions, b = bp / positions;
  const int nch = d / 8;
  bf16_t* kl = kv_lds[wave][0];
  bf16_t* vl = kv_lds[wave][1];
  // stage K, V of this item: frames x d
  for (int idx = lane; idx < frames * nch; idx += 64) {
    const int f = idx / nch, c = idx - f * nch;
    const int64_t row = (b * frames + f) * positions + p;
    *(uint4*)(kl + f * d + c * 8) = *(const uint4*)(k + row * ld + (int64_t)h * d + c * 8);
    *(uint4*)(vl + f * d + c * 8) = *(const uint4*)(v + row * ld + (int64_t)h * d + c * 8);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  const int fq = lane / LPQ, part = lane % LPQ;
  const bool qvalid = fq < frames;
  const int64_t qrow = (b * frames + (qvalid ? fq : 0)) * positions + p;
  constexpr int MAXC = (20 + LPQ - 1) / LPQ;  // chunks per lane (d <= 160)
  float qv[MAXC][8];
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = part + i * LPQ;
    if (c < nch) unpack8(*(const uint4*)(q + qrow * ld + (int64_t)h * d + c * 8), qv[i]);
  }
  float sc[FMAX];
#pragma unroll
  for (int kk = 0; kk < FMAX; ++kk) {
    float acc = 0.f;
    if (kk < frames) {
#pragma unroll
      for (int i = 0; i < MAXC; ++i) {
        const int c = part + i * LPQ;
        if (c < nch) {
          float kf[8];
          unpack8(*(const uint4*)(kl + kk * d + c * 8), kf);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc = fmaf(qv[i][e], kf[e], acc);
        }
      }
    }
#pragma unroll
    for (int off = 1; off < LPQ; off <<= 1) acc += __shfl_xor(acc, off, 64);
    sc[kk] = kk < frames ? acc * scale_log2 : -INFINITY;
  }
  float mx = -INFINITY;
#pragma unroll
  for (int kk = 0; kk < FMAX; ++kk) mx = fmaxf(mx, sc[kk]);
  float sum = 0.f;
#pragma unroll
  for (int kk = 0; kk < FMAX; ++kk) {
    sc[kk] = exp2f(sc[kk] - mx);
    sum += sc[kk];
  }
  const float inv = 1.0f / sum;
  if (!qvalid) return;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = part + i * LPQ;
    if (c < nch) {
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int kk = 0; kk < FMAX; ++kk) {
        if (kk < frames) {
          float vf[8];
          unpack8(*(const uint4*)(vl + kk * d + c * 8), vf);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] = fmaf(sc[kk], vf[e], acc[e]);
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] *= inv;
      *(uint4*)(o + qrow * ldo + (int64_t)h * d + c * 8) = pack8(acc);
    }
  }
}

// ------------------------------------------------------- temporal (MFMA)
// frames <= 16: one (b, p, h) item per wave iteration on v_mfma_f32_16x16x32_bf16.
//   S^T[key][q] = K . Q^T   A = K rows, B = Q^T, both straight from the NHWC rows
//                           (lane (fr, fq) holds row fr, dims 32*ks + 8*fq .. +7);
//   softmax over the 16 keys of query fr: 4 keys per lane, two xor-shuffles;
//   O^T[d][q] = V^T . P^T   P^T's k-slot (fq, j) is key 4*fq + j for j < 4 and an
//                           empty slot (P = 0) for j >= 4, so the S^T accumulator
//                           IS the B operand (no lane movement); V^T comes from a
//                           per-wave LDS image with ds_read_b64_tr_b16 (T10), whose
//                           column D is 1.0: row D of O^T is the softmax row sum.
// Memory-bound (3 reads + 1 write of the head's 16 rows); 4 waves per block,
// items strided over the grid so the LDS padding is written once per wave.
template <int D>
struct TmCfg {
  static constexpr int KSTEPS = (D + 31) / 32;
  static constexpr int DB = (D + 1 + 15) / 16;   // O^T row blocks incl. the ones row
  static constexpr int VS = 16 * (DB | 1);       // LDS row (elements): 32 B x odd -> conflict-free tr reads
  static constexpr int DCH = D / 8;
};

// Query and key frames may differ (vd_temporal_attention_kv: a frame-sharded rank's own
// qframes queries against all kframes keys gathered from every rank, SURVEY §8e's K/V
// all-gather); q/o rows are (b, qframes, p) at stride ldq/ldo, k/v rows (b, kframes, p) at
// stride ldkv.  The self-attention call passes qframes == kframes and one stride.
template <int D>
__global__ __launch_bounds__(NT) void temporal_mfma_kernel(
    const bf16_t* __restrict__ q, int64_t ldq, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    int64_t ldkv, bf16_t* __restrict__ o, int64_t ldo, int64_t batch, int qframes, int frames, int64_t positions,
    int heads, float c) {
  using C = TmCfg<D>;
  __shared__ __attribute__((aligned(16))) bf16_t vimg[4][16 * C::VS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  bf16_t* vl = vimg[wave];
  // padding columns [D, VS) of every row: 1.0 at column D, 0 elsewhere (never overwritten);
  // rows >= frames stay zero (their P is 0)
  for (int idx = lane; idx < 16 * C::VS / 8; idx += 64) *(uint4*)(vl + idx * 8) = make_uint4(0, 0, 0, 0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane < 16) vl[lane * C::VS + D] = (bf16_t)0x3F80;
  const int64_t nitems = batch * positions * heads;
  const int64_t stride = (int64_t)gridDim.x * 4;
  const bool unitc = c == 1.0f;
  const int vtr = (4 * fq + (fr >> 2)) * C::VS + 4 * (fr & 3);  // tr-read lane offset in a column block
  // XCD-aware (T1): the blocks holding the other heads of the same position (whose 80-byte
  // head slices share 128-byte lines of the Q/K/V/O rows) get adjacent logical ids, which
  // xcd_remap keeps on one XCD, so a shared line is fetched into one L2, not two
  const int64_t lblk = xcd_remap(blockIdx.x, gridDim.x);
  // Software-pipelined (round 2): the K/Q fragments and V chunks of the wave's NEXT item are
  // loaded into registers while the current item computes, so a wave keeps one item of loads
  // in flight behind its MFMAs, softmax and stores (the kernel is memory-latency bound: 3.3
  // TB/s at L1 with one item's loads outstanding at a time).
  constexpr int VN = (16 * C::DCH + 63) / 64;  // V chunks per lane (frames <= 16)
  const bool fok = fr < frames, qok = fr < qframes;
  uint4 kn[C::KSTEPS], qn[C::KSTEPS], vn[VN];
  // (a macro, not a lambda: a lambda capturing the register arrays by reference left them on
  // the scratch stack)
#define TM_LOAD_ITEM(IT)                                                                              \
  {                                                                                                   \
    const int h_ = (int)((IT) % heads);                                                              \
    const int64_t bp_ = (IT) / heads;                                                                 \
    const int64_t p_ = bp_ % positions, b_ = bp_ / positions;                                         \
    const int64_t row0_ = b_ * frames * positions + p_;                                               \
    const int64_t rf_ = (row0_ + (fok ? fr : 0) * positions) * ldkv + (int64_t)h_ * D;                \
    const int64_t rq_ = ((b_ * qframes * positions + p_) + (qok ? fr : 0) * positions) * ldq + (int64_t)h_ * D; \
    _Pragma("unroll") for (int ks = 0; ks < C::KSTEPS; ++ks) {                                        \
      const int dd = ks * 32 + 8 * fq;                                                                \
      kn[ks] = make_uint4(0, 0, 0, 0);                                                                \
      qn[ks] = make_uint4(0, 0, 0, 0);                                                                \
      if (dd < D) {                                                                                   \
        if (fok) kn[ks] = *(const uint4*)(k + rf_ + dd);                                              \
        if (qok) qn[ks] = *(const uint4*)(q + rq_ + dd);                                              \
      }                                                                                               \
    }                                                                                                 \
    _Pragma("unroll") for (int r = 0; r < VN; ++r) {                                                  \
      const int idx = lane + 64 * r;                                                                  \
      const int f = idx / C::DCH, cc = idx - f * C::DCH;                                              \
      vn[r] = make_uint4(0, 0, 0, 0);                                                                 \
      if (idx < frames * C::DCH)                                                                      \
        vn[r] = *(const uint4*)(v + (row0_ + (int64_t)f * positions) * ldkv + (int64_t)h_ * D + cc * 8); \
    }                                                                                                 \
  }
  int64_t item = lblk * 4 + wave;
  if (item < nitems) TM_LOAD_ITEM(item)
  for (; item < nitems; item += stride) {
    uint4 kc[C::KSTEPS], qc[C::KSTEPS], vc[VN];
#pragma unroll
    for (int ks = 0; ks < C::KSTEPS; ++ks) {
      kc[ks] = kn[ks];
      qc[ks] = qn[ks];
    }
#pragma unroll
    for (int r = 0; r < VN; ++r) vc[r] = vn[r];
    const int h = (int)(item % heads);
    const int64_t bp = item / heads;
    const int64_t p = bp % positions, b = bp / positions;
    const int64_t qrow0 = b * qframes * positions + p;  // query / output row of frame 0
    if (item + stride < nitems) TM_LOAD_ITEM(item + stride)
    // ---- V chunks -> LDS image (d < D only)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // previous item's tr reads done
#pragma unroll
    for (int r = 0; r < VN; ++r) {
      const int idx = lane + 64 * r;
      const int f = idx / C::DCH, cc = idx - f * C::DCH;
      if (idx < frames * C::DCH) *(uint4*)(vl + f * C::VS + cc * 8) = vc[r];
    }
    // ---- S^T = K . Q^T
    f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < C::KSTEPS; ++ks)
      s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kc[ks]), __builtin_bit_cast(bf16x8, qc[ks]),
                                                  s, 0, 0, 0);
    // ---- softmax over keys 4*fq + j of query fr (log2 units)
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (4 * fq + j >= frames) s[j] = -INFINITY;
      else if (!unitc) s[j] *= c;
      mx = fmaxf(mx, s[j]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    bf16x8 pf;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pf[j] = (__bf16)__builtin_amdgcn_exp2f(s[j] - mx);
      pf[4 + j] = (__bf16)0.0f;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // V image written (the prefetch stays in flight)
    __builtin_amdgcn_wave_barrier();
    // ---- O^T = V^T . P^T, one 16-row block of d at a time
    f32x4 ot[C::DB];
#pragma unroll
    for (int a = 0; a < C::DB; ++a) {
      const bf16x4 t = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
          (bf16x4 __attribute__((address_space(3)))*)(vl + vtr + 16 * a));
      const bf16x8 vf = {t[0], t[1], t[2], t[3], (__bf16)0.0f, (__bf16)0.0f, (__bf16)0.0f, (__bf16)0.0f};
      ot[a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    }
    // row sum = O^T row D: block D/16, lane group (D%16)/4, element D%4
    const float l = __shfl(ot[D / 16][(D % 16) % 4], ((D % 16) / 4) * 16 + fr, 64);
    const float inv = __builtin_amdgcn_rcpf(l);
    if (qok) {
      bf16_t* orow = o + (qrow0 + (int64_t)fr * positions) * ldo + (int64_t)h * D;
#pragma unroll
      for (int a = 0; a < C::DB; ++a) {
        const int dd = 16 * a + 4 * fq;
        if (dd + 4 <= D)
          *(uint2*)(orow + dd) = make_uint2(pack2(ot[a][0] * inv, ot[a][1] * inv), pack2(ot[a][2] * inv, ot[a][3] * inv));
      }
    }
  }
#undef TM_LOAD_ITEM
}

// 17..32 frames (the DiT's 32-frame temporal blocks): the 16-frame kernel's scheme on two
// key blocks and two query blocks.  Per query block, S^T blocks (keys 16kb + 4fq + j,
// query 16qb + fr) give each lane 8 keys of its query; P^T's k-slot (fq, j) is key
// 4fq + j for j < 4 and 16 + 4fq + (j - 4) for j >= 4, and V^T's fragment takes the
// same keys from two tr reads 16 LDS rows apart, so one 16x16x32 MFMA per d-block sums
// all 32 keys.  The V^T fragments are read once per item and reused by both query blocks.
// ROPE (D = 64, the DiT's temporal blocks): the 1-D temporal RoPE of vd_rope_qk mode 1 is
// applied to the Q/K fragments as they are loaded — a lane's chunk at d-step 0 (dims
// 8fq..8fq+7) and d-step 1 (dims 32 + 8fq..) are exactly a rotate-half pair set, rotated
// by its frame f at angle f * theta^(-2i/64) in fp32 and rounded to bf16 as dit.hip's
// rope_kernel does — so the separate in-place RoPE pass over the Q/K rows disappears.
template <int D, bool ROPE = false>
__global__ __launch_bounds__(NT) void temporal_mfma32_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v, int64_t ld,
    bf16_t* __restrict__ o, int64_t ldo, int64_t batch, int frames, int64_t positions, int heads,
    float c, float log2_theta) {
  static_assert(!ROPE || D == 64, "fused temporal RoPE: d = 64 only");
  using C = TmCfg<D>;
  __shared__ __attribute__((aligned(16))) bf16_t vimg[4][32 * C::VS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  bf16_t* vl = vimg[wave];
  for (int idx = lane; idx < 32 * C::VS / 8; idx += 64) *(uint4*)(vl + idx * 8) = make_uint4(0, 0, 0, 0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane < 32) vl[lane * C::VS + D] = (bf16_t)0x3F80;
  const int64_t nitems = batch * positions * heads;
  const int64_t stride = (int64_t)gridDim.x * 4;
  const bool unitc = c == 1.0f;
  const int vtr = (4 * fq + (fr >> 2)) * C::VS + 4 * (fr & 3);
  const int64_t lblk = xcd_remap(blockIdx.x, gridDim.x);
  for (int64_t item = lblk * 4 + wave; item < nitems; item += stride) {
    const int h = (int)(item % heads);
    const int64_t bp = item / heads;
    const int64_t p = bp % positions, b = bp / positions;
    const int64_t row0 = b * frames * positions + p;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // previous item's tr reads done
    for (int idx = lane; idx < frames * C::DCH; idx += 64) {
      const int f = idx / C::DCH, cc = idx - f * C::DCH;
      *(uint4*)(vl + f * C::VS + cc * 8) =
          *(const uint4*)(v + (row0 + (int64_t)f * positions) * ld + (int64_t)h * D + cc * 8);
    }
    // ---- S^T blocks: [qb][kb]
    f32x4 s[2][2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) s[qb][kb] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (ROPE) {
      uint4 kq[2][2], qq[2][2];  // [d-step][frame block]
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int f = 16 * t + fr;
          kq[ks][t] = qq[ks][t] = make_uint4(0, 0, 0, 0);
          if (f < frames) {
            const int64_t rf = (row0 + (int64_t)f * positions) * ld + (int64_t)h * D + ks * 32 + 8 * fq;
            kq[ks][t] = *(const uint4*)(k + rf);
            qq[ks][t] = *(const uint4*)(q + rf);
          }
        }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const float pos = (float)(16 * t + fr);
        float ka[8], kb8[8], qa[8], qb8[8];
        unpack8(kq[0][t], ka); unpack8(kq[1][t], kb8);
        unpack8(qq[0][t], qa); unpack8(qq[1][t], qb8);
        float oka[8], okb[8], oqa[8], oqb[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float inv_freq = exp2f(-log2_theta * (float)(2 * (8 * fq + j)) / (float)D);
          float sn, cs;
          __sincosf(pos * inv_freq, &sn, &cs);
          oka[j] = ka[j] * cs - kb8[j] * sn;
          okb[j] = kb8[j] * cs + ka[j] * sn;
          oqa[j] = qa[j] * cs - qb8[j] * sn;
          oqb[j] = qb8[j] * cs + qa[j] * sn;
        }
        kq[0][t] = pack8(oka); kq[1][t] = pack8(okb);
        qq[0][t] = pack8(oqa); qq[1][t] = pack8(oqb);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
#pragma unroll
          for (int kb = 0; kb < 2; ++kb)
            s[qb][kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kq[ks][kb]),
                                                                __builtin_bit_cast(bf16x8, qq[ks][qb]), s[qb][kb], 0, 0,
                                                                0);
    } else {
#pragma unroll
    for (int ks = 0; ks < C::KSTEPS; ++ks) {
      const int dd = ks * 32 + 8 * fq;
      uint4 kq[2], qq[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int f = 16 * t + fr;
        kq[t] = qq[t] = make_uint4(0, 0, 0, 0);
        if (dd < D && f < frames) {
          const int64_t rf = (row0 + (int64_t)f * positions) * ld + (int64_t)h * D + dd;
          kq[t] = *(const uint4*)(k + rf);
          qq[t] = *(const uint4*)(q + rf);
        }
      }
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
          s[qb][kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kq[kb]),
                                                              __builtin_bit_cast(bf16x8, qq[qb]), s[qb][kb], 0, 0, 0);
    }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // V image written
    __builtin_amdgcn_wave_barrier();
    bf16x8 vf[C::DB];
#pragma unroll
    for (int a = 0; a < C::DB; ++a) {
      const bf16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
          (bf16x4 __attribute__((address_space(3)))*)(vl + vtr + 16 * a));
      const bf16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
          (bf16x4 __attribute__((address_space(3)))*)(vl + 16 * C::VS + vtr + 16 * a));
      vf[a] = bf16x8{t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
    }
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (16 * kb + 4 * fq + j >= frames) s[qb][kb][j] = -INFINITY;
          else if (!unitc) s[qb][kb][j] *= c;
          mx = fmaxf(mx, s[qb][kb][j]);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      bf16x8 pf;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pf[j] = (__bf16)__builtin_amdgcn_exp2f(s[qb][0][j] - mx);
        pf[4 + j] = (__bf16)__builtin_amdgcn_exp2f(s[qb][1][j] - mx);
      }
      f32x4 ot[C::DB];
#pragma unroll
      for (int a = 0; a < C::DB; ++a)
        ot[a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[a], pf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      const float l = __shfl(ot[D / 16][(D % 16) % 4], ((D % 16) / 4) * 16 + fr, 64);
      const float inv = __builtin_amdgcn_rcpf(l);
      const int f = 16 * qb + fr;
      if (f < frames) {
        bf16_t* orow = o + (row0 + (int64_t)f * positions) * ldo + (int64_t)h * D;
#pragma unroll
        for (int a = 0; a < C::DB; ++a) {
          const int dd = 16 * a + 4 * fq;
          if (dd + 4 <= D)
            *(uint2*)(orow + dd) = make_uint2(pack2(ot[a][0] * inv, ot[a][1] * inv), pack2(ot[a][2] * inv, ot[a][3] * inv));
        }
      }
    }
  }
}

// Row softmax for the materialised-score attention of the VAE mid block (one head,
// d = 512: S = 4096 keys per frame fits HBM easily, the flash kernels stop at d = 160).
// Scores arrive fp32 in log2 units (the caller folded d^-1/2 * log2(e) into q):
// p = exp2(s - max) / sum, written bf16 as the A operand of the P.V GEMM.  One
// workgroup per row, 4 columns per thread-step, three passes over the row (max,
// sum, write) — the row (16 KiB at 4096 keys) stays in L1/L2 between them.
__global__ __launch_bounds__(NT) void softmax_rows_kernel(const float* __restrict__ s, int64_t lds,
                                                          int64_t cols, bf16_t* __restrict__ p,
                                                          int64_t ldp) {
  __shared__ float red[NT / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float* row = s + (int64_t)blockIdx.x * lds;
  bf16_t* out = p + (int64_t)blockIdx.x * ldp;
  float m = -INFINITY;
  for (int64_t c = 4 * tid; c < cols; c += 4 * NT) {
    const float4 v = *(const float4*)(row + c);
    m = fmaxf(m, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
  }
  m = wave_max(m);
  if (lane == 0) red[w] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.f;
  for (int64_t c = 4 * tid; c < cols; c += 4 * NT) {
    const float4 v = *(const float4*)(row + c);
    sum += (exp2f(v.x - m) + exp2f(v.y - m)) + (exp2f(v.z - m) + exp2f(v.w - m));
  }
  sum = wave_sum(sum);
  if (lane == 0) red[w] = sum;
  __syncthreads();
  const float inv = 1.f / ((red[0] + red[1]) + (red[2] + red[3]));
  for (int64_t c = 4 * tid; c < cols; c += 4 * NT) {
    const float4 v = *(const float4*)(row + c);
    *(uint2*)(out + c) = make_uint2(pack2(exp2f(v.x - m) * inv, exp2f(v.y - m) * inv),
                                    pack2(exp2f(v.z - m) * inv, exp2f(v.w - m) * inv));
  }
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

// attention_d512.hip: the VAE mid-block attention (d = 512)
int launch_flash512(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv, void* o,
                    int64_t ldo, int64_t batch, int heads, int64_t sq, int64_t skv, int64_t kv_div, float scale,
                    hipStream_t s, int out_f32);

static int attention_entry(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v,
                            int64_t ldv, void* o, int64_t ldo, int64_t batch, int32_t heads,
                            int64_t sq, int64_t skv, int32_t d, int64_t kv_div, float scale,
                            vd_stream_t stream, int out_f32, int kernel) {
  VD_CHECK_ARG(q && k && v && o && al16(q) && al16(k) && al16(v) && ((uintptr_t)o & 7) == 0);
  VD_CHECK_ARG(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldo % 4 == 0);
  if (out_f32) VD_CHECK_ARG(((uintptr_t)o & 15) == 0);
  VD_CHECK_ARG(batch > 0 && heads > 0 && sq > 0 && skv > 0 && kv_div > 0 && batch % kv_div == 0);
  VD_CHECK_ARG(batch <= 65535 && heads <= 65535);
  VD_CHECK_ARG(skv * ldk < 0x7fffffff && skv * ldv < 0x7fffffff);
  VD_CHECK_ARG(kernel >= 0 && kernel <= 3);
  hipStream_t s = (hipStream_t)stream;
  switch (d) {
    case 32: return launch_flash<32>(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, sq, skv, kv_div, scale, s, out_f32, kernel);
    case 40: return launch_flash<40>(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, sq, skv, kv_div, scale, s, out_f32, kernel);
    case 64: return launch_flash<64>(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, sq, skv, kv_div, scale, s, out_f32, kernel);
    case 80: return launch_flash<80>(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, sq, skv, kv_div, scale, s, out_f32, kernel);
    case 128: return launch_flash<128>(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, sq, skv, kv_div, scale, s, out_f32, kernel);
    case 160: return launch_flash<160>(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, sq, skv, kv_div, scale, s, out_f32, kernel);
    case 512: return launch_flash512(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, sq, skv, kv_div, scale, s, out_f32);
    default: return VD_EUNSUPPORTED;
  }
}

extern "C" int vd_attention(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v,
                            int64_t ldv, void* o, int64_t ldo, int64_t batch, int32_t heads,
                            int64_t sq, int64_t skv, int32_t d, int64_t kv_div, float scale,
                            vd_stream_t stream) {
  return attention_entry(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, sq, skv, d, kv_div, scale, stream, 0, 0);
}

extern "C" int vd_attention_f32(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v,
                                int64_t ldv, float* o, int64_t ldo, int64_t batch, int32_t heads,
                                int64_t sq, int64_t skv, int32_t d, int64_t kv_div, float scale,
                                vd_stream_t stream) {
  return attention_entry(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, sq, skv, d, kv_div, scale, stream, 1, 0);
}

extern "C" int vd_attention_ex(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v,
                               int64_t ldv, void* o, int64_t ldo, int64_t batch, int32_t heads, int64_t sq,
                               int64_t skv, int32_t d, int64_t kv_div, float scale, int32_t out_f32,
                               int32_t kernel, vd_stream_t stream) {
  return attention_entry(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, sq, skv, d, kv_div, scale, stream,
                         out_f32 != 0, kernel);
}

static int temporal_entry(const void* q, const void* k, const void* v, int64_t ld, void* o, int64_t ldo,
                          int64_t batch, int32_t frames, int64_t positions, int32_t heads, int32_t d, float scale,
                          bool valu, vd_stream_t stream) {
  VD_CHECK_ARG(q && k && v && o && al16(q) && al16(k) && al16(v) && al16(o));
  VD_CHECK_ARG(ld % 8 == 0 && ldo % 8 == 0 && d % 8 == 0 && d > 0 && d <= 160);
  VD_CHECK_ARG(frames >= 1 && frames <= 32 && batch > 0 && positions > 0 && heads > 0);
  const int64_t items = batch * positions * heads;
  const unsigned grid = (unsigned)((items + 3) / 4);
  const float sl2 = scale * 1.4426950408889634f;
  hipStream_t s = (hipStream_t)stream;
  if (!valu && (d == 40 || d == 64 || d == 80 || d == 160 || (d == 32 && frames <= 16)) && ld % 8 == 0 &&
      ldo % 4 == 0) {
    const int64_t g = (items + 3) / 4;
    const unsigned grid2 = (unsigned)(g < 8192 ? g : 8192);
#define TM_LAUNCH(KERN, DD)                                                                                 \
    hipLaunchKernelGGL(KERN<DD>, dim3(grid2), dim3(NT), 0, s, (const bf16_t*)q, ld, (const bf16_t*)k,       \
                       (const bf16_t*)v, ld, (bf16_t*)o, ldo, batch, frames, frames, positions, heads, sl2)
    if (frames <= 16) {
      if (d == 32) TM_LAUNCH(temporal_mfma_kernel, 32);
      else if (d == 40) TM_LAUNCH(temporal_mfma_kernel, 40);
      else if (d == 64) TM_LAUNCH(temporal_mfma_kernel, 64);
      else if (d == 80) TM_LAUNCH(temporal_mfma_kernel, 80);
      else TM_LAUNCH(temporal_mfma_kernel, 160);
    } else {
#define TM32_LAUNCH(DD)                                                                                     \
    hipLaunchKernelGGL(temporal_mfma32_kernel<DD>, dim3(grid2), dim3(NT), 0, s, (const bf16_t*)q,           \
                       (const bf16_t*)k, (const bf16_t*)v, ld, (bf16_t*)o, ldo, batch, frames, positions,     \
                       heads, sl2, 0.f)
      if (d == 40) TM32_LAUNCH(40);
      else if (d == 64) TM32_LAUNCH(64);
      else if (d == 80) TM32_LAUNCH(80);
      else TM32_LAUNCH(160);
#undef TM32_LAUNCH
    }
#undef TM_LAUNCH
    return vd_launch_status();
  }
  if (frames <= 8)
    hipLaunchKernelGGL(temporal_attn_kernel<8>, dim3(grid), dim3(NT), 0, s, (const bf16_t*)q,
                       (const bf16_t*)k, (const bf16_t*)v, ld, (bf16_t*)o, ldo, batch, frames,
                       positions, heads, d, sl2);
  else if (frames <= 16)
    hipLaunchKernelGGL(temporal_attn_kernel<16>, dim3(grid), dim3(NT), 0, s, (const bf16_t*)q,
                       (const bf16_t*)k, (const bf16_t*)v, ld, (bf16_t*)o, ldo, batch, frames,
                       positions, heads, d, sl2);
  else
    hipLaunchKernelGGL(temporal_attn_kernel<32>, dim3(grid), dim3(NT), 0, s, (const bf16_t*)q,
                       (const bf16_t*)k, (const bf16_t*)v, ld, (bf16_t*)o, ldo, batch, frames,
                       positions, heads, d, sl2);
  return vd_launch_status();
}

extern "C" int vd_temporal_attention(const void* q, const void* k, const void* v, int64_t ld,
                                     void* o, int64_t ldo, int64_t batch, int32_t frames,
                                     int64_t positions, int32_t heads, int32_t d, float scale,
                                     vd_stream_t stream) {
  return temporal_entry(q, k, v, ld, o, ldo, batch, frames, positions, heads, d, scale, false, stream);
}

extern "C" int vd_temporal_attention_valu(const void* q, const void* k, const void* v, int64_t ld,
                                          void* o, int64_t ldo, int64_t batch, int32_t frames,
                                          int64_t positions, int32_t heads, int32_t d, float scale,
                                          vd_stream_t stream) {
  return temporal_entry(q, k, v, ld, o, ldo, batch, frames, positions, heads, d, scale, true, stream);
}

extern "C" int vd_temporal_attention_kv(const void* q, int64_t ldq, const void* k, const void* v, int64_t ldkv,
                                        void* o, int64_t ldo, int64_t batch, int32_t qframes, int32_t kframes,
                                        int64_t positions, int32_t heads, int32_t d, float scale,
                                        vd_stream_t stream) {
  VD_CHECK_ARG(q && k && v && o && al16(q) && al16(k) && al16(v) && al16(o));
  VD_CHECK_ARG(ldq % 8 == 0 && ldkv % 8 == 0 && ldo % 4 == 0);
  VD_CHECK_ARG(qframes >= 1 && qframes <= kframes && kframes <= 16 && batch > 0 && positions > 0 && heads > 0);
  if (!(d == 32 || d == 40 || d == 64 || d == 80 || d == 160)) return VD_EUNSUPPORTED;
  const int64_t g = (batch * positions * heads + 3) / 4;
  const unsigned grid = (unsigned)(g < 8192 ? g : 8192);
  const float sl2 = scale * 1.4426950408889634f;
  hipStream_t s = (hipStream_t)stream;
#define TKV_LAUNCH(DD)                                                                                      \
  hipLaunchKernelGGL(temporal_mfma_kernel<DD>, dim3(grid), dim3(NT), 0, s, (const bf16_t*)q, ldq,           \
                     (const bf16_t*)k, (const bf16_t*)v, ldkv, (bf16_t*)o, ldo, batch, qframes, kframes,       \
                     positions, heads, sl2)
  if (d == 32) TKV_LAUNCH(32);
  else if (d == 40) TKV_LAUNCH(40);
  else if (d == 64) TKV_LAUNCH(64);
  else if (d == 80) TKV_LAUNCH(80);
  else TKV_LAUNCH(160);
#undef TKV_LAUNCH
  return vd_launch_status();
}

extern "C" int vd_temporal_attention_rope(const void* q, const void* k, const void* v, int64_t ld, void* o,
                                          int64_t ldo, int64_t batch, int32_t frames, int64_t positions,
                                          int32_t heads, int32_t d, float scale, float theta,
                                          vd_stream_t stream) {
  VD_CHECK_ARG(q && k && v && o && al16(q) && al16(k) && al16(v) && al16(o));
  VD_CHECK_ARG(ld % 8 == 0 && ldo % 4 == 0 && d == 64 && theta > 1.f);
  VD_CHECK_ARG(frames >= 17 && frames <= 32 && batch > 0 && positions > 0 && heads > 0);
  const int64_t g = (batch * positions * heads + 3) / 4;
  hipLaunchKernelGGL((temporal_mfma32_kernel<64, true>), dim3((unsigned)(g < 8192 ? g : 8192)), dim3(NT), 0,
                     (hipStream_t)stream, (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, ld, (bf16_t*)o, ldo,
                     batch, frames, positions, heads, scale * 1.4426950408889634f, log2f(theta));
  return vd_launch_status();
}

extern "C" int vd_softmax_rows(const float* s, int64_t ld_s, int64_t rows, int64_t cols, void* p, int64_t ld_p,
                               vd_stream_t stream) {
  VD_CHECK_ARG(s && p && rows > 0 && cols > 0 && cols % 4 == 0 && ld_s % 4 == 0 && ld_p % 4 == 0);
  VD_CHECK_ARG(ld_s >= cols && ld_p >= cols && al16(s) && ((uintptr_t)p & 7) == 0 && rows < 0x7fffffff);
  hipLaunchKernelGGL(softmax_rows_kernel, dim3((unsigned)rows), dim3(NT), 0, (hipStream_t)stream, s, ld_s, cols,
                     (bf16_t*)p, ld_p);
  return vd_launch_status();
}
