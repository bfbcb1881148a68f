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
  static constexpr int KS = DQK + 8;                      // K LDS row (elements): odd # of 16B
  static constexpr int VS = ((DV * 2 + 31) / 64 * 64 + 32) / 2;  // V LDS row: 32B * odd
  static constexpr int KCH = DQK / 8;                     // K 16-byte chunks per row
  static constexpr int VCH = DV / 8;
  static constexpr int KREG = (KT * KCH + NT - 1) / NT;   // staged chunks per thread
  static constexpr int VREG = (KT * VCH + NT - 1) / NT;
};

// Cross-lane max over the 4 lanes holding one query (l, l^16, l^32, l^48):
// v_permlane32_swap / v_permlane16_swap + max, no LDS traffic (T12).
__device__ __forceinline__ float max_over_query_lanes(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  auto t = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(t[0]), __uint_as_float(t[1]));
}

template <int D, int QBLK>
__global__ __launch_bounds__(NT, 2) void flash_attn_kernel(
    const bf16_t* __restrict__ q, int64_t ldq, const bf16_t* __restrict__ k, int64_t ldk,
    const bf16_t* __restrict__ v, int64_t ldv, bf16_t* __restrict__ o, int64_t ldo, int heads,
    int64_t sq, int64_t skv, int64_t kv_div, float c) {
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

  uint4 kreg[C::KREG], vreg[C::VREG];
  auto load_kv = [&](int t) {
    const int64_t key0 = (int64_t)t * KT;
#pragma unroll
    for (int i = 0; i < C::KREG; ++i) {
      const int idx = tid + i * NT;
      const int r = idx / C::KCH, cc = idx - r * C::KCH;
      uint4 u = make_uint4(0, 0, 0, 0);
      if (r < KT && key0 + r < skv && cc * 8 < D) u = *(const uint4*)(kb_ptr + (key0 + r) * ldk + cc * 8);
      kreg[i] = u;
    }
#pragma unroll
    for (int i = 0; i < C::VREG; ++i) {
      const int idx = tid + i * NT;
      const int r = idx / C::VCH, cc = idx - r * C::VCH;
      uint4 u = make_uint4(0, 0, 0, 0);
      if (r < KT && key0 + r < skv && cc * 8 < D) u = *(const uint4*)(vb_ptr + (key0 + r) * ldv + cc * 8);
      if (ONES && cc == D / 8) u.x = 0x3F80u;  // bf16 1.0 in column D
      vreg[i] = u;
    }
  };
  auto store_kv = [&](int buf) {
#pragma unroll
    for (int i = 0; i < C::KREG; ++i) {
      const int idx = tid + i * NT;
      const int r = idx / C::KCH, cc = idx - r * C::KCH;
      if (r < KT) *(uint4*)(&ks_lds[buf][r * C::KS + cc * 8]) = kreg[i];
    }
#pragma unroll
    for (int i = 0; i < C::VREG; ++i) {
      const int idx = tid + i * NT;
      const int r = idx / C::VCH, cc = idx - r * C::VCH;
      if (r < KT) *(uint4*)(&vs_lds[buf][r * C::VS + cc * 8]) = vreg[i];
    }
  };

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
  load_kv(0);
  store_kv(0);
  __syncthreads();
  const int qq = fr >> 2, pp = fr & 3;  // tr-read geometry: lane 4*qq+pp -> row qq, cols 4*pp..

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) load_kv(t + 1);
    const bf16_t* kl = ks_lds[buf];
    const bf16_t* vl = vs_lds[buf];

    // ---- S^T = K . Q^T
    f32x4 s[4][QBLK];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int qb = 0; qb < QBLK; ++qb) s[kb][qb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dc = 0; dc < C::DQK / 32; ++dc) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const bf16x8 kf = *(const bf16x8*)(kl + (kb * 16 + fr) * C::KS + dc * 32 + 8 * fg);
#pragma unroll
        for (int qb = 0; qb < QBLK; ++qb)
          s[kb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qb][dc], s[kb][qb], 0, 0, 0);
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
#pragma unroll
    for (int a = 0; a < C::DV / 16; ++a) {
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16_t* p0 = vl + (32 * st + 4 * fg + qq) * C::VS + a * 16 + 4 * pp;
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (bf16x4 __attribute__((address_space(3)))*)(p0));
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (bf16x4 __attribute__((address_space(3)))*)(p0 + 16 * C::VS));
        const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int qb = 0; qb < QBLK; ++qb)
          oacc[a][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[st][qb], oacc[a][qb], 0, 0, 0);
      }
    }
    if (t + 1 < ntiles) store_kv(buf ^ 1);
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
#pragma unroll
    for (int a = 0; a < C::DV / 16; ++a) {
      const int dd = a * 16 + 4 * fg;
      if (dd < D) {
        *(uint2*)(orow + dd) = make_uint2(pack2(oacc[a][qb][0] * inv, oacc[a][qb][1] * inv),
                                          pack2(oacc[a][qb][2] * inv, oacc[a][qb][3] * inv));
      }
    }
  }
}

template <int D>
int launch_flash(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                 void* o, int64_t ldo, int64_t batch, int heads, int64_t sq, int64_t skv,
                 int64_t kv_div, float scale, hipStream_t s) {
  const float c = scale * 1.4426950408889634f;
  if (sq >= 1024 && D <= 64) {
    const dim3 grid((unsigned)((sq + 255) / 256), (unsigned)heads, (unsigned)batch);
    hipLaunchKernelGGL((flash_attn_kernel<D, 4>), grid, dim3(NT), 0, s, (const bf16_t*)q, ldq,
                       (const bf16_t*)k, ldk, (const bf16_t*)v, ldv, (bf16_t*)o, ldo, heads, sq, skv,
                       kv_div, c);
  } else {
    const dim3 grid((unsigned)((sq + 127) / 128), (unsigned)heads, (unsigned)batch);
    hipLaunchKernelGGL((flash_attn_kernel<D, 2>), grid, dim3(NT), 0, s, (const bf16_t*)q, ldq,
                       (const bf16_t*)k, ldk, (const bf16_t*)v, ldv, (bf16_t*)o, ldo, heads, sq, skv,
                       kv_div, c);
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

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" int vd_attention(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v,
                            int64_t ldv, void* o, int64_t ldo, int64_t batch, int32_t heads,
                            int64_t sq, int64_t skv, int32_t d, int64_t kv_div, float scale,
                            vd_stream_t stream) {
  VD_CHECK_ARG(q && k && v && o && al16(q) && al16(k) && al16(v) && ((uintptr_t)o & 7) == 0);
  VD_CHECK_ARG(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldo % 4 == 0);
  VD_CHECK_ARG(batch > 0 && heads > 0 && sq > 0 && skv > 0 && kv_div > 0 && batch % kv_div == 0);
  VD_CHECK_ARG(batch <= 65535 && heads <= 65535);
  hipStream_t s = (hipStream_t)stream;
  switch (d) {
    case 32: return launch_flash<32>(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, sq, skv, kv_div, scale, s);
    case 40: return launch_flash<40>(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, sq, skv, kv_div, scale, s);
    case 64: return launch_flash<64>(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, sq, skv, kv_div, scale, s);
    case 80: return launch_flash<80>(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, sq, skv, kv_div, scale, s);
    case 128: return launch_flash<128>(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, sq, skv, kv_div, scale, s);
    case 160: return launch_flash<160>(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, sq, skv, kv_div, scale, s);
    default: return VD_EUNSUPPORTED;
  }
}

extern "C" int vd_temporal_attention(const void* q, const void* k, const void* v, int64_t ld,
                                     void* o, int64_t ldo, int64_t batch, int32_t frames,
                                     int64_t positions, int32_t heads, int32_t d, float scale,
                                     vd_stream_t stream) {
  VD_CHECK_ARG(q && k && v && o && al16(q) && al16(k) && al16(v) && al16(o));
  VD_CHECK_ARG(ld % 8 == 0 && ldo % 8 == 0 && d % 8 == 0 && d > 0 && d <= 160);
  VD_CHECK_ARG(frames >= 1 && frames <= 32 && batch > 0 && positions > 0 && heads > 0);
  const int64_t items = batch * positions * heads;
  const unsigned grid = (unsigned)((items + 3) / 4);
  const float sl2 = scale * 1.4426950408889634f;
  hipStream_t s = (hipStream_t)stream;
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
