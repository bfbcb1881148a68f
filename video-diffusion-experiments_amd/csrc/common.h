// Shared helpers for the gfx950 kernels of libvdiff_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/vdiff.h"

typedef uint16_t bf16_t;  // raw bf16 storage
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

#define VD_CHECK_ARG(cond) \
  do {                     \
    if (!(cond)) return VD_EINVAL; \
  } while (0)

static inline int vd_launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? VD_OK : (int)e;
}

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

// Round-to-nearest-even float -> bf16 (the cast lowers to v_cvt_pk_bf16_f32 on gfx950).
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
// two floats -> packed bf16x2 in ONE v_cvt_pk_bf16_f32 (RNE, as f2bf); the scalar casts
// combined with a shift and an or compiled to four instructions (round 4)
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t));
}

// 8 bf16 <-> 8 floats through a 16-byte vector.
__device__ __forceinline__ void unpack8(const uint4& u, float* f) {
  f[0] = bf_lo(u.x); f[1] = bf_hi(u.x); f[2] = bf_lo(u.y); f[3] = bf_hi(u.y);
  f[4] = bf_lo(u.z); f[5] = bf_hi(u.z); f[6] = bf_lo(u.w); f[7] = bf_hi(u.w);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

// SiLU with the hardware reciprocal (v_rcp_f32, ~1 ulp) instead of an IEEE divide.
__device__ __forceinline__ float silu_f(float x) {
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}
// erf(x): Abramowitz & Stegun 7.1.26-style rational/exp form refined as
// erf(x) = 1 - t*P(t)*exp(-x^2), t = 1/(1 + p|x|), max abs error 4.7e-7 in fp32 —
// GELU rel. error <= 2e-4 (at |y| ~ 1e-3), 20x below bf16 rounding.  One v_rcp, one
// v_exp, six FMAs (libm erff costs ~3x more issue slots).
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(-1.4426950408889634f * ax * ax);
  const float r = fmaf(-p * t, e, 1.0f);
  return copysignf(r, x);
}
// diffusers GEGLU/FeedForward gelu(approximate="none"): 0.5 x (1 + erf(x / sqrt 2))
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }
// gelu_erf of two values with the same operations in the same order (bit-identical per element),
// the multiplies / FMAs as packed fp32 (v_pk_mul_f32 / v_pk_fma_f32: two lanes' worth per issue
// slot — the GEGLU epilogue is VALU-bound, round 4); the transcendentals and the sign stay scalar.
typedef f32x2_t f32x2;
__device__ __forceinline__ f32x2 gelu_erf2(f32x2 x) {
  const f32x2 y = x * 0.70710678118654752f;
  const f32x2 ax = {fabsf(y[0]), fabsf(y[1])};
  f32x2 t = __builtin_elementwise_fma(f32x2{0.3275911f, 0.3275911f}, ax, f32x2{1.0f, 1.0f});
  t = f32x2{__builtin_amdgcn_rcpf(t[0]), __builtin_amdgcn_rcpf(t[1])};
  f32x2 p = __builtin_elementwise_fma(f32x2{1.061405429f, 1.061405429f}, t, f32x2{-1.453152027f, -1.453152027f});
  p = __builtin_elementwise_fma(p, t, f32x2{1.421413741f, 1.421413741f});
  p = __builtin_elementwise_fma(p, t, f32x2{-0.284496736f, -0.284496736f});
  p = __builtin_elementwise_fma(p, t, f32x2{0.254829592f, 0.254829592f});
  const f32x2 ea = (-1.4426950408889634f * ax) * ax;
  const f32x2 e = {__builtin_amdgcn_exp2f(ea[0]), __builtin_amdgcn_exp2f(ea[1])};
  const f32x2 r = __builtin_elementwise_fma(-p * t, e, f32x2{1.0f, 1.0f});
  const f32x2 erf = {copysignf(r[0], y[0]), copysignf(r[1], y[1])};
  return (0.5f * x) * (1.0f + erf);
}
// pointwise GEMM epilogue activation: VD_ACT_SILU or VD_ACT_GELU (erf form)
__device__ __forceinline__ float act_pw(int act, float x) { return act == VD_ACT_GELU ? gelu_erf(x) : silu_f(x); }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware remap of a 1-D block id (cdna_hip_programming.md §5
// "XCD swizzle must be bijective"): blocks b and b+8 share an XCD, so give
// each XCD group a contiguous range of logical tiles.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// The frame-sharded motion module's re-shard row permutation (round 5): rows
// m = ((i0*n1 + i1)*n2 + i2)*inner + j  ->  ((i2*n1 + i1)*n0 + i0)*inner + j  ("rev3": the three
// outer axes reversed; vdiff.dist.FrameShard.send_perm / return_perm), n1, n2, inner powers of
// two (checked by the callers), n0 = rows / (n1*n2*inner).  Shifts and masks only, all of them
// wave-uniform: the map costs a few VALU per row and no VGPR that outlives it.  inner == 0:
// identity.
struct Rev3 {
  int n0, sh1, sh2, shi;  // shi < 0: identity
  __host__ __device__ static int lg(int64_t v) {
    int s = 0;
    while (s < 62 && (int64_t{1} << s) < v) ++s;
    return s;
  }
  __host__ __device__ Rev3(int64_t rows, int64_t n1, int64_t n2, int64_t inner)
      : n0(0), sh1(0), sh2(0), shi(-1) {
    if (inner <= 0) return;
    sh1 = lg(n1); sh2 = lg(n2); shi = lg(inner);
    n0 = (int)(rows >> (sh1 + sh2 + shi));
  }
  __host__ __device__ static bool ok(int64_t rows, int64_t n1, int64_t n2, int64_t inner) {
    auto p2 = [](int64_t v) { return v > 0 && (v & (v - 1)) == 0; };
    return inner == 0 || (p2(n1) && p2(n2) && p2(inner) && rows % (n1 * n2 * inner) == 0 && rows < 0x7fffffff);
  }
  __device__ __forceinline__ int operator()(int m) const {
    if (shi < 0) return m;
    const uint32_t u = (uint32_t)m;
    const uint32_t j = u & ((1u << shi) - 1u), q = u >> shi;
    const uint32_t i2 = q & ((1u << sh2) - 1u), q1 = q >> sh2;
    const uint32_t i1 = q1 & ((1u << sh1) - 1u), i0 = q1 >> sh1;
    return (int)(((((i2 << sh1) + i1) * (uint32_t)n0 + i0) << shi) + j);
  }
};

// LayerNorm-fold statistics (v8 / the fused motion QKV attention): var1 = E[x²] − mean² from the
// fp32 MFMA sums, relative error ≈ 1e-7·(1 + mean²/var).  Where any row of the wave has
// |mean| / std > 16 (mean² > 256 var1), the wave takes the exact second pass Σ(x − mean)² over
// the row fragments it holds — lane (fr, fq) has row fr's elements 32 ks + 8 fq .. +7, so the
// four lanes fr + 16 fq hold the whole row.  The branch is wave-uniform and never
// taken on the UNet's rows (|mean| / std ≤ 0.1).
template <int KS>
__device__ __forceinline__ float row_var_guarded(const bf16x8 (&x)[KS], float mean, float var1, float rk) {
  if (__any(mean * mean > 256.f * var1)) {
    float ss = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = (float)x[ks][e] - mean;
        ss = fmaf(v, v, ss);
      }
    ss += __shfl_xor(ss, 16, 64);
    ss += __shfl_xor(ss, 32, 64);
    return ss * rk;
  }
  return fmaxf(var1, 0.f);
}
