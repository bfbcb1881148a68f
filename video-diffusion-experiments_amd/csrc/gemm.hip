// bf16 MFMA GEMM + implicit-GEMM 3x3 conv for gfx950 (CDNA4).
//
// Replaces every matmul-shaped op of diffusers:UNetMotionModel.forward
// (SURVEY.md §8a a3-a5, a8, a10): ResnetBlock2D conv1/conv2/conv_shortcut,
// Down/Upsample2D convs, conv_in/conv_out, Transformer2DModel proj_in/proj_out,
// Attention to_q/k/v/out, FeedForward GEGLU + Linear, motion proj_in/out.
//
// Orientation: the MFMA computes C^T = W . A^T, i.e. the weight tile is the
// MFMA A operand (rows = output channels n) and the activation tile the B
// operand (rows = pixels/tokens m).  With v_mfma_f32_16x16x32_bf16 each lane
// then owns 4 CONSECUTIVE output channels of one pixel, so the NHWC store is
// one 8-byte (bf16) / 16-byte (fp32) write per lane and the GEGLU pair
// (hidden block, gate block) lands in the same lane.
//
// Tile BM x BN x 64, 256 threads = 4 waves as 2(M) x 2(N); operands staged
// global -> registers -> LDS (register staging so the conv gather, the channel
// concat and the nearest-x2 upsample happen in the load), double-buffered LDS
// with the next tile's global loads issued before the MFMAs of the current one
// (cdna_hip_programming.md T14), 16-B chunks XOR-swizzled by (row & 7) so the
// ds_read_b128 fragment reads spread over the bank row (T2), and an XCD-aware
// tile order (T1).
#include "common.h"

namespace {

constexpr int BK = 64;    // K elements per LDS tile row (128 bytes = 8 chunks)
constexpr int NT = 256;   // threads per block

__device__ __forceinline__ int lds_off(int row, int chunk) {
  return row * BK + ((chunk ^ (row & 7)) << 3);
}

// a / b for 0 <= a < 2^31 and a wave-uniform b > 0 (round 3): every image size, row width and
// frame count of the UNet is a power of two, so the common case is a shift; hipcc's 32-bit
// division is ~25 VALU, the 64-bit one (an int64 row index) ~100
struct Div {
  int b, sh;
  __device__ __forceinline__ explicit Div(int b_) : b(b_), sh((b_ & (b_ - 1)) == 0 ? __builtin_ctz((uint32_t)b_) : -1) {}
  __device__ __forceinline__ int operator()(int a) const {
    return sh >= 0 ? (int)((uint32_t)a >> sh) : (int)((uint32_t)a / (uint32_t)b);
  }
};

// PERM: the vd_gemm_desc.rmap_* output-row map (instantiated only by the kernels the plan gives
// an rmap request — v6, v1; the v2 / v3 / v5 pipelines sit at 256 VGPRs and spill with it)
template <int MB, int NB, bool PERM = false>
__device__ __forceinline__ void gemm_epilogue(const vd_gemm_desc& d, f32x4 (&acc)[NB][MB], int mbase,
                                              int nbase, int lane, int nodd = -1) {
  // acc[a][b][j] = C[m = mbase + b*16 + fr][n = nbase + a*16 + 4*fq + j]  (the wave's sub-tile);
  // nodd >= 0 moves the odd last block (NB odd) to columns nodd .. nodd + 15 instead
  // All offsets fit 32 bits (M*ldc < 2^31 is checked on the host).
  const int M = (int)d.M, N = (int)d.N;
  const int fr = lane & 15, fq = lane >> 4;
  const int nw = nbase;
  const Rev3 perm = PERM ? Rev3(d.M, d.rmap_n1, d.rmap_n2, d.rmap_inner) : Rev3(0, 0, 0, 0);
  // per-row values are recomputed inside each loop (arrays of MB row pointers kept
  // live across the whole epilogue cost 3 x MB VGPRs beside MB x NB x 4 accumulators)
#define VD_EPI_ROW(b)                                       \
  const int m_ = mbase + (b) * 16 + fr;                     \
  const bool mok_ = m_ < M;                                 \
  const int mrow_ = mok_ ? (PERM ? perm(m_) : m_) : 0;
  // Wide path (T21 for the 16x16 layout): v_permlane16_swap of 16-column blocks
  // (a, a+1) leaves each lane 8 CONSECUTIVE channels — lane group g of the pair
  // holds columns 16a + 16(g&1) + 8(g>>1) .. +7 — so residual loads and bf16
  // stores are 16 B and each store instruction writes 64 contiguous bytes per row
  // (full 64-B write granules) instead of 32.
  const bool wide = (N % 8) == 0 && !d.out_f32 && (d.ldc % 8) == 0 && (((uintptr_t)d.out) & 15) == 0 &&
                    (!d.res || ((d.ld_res % 8) == 0 && (((uintptr_t)d.res) & 15) == 0));
  const int wcol = 16 * (fq & 1) + 8 * (fq >> 1);  // lane's column offset inside a swapped pair
  // the row-bias row of each of the lane's MB rows, divided once (not per column block)
  int rbr[MB];
  if (d.rowbias) {
    const Div rdiv((int)d.rb_div);
#pragma unroll
    for (int b = 0; b < MB; ++b) {
      const int m = mbase + b * 16 + fr;
      rbr[b] = rdiv(m < M ? m : 0);
    }
  }
  if (d.act == VD_ACT_GEGLU) {
    if constexpr (NB % 4 == 0) {
      if (wide) {
        bf16_t* out = (bf16_t*)d.out;
#pragma unroll
        for (int a = 0; a < NB; a += 4) {  // hidden/gate blocks (a, a+1) and (a+2, a+3)
          const int nh0 = nw + a * 16 + 4 * fq, nh1 = nh0 + 32;
          float bh0[4] = {0, 0, 0, 0}, bg0[4] = {0, 0, 0, 0}, bh1[4] = {0, 0, 0, 0}, bg1[4] = {0, 0, 0, 0};
          if (d.bias) {
            const float4 t0 = *(const float4*)(d.bias + (nh0 < N ? nh0 : 0));
            const float4 t1 = *(const float4*)(d.bias + (nh0 + 16 < N ? nh0 + 16 : 0));
            const float4 t2 = *(const float4*)(d.bias + (nh1 < N ? nh1 : 0));
            const float4 t3 = *(const float4*)(d.bias + (nh1 + 16 < N ? nh1 + 16 : 0));
            bh0[0] = t0.x; bh0[1] = t0.y; bh0[2] = t0.z; bh0[3] = t0.w;
            bg0[0] = t1.x; bg0[1] = t1.y; bg0[2] = t1.z; bg0[3] = t1.w;
            bh1[0] = t2.x; bh1[1] = t2.y; bh1[2] = t2.z; bh1[3] = t2.w;
            bg1[0] = t3.x; bg1[1] = t3.y; bg1[2] = t3.z; bg1[3] = t3.w;
          }
          const int nout = nw / 2 + (a / 2) * 16 + wcol;
#pragma unroll
          for (int b = 0; b < MB; ++b) {
            VD_EPI_ROW(b)
            uint32_t x[2], y[2];
#pragma unroll
            for (int h2 = 0; h2 < 2; ++h2) {
              const f32x2 go = gelu_erf2(f32x2{acc[a + 1][b][2 * h2], acc[a + 1][b][2 * h2 + 1]} +
                                         f32x2{bg0[2 * h2], bg0[2 * h2 + 1]});
              const f32x2 gp = gelu_erf2(f32x2{acc[a + 3][b][2 * h2], acc[a + 3][b][2 * h2 + 1]} +
                                         f32x2{bg1[2 * h2], bg1[2 * h2 + 1]});
              const f32x2 oo =
                  (f32x2{acc[a][b][2 * h2], acc[a][b][2 * h2 + 1]} + f32x2{bh0[2 * h2], bh0[2 * h2 + 1]}) * go;
              const f32x2 pp =
                  (f32x2{acc[a + 2][b][2 * h2], acc[a + 2][b][2 * h2 + 1]} + f32x2{bh1[2 * h2], bh1[2 * h2 + 1]}) * gp;
              const float o0 = oo[0], o1 = oo[1], p0 = pp[0], p1 = pp[1];
              auto r = __builtin_amdgcn_permlane16_swap(pack2(o0, o1), pack2(p0, p1), false, false);
              x[h2] = r[0];
              y[h2] = r[1];
            }
            if (mok_ && 2 * nout < N)
              *(uint4*)(out + (uint32_t)(mrow_ * (int)d.ldc + nout)) = make_uint4(x[0], x[1], y[0], y[1]);
          }
        }
        return;
      }
    }
    if constexpr (NB % 2 == 0) {
      bf16_t* out = (bf16_t*)d.out;
#pragma unroll
      for (int a = 0; a < NB; a += 2) {
        const int nh = nw + a * 16 + 4 * fq;  // packed hidden column
        const int ng = nh + 16;                // packed gate column
        if (ng >= N) continue;
        const int nout = nw / 2 + (a / 2) * 16 + 4 * fq;
        float bh[4] = {0, 0, 0, 0}, bg[4] = {0, 0, 0, 0};
        if (d.bias) {
          const float4 t0 = *(const float4*)(d.bias + nh);
          const float4 t1 = *(const float4*)(d.bias + ng);
          bh[0] = t0.x; bh[1] = t0.y; bh[2] = t0.z; bh[3] = t0.w;
          bg[0] = t1.x; bg[1] = t1.y; bg[2] = t1.z; bg[3] = t1.w;
        }
#pragma unroll
        for (int b = 0; b < MB; ++b) {
          VD_EPI_ROW(b)
          if (!mok_) continue;
          float o[4];
          const f32x2 g01 = gelu_erf2(f32x2{acc[a + 1][b][0] + bg[0], acc[a + 1][b][1] + bg[1]});
          const f32x2 g23 = gelu_erf2(f32x2{acc[a + 1][b][2] + bg[2], acc[a + 1][b][3] + bg[3]});
          o[0] = (acc[a][b][0] + bh[0]) * g01[0];
          o[1] = (acc[a][b][1] + bh[1]) * g01[1];
          o[2] = (acc[a][b][2] + bh[2]) * g23[0];
          o[3] = (acc[a][b][3] + bh[3]) * g23[1];
          *(uint2*)(out + (uint32_t)(mrow_ * (int)d.ldc + nout)) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
        }
      }
    }
    return;
  }
  if (wide) {
    bf16_t* out = (bf16_t*)d.out;
#pragma unroll
    for (int a = 0; a + 1 < NB; a += 2) {
      const int n = nw + a * 16 + wcol;  // first of this lane's 8 columns after the swap
      const bool nok = n < N;
      const int nn = nok ? n : 0;
      float bv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (d.bias) {
        const float4 t0 = *(const float4*)(d.bias + nn), t1 = *(const float4*)(d.bias + nn + 4);
        bv[0] = t0.x; bv[1] = t0.y; bv[2] = t0.z; bv[3] = t0.w;
        bv[4] = t1.x; bv[5] = t1.y; bv[6] = t1.z; bv[7] = t1.w;
      }
      uint4 rsv[MB];  // residual rows loaded together ahead of the stores (as epi_ln, round 2)
      if (d.res) {
#pragma unroll
        for (int b = 0; b < MB; ++b) {
          VD_EPI_ROW(b)
          rsv[b] = *(const uint4*)((const bf16_t*)d.res + (uint32_t)(mrow_ * (int)d.ld_res + nn));
        }
      }
#pragma unroll
      for (int b = 0; b < MB; ++b) {
        VD_EPI_ROW(b)
        float o[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[a][b][j]), __float_as_uint(acc[a + 1][b][j]),
                                                    false, false);
          o[j] = __uint_as_float(r[0]) + bv[j];
          o[4 + j] = __uint_as_float(r[1]) + bv[4 + j];
        }
        if (!mok_ || !nok) continue;
        if (d.rowbias) {
          const float* rbrow = d.rowbias + (int64_t)rbr[b] * d.ld_rb;
          const float4 t0 = *(const float4*)(rbrow + n), t1 = *(const float4*)(rbrow + n + 4);
          o[0] += t0.x; o[1] += t0.y; o[2] += t0.z; o[3] += t0.w;
          o[4] += t1.x; o[5] += t1.y; o[6] += t1.z; o[7] += t1.w;
        }
        if (d.act == VD_ACT_SILU || d.act == VD_ACT_GELU) {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = act_pw(d.act, o[j]);
        }
        if (d.res) {
          float rf[8];
          unpack8(rsv[b], rf);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += rf[j];
        }
        *(uint4*)(out + (uint32_t)(mrow_ * (int)d.ldc + n)) = pack8(o);
      }
    }
    if constexpr (NB % 2 == 0) return;
  }
#pragma unroll
  for (int a = 0; a < NB; ++a) {  // narrow path (or, when wide, the odd last block)
    if (wide && a + 1 < NB) continue;
    const int n = (nodd >= 0 && a == NB - 1 ? nodd : nw + a * 16) + 4 * fq;
    if (n >= N) continue;
    float bv[4] = {0, 0, 0, 0};
    if (d.bias) {
      const float4 t = *(const float4*)(d.bias + n);
      bv[0] = t.x; bv[1] = t.y; bv[2] = t.z; bv[3] = t.w;
    }
#pragma unroll
    for (int b = 0; b < MB; ++b) {
      VD_EPI_ROW(b)
      if (!mok_) continue;
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = acc[a][b][j] + bv[j];
      if (d.rowbias) {
        const float4 t = *(const float4*)(d.rowbias + (int64_t)rbr[b] * d.ld_rb + n);
        o[0] += t.x; o[1] += t.y; o[2] += t.z; o[3] += t.w;
      }
      if (d.act == VD_ACT_SILU || d.act == VD_ACT_GELU) {
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = act_pw(d.act, o[j]);
      }
      if (d.res) {
        const uint2 r = *(const uint2*)((const bf16_t*)d.res + (uint32_t)(mrow_ * (int)d.ld_res + n));
        o[0] += bf_lo(r.x); o[1] += bf_hi(r.x); o[2] += bf_lo(r.y); o[3] += bf_hi(r.y);
      }
      const uint32_t off = (uint32_t)(mrow_ * (int)d.ldc + n);
      if (d.out_f32) {
        *(float4*)((float*)d.out + off) = make_float4(o[0], o[1], o[2], o[3]);
      } else {
        *(uint2*)((bf16_t*)d.out + off) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
      }
    }
  }
}

#undef VD_EPI_ROW

template <int BM, int BN, int MODE>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(const vd_gemm_desc d) {
  constexpr int RA = BM / 32;        // A chunks staged per thread
  constexpr int RW = BN / 32;        // W chunks staged per thread
  constexpr int MB = BM / 2 / 16;    // 16-row m blocks per wave
  constexpr int NB = BN / 2 / 16;    // 16-row n blocks per wave
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * (BM + BN) * BK];
  bf16_t* As = smem;
  bf16_t* Ws = smem + 2 * BM * BK;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  const int64_t M = d.M, N = d.N, K = d.K;
  const int tiles_n = (int)((N + BN - 1) / BN);
  const int tiles_m = (int)((M + BM - 1) / BM);
  const int id = xcd_remap(blockIdx.x, tiles_n * tiles_m);
  const int64_t m0 = (int64_t)(id / tiles_n) * BM;
  const int64_t n0 = (int64_t)(id % tiles_n) * BN;

  const int sc = tid & 7;    // staged chunk (8 bf16) within the 64-wide K tile
  const int sr = tid >> 3;   // staged row base (rows sr + 32*i)

  const bf16_t* a0 = (const bf16_t*)d.a0;
  const bf16_t* a1 = (const bf16_t*)d.a1;
  const bf16_t* w = (const bf16_t*)d.w;

  // Per staged A row: pixel coordinates for the conv gather.  pimg = the input image of
  // temporal tap 0, pfr = its frame index inside the video (valid range [0, frames_in)).
  int pimg[RA], pfr[RA], poh[RA], pow_[RA];
  bool prow[RA];
  int cin = 0, hgrid = 0, wgrid = 0;
  if constexpr (MODE == VD_A_CONV3X3) {
    cin = (int)d.K / (d.ks * d.ks * d.kt);
    hgrid = d.upsample ? 2 * d.h_in : d.h_in;
    wgrid = d.upsample ? 2 * d.w_in : d.w_in;
    const int hw = d.h_out * d.w_out;
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const int64_t m = m0 + sr + 32 * i;
      prow[i] = m < M;
      const int mm = prow[i] ? (int)m : 0;
      const int img = mm / hw;
      const int vid = img / d.frames_out;
      pfr[i] = img - vid * d.frames_out + d.t_off - d.kt / 2;
      pimg[i] = vid * d.frames_in + pfr[i];
      const int p = mm - img * hw;
      poh[i] = p / d.w_out;
      pow_[i] = p - poh[i] * d.w_out;
    }
  }

  uint4 ra[RA], rw[RW];

  auto load_tile = [&](int kt) {
    const int64_t k = (int64_t)kt * BK + sc * 8;
    if constexpr (MODE == VD_A_DENSE) {
      const bool in0 = k < d.k0;
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        const int64_t m = m0 + sr + 32 * i;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (m < M && k < K) {
          const bf16_t* p = in0 ? a0 + m * d.lda0 + k : a1 + m * d.lda1 + (k - d.k0);
          v = *(const uint4*)p;
        }
        ra[i] = v;
      }
    } else {
      const bool kin = k < K;
      const int tap27 = kin ? (int)(k / cin) : 0;
      const int ci = (int)k - tap27 * cin;
      const int ks2 = d.ks * d.ks;
      const int dt = tap27 / ks2, tap = tap27 - ks2 * dt;
      const int dy = d.ks == 3 ? tap / 3 : 1, dx = d.ks == 3 ? tap - 3 * (tap / 3) : 1;
      const bool in0 = ci < d.k0;
      const bf16_t* base = in0 ? a0 + ci : a1 + (ci - d.k0);
      const int64_t ld = in0 ? d.lda0 : d.lda1;
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        int ih = poh[i] * d.stride + dy - 1;
        int iw = pow_[i] * d.stride + dx - 1;
        const int fin = pfr[i] + dt;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (kin && prow[i] && ih >= 0 && ih < hgrid && iw >= 0 && iw < wgrid && fin >= 0 && fin < d.frames_in) {
          ih >>= d.upsample;
          iw >>= d.upsample;
          const int64_t pix = ((int64_t)(pimg[i] + dt) * d.h_in + ih) * d.w_in + iw;
          v = *(const uint4*)(base + pix * ld);
        }
        ra[i] = v;
      }
    }
#pragma unroll
    for (int i = 0; i < RW; ++i) {
      const int64_t n = n0 + sr + 32 * i;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (n < N && k < K) v = *(const uint4*)(w + n * d.ldw + k);
      rw[i] = v;
    }
  };
  auto store_tile = [&](int buf) {
    bf16_t* as = As + buf * BM * BK;
    bf16_t* ws = Ws + buf * BN * BK;
#pragma unroll
    for (int i = 0; i < RA; ++i) *(uint4*)(as + lds_off(sr + 32 * i, sc)) = ra[i];
#pragma unroll
    for (int i = 0; i < RW; ++i) *(uint4*)(ws + lds_off(sr + 32 * i, sc)) = rw[i];
  };

  f32x4 acc[NB][MB];
#pragma unroll
  for (int a = 0; a < NB; ++a)
#pragma unroll
    for (int b = 0; b < MB; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (int)((K + BK - 1) / BK);
  load_tile(0);
  store_tile(0);
  __syncthreads();

  const int fr = lane & 15;   // fragment row within a 16-block
  const int fq = lane >> 4;   // which 8-wide k slice (0..3)
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tile(kt + 1);
    const bf16_t* as = As + cur * BM * BK;
    const bf16_t* ws = Ws + cur * BN * BK;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 wf[NB], xf[MB];
#pragma unroll
      for (int a = 0; a < NB; ++a)
        wf[a] = *(const bf16x8*)(ws + lds_off(wn * (BN / 2) + a * 16 + fr, ks * 4 + fq));
#pragma unroll
      for (int b = 0; b < MB; ++b)
        xf[b] = *(const bf16x8*)(as + lds_off(wm * (BM / 2) + b * 16 + fr, ks * 4 + fq));
#pragma unroll
      for (int a = 0; a < NB; ++a)
#pragma unroll
        for (int b = 0; b < MB; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[a], xf[b], acc[a][b], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }

  if (d.rmap_inner)
    gemm_epilogue<MB, NB, true>(d, acc, (int)m0 + wm * MB * 16, (int)n0 + wn * (BN / 2), lane);
  else
    gemm_epilogue<MB, NB>(d, acc, (int)m0 + wm * MB * 16, (int)n0 + wn * (BN / 2), lane);
}

// ============================================================================ v9
// Skinny GEMM, M <= 16: the time-embedding MLP and the resnets' concatenated time_emb_proj (M = the
// UNet batch, 2 with CFG) — weight streaming, HBM-bound.  v1's 128 x 160 tiles put these on 8 / 126
// workgroups (22 / 31 us per launch at N = 1280 / 20160).  One wave owns 16 output columns and all
// of K; its MFMA chain is v1's (C^T = W . A^T by v_mfma_f32_16x16x32_bf16, k ascending, one
// accumulator, zero-filled past K), so the result is bit-identical to v1's.  The fragments come
// straight from global memory (no LDS): lane (fr, fq) holds W row n0 + fr and A row fr (zero for
// fr >= M), k slice 8*fq .. +7 of each 32-k step; G9_U steps of loads are in flight ahead of the
// MFMAs that consume the previous G9_U.  The epilogue is gemm_epilogue's narrow path (MB = NB = 1).
constexpr int G9_NW = 4, G9_U = 8, G9_MMAX = 16;
__global__ __launch_bounds__(G9_NW * 64) void gemm9_kernel(const vd_gemm_desc d) {
  const int lane = threadIdx.x & 63;
  const int fr = lane & 15, fq = lane >> 4;
  const int n0 = (blockIdx.x * G9_NW + (threadIdx.x >> 6)) * 16;
  const int N = (int)d.N, M = (int)d.M, K = (int)d.K;
  if (n0 >= N) return;  // wave-uniform; no barriers below
  const bool nok = n0 + fr < N, mok = fr < M;
  const bf16_t* wp = (const bf16_t*)d.w + (int64_t)(nok ? n0 + fr : 0) * d.ldw + 8 * fq;
  const bf16_t* ap = (const bf16_t*)d.a0 + (int64_t)(mok ? fr : 0) * d.lda0 + 8 * fq;
  const int nsteps = (K + 31) / 32;
  uint4 wc[G9_U], ac[G9_U], wn[G9_U], an[G9_U];
  auto load = [&](int s0, uint4 (&wv)[G9_U], uint4 (&av)[G9_U]) {
#pragma unroll
    for (int u = 0; u < G9_U; ++u) {
      const int k = (s0 + u) * 32;
      const bool kok = k + 8 * fq < K;
      wv[u] = nok && kok ? *(const uint4*)(wp + k) : make_uint4(0, 0, 0, 0);
      av[u] = mok && kok ? *(const uint4*)(ap + k) : make_uint4(0, 0, 0, 0);
    }
  };
  f32x4 acc[1][1] = {{f32x4{0.f, 0.f, 0.f, 0.f}}};
  load(0, wc, ac);
  for (int s0 = 0; s0 < nsteps; s0 += G9_U) {
    if (s0 + G9_U < nsteps) load(s0 + G9_U, wn, an);
#pragma unroll
    for (int u = 0; u < G9_U; ++u)
      if (s0 + u < nsteps)
        acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wc[u]),
                                                             __builtin_bit_cast(bf16x8, ac[u]), acc[0][0], 0, 0, 0);
#pragma unroll
    for (int u = 0; u < G9_U; ++u) {
      wc[u] = wn[u];
      ac[u] = an[u];
    }
  }
  gemm_epilogue<1, 1>(d, acc, 0, n0, lane);
}

// ============================================================================ v2
// LDS-DMA GEMM: BM = 256, BN in {128, 160}, BK = 64, 512 threads = 8 waves as
// 4(M) x 2(N), each wave 64 x BN/2.  Operands reach LDS by `buffer_load_dwordx4
// ... lds` (no VGPR staging, no ds_write pass) into a 3-stage ring, two tiles in
// flight, ONE raw s_barrier per K-tile behind a counted vmcnt (guide §5
// "Pipelining across barriers").  The LDS image is lane-linear; the (row & 7)
// XOR swizzle is applied on the per-lane SOURCE address (rule 21).  Conv taps
// outside the image are zero-filled by the buffer range check (voffset beyond
// num_records returns 0).  Per-tile address work: one integer add per load.
constexpr int G2_BM = 256, G2_NT = 512, G2_STAGES = 3;
int g_num_cus = 256;  // MI355X; the device's CU count, read once per process (read_num_cus)
constexpr uint32_t G2_OOB = 0x80000000u;

template <int BN>
struct G2 {
  static constexpr int A_BYTES = G2_BM * BK * 2;   // 32 KiB
  static constexpr int B_BYTES = BN * BK * 2;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int NA = 4;                     // A DMA instructions per wave per tile
  static constexpr int NBI = BN / 8;               // B DMA instructions per tile (whole block)
  static constexpr int NBMAX = (NBI + 7) / 8;      // per wave, upper bound
  static constexpr int MB = 4, NB = BN / 32;
};

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, voff, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  else if constexpr (N == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
}

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// Fragment-read order (round 2): without a pin hipcc sinks each X fragment read to its 4 MFMAs
// behind an lgkmcnt(0) — 8 exposed LDS latencies per K-tile.  k-step 0's 9 reads issue right
// after the barrier (sched_barrier), then k-step 1's reads interleave one per two of k-step 0's
// MFMAs (sched_group_barrier), so the MFMA chain waits on counted lgkmcnt only (52.79 vs 53.50
// ms/step for the unpinned order, 53.11 with all reads ahead; profiles/r02f_fragment_order.txt).

template <int BN, int MODE>
__global__ __launch_bounds__(G2_NT, 1) void gemm2_kernel(const vd_gemm_desc d, uint32_t a0_bytes,
                                                         uint32_t a1_bytes, uint32_t w_bytes,
                                                         int split) {
  using C = G2<BN>;
  __shared__ __attribute__((aligned(1024))) char smem[G2_STAGES * C::STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int64_t M = d.M, N = d.N, K = d.K;
  const int tiles_n = (int)((N + BN - 1) / BN);
  const int tiles_m = (int)((M + G2_BM - 1) / G2_BM);
  const int units = tiles_n * tiles_m * split;
  // Persistent, strided: this workgroup owns units lid, lid + G, lid + 2G, ...
  // (G = gridDim.x <= #CUs, all resident).  A unit is (output tile, split-K
  // slice), tiles N-fastest.  lid is XCD-contiguous (xcd_remap), so at every
  // round the ~32 workgroups of one XCD run ~32 CONSECUTIVE units — the N-tiles
  // of the same few A row-panels — and each A panel comes from HBM once and is
  // shared through that XCD's L2 (a contiguous per-workgroup range instead puts
  // 32 different panels in flight per XCD, thrashes L2 and re-reads A from HBM
  // once per N-tile).
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int G = gridDim.x;
  const int u_begin = lid;
  const int nk_all = (int)(K / BK);

  const int rb = lane >> 3;                                  // row within the 8-row DMA block
  const uint32_t lc16 = (uint32_t)(((lane & 7) ^ rb) * 16);  // swizzled source chunk (bytes)
  const __amdgpu_buffer_rsrc_t ra0 = __builtin_amdgcn_make_buffer_rsrc((void*)d.a0, 0, a0_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ra1 =
      __builtin_amdgcn_make_buffer_rsrc((void*)(d.a1 ? d.a1 : d.a0), 0, d.a1 ? a1_bytes : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)d.w, 0, w_bytes, 0x00020000);
  const int nbw = (C::NBI - wid + 7) / 8;  // this wave's B DMA instructions per K-tile
  const int cin = MODE == VD_A_CONV3X3 ? (int)(K / (d.ks * d.ks * d.kt)) : 0;
  const int hgrid = d.upsample ? 2 * d.h_in : d.h_in;
  const int wgrid = d.upsample ? 2 * d.w_in : d.w_in;

  // ---- issue cursor: the (unit, k-tile) whose DMA goes out next
  int iu = u_begin, ikt = 0, ikt1 = 0;
  uint32_t boff[C::NBMAX], aoff0[C::NA], aoff1[C::NA];
  int poh[C::NA], pow_[C::NA], pimg[C::NA], pfr[C::NA];
  int c_tap = 0, c_ci = 0;
  bool c_new = true;
  // (an early-out for split == 1 here measured 15 % slower on the dense v2 GEMMs, same box,
  // profiles/r03t_unit_kr_bisect.txt: it changes how hipcc lays out the persistent unit loop)
  auto unit_kr = [&](int u, int& kt0, int& kt1) {
    const int sp = u % split;
    kt0 = (int)((int64_t)nk_all * sp / split);
    kt1 = (int)((int64_t)nk_all * (sp + 1) / split);
  };
  auto setup_unit = [&](int u) {  // per-unit row offsets for the issue cursor
    const int tile = u / split;
    const int64_t m0 = (int64_t)(tile / tiles_n) * G2_BM, n0 = (int64_t)(tile % tiles_n) * BN;
    int kt0;
    unit_kr(u, kt0, ikt1);
    ikt = kt0;
#pragma unroll
    for (int j = 0; j < C::NBMAX; ++j) {
      int64_t n = n0 + (j * 8 + wid) * 8 + rb;
      n = n < N ? n : N - 1;
      boff[j] = (uint32_t)(n * d.ldw * 2) + lc16;
    }
    if constexpr (MODE == VD_A_DENSE) {
#pragma unroll
      for (int j = 0; j < C::NA; ++j) {
        int64_t m = m0 + (wid * 4 + j) * 8 + rb;
        m = m < M ? m : M - 1;
        aoff0[j] = (uint32_t)(m * d.lda0 * 2) + lc16;
        aoff1[j] = (uint32_t)(m * d.lda1 * 2) + lc16;
      }
    } else {  // 32-bit rows, shifts for power-of-two sizes (round 3; int64 divisions: -2-3 %)
      const int hw = d.h_out * d.w_out;
      const Div dhw(hw), dfr(d.frames_out), dw(d.w_out);
#pragma unroll
      for (int j = 0; j < C::NA; ++j) {
        int m = (int)m0 + (wid * 4 + j) * 8 + rb;
        m = m < (int)M ? m : (int)M - 1;
        const int img = dhw(m);
        const int vid = dfr(img);
        pfr[j] = img - vid * d.frames_out + d.t_off - d.kt / 2;  // frame of temporal tap 0
        pimg[j] = vid * d.frames_in + pfr[j];
        const int p = m - img * hw;
        poh[j] = dw(p);
        pow_[j] = p - poh[j] * d.w_out;
      }
    }
    if constexpr (MODE != VD_A_DENSE) {
      c_tap = kt0 * BK / cin;
      c_ci = kt0 * BK - c_tap * cin;
      c_new = true;
    }
  };
  auto issue = [&](int stage) {  // DMA of the cursor's k-tile into `stage`, then advance it
    char* la = smem + stage * C::STAGE;
    char* lb = la + C::A_BYTES;
    const int kb = ikt * BK;
    if constexpr (MODE == VD_A_DENSE) {
      const bool s0 = kb < (int)d.k0;
      const uint32_t koff = (uint32_t)(s0 ? kb : kb - (int)d.k0) * 2;
#pragma unroll
      for (int j = 0; j < C::NA; ++j)
        dma16(s0 ? ra0 : ra1, la + (wid * 4 + j) * 1024, (s0 ? aoff0[j] : aoff1[j]) + koff);
    } else {
      if (c_new) {  // new tap: recompute the rows' pixel offsets
        c_new = false;
        const int ks2 = d.ks * d.ks;
        const int dt = c_tap / ks2, t9 = c_tap - ks2 * dt;
        const int dy = d.ks == 3 ? t9 / 3 : 1, dx = d.ks == 3 ? t9 - 3 * (t9 / 3) : 1;
        // branch-free (round 3): unsigned range checks combined with &, so hipcc emits no
        // exec-mask branches per row (the && chain compiled to three nested saveexec blocks)
#pragma unroll
        for (int j = 0; j < C::NA; ++j) {
          const int ih = poh[j] * d.stride + dy - 1, iw = pow_[j] * d.stride + dx - 1;
          const int fin = pfr[j] + dt;
          const bool ok = ((uint32_t)ih < (uint32_t)hgrid) & ((uint32_t)iw < (uint32_t)wgrid) &
                          ((uint32_t)fin < (uint32_t)d.frames_in);
          const uint32_t pix = (uint32_t)(((pimg[j] + dt) * d.h_in + (ih >> d.upsample)) * d.w_in + (iw >> d.upsample));
          aoff0[j] = ok ? pix * (uint32_t)(d.lda0 * 2) + lc16 : G2_OOB;
          aoff1[j] = ok ? pix * (uint32_t)(d.lda1 * 2) + lc16 : G2_OOB;
        }
      }
      const bool s0 = c_ci < (int)d.k0;
      const uint32_t coff = (uint32_t)(s0 ? c_ci : c_ci - (int)d.k0) * 2;
      // a tap outside the image keeps G2_OOB + coff >= 2^31 > the buffer's num_records (< 2^31,
      // checked by plan()): still out of range, read as zeros — no per-piece select
#pragma unroll
      for (int j = 0; j < C::NA; ++j)
        dma16(s0 ? ra0 : ra1, la + (wid * 4 + j) * 1024, (s0 ? aoff0[j] : aoff1[j]) + coff);
      c_ci += BK;
      if (c_ci == cin) { c_ci = 0; ++c_tap; c_new = true; }
    }
#pragma unroll
    for (int j = 0; j < C::NBMAX; ++j)
      if (j < nbw) dma16(rw, lb + (j * 8 + wid) * 1024, boff[j] + (uint32_t)kb * 2);
    if (++ikt == ikt1 && (iu += G) < units) setup_unit(iu);
  };

  f32x4 acc[C::NB][C::MB];
#pragma unroll
  for (int a = 0; a < C::NB; ++a)
#pragma unroll
    for (int b = 0; b < C::MB; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // total k-tiles this workgroup streams
  int n_it = 0;
  for (int u = u_begin; u < units; u += G) {
    int a0_, a1_;
    unit_kr(u, a0_, a1_);
    n_it += a1_ - a0_;
  }
  if (n_it == 0) return;
  setup_unit(u_begin);
  issue(0);
  if (n_it > 1) issue(1);
  // per-lane LDS byte offsets of the first fragment of each operand for k-step
  // ks (rows differ by multiples of 16 between fragments, so the (row & 7) XOR
  // swizzle is the same and fragment a/b adds a constant)
  // Column map (BN = 160, 5 blocks per wave): wave wn owns the 64 columns 64 wn .. 64 wn + 63 as
  // two 16-B-store pairs, and the odd block at 128 + 16 wn, so every bf16 store segment is 64-B
  // aligned (an 80-column wave tile put wave 1's pairs across 64-B granules and wrote 1.6x,
  // profiles/r03w_gemm_traffic.txt). Rows stay 16-multiples apart: the LDS XOR is unchanged.
  constexpr bool ODDMAP = (C::NB % 2) == 1 && C::NB > 1;
  const int wcb = ODDMAP ? wn * 16 * (C::NB - 1) : wn * (BN / 2);  // the wave's first column
  const int wodd = ODDMAP ? 32 * (C::NB - 1) + 16 * wn : wcb + 16 * (C::NB - 1);  // odd block's column
  uint32_t wlane[BK / 32], xlane[BK / 32], wlodd[BK / 32];
#pragma unroll
  for (int ks = 0; ks < BK / 32; ++ks) {
    wlane[ks] = C::A_BYTES + 2 * lds_off(wcb + (lane & 15), ks * 4 + (lane >> 4));
    wlodd[ks] = wlane[ks] + (uint32_t)(wodd - wcb) * BK * 2;
    xlane[ks] = 2 * lds_off(wm * 64 + (lane & 15), ks * 4 + (lane >> 4));
  }
  // ---- compute cursor
  int cu = u_begin, ckt, ckt1;
  unit_kr(cu, ckt, ckt1);
  const int fr = lane & 15, fq = lane >> 4;
  int stage = 0;
  for (int it = 0; it < n_it; ++it) {
    // this wave's DMA for k-tile `it` has landed once at most k-tile it+1's remain
    // outstanding (everything issued before that, epilogue stores included, is done)
    if (it + 1 < n_it) {
      if (nbw == C::NBMAX) wait_vm<C::NA + C::NBMAX>();
      else wait_vm<C::NA + C::NBMAX - 1>();
    } else {
      wait_vm<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's DMA for `it` landed; stage (it-1)%3 fully read
    const char* sbase = smem + stage * C::STAGE;
    {
      bf16x8 wf[BK / 32][C::NB], xf[BK / 32][C::MB];
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
#pragma unroll
        for (int b = 0; b < C::MB; ++b) xf[ks][b] = *(const bf16x8*)(sbase + xlane[ks] + b * 16 * BK * 2);
#pragma unroll
        for (int a = 0; a < C::NB; ++a)
          wf[ks][a] = *(const bf16x8*)(sbase + (a == C::NB - 1 ? wlodd[ks] : wlane[ks] + a * 16 * BK * 2));
        if (ks == 0) __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks)
#pragma unroll
        for (int a = 0; a < C::NB; ++a)
#pragma unroll
          for (int b = 0; b < C::MB; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ks][a], xf[ks][b], acc[a][b], 0, 0, 0);
      {  // k-step 1's reads one per two of k-step 0's MFMAs
        constexpr int NR = C::MB + C::NB, NM = 2 * C::MB * C::NB;
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NM - 2 * NR, 0);
      }
    }
    if (++ckt == ckt1) {  // unit finished: epilogue (its memory ops precede the next DMA)
      const int tile = cu / split, sp = cu % split;
      const int64_t m0 = (int64_t)(tile / tiles_n) * G2_BM, n0 = (int64_t)(tile % tiles_n) * BN;
      if (split == 1) {
        gemm_epilogue<C::MB, C::NB>(d, acc, (int)m0 + wm * C::MB * 16, (int)n0 + wcb, lane,
                                    ODDMAP ? (int)n0 + wodd : -1);
      } else {  // split-K: raw fp32 slab ws[sp][m][n]; gemm_splitk_reduce applies the epilogue
        float* slab = (float*)d.ws + (int64_t)sp * M * N;
#pragma unroll
        for (int a = 0; a < C::NB; ++a) {
          const int64_t n = n0 + (a == C::NB - 1 ? wodd : wcb + a * 16) + 4 * fq;
          if (n >= N) continue;
#pragma unroll
          for (int b = 0; b < C::MB; ++b) {
            const int64_t m = m0 + wm * 64 + b * 16 + fr;
            if (m < M)
              *(float4*)(slab + m * N + n) = make_float4(acc[a][b][0], acc[a][b][1], acc[a][b][2], acc[a][b][3]);
          }
        }
      }
#pragma unroll
      for (int a = 0; a < C::NB; ++a)
#pragma unroll
        for (int b = 0; b < C::MB; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
      if ((cu += G) < units) unit_kr(cu, ckt, ckt1);
    }
    if (it + 2 < n_it) issue(stage == 0 ? 2 : stage - 1);
    stage = stage == 2 ? 0 : stage + 1;
  }
}



// Load-free epilogue (v5, split == 1, bf16 out, no residual / row bias): the bias
// comes from the unit's LDS slot (DMA'd with its first k-step) and every store is
// an UNCONDITIONAL buffer store whose out-of-range lanes carry an offset past the
// resource's num_records (dropped by the hardware).  So the epilogue issues no
// vector-memory load — nothing makes the wave wait for the k-steps still in flight
// — and a compile-time number of stores, which the k-loop's counted vmcnt then
// leaves outstanding instead of draining.  Returns that number.
template <int MB, int NB>
__device__ __forceinline__ int epi_fast(const vd_gemm_desc& d, f32x4 (&acc)[NB][MB], int mbase, int nbase, int lane,
                                        const float* bsl, int n0, __amdgpu_buffer_rsrc_t ro) {
  static_assert(NB % 2 == 0, "epi_fast: whole 16-column pairs");
  const int M = (int)d.M, N = (int)d.N, ldc = (int)d.ldc;
  const int fr = lane & 15, fq = lane >> 4;
  const int wcol = 16 * (fq & 1) + 8 * (fq >> 1);
  int nst = 0;
  if (d.act == VD_ACT_GEGLU) {
    // pairs (a, a+1) = (hidden, gate) blocks -> 16 output columns; pair-pairs swapped
    // by permlane16 into 8 consecutive columns per lane (16-B stores), a lone last
    // pair stores 4 columns (8 B)
    constexpr int NP = NB / 2;
#pragma unroll
    for (int pp = 0; pp + 1 < NP; pp += 2) {
      const int a = 2 * pp;
      const int c0 = nbase - n0 + a * 16 + 4 * fq;  // column of acc[a][.][0] inside the tile
      const float4 th0 = *(const float4*)(bsl + c0), tg0 = *(const float4*)(bsl + c0 + 16);
      const float4 th1 = *(const float4*)(bsl + c0 + 32), tg1 = *(const float4*)(bsl + c0 + 48);
      const float bh0[4] = {th0.x, th0.y, th0.z, th0.w}, bg0[4] = {tg0.x, tg0.y, tg0.z, tg0.w};
      const float bh1[4] = {th1.x, th1.y, th1.z, th1.w}, bg1[4] = {tg1.x, tg1.y, tg1.z, tg1.w};
      const int nout = nbase / 2 + pp * 16 + wcol;
#pragma unroll
      for (int b = 0; b < MB; ++b) {
        const int m = mbase + b * 16 + fr;
        uint32_t x[2], y[2];
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          // (h + bh) * gelu(g + bg) on value pairs: packed adds / multiplies, the same bits
          const f32x2 go = gelu_erf2(f32x2{acc[a + 1][b][2 * h2], acc[a + 1][b][2 * h2 + 1]} +
                                     f32x2{bg0[2 * h2], bg0[2 * h2 + 1]});
          const f32x2 gp = gelu_erf2(f32x2{acc[a + 3][b][2 * h2], acc[a + 3][b][2 * h2 + 1]} +
                                     f32x2{bg1[2 * h2], bg1[2 * h2 + 1]});
          const f32x2 oo = (f32x2{acc[a][b][2 * h2], acc[a][b][2 * h2 + 1]} + f32x2{bh0[2 * h2], bh0[2 * h2 + 1]}) * go;
          const f32x2 pp = (f32x2{acc[a + 2][b][2 * h2], acc[a + 2][b][2 * h2 + 1]} + f32x2{bh1[2 * h2], bh1[2 * h2 + 1]}) * gp;
          const float o0 = oo[0], o1 = oo[1], p0 = pp[0], p1 = pp[1];
          auto r = __builtin_amdgcn_permlane16_swap(pack2(o0, o1), pack2(p0, p1), false, false);
          x[h2] = r[0];
          y[h2] = r[1];
        }
        const bool ok = m < M && 2 * nout < N;
        const uint32_t off = ok ? (uint32_t)(m * ldc + nout) * 2u : G2_OOB;
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{x[0], x[1], y[0], y[1]}, ro, off, 0, 0);
        ++nst;
      }
    }
    if constexpr (NP % 2 == 1) {
      const int a = NB - 2;
      const int c0 = nbase - n0 + a * 16 + 4 * fq;
      const float4 th = *(const float4*)(bsl + c0), tg = *(const float4*)(bsl + c0 + 16);
      const float bh[4] = {th.x, th.y, th.z, th.w}, bg[4] = {tg.x, tg.y, tg.z, tg.w};
      const int nout = nbase / 2 + (a / 2) * 16 + 4 * fq;
#pragma unroll
      for (int b = 0; b < MB; ++b) {
        const int m = mbase + b * 16 + fr;
        float o[4];
        const f32x2 g01 = gelu_erf2(f32x2{acc[a + 1][b][0] + bg[0], acc[a + 1][b][1] + bg[1]});
        const f32x2 g23 = gelu_erf2(f32x2{acc[a + 1][b][2] + bg[2], acc[a + 1][b][3] + bg[3]});
        o[0] = (acc[a][b][0] + bh[0]) * g01[0];
        o[1] = (acc[a][b][1] + bh[1]) * g01[1];
        o[2] = (acc[a][b][2] + bh[2]) * g23[0];
        o[3] = (acc[a][b][3] + bh[3]) * g23[1];
        const bool ok = m < M && 2 * nout < N;
        const uint32_t off = ok ? (uint32_t)(m * ldc + nout) * 2u : G2_OOB;
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{pack2(o[0], o[1]), pack2(o[2], o[3])}, ro, off, 0, 0);
        ++nst;
      }
    }
    return nst;
  }
#pragma unroll
  for (int a = 0; a < NB; a += 2) {
    const int n = nbase + a * 16 + wcol;  // first of this lane's 8 columns after the swap
    const float4 t0 = *(const float4*)(bsl + (n - n0)), t1 = *(const float4*)(bsl + (n - n0) + 4);
    const float bv[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
#pragma unroll
    for (int b = 0; b < MB; ++b) {
      const int m = mbase + b * 16 + fr;
      float o[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[a][b][j]), __float_as_uint(acc[a + 1][b][j]),
                                                  false, false);
        o[j] = __uint_as_float(r[0]) + bv[j];
        o[4 + j] = __uint_as_float(r[1]) + bv[4 + j];
      }
      if (d.act == VD_ACT_SILU || d.act == VD_ACT_GELU) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = act_pw(d.act, o[j]);
      }
      const uint4 pk = pack8(o);
      const bool ok = m < M && n < N;
      const uint32_t off = ok ? (uint32_t)(m * ldc + n) * 2u : G2_OOB;
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{pk.x, pk.y, pk.z, pk.w}, ro, off, 0, 0);
      ++nst;
    }
  }
  return nst;
}

// ============================================================================ v3
// 256x256 tile, 8 waves as 2(M) x 4(N) (128 x 64 per wave: 0.375 LDS fragment
// reads per MFMA vs 0.45 for v2's 64 x 80), after the 8-phase template of
// cdna_hip_programming.md §5 "The 256² 8-phase template":
//  * a K-tile (BK = 64) is 4 phases, each one quadrant of the wave's C
//    (64 m x 32 n x K 64 = 16 MFMAs): Q(x0,w0) Q(x0,w1) Q(x1,w1) Q(x1,w0), so
//    the phases read 12 / 4 / 8 / 0 fragments (W0+X0, W1, X1, -);
//  * each K-tile's operands are four 16-KiB parts — X0 = A rows with
//    (r & 127) < 64, X1 the other A rows, W0 = W rows with (n & 63) < 32, W1 the
//    rest — one part DMA'd (buffer_load ... lds, 2 instructions per wave) per
//    phase, 6-7 phases before its first read, into the stage of the K-tile two
//    back (2 x 64 KiB); every part is restaged >= 1 phase after its last read
//    (lgkmcnt(0) retired the reads before the phase's MFMAs) and waited for by
//    a uniform counted vmcnt(10) (5 parts in flight) before the barrier ahead of
//    its first read;
//  * phase = [ds_reads | DMA | vmcnt] barrier lgkmcnt(0) setprio(1) MFMAs
//    setprio(0) barrier, and the wr = 1 wave group runs ONE BARRIER BEHIND the
//    wr = 0 group: on every SIMD (one wave of each group) one wave issues MFMAs
//    while the other reads LDS and issues DMA (ping-pong);
//  * the A (X) parts a wave group reads are DMA'd by that group only, so the
//    stagger never lets one group overwrite rows the other has yet to read; the
//    W parts, read by both groups, are restaged >= 2 phases after their reads.
// Persistent (round 2): a workgroup walks units lid, lid + G, ... (unit = output tile or
// one split-K slice of it, XCD-aware order with the N tiles of an A row-panel adjacent),
// and the K-tiles of all its units form ONE flat stream: the DMA of the next unit's first
// two K-tiles goes out during the last K-tiles of the current one, so the prologue's HBM
// burst and most of the epilogue's store tail overlap MFMA work (per-tile fixed cost,
// profiles/r02_v3_k_sweep.txt: 9.4 us per 256^2 tile vs 4.8 for hipBLASLt).  At a unit
// boundary the two wave groups re-align (group 0 one extra barrier), both run the
// epilogue, and group 1 re-staggers (one extra barrier) before the next unit's phase 0.
// Grid = units gives one unit per workgroup (the round-1 non-persistent kernel).
constexpr int G3_BM = 256, G3_BN = 256, G3_NT = 512;
constexpr int G3_A_BYTES = G3_BM * BK * 2;     // 32 KiB
constexpr int G3_STAGE = 2 * G3_A_BYTES;       // A + W: 64 KiB
// Load-free epilogue (round 2): for plain bf16 outputs (no residual / row bias, unsplit) with
// N <= G3_BIAS_N the whole bias vector is copied into LDS once, before the first DMA, and the
// epilogue is v5's epi_fast (bias from LDS, unconditional buffer stores).  gemm_epilogue's
// global bias loads made hipcc wait vmcnt(0) at every unit boundary — draining the next
// unit's two K-tiles of DMA under the epilogue (20 units per CU at the L1 GEGLU).
constexpr int G3_BIAS_N = 5120;

struct G3Cursor {  // a position (unit, local K-tile) in the workgroup's flat K-tile stream
  int u, t, kt0, nk, m0, n0;
};

template <int MODE>
__global__ __launch_bounds__(G3_NT, 1) void gemm3_kernel(const vd_gemm_desc d, uint32_t a0_bytes,
                                                         uint32_t a1_bytes, uint32_t w_bytes, int split,
                                                         int fast) {
  static_assert(MODE == VD_A_DENSE, "gemm3: dense A only");
  __shared__ __attribute__((aligned(1024))) char smem[2 * G3_STAGE + G3_BIAS_N * 4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int M = (int)d.M, N = (int)d.N;
  const int tiles_n = (N + G3_BN - 1) / G3_BN;
  const int units = ((M + G3_BM - 1) / G3_BM) * tiles_n * split;
  const int lid = xcd_remap(blockIdx.x, gridDim.x), G = gridDim.x;
  const int nk_all = (int)(d.K / BK);

  auto set_unit = [&](G3Cursor& c, int u) {
    c.u = u;
    c.t = 0;
    if (u < units) {
      const int tile = u / split, sp = u % split;
      c.kt0 = split == 1 ? 0 : nk_all * sp / split;  // 32-bit: nk_all * split < 2^31
      c.nk = (split == 1 ? nk_all : nk_all * (sp + 1) / split) - c.kt0;
      c.m0 = (tile / tiles_n) * G3_BM;
      c.n0 = (tile % tiles_n) * G3_BN;
    }
  };
  auto advance = [&](G3Cursor& c) {
    if (++c.t == c.nk) set_unit(c, c.u + G);
  };
  int total = 0;  // K-tiles this workgroup streams
  for (int u = lid; u < units; u += G) {
    G3Cursor c;
    set_unit(c, u);
    total += c.nk;
  }
  if (total == 0) return;

  const int rb = lane >> 3;
  const uint32_t lc16 = (uint32_t)(((lane & 7) ^ rb) * 16);
  const __amdgpu_buffer_rsrc_t ra0 = __builtin_amdgcn_make_buffer_rsrc((void*)d.a0, 0, a0_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ra1 =
      __builtin_amdgcn_make_buffer_rsrc((void*)(d.a1 ? d.a1 : d.a0), 0, d.a1 ? a1_bytes : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)d.w, 0, w_bytes, 0x00020000);
  const uint32_t lda0b = (uint32_t)d.lda0 * 2, lda1b = (uint32_t)d.lda1 * 2, ldwb = (uint32_t)d.ldw * 2;
  float* const bias_lds = (float*)(smem + 2 * G3_STAGE);
  const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(d.out, 0, (uint32_t)(M * d.ldc * 2), 0x00020000);
  if (fast) {  // the bias (or zeros) into LDS before any DMA is in flight; the prologue's
               // lgkmcnt(0) + s_barrier publish it
    for (int i = 4 * tid; i < N; i += 4 * G3_NT)
      *(float4*)(bias_lds + i) = d.bias ? *(const float4*)(d.bias + i) : make_float4(0.f, 0.f, 0.f, 0.f);
    __builtin_amdgcn_sched_barrier(0);
  }

  // DMA slots (wave-uniform LDS offsets; per-lane source rows from the cursor's tile): X part
  // q, slot j covers A rows 128*wr + 64*q + 8*(2*wc + j) + 0..7; W part q, slot j covers W
  // rows 64*c + 32*q + rr + 0..7 with (c, rr) from g = 2*wid + j.
  auto dma_x = [&](int q, const G3Cursor& c, int T) {  // X part q of flat K-tile T (at cursor c)
    char* st = smem + (T & 1) * G3_STAGE;
    const int kb = (c.kt0 + c.t) * BK;
    const bool s0 = kb < (int)d.k0;
    const uint32_t koff = (uint32_t)(s0 ? kb : kb - (int)d.k0) * 2;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int xr = 128 * wr + 64 * q + 8 * (2 * wc + j);
      int m = c.m0 + xr + rb;
      m = m < M ? m : M - 1;
      dma16(s0 ? ra0 : ra1, st + xr * 128, (uint32_t)m * (s0 ? lda0b : lda1b) + lc16 + koff);
    }
  };
  auto dma_w = [&](int q, const G3Cursor& c, int T) {
    char* st = smem + (T & 1) * G3_STAGE;
    const uint32_t koff = (uint32_t)((c.kt0 + c.t) * BK) * 2;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int g = 2 * wid + j;
      const int wrow = 64 * (g >> 2) + 32 * q + 8 * (g & 3);
      int n = c.n0 + wrow + rb;
      n = n < N ? n : N - 1;
      dma16(rw, st + G3_A_BYTES + wrow * 128, (uint32_t)n * ldwb + lc16 + koff);
    }
  };

  // fragment LDS offsets (bytes within a stage): rows differ by multiples of 16
  // between the blocks of one operand, so the (row & 7) XOR is shared
  const int fr = lane & 15, fq = lane >> 4;
  uint32_t xl[2][2], wl[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      xl[h][ks] = 2 * lds_off(128 * wr + 64 * h + fr, ks * 4 + fq);
      wl[h][ks] = G3_A_BYTES + 2 * lds_off(64 * wc + 32 * h + fr, ks * 4 + fq);
    }

  f32x4 acc[4][8];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // cursors of flat K-tiles T (compute), T+1 and T+2 (DMA)
  G3Cursor c0, c1, c2;
  set_unit(c0, lid);
  c1 = c0;
  advance(c1);
  c2 = c1;
  advance(c2);
  // ---- prologue: K-tile 0 complete, K-tile 1's X0/W0/W1 in flight
  dma_x(0, c0, 0); dma_w(0, c0, 0); dma_w(1, c0, 0); dma_x(1, c0, 0);
  if (total > 1) {
    dma_x(0, c1, 1); dma_w(0, c1, 1); dma_w(1, c1, 1);
    wait_vm<10>();
  } else {
    wait_vm<0>();
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // the stagger

  bf16x8 w0f[2][2], w1f[2][2], xf[4][2];
  for (int T = 0; T < total; ++T) {
    const char* st = smem + (T & 1) * G3_STAGE;
    const bool deep = T + 2 < total;
#define G3_SYNC_MFMA(H, G_, WF)                                                                    \
    if (deep) wait_vm<10>(); else wait_vm<0>();                                                     \
    __builtin_amdgcn_s_barrier();                                                                   \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                              \
    __builtin_amdgcn_s_setprio(1);                                                                  \
    _Pragma("unroll") for (int ks = 0; ks < 2; ++ks)                                                \
      _Pragma("unroll") for (int a = 0; a < 2; ++a)                                                 \
        _Pragma("unroll") for (int b = 0; b < 4; ++b)                                               \
          acc[2 * (G_) + a][4 * (H) + b] =                                                          \
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(WF[a][ks], xf[b][ks], acc[2 * (G_) + a][4 * (H) + b], 0, 0, 0); \
    __builtin_amdgcn_s_setprio(0);                                                                  \
    __builtin_amdgcn_s_barrier();
    // ---- phase 0: read W0, X0; DMA X1 of T+1; Q(x0, w0)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) w0f[a][ks] = *(const bf16x8*)(st + wl[0][ks] + a * 16 * BK * 2);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) xf[b][ks] = *(const bf16x8*)(st + xl[0][ks] + b * 16 * BK * 2);
    if (T + 1 < total) dma_x(1, c1, T + 1);
    G3_SYNC_MFMA(0, 0, w0f)
    // ---- phase 1: read W1; DMA X0 of T+2; Q(x0, w1)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) w1f[a][ks] = *(const bf16x8*)(st + wl[1][ks] + a * 16 * BK * 2);
    if (deep) dma_x(0, c2, T + 2);
    G3_SYNC_MFMA(0, 1, w1f)
    // ---- phase 2: read X1; DMA W0 of T+2; Q(x1, w1)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) xf[b][ks] = *(const bf16x8*)(st + xl[1][ks] + b * 16 * BK * 2);
    if (deep) dma_w(0, c2, T + 2);
    G3_SYNC_MFMA(1, 1, w1f)
    // ---- phase 3: DMA W1 of T+2; Q(x1, w0)
    if (deep) dma_w(1, c2, T + 2);
    G3_SYNC_MFMA(1, 0, w0f)
#undef G3_SYNC_MFMA
    if (c0.t + 1 == c0.nk) {  // unit finished
      if (wr == 0) __builtin_amdgcn_s_barrier();  // re-align the groups
      const int mbase = c0.m0 + 128 * wr, nbase = c0.n0 + 64 * wc;
      if (fast) {
        epi_fast<8, 4>(d, acc, mbase, nbase, lane, bias_lds + c0.n0, c0.n0, rout);
      } else if (split == 1) {
        gemm_epilogue<8, 4>(d, acc, mbase, nbase, lane);
      } else {  // split-K: raw fp32 slab ws[sp][m][n]; gemm_splitk_reduce applies the epilogue
        float* slab = (float*)d.ws + (int64_t)(c0.u % split) * d.M * d.N;
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          const int64_t n = nbase + a * 16 + 4 * fq;
          if (n >= N) continue;
#pragma unroll
          for (int b = 0; b < 8; ++b) {
            const int64_t m = mbase + b * 16 + fr;
            if (m < M) *(float4*)(slab + m * d.N + n) = make_float4(acc[a][b][0], acc[a][b][1], acc[a][b][2], acc[a][b][3]);
          }
        }
      }
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (wr == 1 && T + 1 < total) __builtin_amdgcn_s_barrier();  // re-stagger
    }
    advance(c0);
    advance(c1);
    advance(c2);
  }
}

// ============================================================================ v5
// Persistent 256 x 320 GEMM / implicit-GEMM conv, BK = 32, 8 waves as 4(M) x 2(N)
// (64 x 160 per wave: 4 x 10 accumulators of 16x16), 4-stage LDS-DMA ring (36 KiB per
// stage, three k-steps in flight), persistent strided unit walk as v2.  320 divides
// every N of the UNet (320 ... 10240): no padding.  One raw s_barrier per k-step behind
// a counted vmcnt; the DMA for k-step it+3 goes out right after the barrier of k-step
// it into the stage read at it-1.  Load-free epilogue (epi_fast) where it applies: the
// stores stay in flight across the next k-steps' counted waits.
// Measured against v2/v3 (tools/kbench.py): wins on the L1 attention QKV
// projection (M 131072, K 320, N 960: 145 vs 169 us), ties or loses elsewhere — the
// k-loop is bound by LDS-read / MFMA phase lock of the two waves on each SIMD and by
// the DMA of 64-B row segments, which neither two workgroups per CU, a dedicated
// L2-prefetch wave nor a two-group ping-pong schedule (all built and measured this
// round) removed.
// LDS operand image: rows of 64 B (4 chunks of 16 B); logical chunk c of row r
// sits in physical chunk c ^ ((r >> 2) & 2), which makes the 16x16x32 fragment
// reads (ds_read_b128: 16-lane groups over rows 0-3/12-15 and 4-11) conflict
// free.  The permutation is applied to the per-lane DMA SOURCE address, the
// image stays lane-linear (cdna_hip_programming.md rule 21).
constexpr int G4_BM = 256, G4_BK = 32;

template <int BN, int WM, int WN, int STAGES>
struct G4 {
  static constexpr int NT = WM * WN * 64;
  static constexpr int NW = WM * WN;
  static constexpr int A_BYTES = G4_BM * G4_BK * 2;  // 16 KiB
  static constexpr int B_BYTES = BN * G4_BK * 2;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int NPA = G4_BM / 16;             // A DMA pieces (16 rows x 64 B = 1 KiB) per k-step
  static constexpr int NPB = BN / 16;                // W DMA pieces per k-step
  // wave w issues A pieces w + NW*j (j < NAMAX) and W pieces w + NW*j (j < NBMAX)
  static constexpr int NAMAX = (NPA + NW - 1) / NW;
  static constexpr int NBMAX = (NPB + NW - 1) / NW;
  static constexpr int WROWS = G4_BM / WM, WCOLS = BN / WN;
  static constexpr int MB = WROWS / 16, NB = WCOLS / 16;
  // a ring of 4 per-unit bias slots (2 KiB each: two 1-KiB DMA pieces) for epi_fast
  static constexpr int BIAS_SLOTS = 4;
  static constexpr int LDS_BYTES = STAGES * STAGE + BIAS_SLOTS * 2048;
  static_assert(BN % (16 * WN) == 0 && G4_BM % (16 * WM) == 0, "tile / wave grid mismatch");
};

__device__ __forceinline__ uint32_t g4_off(int row, int chunk) {  // byte offset in an operand image
  return (uint32_t)(row * 64 + ((chunk ^ ((row >> 2) & 2)) << 4));
}

// s_waitcnt vmcnt(n) (expcnt / lgkmcnt left at max) for a wave-uniform runtime n;
// n > 63 waits for 63 (more than asked: always safe).
template <int N>
__device__ __forceinline__ void s_wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}
__device__ __forceinline__ void wait_vm_rt(int n) {
#define VM4(B) case B: s_wait_vm<B>(); break; case B + 1: s_wait_vm<B + 1>(); break; \
               case B + 2: s_wait_vm<B + 2>(); break; case B + 3: s_wait_vm<B + 3>(); break;
  switch (n) {
    VM4(0) VM4(4) VM4(8) VM4(12) VM4(16) VM4(20) VM4(24) VM4(28)
    VM4(32) VM4(36) VM4(40) VM4(44) VM4(48) VM4(52) VM4(56) VM4(60)
    default: s_wait_vm<63>(); break;
  }
#undef VM4
}

// Epilogue with the next LayerNorm fused (vd_gemm_desc.ln_out; v5 with N == BN == 320, so
// the workgroup's tile owns whole rows): x = bf16(acc + bias (+ res)) is stored as usual and
// kept in registers; row sums of the rounded x (lane: 4 columns x NB blocks; then the 4 lanes
// of a row by xor shuffles; then the WN = 2 column waves through `red` in LDS), mean, the
// two-pass variance the same way, and ln_out = fmaf((x - mean) * rstd, gamma, beta) (+ pe)
// — vd_layernorm's arithmetic on the same bf16 x (only the fp32 summation order differs).
// Every wave of the workgroup runs it (two s_barriers).
template <int MB, int NB>
__device__ __forceinline__ void epi_ln(const vd_gemm_desc& d, f32x4 (&acc)[NB][MB], int mbase, int nbase, int lane,
                                       int rloc, int wn, float* red) {
  static_assert(NB % 2 == 0, "epi_ln: whole 16-column pairs");
  const int M = (int)d.M, N = (int)d.N;
  const int fr = lane & 15, fq = lane >> 4;
  const int wcol = 16 * (fq & 1) + 8 * (fq >> 1);  // lane's first column inside a swapped pair
  bf16_t* out = (bf16_t*)d.out;
  // x: v_permlane16_swap of blocks (a, a+1) leaves each lane 8 consecutive columns of its row
  // (16-B residual loads and stores, as gemm_epilogue's wide path); the rounded x stays in acc
  // in that swapped order (a row's statistics do not depend on it)
#pragma unroll
  for (int a = 0; a < NB; a += 2) {
    const int n = nbase + a * 16 + wcol;
    float bv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (d.bias) {
      const float4 t0 = *(const float4*)(d.bias + n), t1 = *(const float4*)(d.bias + n + 4);
      bv[0] = t0.x; bv[1] = t0.y; bv[2] = t0.z; bv[3] = t0.w;
      bv[4] = t1.x; bv[5] = t1.y; bv[6] = t1.z; bv[7] = t1.w;
    }
    // the MB residual rows of this column pair load together, ahead of the stores below (round 2):
    // hipcc cannot move a residual load above an earlier `out` store (they may alias), so one
    // load per row interleaved with the stores made MB dependent HBM round trips per pair
    // (fused LN + residual at L1: 119 -> 110 us; gamma / beta staged in LDS as well spilled)
    uint4 rsv[MB];
    if (d.res) {
#pragma unroll
      for (int b = 0; b < MB; ++b) {
        const int m = mbase + b * 16 + fr;
        rsv[b] = *(const uint4*)((const bf16_t*)d.res + (uint32_t)((m < M ? m : 0) * (int)d.ld_res + n));
      }
    }
#pragma unroll
    for (int b = 0; b < MB; ++b) {
      const int m = mbase + b * 16 + fr;
      const bool mok = m < M;
      const int mrow = mok ? m : 0;
      float o[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[a][b][j]), __float_as_uint(acc[a + 1][b][j]),
                                                  false, false);
        o[j] = __uint_as_float(r[0]) + bv[j];
        o[4 + j] = __uint_as_float(r[1]) + bv[4 + j];
      }
      if (d.res) {
        float rf[8];
        unpack8(rsv[b], rf);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += rf[j];
      }
      const uint4 pk = pack8(o);
      if (mok) *(uint4*)(out + (uint32_t)(mrow * (int)d.ldc + n)) = pk;
      float x8[8];
      unpack8(pk, x8);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[a][b][j] = x8[j];
        acc[a + 1][b][j] = x8[4 + j];
      }
    }
  }
  float mean[MB], rstd[MB];
#pragma unroll
  for (int b = 0; b < MB; ++b) {
    float sm = 0.f;
#pragma unroll
    for (int a = 0; a < NB; ++a)
#pragma unroll
      for (int j = 0; j < 4; ++j) sm += acc[a][b][j];
    sm += __shfl_xor(sm, 16, 64);
    sm += __shfl_xor(sm, 32, 64);
    mean[b] = sm;
    if (fq == 0) red[wn * 256 + rloc + b * 16 + fr] = sm;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int b = 0; b < MB; ++b) mean[b] = (mean[b] + red[(1 - wn) * 256 + rloc + b * 16 + fr]) / (float)N;
#pragma unroll
  for (int b = 0; b < MB; ++b) {
    float s2 = 0.f;
#pragma unroll
    for (int a = 0; a < NB; ++a)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float t = acc[a][b][j] - mean[b];
        s2 = fmaf(t, t, s2);
      }
    s2 += __shfl_xor(s2, 16, 64);
    s2 += __shfl_xor(s2, 32, 64);
    rstd[b] = s2;
    if (fq == 0) red[512 + wn * 256 + rloc + b * 16 + fr] = s2;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int b = 0; b < MB; ++b)
    rstd[b] = rsqrtf((rstd[b] + red[512 + (1 - wn) * 256 + rloc + b * 16 + fr]) / (float)N + d.ln_eps);
  bf16_t* y = (bf16_t*)d.ln_out;
  int perow[MB];  // element offset of row m's PE row (m clamped; unused without ln_pe)
#pragma unroll
  for (int b = 0; b < MB; ++b) {
    const int m = mbase + b * 16 + fr;
    perow[b] = d.ln_pe ? ((m < M ? m : 0) / (int)d.ln_pe_div) % (int)d.ln_pe_period * N : 0;
  }
#pragma unroll
  for (int a = 0; a < NB; a += 2) {
    const int n = nbase + a * 16 + wcol;
    const float4 g0 = *(const float4*)(d.ln_gamma + n), g1 = *(const float4*)(d.ln_gamma + n + 4);
    const float4 b0 = *(const float4*)(d.ln_beta + n), b1 = *(const float4*)(d.ln_beta + n + 4);
    const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
    for (int b = 0; b < MB; ++b) {
      const int m = mbase + b * 16 + fr;
      if (m >= M) continue;
      float o[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[j] = fmaf((acc[a][b][j] - mean[b]) * rstd[b], gg[j], bb[j]);
        o[4 + j] = fmaf((acc[a + 1][b][j] - mean[b]) * rstd[b], gg[4 + j], bb[4 + j]);
      }
      if (d.ln_pe) {
        const float4 t0 = *(const float4*)(d.ln_pe + perow[b] + n), t1 = *(const float4*)(d.ln_pe + perow[b] + n + 4);
        o[0] += t0.x; o[1] += t0.y; o[2] += t0.z; o[3] += t0.w;
        o[4] += t1.x; o[5] += t1.y; o[6] += t1.z; o[7] += t1.w;
      }
      *(uint4*)(y + (uint32_t)(m * (int)d.ld_ln + n)) = pack8(o);
    }
  }
}

template <int BN, int WM, int WN, int STAGES, int MODE, bool LN = false>
__global__ __attribute__((amdgpu_flat_work_group_size(1, WM * WN * 64), amdgpu_waves_per_eu(2))) void gemm4_kernel(
    const vd_gemm_desc d, uint32_t a0_bytes, uint32_t a1_bytes, uint32_t w_bytes, int split) {
  using C = G4<BN, WM, WN, STAGES>;
  __shared__ __attribute__((aligned(1024))) char smem[C::LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int64_t M = d.M, N = d.N, K = d.K;
  const int tiles_n = (int)((N + BN - 1) / BN);
  const int tiles_m = (int)((M + G4_BM - 1) / G4_BM);
  const int units = tiles_n * tiles_m * split;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);  // see v2: XCD-contiguous strided walk
  const int G = gridDim.x;
  const int nk_all = (int)(K / G4_BK);

  const int rb = lane >> 2;                                               // row within the 16-row DMA piece
  const uint32_t lc16 = (uint32_t)(((lane & 3) ^ ((rb >> 2) & 2)) * 16);  // logical source chunk (bytes)
  const __amdgpu_buffer_rsrc_t ra0 = __builtin_amdgcn_make_buffer_rsrc((void*)d.a0, 0, a0_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ra1 =
      __builtin_amdgcn_make_buffer_rsrc((void*)(d.a1 ? d.a1 : d.a0), 0, d.a1 ? a1_bytes : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)d.w, 0, w_bytes, 0x00020000);
  // this wave's pieces per k-step
  const int na_w = (C::NPA - wid + C::NW - 1) / C::NW;
  const int nb_w = (C::NPB - wid + C::NW - 1) / C::NW;
  const int per_step = na_w + nb_w;
  const int cin = MODE == VD_A_CONV3X3 ? (int)(K / 9) : 0;
  const int hgrid = d.upsample ? 2 * d.h_in : d.h_in;
  const int wgrid = d.upsample ? 2 * d.w_in : d.w_in;
  // load-free epilogue (epi_fast) for plain bf16 outputs
  const bool fast = !LN && split == 1 && !d.res && !d.rowbias && !d.out_f32 && !d.rmap_inner && (N % 8) == 0 &&
                    (d.ldc % 8) == 0 && (((uintptr_t)d.out) & 15) == 0;
  const __amdgpu_buffer_rsrc_t rbias = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(d.bias ? d.bias : (const float*)d.a0), 0, d.bias ? (uint32_t)(N * 4) : 0u, 0x00020000);
  const __amdgpu_buffer_rsrc_t rout =
      __builtin_amdgcn_make_buffer_rsrc(d.out, 0, (uint32_t)(M * d.ldc * 2), 0x00020000);
  int iun = 0, cun = 0;  // per-workgroup unit ordinals of the issue and compute cursors (bias slot)

  // ---- issue cursor: the (unit, k-step) whose DMA goes out next
  int iu = lid, ikt = 0, ikt1 = 0;
  uint32_t boff[C::NBMAX], aoff0[C::NAMAX], aoff1[C::NAMAX];
  // conv rows: base pixel of the row's image and its (oh, ow) packed 16:16
  int pimg[C::NAMAX], pohw[C::NAMAX];
  int c_tap = 0, c_ci = 0;
  bool c_new = true;
  // (an early-out for split == 1 here measured 15 % slower on the dense v2 GEMMs, same box,
  // profiles/r03t_unit_kr_bisect.txt: it changes how hipcc lays out the persistent unit loop)
  auto unit_kr = [&](int u, int& kt0, int& kt1) {
    const int sp = u % split;
    kt0 = (int)((int64_t)nk_all * sp / split);
    kt1 = (int)((int64_t)nk_all * (sp + 1) / split);
  };
  auto setup_unit = [&](int u) {
    const int tile = u / split;
    const int64_t m0 = (int64_t)(tile / tiles_n) * G4_BM, n0 = (int64_t)(tile % tiles_n) * BN;
    int kt0;
    unit_kr(u, kt0, ikt1);
    ikt = kt0;
#pragma unroll
    for (int j = 0; j < C::NBMAX; ++j) {
      int64_t n = n0 + (wid + C::NW * j) * 16 + rb;
      n = n < N ? n : N - 1;
      boff[j] = (uint32_t)(n * d.ldw * 2) + lc16;
    }
    if constexpr (MODE == VD_A_DENSE) {
#pragma unroll
      for (int j = 0; j < C::NAMAX; ++j) {
        int64_t m = m0 + (wid + C::NW * j) * 16 + rb;
        m = m < M ? m : M - 1;
        aoff0[j] = (uint32_t)(m * d.lda0 * 2) + lc16;
        aoff1[j] = (uint32_t)(m * d.lda1 * 2) + lc16;
      }
    } else {
      const int hw = d.h_out * d.w_out;
      const Div dhw(hw), dw(d.w_out);
#pragma unroll
      for (int j = 0; j < C::NAMAX; ++j) {
        int m = (int)m0 + (wid + C::NW * j) * 16 + rb;
        m = m < (int)M ? m : (int)M - 1;
        const int img = dhw(m);
        const int p = m - img * hw;
        const int oh = dw(p);
        pimg[j] = img * d.h_in * d.w_in;
        pohw[j] = (oh << 16) | (p - oh * d.w_out);
      }
      c_tap = kt0 * G4_BK / cin;
      c_ci = kt0 * G4_BK - c_tap * cin;
      c_new = true;
    }
  };
  auto issue = [&](int stage) {  // DMA of the cursor's k-step into `stage`, then advance the cursor
    char* la = smem + stage * C::STAGE;
    char* lb = la + C::A_BYTES;
    const int kb = ikt * G4_BK;
    {
      if (fast && wid == 0 && ikt == (int)((int64_t)nk_all * (iu % split) / split)) {
        // first k-step of a unit: its BN bias values (zeros past N or without bias) into slot iun & 3
        char* bs = smem + STAGES * C::STAGE + (iun & (C::BIAS_SLOTS - 1)) * 2048;
        const uint32_t nb0 = (uint32_t)((iu / split) % tiles_n) * BN * 4 + lane * 16;
        dma16(rbias, bs, nb0);
        dma16(rbias, bs + 1024, nb0 + 1024);
      }
      if constexpr (MODE == VD_A_DENSE) {
        const bool s0 = kb < (int)d.k0;
        const uint32_t koff = (uint32_t)(s0 ? kb : kb - (int)d.k0) * 2;
#pragma unroll
        for (int j = 0; j < C::NAMAX; ++j)
          if (j < na_w) dma16(s0 ? ra0 : ra1, la + (wid + C::NW * j) * 1024, (s0 ? aoff0[j] : aoff1[j]) + koff);
      } else {
        if (c_new) {  // new tap: recompute the rows' pixel offsets
          c_new = false;
          const int dy = c_tap / 3, dx = c_tap - 3 * dy;
#pragma unroll
          for (int j = 0; j < C::NAMAX; ++j) {
            int ih = (pohw[j] >> 16) * d.stride + dy - 1, iw = (pohw[j] & 0xffff) * d.stride + dx - 1;
            const bool ok = ((uint32_t)ih < (uint32_t)hgrid) & ((uint32_t)iw < (uint32_t)wgrid);  // branch-free
            ih >>= d.upsample;
            iw >>= d.upsample;
            const uint32_t pix = (uint32_t)(pimg[j] + ih * d.w_in + iw);
            aoff0[j] = ok ? pix * (uint32_t)(d.lda0 * 2) + lc16 : G2_OOB;
            aoff1[j] = ok ? pix * (uint32_t)(d.lda1 * 2) + lc16 : G2_OOB;
          }
        }
        const bool s0 = c_ci < (int)d.k0;
        const uint32_t coff = (uint32_t)(s0 ? c_ci : c_ci - (int)d.k0) * 2;
#pragma unroll
        for (int j = 0; j < C::NAMAX; ++j) {
          const uint32_t o = s0 ? aoff0[j] : aoff1[j];
          if (j < na_w) dma16(s0 ? ra0 : ra1, la + (wid + C::NW * j) * 1024, o + coff);
        }
      }
#pragma unroll
      for (int j = 0; j < C::NBMAX; ++j)
        if (j < nb_w) dma16(rw, lb + (wid + C::NW * j) * 1024, boff[j] + (uint32_t)kb * 2);
    }
    if constexpr (MODE == VD_A_CONV3X3) {
      c_ci += G4_BK;
      if (c_ci == cin) { c_ci = 0; ++c_tap; c_new = true; }
    }
    if (++ikt == ikt1) {
      ++iun;
      if ((iu += G) < units) setup_unit(iu);
    }
  };

  f32x4 acc[C::NB][C::MB];
#pragma unroll
  for (int a = 0; a < C::NB; ++a)
#pragma unroll
    for (int b = 0; b < C::MB; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  int n_it = 0;
  for (int u = lid; u < units; u += G) {
    int a0_, a1_;
    unit_kr(u, a0_, a1_);
    n_it += a1_ - a0_;
  }
  if (n_it == 0) return;
  setup_unit(lid);
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < n_it) issue(s);
  const int fr = lane & 15, fq = lane >> 4;
  const uint32_t wlane = C::A_BYTES + g4_off(wn * C::WCOLS + fr, fq);
  const uint32_t xlane = g4_off(wm * C::WROWS + fr, fq);
  int cu = lid, ckt, ckt1;
  unit_kr(cu, ckt, ckt1);
  int stage = 0;
  int st1 = 0, st2 = 0, st3 = 0;  // epilogue stores issued 1, 2, 3 iterations ago (still younger than k-step it's DMA)
  for (int it = 0; it < n_it; ++it) {
    // this wave's DMA for k-step `it` has landed once only the younger k-steps' (at
    // most S-2 of them) remain outstanding, plus the epilogue stores issued since
    // k-step it's DMA went out (iterations it-S+1 .. it-1); the barrier then publishes
    // every wave's part and certifies that stage (it-1)%S, the target of the next
    // issue, is no longer read.
    {
      const int younger = n_it - 1 - it < STAGES - 2 ? n_it - 1 - it : STAGES - 2;
      const int pend = st1 + (STAGES >= 3 ? st2 : 0) + (STAGES >= 4 ? st3 : 0);
      wait_vm_rt(younger * per_step + pend);
    }
    st3 = st2;
    st2 = st1;
    st1 = 0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (it + STAGES - 1 < n_it) issue(stage == 0 ? STAGES - 1 : stage - 1);
    const char* sbase = smem + stage * C::STAGE;
    if constexpr (C::MB == 8) {
      // W once, X in two halves of 4 (caps the live fragment registers)
      bf16x8 wf[C::NB], xf[4];
#pragma unroll
      for (int a = 0; a < C::NB; ++a) wf[a] = *(const bf16x8*)(sbase + wlane + a * 1024);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int b = 0; b < 4; ++b) xf[b] = *(const bf16x8*)(sbase + xlane + (4 * h + b) * 1024);
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
          for (int a = 0; a < C::NB; ++a)
            acc[a][4 * h + b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[a], xf[b], acc[a][4 * h + b], 0, 0, 0);
      }
    } else {
      // X once; W fragments two ahead in a rolling window (round 2): each W read issues under the
      // MFMAs of the fragment two before it, pinned by sched_group_barrier — the halves below let
      // hipcc wait lgkmcnt on every pair right before its MFMAs
      bf16x8 xf[C::MB];
#pragma unroll
      for (int b = 0; b < C::MB; ++b) xf[b] = *(const bf16x8*)(sbase + xlane + b * 1024);
      bf16x8 w0 = *(const bf16x8*)(sbase + wlane), w1 = *(const bf16x8*)(sbase + wlane + 1024);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int a = 0; a < C::NB; ++a) {
        bf16x8 wn = w1;
        if (a + 2 < C::NB) wn = *(const bf16x8*)(sbase + wlane + (a + 2) * 1024);
#pragma unroll
        for (int b = 0; b < C::MB; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, xf[b], acc[a][b], 0, 0, 0);
        w0 = w1;
        w1 = wn;
      }
#pragma unroll
      for (int a = 0; a < C::NB; ++a) {
        if (a + 2 < C::NB) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, C::MB, 0);
      }
    }
    if (++ckt == ckt1) {  // unit finished: epilogue
      const int tile = cu / split, sp = cu % split;
      const int64_t m0 = (int64_t)(tile / tiles_n) * G4_BM, n0 = (int64_t)(tile % tiles_n) * BN;
      bool done = false;
      if constexpr (LN) {  // plan: N == BN, split == 1; the bias slots (unused without `fast`) hold `red`
        static_assert(WN == 2 && C::BIAS_SLOTS * 2048 >= 4096, "epi_ln: two column waves, 4 KiB of LDS");
        epi_ln<C::MB, C::NB>(d, acc, (int)m0 + wm * C::WROWS, (int)n0 + wn * C::WCOLS, lane, wm * C::WROWS, wn,
                             (float*)(smem + STAGES * C::STAGE));
        done = true;
      } else if (fast) {
        const float* bsl = (const float*)(smem + STAGES * C::STAGE + (cun & (C::BIAS_SLOTS - 1)) * 2048);
        st1 = epi_fast<C::MB, C::NB>(d, acc, (int)m0 + wm * C::WROWS, (int)n0 + wn * C::WCOLS, lane, bsl,
                                     (int)n0, rout);
        done = true;
      }
      if (!LN && !done) {
        if (split == 1) {
          gemm_epilogue<C::MB, C::NB>(d, acc, (int)m0 + wm * C::WROWS, (int)n0 + wn * C::WCOLS, lane);
        } else {  // split-K: raw fp32 slab ws[sp][m][n]; gemm_splitk_reduce applies the epilogue
          float* slab = (float*)d.ws + (int64_t)sp * M * N;
#pragma unroll
          for (int a = 0; a < C::NB; ++a) {
            const int64_t n = n0 + wn * C::WCOLS + a * 16 + 4 * fq;
            if (n >= N) continue;
#pragma unroll
            for (int b = 0; b < C::MB; ++b) {
              const int64_t m = m0 + wm * C::WROWS + b * 16 + fr;
              if (m < M)
                *(float4*)(slab + m * N + n) = make_float4(acc[a][b][0], acc[a][b][1], acc[a][b][2], acc[a][b][3]);
            }
          }
        }
      }
#pragma unroll
      for (int a = 0; a < C::NB; ++a)
#pragma unroll
        for (int b = 0; b < C::MB; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
      ++cun;
      if ((cu += G) < units) unit_kr(cu, ckt, ckt1);
    }
    stage = stage == STAGES - 1 ? 0 : stage + 1;
  }
}

// ============================================================================ v6
// Small-M GEMM / implicit-GEMM conv: tile 64 x 64, BK = 64, 4 waves as 2 x 2 (32 x 32
// per wave), 3-stage LDS-DMA ring (48 KiB: three workgroups per CU), one workgroup
// per (tile, K-slice) — non-persistent, so the grid fills the chip at the M of a
// frame-sharded rank (M = 256 ... 16384 rows at 2-8 frames per GPU), where the
// 256-row v2/v3/v5 tiles leave most CUs idle and split K into a separate reduce
// launch.  Split K is reduced IN the kernel: every slice writes its fp32 slab, and the
// last slice to arrive at the tile's counter sums the slabs and runs the epilogue
// (cdna_hip_programming.md §5 "Projection GEMM at M = 256" item 2: plain slab stores
// -> every wave s_waitcnt vmcnt(0) -> barrier -> lane 0 agent release fence + asm
// vmcnt(0) -> relaxed agent atomic add; the last arriver: agent acquire fence + asm
// vmcnt(0) -> barrier -> plain slab loads).  The counters live in the workspace after
// the slabs and are zeroed by a memset node ahead of the launch; the last arriver
// also resets its counter.
// The ring depth S is picked per launch: 3 stages (48 KiB, three workgroups per CU) when
// the grid oversubscribes the CUs, 4 / 6 stages (2 / 1 per CU) on small grids, where
// each workgroup's k-loop is latency-bound and more tiles in flight pay directly.
// LNF (round 5, vd_gemm_desc.ln_fold_s; dense, unsplit): the LayerNorm of A's rows folded in, as
// v8's: per k-step two more MFMAs per X fragment the wave already holds — ones·x (Σx in every entry)
// and x·xᵀ (Σx² on the Gram block's diagonal) — in a loop that runs far below the MFMA pipe's rate at
// these M (dot-2 VALU for the same sums cost ≈ 10 cycles each beside the MFMAs and 1.5-3x the time,
// MI355X_MICROARCH.md "price of one filler"); the accumulators become rstd·(acc − mean·s[n]) before
// the common epilogue adds b' (the folded bias) and any row bias (the motion block's W·pe[frame]).
// Rows with |mean| / std > 16 take v8's exact second pass (re-read from L2).
constexpr int G6_BM = 64, G6_BN = 64, G6_NT = 256;
constexpr int G6_A = G6_BM * BK * 2, G6_W = G6_BN * BK * 2, G6_STAGE = G6_A + G6_W;  // 8 + 8 KiB

template <int MODE, int G6_S, bool LNF = false>  // all fragment reads of a K-tile ahead of its MFMAs (as gemm2)
__global__ __launch_bounds__(G6_NT, G6_S == 3 ? 3 : (G6_S == 4 ? 2 : 1)) void gemm6_kernel(
    const vd_gemm_desc d, uint32_t a0_bytes, uint32_t a1_bytes, uint32_t w_bytes, int split) {
  constexpr int MB = 2, NB = 2;
  __shared__ __attribute__((aligned(1024))) char smem[G6_S * G6_STAGE + 16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int64_t M = d.M, N = d.N, K = d.K;
  const int tiles_n = (int)((N + G6_BN - 1) / G6_BN);
  const int lid = xcd_remap(blockIdx.x, gridDim.x);  // a tile's K-slices adjacent (one XCD)
  const int tile = lid / split, sp = lid % split;
  const int64_t m0 = (int64_t)(tile / tiles_n) * G6_BM, n0 = (int64_t)(tile % tiles_n) * G6_BN;
  const int nk_all = (int)(K / BK);
  const int kt0 = split == 1 ? 0 : nk_all * sp / split, kt1 = split == 1 ? nk_all : nk_all * (sp + 1) / split;
  const int nk = kt1 - kt0;

  const int rb = lane >> 3;
  const uint32_t lc16 = (uint32_t)(((lane & 7) ^ rb) * 16);
  const __amdgpu_buffer_rsrc_t ra0 = __builtin_amdgcn_make_buffer_rsrc((void*)d.a0, 0, a0_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ra1 =
      __builtin_amdgcn_make_buffer_rsrc((void*)(d.a1 ? d.a1 : d.a0), 0, d.a1 ? a1_bytes : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)d.w, 0, w_bytes, 0x00020000);
  // DMA pieces: 8 rows x 128 B; A rows 16*wid + 8*j + rb, W rows the same (j = 0, 1)
  uint32_t aoff0[2], aoff1[2], boff[2];
  int pimg[2], pohw[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    int64_t n = n0 + 16 * wid + 8 * j + rb;
    n = n < N ? n : N - 1;
    boff[j] = (uint32_t)(n * d.ldw * 2) + lc16;
    int64_t m = m0 + 16 * wid + 8 * j + rb;
    m = m < M ? m : M - 1;
    if constexpr (MODE == VD_A_DENSE) {
      aoff0[j] = (uint32_t)(m * d.lda0 * 2) + lc16;
      aoff1[j] = (uint32_t)(m * d.lda1 * 2) + lc16;
    } else {
      const int hw = d.h_out * d.w_out;
      const int img = Div(hw)((int)m);
      const int p = (int)m - img * hw;
      const int oh = Div(d.w_out)(p);
      pimg[j] = img * d.h_in * d.w_in;
      pohw[j] = (oh << 16) | (p - oh * d.w_out);
    }
  }
  const int cin = MODE == VD_A_CONV3X3 ? (int)(K / 9) : 0;
  const int hgrid = d.upsample ? 2 * d.h_in : d.h_in;
  const int wgrid = d.upsample ? 2 * d.w_in : d.w_in;
  int c_tap = 0, c_ci = 0, ikt = kt0;
  bool c_new = true;
  if constexpr (MODE == VD_A_CONV3X3) {
    c_tap = kt0 * BK / cin;
    c_ci = kt0 * BK - c_tap * cin;
  }
  auto issue = [&](int stage) __attribute__((always_inline)) {
    char* la = smem + stage * G6_STAGE;
    char* lb = la + G6_A;
    const int kb = ikt * BK;
    if constexpr (MODE == VD_A_DENSE) {
      const bool s0 = kb < (int)d.k0;
      const uint32_t koff = (uint32_t)(s0 ? kb : kb - (int)d.k0) * 2;
#pragma unroll
      for (int j = 0; j < 2; ++j) dma16(s0 ? ra0 : ra1, la + (2 * wid + j) * 1024, (s0 ? aoff0[j] : aoff1[j]) + koff);
    } else {
      if (c_new) {
        c_new = false;
        const int dy = c_tap / 3, dx = c_tap - 3 * dy;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          int ih = (pohw[j] >> 16) * d.stride + dy - 1, iw = (pohw[j] & 0xffff) * d.stride + dx - 1;
          const bool ok = ((uint32_t)ih < (uint32_t)hgrid) & ((uint32_t)iw < (uint32_t)wgrid);  // branch-free
          ih >>= d.upsample;
          iw >>= d.upsample;
          const uint32_t pix = (uint32_t)(pimg[j] + ih * d.w_in + iw);
          aoff0[j] = ok ? pix * (uint32_t)(d.lda0 * 2) + lc16 : G2_OOB;
          aoff1[j] = ok ? pix * (uint32_t)(d.lda1 * 2) + lc16 : G2_OOB;
        }
      }
      const bool s0 = c_ci < (int)d.k0;
      const uint32_t coff = (uint32_t)(s0 ? c_ci : c_ci - (int)d.k0) * 2;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t o = s0 ? aoff0[j] : aoff1[j];
        dma16(s0 ? ra0 : ra1, la + (2 * wid + j) * 1024, o + coff);
      }
      c_ci += BK;
      if (c_ci == cin) { c_ci = 0; ++c_tap; c_new = true; }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) dma16(rw, lb + (2 * wid + j) * 1024, boff[j] + (uint32_t)kb * 2);
    ++ikt;
  };

  f32x4 acc[NB][MB];
#pragma unroll
  for (int a = 0; a < NB; ++a)
#pragma unroll
    for (int b = 0; b < MB; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < G6_S - 1; ++j)
    if (j < nk) issue(j);
  const int fr = lane & 15, fq = lane >> 4;
  f32x4 sacc[LNF ? MB : 1], gacc[LNF ? MB : 1];  // LNF: ones·x and x·xᵀ per row block
#pragma unroll
  for (int b = 0; b < (LNF ? MB : 1); ++b) sacc[b] = gacc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bf16x8 ones = __builtin_bit_cast(bf16x8, make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u));
  int stage = 0;
  for (int it = 0; it < nk; ++it) {
    // k-steps it+1 .. it+S-2 (4 pieces each) may stay in flight
    const int ahead = nk - 1 - it < G6_S - 2 ? nk - 1 - it : G6_S - 2;
    if constexpr (G6_S == 3) {
      if (ahead) wait_vm<4>();
      else wait_vm<0>();
    } else {
      wait_vm_rt(4 * ahead);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (it + G6_S - 1 < nk) issue(stage == 0 ? G6_S - 1 : stage - 1);
    const char* sb = smem + stage * G6_STAGE;
    {
      bf16x8 wf[BK / 32][NB], xf[BK / 32][MB];
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
#pragma unroll
        for (int b = 0; b < MB; ++b) xf[ks][b] = *(const bf16x8*)(sb + 2 * lds_off(wm * 32 + b * 16 + fr, ks * 4 + fq));
#pragma unroll
        for (int a = 0; a < NB; ++a)
          wf[ks][a] = *(const bf16x8*)(sb + G6_A + 2 * lds_off(wn * 32 + a * 16 + fr, ks * 4 + fq));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks)
#pragma unroll
        for (int a = 0; a < NB; ++a)
#pragma unroll
          for (int b = 0; b < MB; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ks][a], xf[ks][b], acc[a][b], 0, 0, 0);
      if constexpr (LNF) {
#pragma unroll
        for (int ks = 0; ks < BK / 32; ++ks)
#pragma unroll
          for (int b = 0; b < MB; ++b) {
            sacc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, xf[ks][b], sacc[b], 0, 0, 0);
            gacc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[ks][b], xf[ks][b], gacc[b], 0, 0, 0);
          }
      }
    }
    stage = stage == G6_S - 1 ? 0 : stage + 1;
  }
  const int mbase = (int)m0 + wm * 32, nbase = (int)n0 + wn * 32;
  if constexpr (LNF) {  // dense, unsplit (plan): the whole row went through this wave
    // the lane's outputs of row block b belong to A row fr: Σx in every entry of sacc[b], Σx² the
    // Gram block's diagonal entry (fr, fr), held by lane fr + 16 (fr >> 2) at index fr & 3
    const float rk = 1.0f / (float)d.K;
    const int j3 = fr & 3;
#pragma unroll
    for (int b = 0; b < MB; ++b) {
      const float gd = j3 == 0 ? gacc[b][0] : j3 == 1 ? gacc[b][1] : j3 == 2 ? gacc[b][2] : gacc[b][3];
      const float sxx = __shfl(gd, fr + 16 * (fr >> 2), 64);
      const float mean = sacc[b][0] * rk;
      float var = fmaf(sxx, rk, -mean * mean);
      if (__any(mean * mean > 256.f * var)) {  // ill-conditioned row(s): exact second pass from L2 (v8's)
        const int m = mbase + b * 16 + fr;
        float ss = 0.f;
#pragma unroll 1
        for (int kk = 8 * fq; kk < (int)K; kk += 32) {
          const bool s0 = kk < (int)d.k0;
          const uint32_t o = m < (int)M ? (uint32_t)m * (uint32_t)((s0 ? d.lda0 : d.lda1) * 2) +
                                              (uint32_t)(s0 ? kk : kk - (int)d.k0) * 2u : G2_OOB;
          const bf16x8 v = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(s0 ? ra0 : ra1, o, 0, 0));
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float t = (float)v[e] - mean;
            ss = fmaf(t, t, ss);
          }
        }
        ss += __shfl_xor(ss, 16, 64);
        ss += __shfl_xor(ss, 32, 64);
        var = ss * rk;
      }
      const float rstd = rsqrtf(fmaxf(var, 0.f) + d.ln_fold_eps);
#pragma unroll
      for (int a = 0; a < NB; ++a) {
        const int n = nbase + a * 16 + 4 * fq;
        const float4 t = n < (int)N ? *(const float4*)(d.ln_fold_s + n) : make_float4(0.f, 0.f, 0.f, 0.f);
        acc[a][b][0] = rstd * fmaf(-mean, t.x, acc[a][b][0]);
        acc[a][b][1] = rstd * fmaf(-mean, t.y, acc[a][b][1]);
        acc[a][b][2] = rstd * fmaf(-mean, t.z, acc[a][b][2]);
        acc[a][b][3] = rstd * fmaf(-mean, t.w, acc[a][b][3]);
      }
    }
    gemm_epilogue<MB, NB>(d, acc, mbase, nbase, lane);
    return;
  }
  if (split == 1) {
    if (d.rmap_inner)
      gemm_epilogue<MB, NB, true>(d, acc, mbase, nbase, lane);
    else
      gemm_epilogue<MB, NB>(d, acc, mbase, nbase, lane);
    return;
  }
  // ---- split K: slab, arrival counter, last arriver reduces.  Round 2: the hand-off is the
  // guide's fence-free form (cdna_hip_programming.md Guideline 16, R1 / "sc1 slab stores"): every
  // slab store is write-through (sc1), every storing wave drains it (vmcnt(0)) before the
  // workgroup barrier, ONE lane adds to the tile's counter (relaxed, agent scope), and the last
  // arriver reads every slab with sc1 loads (past this CU's L1), so neither side needs an
  // agent-scope fence — the release fence of round 1 wrote back the XCD's whole L2 (~25 us).
  float* slabs = (float*)d.ws;
  const __amdgpu_buffer_rsrc_t rws =
      __builtin_amdgcn_make_buffer_rsrc(d.ws, 0, (uint32_t)((int64_t)split * M * N * 4), 0x00020000);
#pragma unroll
  for (int a = 0; a < NB; ++a) {
    const int64_t n = nbase + a * 16 + 4 * fq;
#pragma unroll
    for (int b = 0; b < MB; ++b) {
      const int64_t m = mbase + b * 16 + fr;
      const uint32_t off = (n < N && m < M) ? (uint32_t)((((int64_t)sp * M + m) * N + n) * 4) : G2_OOB;
      __builtin_amdgcn_raw_buffer_store_b128(
          u32x4{__float_as_uint(acc[a][b][0]), __float_as_uint(acc[a][b][1]), __float_as_uint(acc[a][b][2]),
                __float_as_uint(acc[a][b][3])},
          rws, off, 0, 16);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  int* cnt = (int*)(slabs + (int64_t)split * M * N);
  int* last_flag = (int*)(smem + G6_S * G6_STAGE);
  if (tid == 0) {
    const int prev = __hip_atomic_fetch_add(cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == split - 1;
    if (last) __hip_atomic_store(cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // the memset node zeroes it too
    *last_flag = last;
  }
  __syncthreads();
  if (!*last_flag) return;
  auto slab4 = [&](int s2, int64_t m, int64_t n) {  // sc1 load of 4 slab floats
    const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rws, (uint32_t)((((int64_t)s2 * M + m) * N + n) * 4), 0, 16);
    return make_float4(__uint_as_float(u[0]), __uint_as_float(u[1]), __uint_as_float(u[2]), __uint_as_float(u[3]));
  };
  // 64 x 64 outputs (GEGLU: 64 x 32), 4 consecutive columns per thread-step
  const bool geglu = d.act == VD_ACT_GEGLU;
  const int ncol = geglu ? G6_BN / 2 : G6_BN;
  for (int e = tid; e < G6_BM * ncol / 4; e += G6_NT) {
    const int r = e / (ncol / 4), c4 = (e % (ncol / 4)) * 4;
    const int64_t m = m0 + r;
    if (m >= M) continue;
    float o4[4];
    if (geglu) {
      // packed column blocks of 16: hidden block i at 32i, gate block at 32i + 16
      const int64_t nh = n0 + (c4 / 16) * 32 + (c4 % 16), ng = nh + 16;
      if (ng >= N) continue;
      float h[4] = {0, 0, 0, 0}, g[4] = {0, 0, 0, 0};
      for (int s2 = 0; s2 < split; ++s2) {
        const float4 a4 = slab4(s2, m, nh);
        const float4 b4 = slab4(s2, m, ng);
        h[0] += a4.x; h[1] += a4.y; h[2] += a4.z; h[3] += a4.w;
        g[0] += b4.x; g[1] += b4.y; g[2] += b4.z; g[3] += b4.w;
      }
      if (d.bias) {
        const float4 a4 = *(const float4*)(d.bias + nh), b4 = *(const float4*)(d.bias + ng);
        h[0] += a4.x; h[1] += a4.y; h[2] += a4.z; h[3] += a4.w;
        g[0] += b4.x; g[1] += b4.y; g[2] += b4.z; g[3] += b4.w;
      }
      for (int j = 0; j < 4; ++j) o4[j] = h[j] * gelu_erf(g[j]);
      const int64_t o = n0 / 2 + c4;
      *(uint2*)((bf16_t*)d.out + m * d.ldc + o) = make_uint2(pack2(o4[0], o4[1]), pack2(o4[2], o4[3]));
      continue;
    }
    const int64_t o = n0 + c4;
    if (o >= N) continue;
    const int64_t mo = Rev3(d.M, d.rmap_n1, d.rmap_n2, d.rmap_inner)((int)m);  // output / residual row
    float v[4] = {0, 0, 0, 0};
    for (int s2 = 0; s2 < split; ++s2) {
      const float4 a4 = slab4(s2, m, o);
      v[0] += a4.x; v[1] += a4.y; v[2] += a4.z; v[3] += a4.w;
    }
    if (d.bias) {
      const float4 a4 = *(const float4*)(d.bias + o);
      v[0] += a4.x; v[1] += a4.y; v[2] += a4.z; v[3] += a4.w;
    }
    if (d.rowbias) {
      const float4 a4 = *(const float4*)(d.rowbias + (int64_t)Div((int)d.rb_div)((int)m) * d.ld_rb + o);
      v[0] += a4.x; v[1] += a4.y; v[2] += a4.z; v[3] += a4.w;
    }
    if (d.act == VD_ACT_SILU || d.act == VD_ACT_GELU)
      for (int j = 0; j < 4; ++j) v[j] = act_pw(d.act, v[j]);
    if (d.res) {
      const uint2 r2 = *(const uint2*)((const bf16_t*)d.res + mo * d.ld_res + o);
      v[0] += bf_lo(r2.x); v[1] += bf_hi(r2.x); v[2] += bf_lo(r2.y); v[3] += bf_hi(r2.y);
    }
    if (d.out_f32)
      *(float4*)((float*)d.out + mo * d.ldc + o) = make_float4(v[0], v[1], v[2], v[3]);
    else
      *(uint2*)((bf16_t*)d.out + mo * d.ldc + o) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
  }
}

// Sum the split-K slabs and apply the GEMM epilogue (4 output columns per thread).
// Index math in 32 bits (M * N < 2^31, checked by vd_gemm: M * ldc): a 64-bit division per element
// was most of this memory-bound kernel's instructions (round 3).
__global__ __launch_bounds__(256) void gemm_splitk_reduce(const vd_gemm_desc d, int split) {
  const int64_t M = d.M, N = d.N;
  const bool geglu = d.act == VD_ACT_GEGLU;
  const int64_t nout = geglu ? N / 2 : N;
  const int total = (int)(M * (nout / 4));
  const Div dq((int)(nout / 4)), drb(d.rowbias ? (int)d.rb_div : 1);
  const float* ws = (const float*)d.ws;
  const Rev3 perm(d.M, d.rmap_n1, d.rmap_n2, d.rmap_inner);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int m32 = dq(i);
    const int64_t m = m32, mo = perm(m32);  // slab row, output / residual row
    const int64_t o = (int64_t)(i - m32 * (int)(nout / 4)) * 4;
    float o4[4];
    if (geglu) {
      const int64_t nh = (o / 16) * 32 + (o % 16), ng = nh + 16;
      float h[4] = {0, 0, 0, 0}, g[4] = {0, 0, 0, 0};
      for (int sp = 0; sp < split; ++sp) {
        const float4 a = *(const float4*)(ws + (sp * M + m) * N + nh);
        const float4 b = *(const float4*)(ws + (sp * M + m) * N + ng);
        h[0] += a.x; h[1] += a.y; h[2] += a.z; h[3] += a.w;
        g[0] += b.x; g[1] += b.y; g[2] += b.z; g[3] += b.w;
      }
      if (d.bias) {
        const float4 a = *(const float4*)(d.bias + nh);
        const float4 b = *(const float4*)(d.bias + ng);
        h[0] += a.x; h[1] += a.y; h[2] += a.z; h[3] += a.w;
        g[0] += b.x; g[1] += b.y; g[2] += b.z; g[3] += b.w;
      }
      for (int j = 0; j < 4; ++j) o4[j] = h[j] * gelu_erf(g[j]);
    } else {
      float v[4] = {0, 0, 0, 0};
      for (int sp = 0; sp < split; ++sp) {
        const float4 a = *(const float4*)(ws + (sp * M + m) * N + o);
        v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
      }
      if (d.bias) {
        const float4 a = *(const float4*)(d.bias + o);
        v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
      }
      if (d.rowbias) {
        const float4 a = *(const float4*)(d.rowbias + (int64_t)drb(m32) * d.ld_rb + o);
        v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
      }
      if (d.act == VD_ACT_SILU || d.act == VD_ACT_GELU)
        for (int j = 0; j < 4; ++j) v[j] = act_pw(d.act, v[j]);
      if (d.res) {
        const uint2 r = *(const uint2*)((const bf16_t*)d.res + mo * d.ld_res + o);
        v[0] += bf_lo(r.x); v[1] += bf_hi(r.x); v[2] += bf_lo(r.y); v[3] += bf_hi(r.y);
      }
      for (int j = 0; j < 4; ++j) o4[j] = v[j];
    }
    if (d.out_f32)
      *(float4*)((float*)d.out + mo * d.ldc + o) = make_float4(o4[0], o4[1], o4[2], o4[3]);
    else
      *(uint2*)((bf16_t*)d.out + mo * d.ldc + o) = make_uint2(pack2(o4[0], o4[1]), pack2(o4[2], o4[3]));
  }
}

// ============================================================================ v8
// Weight-stationary GEMM for the short-K, tall-M L1 projections (K = 320, M >= 65536: the
// attention / motion projections and the fused QKV of the 64 x 64 level).  Every other kernel
// restages a W k-tile through LDS per 256-row tile and synchronises the workgroup per k-tile;
// here a workgroup loads ONE 160-column W tile (160 x 320 bf16 = 100 KiB) and its bias into LDS
// once and keeps them, and each of its 8 waves streams 16-row blocks of A straight from global
// memory into MFMA B-operand registers — no A staging, no barrier after the W fill:
//  * per row block a wave runs 10 k-steps x 10 column blocks = 100 MFMAs
//    (v_mfma_f32_16x16x32_bf16); the W fragments are double-buffered in registers (k-step
//    ks + 1's 10 ds_read_b128 go out before k-step ks's MFMAs);
//  * the A registers are double-buffered: the next row block's 10 loads (and this block's
//    residual rows) go out before this block's first MFMA, so each load has a whole row block
//    of MFMA work to land, and the epilogue issues no load (bias from LDS, residual already in
//    registers) — nothing in it waits for the prefetch;
//  * the epilogue stages the wave's 16 x 160 output tile through LDS and writes it back as
//    320-B row segments (1 KiB per store instruction over 3-4 rows) instead of 16 rows x 64 B;
//  * blockIdx % 8 is the XCD; the row blocks are split into 8 contiguous ranges, one per XCD,
//    and inside an XCD each 160-column W tile has 32 / tiles_n workgroups walking the XCD's row
//    blocks in the same order, so an A row block is fetched from HBM once and served from that
//    XCD's L2 to the other column tiles;
//  * the k-order per output (k-steps 0..9, 32 deep each) and the epilogue arithmetic are v2's,
//    so the results equal v2's bits (tests/test_gpu_kernels.py::test_gemm_v8_weight_stationary).
// Measured (tools/kbench.py, 32 images, profiles/r04_gemm_v8.txt): L1 projection 36 vs 52 us,
// with residual 45-50 vs 73-80 us, fused QKV N = 960 125 vs 137 us (v5).  Variants measured
// and not kept: 32-row blocks (4 waves, accumulators in AGPRs: 0.5 W reads per MFMA, slower),
// triple-buffered A, 12 waves per CU, unstaged 64-B stores.
constexpr int G8_BN = 160, G8_KMAX = 320, G8_NW = 8;
constexpr int G8_SUB = G8_BN * BK * 2;  // one 64-deep W sub-tile: 20 KiB

// LNF (round 5, vd_gemm_desc.ln_fold_s): the LayerNorm of A's rows folded in.  Per k-step two
// more MFMAs on the A fragments the wave already holds — ones·x (every output column = the row
// sum) and x·xᵀ (the 16 x 16 Gram block, whose diagonal is the row's sum of squares) — so the
// statistics cost no VALU inside the loop; the epilogue forms rstd·(acc − mean·s[n]) + b'[n]
// with s and b' in LDS next to the bias.  var = E[x²] − mean² in fp32 has a relative error of
// ≈ 1e-7·(1 + mean²/var); where a row's |mean| / std passes 16 (never in the UNet: ≤ 0.1,
// profiles/r06_motion_bisect.txt) the wave takes the exact second pass Σ(x − mean)², re-reading
// its rows from L2 (test_gemm_ln_fold runs rows offset by 30 / 100 / 300 std).
template <bool RES, bool GEGLU, bool PERM = false, bool LNF = false>
__global__ __launch_bounds__(G8_NW * 64, 1) void gemm8_kernel(const vd_gemm_desc d, uint32_t a0_bytes,
                                                             uint32_t w_bytes, uint32_t c_bytes, int tiles_n,
                                                             int groups) {
  constexpr int KS = G8_KMAX / 32, NB = G8_BN / 16, NW = G8_NW;
  constexpr int OROW = G8_BN * 2 + 16;  // staged output row (bytes, padded)
  __shared__ __attribute__((aligned(1024))) char smem[(G8_KMAX / BK) * G8_SUB + G8_BN * 8 + NW * 16 * OROW];
  float* sbias = (float*)(smem + (G8_KMAX / BK) * G8_SUB);
  float* ssum = sbias + G8_BN;  // LNF: s[n] of the tile's columns
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  char* obuf = smem + (G8_KMAX / BK) * G8_SUB + G8_BN * 8 + wid * 16 * OROW;
  const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  if (j >= groups * tiles_n) return;  // the XCD's workgroups beyond a whole number of W tiles
  const int nt = j % tiles_n, grp = j / tiles_n;
  const int M = (int)d.M, n0 = nt * G8_BN;
  const int rbs = (M + 15) / 16;
  const int rb0 = (int)((int64_t)rbs * xcd / 8), rb1 = (int)((int64_t)rbs * (xcd + 1) / 8);
  const int gw = grp * NW + wid, GW = groups * NW;

  // ---- W tile -> LDS (5 sub-tiles of 160 rows x 64 k, v2's swizzled B image) + bias, once
  {
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)d.w, 0, w_bytes, 0x00020000);
    const int rb = lane >> 3;
    const uint32_t lc16 = (uint32_t)(((lane & 7) ^ rb) * 16);
    constexpr int PIECES = (G8_KMAX / BK) * (G8_BN / 8);
    for (int p = wid; p < PIECES; p += NW) {
      const int s = p / (G8_BN / 8), pr = p - s * (G8_BN / 8);
      const uint32_t n = (uint32_t)(n0 + pr * 8 + rb);
      dma16(rw, smem + s * G8_SUB + pr * 1024, n * (uint32_t)(d.ldw * 2) + (uint32_t)(s * BK * 2) + lc16);
    }
    if (tid < G8_BN) {
      sbias[tid] = d.bias ? d.bias[n0 + tid] : 0.f;
      if constexpr (LNF) ssum[tid] = d.ln_fold_s[n0 + tid];
    }
    wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  int r = rb0 + gw;
  if (r >= rb1) return;  // no barrier follows
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)d.a0, 0, a0_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc((void*)d.out, 0, c_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rr =
      __builtin_amdgcn_make_buffer_rsrc((void*)(RES ? d.res : d.out), 0, RES ? (uint32_t)(d.M * d.ld_res * 2) : 0u,
                                        0x00020000);
  const int fr = lane & 15, fq = lane >> 4;
  const int wcol = 16 * (fq & 1) + 8 * (fq >> 1);  // lane's column offset inside a swapped pair
  const Rev3 perm = PERM ? Rev3(d.M, d.rmap_n1, d.rmap_n2, d.rmap_inner) : Rev3(0, 0, 0, 0);  // row map
  // this lane's A fragments of row block rb: past the buffer (read as zeros, no traffic) for
  // rows >= M and for row blocks past the XCD's range
  auto load_a = [&](bf16x8 (&x)[KS], int rb) {
    const int m = rb * 16 + fr;
    const uint32_t o = (rb < rb1 && m < M) ? (uint32_t)m * (uint32_t)(d.lda0 * 2) + (uint32_t)(fq * 16) : G2_OOB;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      x[ks] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ra, o + (uint32_t)(ks * 64), 0, 0));
  };
  u32x4 rsv[NB / 2];
  auto load_res = [&](int rb) {
    const int m = rb * 16 + fr;
#pragma unroll
    for (int pr = 0; pr < NB / 2; ++pr) {
      const uint32_t off = m < M ? (uint32_t)((PERM ? perm(m) : m) * (int)d.ld_res + n0 + pr * 32 + wcol) * 2u : G2_OOB;
      rsv[pr] = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0);
    }
  };
  const uint32_t wl = 2 * lds_off(fr, fq);  // lane's W fragment byte offset (column block 0, k-step 0)
  auto block = [&](const bf16x8 (&x)[KS], int rb) {
    f32x4 acc[NB];
#pragma unroll
    for (int a = 0; a < NB; ++a) acc[a] = f32x4{0.f, 0.f, 0.f, 0.f};
    // k-step ks = sub-tile ks / 2, chunks 4 (ks & 1) + fq: the XOR with (row & 7) is the same
    // for every 16-row column block, so (ks & 1) flips bit 2 of the chunk index (byte bit 6)
    bf16x8 wf[2][NB];
    auto read_w = [&](bf16x8 (&f)[NB], int ks) {
      const char* sb = smem + (ks >> 1) * G8_SUB;
      const uint32_t wk = (ks & 1) ? (wl ^ 64u) : wl;
#pragma unroll
      for (int a = 0; a < NB; ++a) f[a] = *(const bf16x8*)(sb + wk + a * 16 * BK * 2);
    };
    f32x4 sacc = f32x4{0.f, 0.f, 0.f, 0.f}, gacc = f32x4{0.f, 0.f, 0.f, 0.f};  // LNF: ones·x, x·xᵀ
    const bf16x8 ones = __builtin_bit_cast(bf16x8, make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u));
    read_w(wf[0], 0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) read_w(wf[(ks + 1) & 1], ks + 1);
#pragma unroll
      for (int a = 0; a < NB; ++a)
        acc[a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ks & 1][a], x[ks], acc[a], 0, 0, 0);
      if constexpr (LNF) {
        sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, x[ks], sacc, 0, 0, 0);
        gacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[ks], x[ks], gacc, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);  // one k-step per region (unpinned, hipcc spilled)
    }
    // LNF: this lane's outputs all belong to A row rb*16 + fr.  Σx is in every entry of sacc;
    // Σx² is the Gram block's diagonal entry (fr, fr), held by lane fr + 16 (fr >> 2) at index fr & 3
    float nmean = 0.f, rstd = 1.f;
    if constexpr (LNF) {
      const int j3 = fr & 3;
      const float gd = j3 == 0 ? gacc[0] : j3 == 1 ? gacc[1] : j3 == 2 ? gacc[2] : gacc[3];
      const float sxx = __shfl(gd, fr + 16 * (fr >> 2), 64);
      constexpr float RK = 1.0f / (float)G8_KMAX;
      const float mean = sacc[0] * RK;
      float var = fmaf(sxx, RK, -mean * mean);
      if (__any(mean * mean > 256.f * var)) {  // ill-conditioned row(s): exact second pass (see above)
        const int m = rb * 16 + fr;
        const uint32_t o = m < M ? (uint32_t)m * (uint32_t)(d.lda0 * 2) + (uint32_t)(fq * 16) : G2_OOB;
        float ss = 0.f;
#pragma unroll 1
        for (int ks = 0; ks < KS; ++ks) {  // re-read from L2 (the fragments' registers are not kept live)
          const bf16x8 v = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ra, o + (uint32_t)(ks * 64), 0, 0));
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float t = (float)v[e] - mean;
            ss = fmaf(t, t, ss);
          }
        }
        ss += __shfl_xor(ss, 16, 64);
        ss += __shfl_xor(ss, 32, 64);
        var = ss * RK;
      }
      rstd = rsqrtf(fmaxf(var, 0.f) + d.ln_fold_eps);
      nmean = -mean;
    }
    if constexpr (GEGLU) {
      // (hidden, gate) 16-column block pairs (a, a+1) -> 16 output columns: the lane's 4 outputs
      // (h + bh) * gelu(g + bg) on fp32 pairs (gemm_epilogue's arithmetic), 8 B into the staged row
#pragma unroll
      for (int a = 0; a < NB; a += 2) {
        const int c = a * 16 + 4 * fq;
        const float4 th = *(const float4*)(sbias + c), tg = *(const float4*)(sbias + c + 16);
        const float thv[4] = {th.x, th.y, th.z, th.w}, tgv[4] = {tg.x, tg.y, tg.z, tg.w};
        float hv[4], gv[4];
        if constexpr (LNF) {
          const float4 sh = *(const float4*)(ssum + c), sg = *(const float4*)(ssum + c + 16);
          const float shv[4] = {sh.x, sh.y, sh.z, sh.w}, sgv[4] = {sg.x, sg.y, sg.z, sg.w};
#pragma unroll
          for (int j4 = 0; j4 < 4; ++j4) {
            hv[j4] = fmaf(rstd, fmaf(nmean, shv[j4], acc[a][j4]), thv[j4]);
            gv[j4] = fmaf(rstd, fmaf(nmean, sgv[j4], acc[a + 1][j4]), tgv[j4]);
          }
        } else {
#pragma unroll
          for (int j4 = 0; j4 < 4; ++j4) {
            hv[j4] = acc[a][j4] + thv[j4];
            gv[j4] = acc[a + 1][j4] + tgv[j4];
          }
        }
        uint32_t pk[2];
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const f32x2 go = gelu_erf2(f32x2{gv[2 * h2], gv[2 * h2 + 1]});
          const f32x2 oo = f32x2{hv[2 * h2], hv[2 * h2 + 1]} * go;
          pk[h2] = pack2(oo[0], oo[1]);
        }
        *(uint2*)(obuf + fr * OROW + ((a / 2) * 16 + 4 * fq) * 2) = make_uint2(pk[0], pk[1]);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int it = 0; it < 3; ++it) {  // 16 rows x 160 B
        const int q = it * 64 + lane, row = q / 10, ch = q - row * 10;
        if (q < 160) {
          const uint4 v = *(const uint4*)(obuf + row * OROW + ch * 16);
          const int m = rb * 16 + row;
          const uint32_t off = m < M ? (uint32_t)(m * (int)d.ldc + n0 / 2 + ch * 8) * 2u : G2_OOB;
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{v.x, v.y, v.z, v.w}, rc, off, 0, 0);
        }
      }
      return;
    }
    // epilogue (gemm_epilogue's wide-path arithmetic): permlane16_swap of column blocks (a, a+1)
    // leaves each lane 8 consecutive columns; bias from LDS, residual from rsv
#pragma unroll
    for (int a = 0; a < NB; a += 2) {
      const int c = a * 16 + wcol;
      const float4 t0 = *(const float4*)(sbias + c), t1 = *(const float4*)(sbias + c + 4);
      const float bv[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
      float o[8];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        auto rp = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[a][jj]), __float_as_uint(acc[a + 1][jj]),
                                                   false, false);
        o[jj] = __uint_as_float(rp[0]);
        o[4 + jj] = __uint_as_float(rp[1]);
      }
      if constexpr (LNF) {
        const float4 u0 = *(const float4*)(ssum + c), u1 = *(const float4*)(ssum + c + 4);
        const float sv[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) o[jj] = fmaf(rstd, fmaf(nmean, sv[jj], o[jj]), bv[jj]);
      } else {
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) o[jj] += bv[jj];
      }
      if (d.act == VD_ACT_SILU || d.act == VD_ACT_GELU) {
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) o[jj] = act_pw(d.act, o[jj]);
      }
      if constexpr (RES) {
        float rf[8];
        const u32x4 rv = rsv[a / 2];
        unpack8(make_uint4(rv[0], rv[1], rv[2], rv[3]), rf);
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) o[jj] += rf[jj];
      }
      *(uint4*)(obuf + fr * OROW + c * 2) = pack8(o);
    }
    // the wave's 16 x 160 tile back out of LDS as 320-B row segments (in-order LDS: no barrier
    // within the wave; out-of-range rows carry an offset past the output buffer, dropped)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int it = 0; it < 5; ++it) {
      const int q = it * 64 + lane, row = q / 20, ch = q - row * 20;
      const uint4 v = *(const uint4*)(obuf + row * OROW + ch * 16);
      const int m = rb * 16 + row;
      const uint32_t off = m < M ? (uint32_t)((PERM ? perm(m) : m) * (int)d.ldc + n0 + ch * 8) * 2u : G2_OOB;
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{v.x, v.y, v.z, v.w}, rc, off, 0, 0);
    }
  };
  bf16x8 x0[KS], x1[KS];
  load_a(x0, r);
  for (;;) {
    if constexpr (RES) load_res(r);
    load_a(x1, r + GW);
    block(x0, r);
    if ((r += GW) >= rb1) break;
    if constexpr (RES) load_res(r);
    load_a(x0, r + GW);
    block(x1, r);
    if ((r += GW) >= rb1) break;
  }
}

template <int BN>
int launch2(const vd_gemm_desc& d, hipStream_t s, uint32_t a0b, uint32_t a1b, uint32_t wb, int split) {
  const int64_t units = ((d.M + G2_BM - 1) / G2_BM) * ((d.N + BN - 1) / BN) * split;
  // persistent: one workgroup per CU, ceil(units / grid) rounds, balanced grid
  const int64_t rounds = (units + g_num_cus - 1) / g_num_cus;
  const int64_t grid = (units + rounds - 1) / rounds;
  if (d.a_mode == VD_A_CONV3X3)
    hipLaunchKernelGGL((gemm2_kernel<BN, VD_A_CONV3X3>), dim3((unsigned)grid), dim3(G2_NT), 0, s, d, a0b, a1b, wb, split);
  else
    hipLaunchKernelGGL((gemm2_kernel<BN, VD_A_DENSE>), dim3((unsigned)grid), dim3(G2_NT), 0, s, d, a0b, a1b, wb, split);
  int rc = vd_launch_status();
  if (rc != VD_OK || split == 1) return rc;
  const int64_t work = d.M * ((d.act == VD_ACT_GEGLU ? d.N / 2 : d.N) / 4);
  const int64_t blocks = (work + 255) / 256;
  hipLaunchKernelGGL(gemm_splitk_reduce, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0, s, d, split);
  return vd_launch_status();
}

template <int BM, int BN>
int launch(const vd_gemm_desc& d, hipStream_t s) {
  const int64_t tiles = ((d.M + BM - 1) / BM) * ((d.N + BN - 1) / BN);
  if (tiles > 0x7fffffff) return VD_EINVAL;
  if (d.a_mode == VD_A_CONV3X3)
    hipLaunchKernelGGL((gemm_kernel<BM, BN, VD_A_CONV3X3>), dim3((unsigned)tiles), dim3(NT), 0, s, d);
  else
    hipLaunchKernelGGL((gemm_kernel<BM, BN, VD_A_DENSE>), dim3((unsigned)tiles), dim3(NT), 0, s, d);
  return vd_launch_status();
}

int launch9(const vd_gemm_desc& d, hipStream_t s) {
  const int64_t waves = (d.N + 15) / 16;
  hipLaunchKernelGGL(gemm9_kernel, dim3((unsigned)((waves + G9_NW - 1) / G9_NW)), dim3(G9_NW * 64), 0, s, d);
  return vd_launch_status();
}

template <int BN, int WM, int WN, int STAGES>
int launch4(const vd_gemm_desc& d, hipStream_t s, uint32_t a0b, uint32_t a1b, uint32_t wb, int split) {
  using C = G4<BN, WM, WN, STAGES>;
  const int64_t units = ((d.M + G4_BM - 1) / G4_BM) * ((d.N + BN - 1) / BN) * split;
  // persistent: one workgroup per CU, ceil(units / grid) rounds, balanced grid
  const int64_t slots = (int64_t)g_num_cus;
  const int64_t rounds = (units + slots - 1) / slots;
  const int64_t grid = (units + rounds - 1) / rounds;
  if (d.a_mode == VD_A_CONV3X3)
    hipLaunchKernelGGL((gemm4_kernel<BN, WM, WN, STAGES, VD_A_CONV3X3>), dim3((unsigned)grid), dim3(C::NT), 0,
                       s, d, a0b, a1b, wb, split);
  else if (d.ln_out)  // plan() only lets a fusable descriptor keep ln_out
    hipLaunchKernelGGL((gemm4_kernel<BN, WM, WN, STAGES, VD_A_DENSE, true>), dim3((unsigned)grid), dim3(C::NT), 0,
                       s, d, a0b, a1b, wb, split);
  else
    hipLaunchKernelGGL((gemm4_kernel<BN, WM, WN, STAGES, VD_A_DENSE>), dim3((unsigned)grid), dim3(C::NT), 0, s,
                       d, a0b, a1b, wb, split);
  int rc = vd_launch_status();
  if (rc != VD_OK || split == 1) return rc;
  const int64_t work = d.M * ((d.act == VD_ACT_GEGLU ? d.N / 2 : d.N) / 4);
  const int64_t blocks = (work + 255) / 256;
  hipLaunchKernelGGL(gemm_splitk_reduce, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0, s, d, split);
  return vd_launch_status();
}

int launch6(const vd_gemm_desc& d, hipStream_t s, uint32_t a0b, uint32_t a1b, uint32_t wb, int split) {
  const int64_t tiles = ((d.M + G6_BM - 1) / G6_BM) * ((d.N + G6_BN - 1) / G6_BN);
  if (tiles * split > 0x7fffffff) return VD_EINVAL;
  if (split > 1) {  // arrival counters after the slabs
    char* cnt = (char*)d.ws + (int64_t)split * d.M * d.N * 4;
    if (hipMemsetAsync(cnt, 0, (size_t)tiles * 4, s) != hipSuccess) return vd_launch_status();
  }
  const int64_t wgs = tiles * split;
  const dim3 grid((unsigned)wgs);
#define G6_LAUNCH(S)                                                                                    \
  if (d.ln_fold_s)                                                                                      \
    hipLaunchKernelGGL((gemm6_kernel<VD_A_DENSE, S, true>), grid, dim3(G6_NT), 0, s, d, a0b, a1b, wb, split); \
  else if (d.a_mode == VD_A_CONV3X3)                                                                    \
    hipLaunchKernelGGL((gemm6_kernel<VD_A_CONV3X3, S>), grid, dim3(G6_NT), 0, s, d, a0b, a1b, wb, split); \
  else                                                                                                  \
    hipLaunchKernelGGL((gemm6_kernel<VD_A_DENSE, S>), grid, dim3(G6_NT), 0, s, d, a0b, a1b, wb, split);
  if (wgs <= g_num_cus) {
    G6_LAUNCH(6)
  } else if (wgs <= 2 * g_num_cus) {
    G6_LAUNCH(4)
  } else {
    G6_LAUNCH(3)
  }
#undef G6_LAUNCH
  return vd_launch_status();
}

int launch8(const vd_gemm_desc& d, hipStream_t s, uint32_t a0b, uint32_t wb) {
  const int per_xcd = g_num_cus / 8;  // one workgroup per CU, blockIdx % 8 = XCD
  const int tiles_n = (int)(d.N / G8_BN);
  const int groups = per_xcd / tiles_n;
  if (groups < 1) return VD_EINVAL;
  const uint32_t cb = (uint32_t)(d.M * d.ldc * 2);
  const dim3 grid((unsigned)(8 * per_xcd)), block(G8_NW * 64);
  if (d.ln_fold_s && d.act == VD_ACT_GEGLU)
    hipLaunchKernelGGL((gemm8_kernel<false, true, false, true>), grid, block, 0, s, d, a0b, wb, cb, tiles_n, groups);
  else if (d.ln_fold_s)
    hipLaunchKernelGGL((gemm8_kernel<false, false, false, true>), grid, block, 0, s, d, a0b, wb, cb, tiles_n, groups);
  else if (d.act == VD_ACT_GEGLU)
    hipLaunchKernelGGL((gemm8_kernel<false, true>), grid, block, 0, s, d, a0b, wb, cb, tiles_n, groups);
  else if (d.res && d.rmap_inner)
    hipLaunchKernelGGL((gemm8_kernel<true, false, true>), grid, block, 0, s, d, a0b, wb, cb, tiles_n, groups);
  else if (d.res)
    hipLaunchKernelGGL((gemm8_kernel<true, false>), grid, block, 0, s, d, a0b, wb, cb, tiles_n, groups);
  else
    hipLaunchKernelGGL((gemm8_kernel<false, false>), grid, block, 0, s, d, a0b, wb, cb, tiles_n, groups);
  return vd_launch_status();
}

int launch3(const vd_gemm_desc& d, hipStream_t s, uint32_t a0b, uint32_t a1b, uint32_t wb, int split) {
  const int64_t units = ((d.M + G3_BM - 1) / G3_BM) * ((d.N + G3_BN - 1) / G3_BN) * split;
  if (units > 0x7fffffff) return VD_EINVAL;
  // persistent: one workgroup per CU, ceil(units / CUs) units each, balanced grid
  const int64_t rounds = (units + g_num_cus - 1) / g_num_cus;
  const int64_t grid = (units + rounds - 1) / rounds;
  const int fast = split == 1 && !d.res && !d.rowbias && !d.out_f32 && !d.rmap_inner && d.N % 8 == 0 &&
                   d.N <= G3_BIAS_N && d.ldc % 8 == 0 && ((uintptr_t)d.out & 15) == 0 &&
                   d.M * d.ldc * 2 < (int64_t)G2_OOB;
  hipLaunchKernelGGL((gemm3_kernel<VD_A_DENSE>), dim3((unsigned)grid), dim3(G3_NT), 0, s, d, a0b, a1b, wb, split,
                     fast);
  int rc = vd_launch_status();
  if (rc != VD_OK || split == 1) return rc;
  const int64_t work = d.M * ((d.act == VD_ACT_GEGLU ? d.N / 2 : d.N) / 4);
  const int64_t blocks = (work + 255) / 256;
  hipLaunchKernelGGL(gemm_splitk_reduce, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0, s, d, split);
  return vd_launch_status();
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
inline bool al8(const void* p) { return ((uintptr_t)p & 7) == 0; }
struct Plan {
  int ver = 1;
  int bn = 128, split = 1;
  bool ln_fused = false;  // v5 writes ln_out in its epilogue
  uint32_t a0b = 0, a1b = 0, wb = 0;
  int64_t ws_bytes = 0;
};

// max K slices of the v2/v3/v5 split path: 32 (L4 convs at 4-8 images per rank, 64 -> 176
// workgroups: 66 -> 38 us, 41 -> 30 us against a cap of 8; neutral elsewhere —
// profiles/r01_gemm_paths.txt)
constexpr int SPLIT_CAP = 32;

inline int64_t nk_of(const vd_gemm_desc& d) { return d.K / BK; }

inline int split_for(int64_t tiles, int64_t nk) {
  if (tiles >= 192 || nk < 16) return 1;
  int64_t sp = (256 + tiles - 1) / tiles;
  sp = sp < nk / 8 ? sp : nk / 8;
  return (int)(sp < SPLIT_CAP ? sp : SPLIT_CAP);
}

// LDS-DMA kernels wherever the operands fit 32-bit buffer offsets: v3 (256x256,
// 8-phase ping-pong) for wide dense shapes that fill the chip, v2 (256 x
// {128,160}, persistent) otherwise; split K when the output tiles cannot fill
// the 256 CUs.
void read_num_cus() {  // once per process: the plan (and the workspace size) depends on it
  static bool cus_read = false;
  if (!cus_read) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      g_num_cus = n;
    cus_read = true;
  }
}

// d.path (per call, stateless): 0 = this automatic plan; 1 / 2 / 3 / 5 / 6 / 8 force v1 / v2 / v3 /
// v5 / v6 / v8 (forced v6 also splits K toward 2 workgroups per CU) wherever that kernel takes the
// shape, else the automatic choice — the parity tests run every path.  d.plan_m > 0 makes
// every decision (kernel, tile count, split-K, LayerNorm fusion) as if M were plan_m while the
// launch covers all M rows: an unsharded run planned with a frame shard's M reproduces that
// shard's arithmetic exactly (split-K fixes the summation order).
Plan plan_core(const vd_gemm_desc& d) {
  read_num_cus();
  Plan p;
  int path = d.path;
  const int64_t M = d.plan_m > 0 ? d.plan_m : d.M;  // the row count the plan is made for
  // v9 (M <= 16 rows, dense, one operand, no GEGLU / LayerNorm / row map): bit-identical to v1.
  // Forced only (path 9): its same-process A/Bs were -0.04 ms on the 8-way rank step and
  // +0.04..0.12 ms on the 16-frame step (profiles/r05_gemm_v9_skinny_ab.txt), and both run the
  // same M = 2 time-embedding GEMMs, so no row count separates the gain from the loss (round 6).
  if (path == 9 && M <= G9_MMAX && d.M <= G9_MMAX && d.a_mode == VD_A_DENSE && d.k0 == d.K &&
      d.act != VD_ACT_GEGLU && !d.ln_out && !d.ln_fold_s && !d.rmap_inner) {
    p.ver = 9;
    return p;
  }
  if (path == 1 || d.K % G4_BK || d.k0 % G4_BK || M < G6_BM || (d.N < 64 && d.N > 32)) return p;
  const int64_t a_rows = d.a_mode == VD_A_CONV3X3
                             ? (int64_t)d.n_img / d.frames_out * d.frames_in * d.h_in * d.w_in : d.M;
  const int64_t a0b = a_rows * d.lda0 * 2, a1b = d.a1 ? a_rows * d.lda1 * 2 : 0, wb = d.N * d.ldw * 2;
  if (a0b >= (int64_t)G2_OOB || a1b >= (int64_t)G2_OOB || wb >= (int64_t)G2_OOB) return p;
  p.a0b = (uint32_t)a0b; p.a1b = (uint32_t)a1b; p.wb = (uint32_t)wb;
  const bool cin32 = d.a_mode != VD_A_CONV3X3 || (d.K / 9) % G4_BK == 0;
  const bool k64 = d.K % BK == 0 && d.k0 % BK == 0 &&
                   (d.a_mode != VD_A_CONV3X3 || (d.K / (d.ks * d.ks * d.kt)) % BK == 0);
  // v8 (weight-stationary, K = 320, dense, M >= 16384): the L1 projections and fused QKV —
  // 36 vs 52 us (projection), 45-50 vs 73-80 us (+ residual), 125 vs 137 us (QKV N = 960) on
  // the previous choices (profiles/r04_gemm_v8.txt); the L1 GEGLU too (same-box step A/B vs v3:
  // -0.1..0.3 ms).  A LayerNorm-fused request is NOT fused on these shapes: v8 + vd_layernorm
  // (≈ 53 + 33 us at M = 131072) beats v5's fused epilogue (≈ 93 us in the step).
  const bool v8ok = d.a_mode == VD_A_DENSE && d.K == G8_KMAX && d.k0 == d.K && !d.a1 && d.N % G8_BN == 0 &&
                    d.N / G8_BN <= g_num_cus / 8 && M >= 4096 && g_num_cus % 8 == 0 && !d.rowbias &&
                    !d.out_f32 && d.ldc % 8 == 0 && al16(d.out) &&
                    d.M * d.ldc * 2 < (int64_t)G2_OOB &&
                    (!d.res || (d.ld_res % 8 == 0 && al16(d.res) && d.M * d.ld_res * 2 < (int64_t)G2_OOB));
  // (M >= 16384: the 4- and 2-frame shards too — 17 vs 20 us, QKV 31-34 vs 35-37 us at M = 32768;
  // even at M = 16384 in kbench, and the 2-frame step 12.47 -> 12.42 ms in a same-box A/B; with
  // the LayerNorm unfused there as well the 4-frame step went 17.47 -> 17.04 ms,
  // profiles/r04_gemm_v8.txt)
  const bool v8auto = v8ok && M >= 16384;
  if (path == 8 && !v8ok) path = 0;  // forced v8 on a shape it does not take: the product plan
  // a folded LayerNorm (ln_fold_s) runs on v8 wherever v8 would run the plain GEMM (or is forced),
  // and on v6 wherever the plain GEMM's plan is an unsplit v6 (levels 2-4 of a frame-sharded rank,
  // the mid block); no other kernel carries it: ver 0 = not runnable, the caller takes the unfolded
  // form.  (Round 5 measured the fold on v2 / v3 too — row statistics by dot-2 VALU: 1.4-1.5x the v2
  // GEMM's time, 20x v3's — and withdrew it: those kernels run at the MFMA / issue limit, and
  // each of their N tiles would recompute the statistics of the same rows.)
  if (d.ln_fold_s) {
    if ((v8auto && path == 0) || (v8ok && path == 8)) {
      p.ver = 8;
      p.bn = G8_BN;
      return p;
    }
    vd_gemm_desc g = d;
    g.ln_fold_s = nullptr;
    const Plan q = plan_core(g);
    if (q.ver == 6 && q.split == 1 && d.a_mode == VD_A_DENSE) return q;
    p.ver = 0;
    return p;
  }
  // an output-row map (rmap; no ln_out, GEGLU or row bias — checked) is carried by v8 (with a
  // residual), v6 and v1 only: the v2 / v3 / v5 pipelines sit at their register limit and spill
  // with it (tests/test_kernel_resources.py).  v6 splits K only where forced (path 6).
  if (d.rmap_inner) {
    if (v8ok && d.res && (path == 0 || path == 8)) {
      p.ver = 8;
      p.bn = G8_BN;
    } else if (k64 && d.N >= 64 && d.kt <= 1 && d.ks != 1 && (path == 0 || path == 6)) {
      p.ver = 6;
      p.bn = 64;
      const int64_t tiles6 = ((M + G6_BM - 1) / G6_BM) * ((d.N + G6_BN - 1) / G6_BN);
      int64_t sp = 1;
      while (path == 6 && tiles6 * sp < 2 * g_num_cus && nk_of(d) / (sp * 2) >= 4 && sp < 16) sp *= 2;
      p.split = (int)sp;
      const int64_t rtiles6 = ((d.M + G6_BM - 1) / G6_BM) * ((d.N + G6_BN - 1) / G6_BN);
      p.ws_bytes = p.split > 1 ? (int64_t)p.split * d.M * d.N * 4 + ((rtiles6 * 4 + 255) / 256) * 256 : 0;
    }
    return p;
  }
  // fused LayerNorm epilogue: one 256 x 320 tile owns whole rows (v5, unsplit; >= 128 tiles so
  // the unsplit grid fills half the chip — smaller M runs the GEMM + vd_layernorm instead)
  if (d.ln_out) {
    p.ln_fused = d.a_mode == VD_A_DENSE && d.N == 320 && d.K % G4_BK == 0 && d.k0 == d.K && !d.a1 &&
                 d.ldc % 8 == 0 && d.ld_ln % 8 == 0 && ((uintptr_t)d.out & 15) == 0 && ((uintptr_t)d.ln_out & 15) == 0 &&
                 (!d.res || (d.ld_res % 8 == 0 && ((uintptr_t)d.res & 15) == 0)) &&
                 (M + G4_BM - 1) / G4_BM >= 128 && !d.rowbias && d.act == VD_ACT_NONE && !d.out_f32 &&
                 (path == 5 || (path == 0 && !v8auto));
    if (p.ln_fused) {
      p.ver = 5;
      p.bn = 320;
      return p;
    }
  }
  // N <= 32 (conv_out, N = 4): 256 x 32 v2 tiles — v1's 128 x 64 tiles ran the full-size
  // conv_out (M 131072, K 2880) in 177 us (profiles/r02b_step_breakdown_f16.txt)
  if (d.N <= 32) {
    if (!k64 || M < G2_BM || d.act == VD_ACT_GEGLU || (path != 0 && path != 2)) return p;
    p.ver = 2;
    p.bn = 32;
    p.split = split_for((M + G2_BM - 1) / G2_BM, d.K / BK);
    p.ws_bytes = p.split > 1 ? (int64_t)p.split * d.M * d.N * 4 : 0;
    return p;
  }
  // fewer rows than one 256-row tile (the deep levels of a 1-2 image rank): 64 x 64 tiles
  // (v1's 128-row tiles left L4's K = 11520 convs on 8 workgroups: 453 us vs ~30)
  if (M < G2_BM) {
    if (!k64 || d.kt > 1 || d.ks == 1 || (path != 0 && path != 6)) return p;  // v6: 2-D 3x3 taps
    p.ver = 6;
    p.bn = 64;
    return p;
  }
  if (d.kt > 1 || d.ks == 1) {  // temporal taps: the v2 loader (or v1 when the channels do not tile by 64)
    if (!k64) return p;
    p.ver = 2;
    const int64_t p128 = (d.N + 127) / 128 * 128, p160 = (d.N + 159) / 160 * 160;
    p.bn = (p160 < p128 || (p160 == p128 && d.N % 160 == 0)) ? 160 : 128;
    p.split = split_for(((M + G2_BM - 1) / G2_BM) * ((d.N + p.bn - 1) / p.bn), d.K / BK);
    p.ws_bytes = p.split > 1 ? (int64_t)p.split * d.M * d.N * 4 : 0;
    return p;
  }
  if ((v8auto && path == 0) || (v8ok && path == 8)) {
    p.ver = 8;
    p.bn = G8_BN;
    return p;
  }
  // v5 (256 x 320, BK 32): forced, where K or k0 is not a multiple of 64, and on the shape
  // it wins (tools/kbench.py: the L1 attention QKV projection M 131072 x N 960 x K 320)
  // (round 2) and the L1 projections N = K = 320 with or without a residual: one 320-column
  // tile covers the whole row (+res 75 vs 85 us on v2, profiles/r02_gemm_paths_vs_hipblaslt_miopen.txt)
  const bool v5auto = d.a_mode == VD_A_DENSE && M >= 65536 && d.K <= 320 && !d.rowbias && d.act != VD_ACT_GEGLU &&
                      ((d.N % 320 == 0 && d.N >= 640 && d.N < 2560 && !d.res) || d.N == 320);
  if (path == 5 || (path == 0 && (!k64 || v5auto))) {
    if (!cin32) return p;
    p.ver = 5;
    p.bn = 320;
    const int64_t tiles = ((M + G4_BM - 1) / G4_BM) * ((d.N + 319) / 320);
    p.split = split_for(tiles, d.K / BK);
    p.ws_bytes = p.split > 1 ? (int64_t)p.split * d.M * d.N * 4 : 0;
    return p;
  }
  if (!k64) return p;
  const int64_t nk = d.K / BK;
  // v6 (64 x 64 tiles, never split automatically): where the 256-row tiles leave the chip
  // underfilled (fewer tiles than CUs: the small M of a frame-sharded rank, or L4 at full
  // size) and K <= 1280 (K <= 2560 when v6 alone gives >= 2 workgroups per CU); wide N only
  // up to 4 workgroups per CU (64 x 64 tiles are L2-bandwidth bound), GEGLU only at tiny M.
  // tools/kb_sweep.sh, profiles/r01_gemm_paths.txt: 4 images L3/L4 projections 21-27 ->
  // 11 us, L4 qkv 24 -> 11 us; v2/v3 stay faster on long K, wide N at M >= 2048, and convs.
  {
    const int64_t tiles6 = ((M + G6_BM - 1) / G6_BM) * ((d.N + G6_BN - 1) / G6_BN);
    const int64_t tiles256 = ((M + G2_BM - 1) / G2_BM) * ((d.N + 159) / 160);
    // (round 4: also the L1 3x3 convs of a 2-frame rank, K = 2880 over >= 4 tiles per CU:
    // 45.5 vs 50.2 us for v2's split-2 + reduce, tools/kbench.py at 4 images)
    const bool v6auto = tiles256 < g_num_cus && (d.N <= 1280 || tiles6 <= 4 * g_num_cus) &&
                        (d.act != VD_ACT_GEGLU || 2 * tiles256 <= g_num_cus) &&
                        (d.K <= 1280 || (d.K <= 2560 && tiles6 >= 2 * g_num_cus) ||
                         (d.a_mode == VD_A_CONV3X3 && d.K <= 2880 && tiles6 >= 4 * g_num_cus));
    if (path == 6 || (path == 0 && v6auto)) {
      p.ver = 6;
      p.bn = 64;
      int64_t sp = 1;
      // forced v6: aim for >= 2 workgroups per CU, each slice >= 4 k-tiles (the automatic
      // choice never splits: the in-kernel reduction's agent-scope release/acquire fences
      // write back / invalidate L2 and cost ~25 us — profiles/r01_gemm_paths.txt)
      while (path == 6 && tiles6 * sp < 2 * g_num_cus && nk / (sp * 2) >= 4 && sp < 16) sp *= 2;
      p.split = (int)sp;
      const int64_t rtiles6 = ((d.M + G6_BM - 1) / G6_BM) * ((d.N + G6_BN - 1) / G6_BN);  // launched tiles
      p.ws_bytes = p.split > 1 ? (int64_t)p.split * d.M * d.N * 4 + ((rtiles6 * 4 + 255) / 256) * 256 : 0;
      return p;
    }
  }
  const bool v3ok = d.a_mode == VD_A_DENSE && d.N >= 256 && path != 2;
  const int64_t p256 = (d.N + 255) / 256 * 256;
  // measured (tools/kbench.py): v3 wins on the wide projections (qkv, GEGLU) once the
  // grid fills the chip without split-K; v2's persistent stream wins on N <= 640 and
  // on few-tile shapes
  // DiT (tools/dit_kbench.py, M 147456): N 1152 = 4.5 tiles still wins on v3 at K >= 1024
  // (426 vs 500 us at K 1152, 1431 vs 1666 us at K 4608), so the padding bound loosens to
  // 1/8 there; no UNet shape has N >= 768 with K >= 1024 at M >= 65536
  // persistent v3 (round 2) also wins at 1/8 padding with short K: L2 qkv N 1920 -> 2048,
  // K 640: 98 vs 109 us on v2 (profiles/r02_gemm3_persistent.txt)
  const bool v3pad = (p256 - d.N) * 8 <= d.N;
  const int64_t tiles3 = ((M + G3_BM - 1) / G3_BM) * (p256 / 256);
  // GEGLU on v3 only from 3 tiles per CU: after the v2 fragment-order fix (round 2) v2's 256 x 128
  // tiles win the 320-640-tile GEGLUs (4 images L1 46 vs 51 us, L2 41 vs 52; 32 images L4 66 vs
  // 81 us; tools/plan_sweep.py, profiles/r02f_plan_sweep.txt)
  const bool v3auto = v3ok && d.N >= 768 && v3pad && tiles3 >= 256 &&
                      (d.act != VD_ACT_GEGLU || tiles3 >= 3 * g_num_cus);
  if (path == 3 ? v3ok : v3auto) {
    p.ver = 3;
    p.bn = 256;
    p.split = split_for(((M + G3_BM - 1) / G3_BM) * (p256 / 256), nk);
  } else {
    p.ver = 2;
    const int64_t p128 = (d.N + 127) / 128 * 128, p160 = (d.N + 159) / 160 * 160;
    p.bn = d.act != VD_ACT_GEGLU && (p160 < p128 || (p160 == p128 && d.N % 160 == 0)) ? 160 : 128;
    p.split = split_for(((M + G2_BM - 1) / G2_BM) * ((d.N + p.bn - 1) / p.bn), nk);
  }
  p.ws_bytes = p.split > 1 ? (int64_t)p.split * d.M * d.N * 4 : 0;
  return p;
}

// a folded LayerNorm only ever runs on v8 or an unsplit v6: every other outcome of the plan (its
// early exits included) is "no kernel"
Plan plan(const vd_gemm_desc& d) {
  Plan p = plan_core(d);
  if (d.ln_fold_s && p.ver != 8 && !(p.ver == 6 && p.split == 1)) {
    p.ver = 0;
    p.split = 1;
    p.ws_bytes = 0;
  }
  return p;
}

}  // namespace

// kt <= 1 (a plain 2-D conv or any dense GEMM): one "frame" per video, no temporal offset,
// so the conv loaders' temporal arithmetic reduces to the 2-D one.
vd_gemm_desc normalized(const vd_gemm_desc& in) {
  vd_gemm_desc d = in;
  if (d.a_mode != VD_A_CONV3X3 || d.ks <= 0) d.ks = 3;
  if (d.a_mode != VD_A_CONV3X3 || d.kt <= 1) {
    d.kt = 1;
    d.frames_in = d.frames_out = 1;
    d.t_off = 0;
  }
  return d;
}

extern "C" int64_t vd_gemm_ws_bytes(const vd_gemm_desc* d) { return d ? plan(normalized(*d)).ws_bytes : 0; }

extern "C" int vd_gemm_plan(const vd_gemm_desc* d, int32_t* kernel, int32_t* split) {
  if (!d || !kernel || !split) return VD_EINVAL;
  const Plan p = plan(normalized(*d));
  *kernel = p.ver;
  *split = p.split;
  return VD_OK;
}

extern "C" int vd_gemm(const vd_gemm_desc* dp, vd_stream_t stream) {
  if (!dp) return VD_EINVAL;
  if (dp->a_mode == VD_A_CONV3X3 && (dp->kt > 1 || dp->ks == 1)) {
    VD_CHECK_ARG((dp->kt <= 1 || dp->kt == 3) && (dp->ks == 1 || dp->ks == 3 || dp->ks == 0));
    VD_CHECK_ARG(dp->upsample == 0);
  }
  if (dp->a_mode == VD_A_CONV3X3 && dp->kt > 1) {
    VD_CHECK_ARG(dp->frames_in > 0 && dp->frames_out > 0);
    VD_CHECK_ARG(dp->n_img % dp->frames_out == 0 && dp->t_off >= 0 && dp->t_off + dp->frames_out <= dp->frames_in);
  }
  const vd_gemm_desc d = normalized(*dp);
  hipStream_t s = (hipStream_t)stream;
  VD_CHECK_ARG(d.M >= 0 && d.N > 0 && d.K > 0);
  if (d.M == 0) return VD_OK;
  VD_CHECK_ARG(d.K % 8 == 0 && d.N % 4 == 0 && d.ldw % 8 == 0 && d.ldw >= d.K);
  VD_CHECK_ARG(d.a0 && d.w && d.out && al16(d.a0) && al16(d.w));
  VD_CHECK_ARG(d.lda0 % 8 == 0 && d.k0 % 8 == 0 && d.k0 > 0);
  if (d.a1) VD_CHECK_ARG(al16(d.a1) && d.lda1 % 8 == 0);
  VD_CHECK_ARG(d.ldc % 4 == 0);
  VD_CHECK_ARG(d.M * d.ldc < 0x7fffffff && (!d.res || d.M * d.ld_res < 0x7fffffff) && d.N < 0x7fffffff);
  VD_CHECK_ARG(d.out_f32 ? al16(d.out) : al8(d.out));
  if (d.bias) VD_CHECK_ARG(al16(d.bias));
  if (d.rowbias) VD_CHECK_ARG(al16(d.rowbias) && d.ld_rb % 4 == 0 && d.rb_div > 0);
  if (d.res) VD_CHECK_ARG(al8(d.res) && d.ld_res % 4 == 0);
  VD_CHECK_ARG(d.act == VD_ACT_NONE || d.act == VD_ACT_SILU || d.act == VD_ACT_GEGLU || d.act == VD_ACT_GELU);
  if (d.a_mode == VD_A_CONV3X3) {
    VD_CHECK_ARG(d.K % (d.ks * d.ks * d.kt) == 0);
    const int64_t cin = d.K / (d.ks * d.ks * d.kt);
    VD_CHECK_ARG(cin % 8 == 0 && d.k0 <= cin);
    if (d.k0 < cin) VD_CHECK_ARG(d.a1 != nullptr);
    VD_CHECK_ARG(d.stride == 1 || d.stride == 2);
    VD_CHECK_ARG(d.upsample == 0 || (d.upsample == 1 && d.stride == 1));
    VD_CHECK_ARG(d.n_img > 0 && d.h_in > 0 && d.w_in > 0 && d.h_out > 0 && d.w_out > 0);
    VD_CHECK_ARG(d.M == (int64_t)d.n_img * d.h_out * d.w_out);
    if (d.upsample) VD_CHECK_ARG(d.h_out == 2 * d.h_in && d.w_out == 2 * d.w_in);
    else VD_CHECK_ARG(d.h_out == (d.h_in - 1) / d.stride + 1 && d.w_out == (d.w_in - 1) / d.stride + 1);
    VD_CHECK_ARG((int64_t)d.n_img / d.frames_out * d.frames_in * d.h_in * d.w_in < 0x7fffffff);
  } else {
    VD_CHECK_ARG(d.a_mode == VD_A_DENSE);
    if (d.k0 < d.K) VD_CHECK_ARG(d.a1 != nullptr);
  }
  if (d.act == VD_ACT_GEGLU) VD_CHECK_ARG(d.N % 32 == 0 && !d.res && !d.rowbias && !d.out_f32);
  VD_CHECK_ARG(d.rmap_inner >= 0);
  if (d.rmap_inner > 0)
    VD_CHECK_ARG(Rev3::ok(d.M, d.rmap_n1, d.rmap_n2, d.rmap_inner) && !d.ln_out && !d.rowbias &&
                 d.act != VD_ACT_GEGLU);
  if (d.ln_fold_s) {
    VD_CHECK_ARG(al16(d.ln_fold_s) && d.ln_fold_eps >= 0.f && !d.res && !d.ln_out && !d.rmap_inner &&
                 d.a_mode == VD_A_DENSE && !d.a1 && d.k0 == d.K);
  }
  if (d.ln_out) {
    VD_CHECK_ARG(!d.out_f32 && d.act != VD_ACT_GEGLU && d.ln_gamma && d.ln_beta && al16(d.ln_gamma) &&
                 al16(d.ln_beta) && d.ld_ln % 4 == 0 && al8(d.ln_out) && d.N % 4 == 0);
    if (d.ln_pe) VD_CHECK_ARG(al16(d.ln_pe) && d.ln_pe_div > 0 && d.ln_pe_period > 0);
  }
  const Plan p = plan(d);
  if (p.ver == 0) return VD_EUNSUPPORTED;  // a folded LayerNorm no kernel takes at this shape
  if (p.ver >= 2 && p.split > 1) VD_CHECK_ARG(d.ws && al16(d.ws) && d.ws_bytes >= p.ws_bytes);
  if (d.ln_out && !p.ln_fused) {  // the GEMM, then vd_layernorm over its output
    vd_gemm_desc g = d;
    g.ln_out = nullptr;
    const int rc = vd_gemm(&g, stream);
    if (rc != VD_OK) return rc;
    return vd_layernorm(d.out, d.ldc, d.M, d.N, d.ln_gamma, d.ln_beta, d.ln_eps, d.ln_pe, d.ln_pe_div,
                        d.ln_pe_period, d.ln_out, d.ld_ln, stream);
  }
  if (p.ver == 9) return launch9(d, s);
  if (p.ver == 8) return launch8(d, s, p.a0b, p.wb);
  if (p.ver == 3) return launch3(d, s, p.a0b, p.a1b, p.wb, p.split);
  if (p.ver == 6) return launch6(d, s, p.a0b, p.a1b, p.wb, p.split);
  if (p.ver == 5) return launch4<320, 4, 2, 4>(d, s, p.a0b, p.a1b, p.wb, p.split);
  if (p.ver == 2)
    return p.bn == 160 ? launch2<160>(d, s, p.a0b, p.a1b, p.wb, p.split)
           : p.bn == 32 ? launch2<32>(d, s, p.a0b, p.a1b, p.wb, p.split)
                        : launch2<128>(d, s, p.a0b, p.a1b, p.wb, p.split);
  if (d.act == VD_ACT_GEGLU) return launch<128, 128>(d, s);
  // N tile: least padding, then fewer tiles.
  if (d.N <= 64) return launch<128, 64>(d, s);
  const int64_t p128 = (d.N + 127) / 128 * 128, p160 = (d.N + 159) / 160 * 160;
  if (p160 < p128 || (p160 == p128 && d.N % 160 == 0)) return launch<128, 160>(d, s);
  return launch<128, 128>(d, s);
}
