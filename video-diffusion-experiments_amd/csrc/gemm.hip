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

  // Per staged A row: pixel coordinates for the conv gather.
  int pimg[RA], poh[RA], pow_[RA];
  bool prow[RA];
  int cin = 0, hgrid = 0, wgrid = 0;
  if constexpr (MODE == VD_A_CONV3X3) {
    cin = (int)d.K / 9;
    hgrid = d.upsample ? 2 * d.h_in : d.h_in;
    wgrid = d.upsample ? 2 * d.w_in : d.w_in;
    const int hw = d.h_out * d.w_out;
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const int64_t m = m0 + sr + 32 * i;
      prow[i] = m < M;
      const int mm = prow[i] ? (int)m : 0;
      pimg[i] = mm / hw;
      const int p = mm - pimg[i] * hw;
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
      const int tap = kin ? (int)(k / cin) : 0;
      const int ci = (int)k - tap * cin;
      const int dy = tap / 3, dx = tap - 3 * (tap / 3);
      const bool in0 = ci < d.k0;
      const bf16_t* base = in0 ? a0 + ci : a1 + (ci - d.k0);
      const int64_t ld = in0 ? d.lda0 : d.lda1;
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        int ih = poh[i] * d.stride + dy - 1;
        int iw = pow_[i] * d.stride + dx - 1;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (kin && prow[i] && ih >= 0 && ih < hgrid && iw >= 0 && iw < wgrid) {
          ih >>= d.upsample;
          iw >>= d.upsample;
          const int64_t pix = ((int64_t)pimg[i] * d.h_in + ih) * d.w_in + iw;
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

  // ---------------------------------------------------------------- epilogue
  // acc[a][b][j] = C[m = m0 + wm*BM/2 + b*16 + fr][n = n0 + wn*BN/2 + a*16 + 4*fq + j]
  const int64_t nw = n0 + wn * (BN / 2);
  if (d.act == VD_ACT_GEGLU) {
    if constexpr (NB % 2 == 0) {
#pragma unroll
      for (int a = 0; a < NB; a += 2) {
        const int64_t nh = nw + a * 16 + 4 * fq;        // packed hidden column
        const int64_t ng = nh + 16;                      // packed gate column
        if (ng >= N) continue;
        const int64_t nout = nw / 2 + (a / 2) * 16 + 4 * fq;
        float bh[4] = {0, 0, 0, 0}, bg[4] = {0, 0, 0, 0};
        if (d.bias) {
          const float4 t0 = *(const float4*)(d.bias + nh);
          const float4 t1 = *(const float4*)(d.bias + ng);
          bh[0] = t0.x; bh[1] = t0.y; bh[2] = t0.z; bh[3] = t0.w;
          bg[0] = t1.x; bg[1] = t1.y; bg[2] = t1.z; bg[3] = t1.w;
        }
#pragma unroll
        for (int b = 0; b < MB; ++b) {
          const int64_t m = m0 + wm * (BM / 2) + b * 16 + fr;
          if (m >= M) continue;
          float o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = (acc[a][b][j] + bh[j]) * gelu_erf(acc[a + 1][b][j] + bg[j]);
          bf16_t* op = (bf16_t*)d.out + m * d.ldc + nout;
          *(uint2*)op = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
        }
      }
    }
    return;
  }
#pragma unroll
  for (int a = 0; a < NB; ++a) {
    const int64_t n = nw + a * 16 + 4 * fq;
    if (n >= N) continue;
    float bv[4] = {0, 0, 0, 0};
    if (d.bias) {
      const float4 t = *(const float4*)(d.bias + n);
      bv[0] = t.x; bv[1] = t.y; bv[2] = t.z; bv[3] = t.w;
    }
#pragma unroll
    for (int b = 0; b < MB; ++b) {
      const int64_t m = m0 + wm * (BM / 2) + b * 16 + fr;
      if (m >= M) continue;
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = acc[a][b][j] + bv[j];
      if (d.rowbias) {
        const float4 t = *(const float4*)(d.rowbias + (m / d.rb_div) * d.ld_rb + n);
        o[0] += t.x; o[1] += t.y; o[2] += t.z; o[3] += t.w;
      }
      if (d.act == VD_ACT_SILU) {
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = silu_f(o[j]);
      }
      if (d.res) {
        const uint2 r = *(const uint2*)((const bf16_t*)d.res + m * d.ld_res + n);
        o[0] += bf_lo(r.x); o[1] += bf_hi(r.x); o[2] += bf_lo(r.y); o[3] += bf_hi(r.y);
      }
      if (d.out_f32) {
        *(float4*)((float*)d.out + m * d.ldc + n) = make_float4(o[0], o[1], o[2], o[3]);
      } else {
        *(uint2*)((bf16_t*)d.out + m * d.ldc + n) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
      }
    }
  }
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

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
inline bool al8(const void* p) { return ((uintptr_t)p & 7) == 0; }

}  // namespace

extern "C" int vd_gemm(const vd_gemm_desc* dp, vd_stream_t stream) {
  if (!dp) return VD_EINVAL;
  const vd_gemm_desc& d = *dp;
  hipStream_t s = (hipStream_t)stream;
  VD_CHECK_ARG(d.M >= 0 && d.N > 0 && d.K > 0);
  if (d.M == 0) return VD_OK;
  VD_CHECK_ARG(d.K % 8 == 0 && d.N % 4 == 0 && d.ldw % 8 == 0 && d.ldw >= d.K);
  VD_CHECK_ARG(d.a0 && d.w && d.out && al16(d.a0) && al16(d.w));
  VD_CHECK_ARG(d.lda0 % 8 == 0 && d.k0 % 8 == 0 && d.k0 > 0);
  if (d.a1) VD_CHECK_ARG(al16(d.a1) && d.lda1 % 8 == 0);
  VD_CHECK_ARG(d.ldc % 4 == 0);
  VD_CHECK_ARG(d.out_f32 ? al16(d.out) : al8(d.out));
  if (d.bias) VD_CHECK_ARG(al16(d.bias));
  if (d.rowbias) VD_CHECK_ARG(al16(d.rowbias) && d.ld_rb % 4 == 0 && d.rb_div > 0);
  if (d.res) VD_CHECK_ARG(al8(d.res) && d.ld_res % 4 == 0);
  VD_CHECK_ARG(d.act == VD_ACT_NONE || d.act == VD_ACT_SILU || d.act == VD_ACT_GEGLU);
  if (d.a_mode == VD_A_CONV3X3) {
    VD_CHECK_ARG(d.K % 9 == 0);
    const int64_t cin = d.K / 9;
    VD_CHECK_ARG(cin % 8 == 0 && d.k0 <= cin);
    if (d.k0 < cin) VD_CHECK_ARG(d.a1 != nullptr);
    VD_CHECK_ARG(d.stride == 1 || d.stride == 2);
    VD_CHECK_ARG(d.upsample == 0 || (d.upsample == 1 && d.stride == 1));
    VD_CHECK_ARG(d.n_img > 0 && d.h_in > 0 && d.w_in > 0 && d.h_out > 0 && d.w_out > 0);
    VD_CHECK_ARG(d.M == (int64_t)d.n_img * d.h_out * d.w_out);
    if (d.upsample) VD_CHECK_ARG(d.h_out == 2 * d.h_in && d.w_out == 2 * d.w_in);
    else VD_CHECK_ARG(d.h_out == (d.h_in - 1) / d.stride + 1 && d.w_out == (d.w_in - 1) / d.stride + 1);
    VD_CHECK_ARG((int64_t)d.n_img * d.h_in * d.w_in < 0x7fffffff);
  } else {
    VD_CHECK_ARG(d.a_mode == VD_A_DENSE);
    if (d.k0 < d.K) VD_CHECK_ARG(d.a1 != nullptr);
  }
  if (d.act == VD_ACT_GEGLU) {
    VD_CHECK_ARG(d.N % 32 == 0 && !d.res && !d.rowbias && !d.out_f32);
    return launch<128, 128>(d, s);
  }
  // N tile: least padding, then fewer tiles.
  if (d.N <= 64) return launch<128, 64>(d, s);
  const int64_t p128 = (d.N + 127) / 128 * 128, p160 = (d.N + 159) / 160 * 160;
  if (p160 < p128 || (p160 == p128 && d.N % 160 == 0)) return launch<128, 160>(d, s);
  return launch<128, 128>(d, s);
}
