// DiT-style video denoiser kernels (BASELINE config 5):
// patchify / unpatchify of (B,C,F,H,W) latents, rotary position embedding applied in
// place to the fused QKV rows, and the adaLN "gated residual + LayerNorm + modulate"
// pass.  The reference has no DiT: the model is build-defined and its
// oracle is oracle/dit_ref.py.  Everything here is HBM-bound elementwise / row work:
// 16-byte coalesced accesses along the contiguous channel axis, one wave per row for
// the row reductions, statistics in fp32.
#include "common.h"

namespace {

constexpr int NT = 256;

unsigned grid_of(int64_t total) {
  const int64_t b = (total + NT - 1) / NT;
  return (unsigned)(b < 32768 ? (b > 0 ? b : 1) : 32768);
}

// latents fp32 (B, C, F, H, W) -> token rows bf16 [(b,f,hp,wp)][kpad], patch vector
// k = (c*p + ph)*p + pw (the flattening of a Conv3d(C, D, (1,p,p)) patch-embed weight),
// zero-padded to kpad; dup = 2 writes the CFG copy at row + B*F*Hp*Wp.
__global__ void patchify_kernel(const float* __restrict__ lat, int64_t B, int64_t C, int64_t F,
                                int64_t H, int64_t W, int p, int dup, float in_div,
                                bf16_t* __restrict__ out, int64_t kpad) {
  const int64_t Hp = H / p, Wp = W / p;
  const int64_t rows = B * F * Hp * Wp;
  const int64_t total = rows * kpad;
  const float inv = 1.0f / in_div;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int64_t r = i / kpad;
    const int k = (int)(i % kpad);
    float v = 0.f;
    if (k < C * p * p) {
      const int c = k / (p * p), ph = (k / p) % p, pw = k % p;
      const int64_t wp = r % Wp, hp = (r / Wp) % Hp, f = (r / (Wp * Hp)) % F, b = r / (Wp * Hp * F);
      v = lat[(((b * C + c) * F + f) * H + hp * p + ph) * W + wp * p + pw] * inv;
    }
    const bf16_t o = f2bf(v);
    out[i] = o;
    if (dup == 2) out[i + rows * kpad] = o;
  }
}

// token rows fp32 [(n,hp,wp)][(ph,pw,c)] (ld_src) -> pixel rows fp32 [(n,h,w)][c]
// (the NHWC eps layout the fused CFG+scheduler kernels read).
__global__ void unpatchify_kernel(const float* __restrict__ src, int64_t ld_src, int64_t n_img,
                                  int64_t H, int64_t W, int p, int C, float* __restrict__ dst) {
  const int64_t total = n_img * H * W * C;
  const int64_t Hp = H / p, Wp = W / p;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int c = (int)(i % C);
    const int64_t pix = i / C;
    const int64_t w = pix % W, h = (pix / W) % H, n = pix / (W * H);
    const int64_t r = (n * Hp + h / p) * Wp + w / p;
    const int k = ((int)(h % p) * p + (int)(w % p)) * C + c;
    dst[i] = src[r * ld_src + k];
  }
}

// Rotary embedding (rotate-half pairing) in place on columns [0, ncols) of token rows
// (the q and k slices of a fused QKV buffer), heads of width d.  Token r = ((b*F + f)*Hp
// + h)*Wp + w.  mode 0 (spatial, 2-D): dims [0, d/2) rotate with position h, [d/2, d)
// with w; mode 1 (temporal, 1-D): all d dims with position f.  Inside a section of
// width S the pairs are (i, i + S/2) at angle pos * theta^(-2i/S).  One thread owns 8
// consecutive pairs (two 16-byte loads / stores).  I = uint32_t when rows * ncols fits
// (index divisions in 32 bits: the 64-bit ones cost more than the pass's HBM time).
template <typename I>
__global__ void rope_kernel(bf16_t* __restrict__ x, int64_t ld, int64_t rows, int ncols, int d,
                            int mode, int64_t F, int64_t Hp, int64_t Wp, float log2_theta) {
  const int S = mode == 0 ? d / 2 : d;       // section width
  const int half = S / 2;
  const int chunks_per_row = ncols / 2 / 8;  // 8-pair chunks per row
  const int chunks_per_sec = half / 8;
  const I total = (I)(rows * chunks_per_row);
  const I uF = (I)F, uHp = (I)Hp, uWp = (I)Wp, ucpr = (I)chunks_per_row;
  for (I i = (I)blockIdx.x * NT + threadIdx.x; i < total; i += (I)gridDim.x * NT) {
    const I r = i / ucpr;
    const int cj = (int)(i - r * ucpr);
    const int sec_global = cj / chunks_per_sec;  // (head, section) index
    const int j0 = (cj % chunks_per_sec) * 8;    // first pair index inside the section
    const int col = sec_global * S + j0;
    const int sec = mode == 0 ? (sec_global % 2) : 0;
    I pos;
    if (mode == 0) pos = sec == 0 ? (r / uWp) % uHp : r % uWp;
    else pos = (r / (uWp * uHp)) % uF;
    bf16_t* p0 = x + (int64_t)r * ld + col;
    bf16_t* p1 = p0 + half;
    float a[8], b[8];
    unpack8(*(const uint4*)p0, a);
    unpack8(*(const uint4*)p1, b);
    float oa[8], ob[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float inv_freq = exp2f(-log2_theta * (float)(2 * (j0 + j)) / (float)S);
      float sn, cs;
      // hardware sin/cos (|angle| < 2^12 rad here; error far below the bf16 output's rounding)
      __sincosf((float)pos * inv_freq, &sn, &cs);
      oa[j] = a[j] * cs - b[j] * sn;
      ob[j] = b[j] * cs + a[j] * sn;
    }
    *(uint4*)p0 = pack8(oa);
    *(uint4*)p1 = pack8(ob);
  }
}

// adaLN pass, one wave per row (C <= 64*8*CPL):
//   xn = x + gate[b] * y      (y optional; gate optional -> plain residual add)
//   x_out = bf16(xn)          (optional; may alias x)
//   h = LN(xn; eps, no affine) * (1 + scale[b]) + shift[b]   (shift/scale optional)
// with b = row / rows_per_b and gate/shift/scale rows of stride ld_mod (fp32).
template <int CPL>
__global__ __launch_bounds__(NT) void res_ln_mod_kernel(
    const bf16_t* x, int64_t ldx, const bf16_t* __restrict__ y, int64_t ldy,
    const float* __restrict__ gate, const float* __restrict__ shift, const float* __restrict__ scale,
    int64_t ld_mod, int64_t rows_per_b, bf16_t* x_out, int64_t ldxo, bf16_t* __restrict__ h,
    int64_t ldh, int64_t rows, int C, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int64_t bidx = row / rows_per_b;
  const int nch = C / 8;
  float v[CPL][8];
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < CPL; ++t) {
    const int ch = lane + 64 * t;
    if (ch < nch) {
      unpack8(*(const uint4*)(x + row * ldx + ch * 8), v[t]);
      if (y) {
        float yy[8];
        unpack8(*(const uint4*)(y + row * ldy + ch * 8), yy);
        if (gate) {
          const float* g = gate + bidx * ld_mod + ch * 8;
          const float4 g0 = *(const float4*)g, g1 = *(const float4*)(g + 4);
          yy[0] *= g0.x; yy[1] *= g0.y; yy[2] *= g0.z; yy[3] *= g0.w;
          yy[4] *= g1.x; yy[5] *= g1.y; yy[6] *= g1.z; yy[7] *= g1.w;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[t][j] = bf2f(f2bf(v[t][j] + yy[j]));  // the stored residual
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[t][j];
    }
  }
  const float mean = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int t = 0; t < CPL; ++t) {
    const int ch = lane + 64 * t;
    if (ch < nch) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float dv = v[t][j] - mean;
        q += dv * dv;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)C + eps);
#pragma unroll
  for (int t = 0; t < CPL; ++t) {
    const int ch = lane + 64 * t;
    if (ch < nch) {
      if (x_out && y) *(uint4*)(x_out + row * ldxo + ch * 8) = pack8(v[t]);
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[t][j] - mean) * rstd;
      if (scale) {
        const float* sc = scale + bidx * ld_mod + ch * 8;
        const float4 a0 = *(const float4*)sc, a1 = *(const float4*)(sc + 4);
        o[0] *= 1.f + a0.x; o[1] *= 1.f + a0.y; o[2] *= 1.f + a0.z; o[3] *= 1.f + a0.w;
        o[4] *= 1.f + a1.x; o[5] *= 1.f + a1.y; o[6] *= 1.f + a1.z; o[7] *= 1.f + a1.w;
      }
      if (shift) {
        const float* sh = shift + bidx * ld_mod + ch * 8;
        const float4 a0 = *(const float4*)sh, a1 = *(const float4*)(sh + 4);
        o[0] += a0.x; o[1] += a0.y; o[2] += a0.z; o[3] += a0.w;
        o[4] += a1.x; o[5] += a1.y; o[6] += a1.z; o[7] += a1.w;
      }
      *(uint4*)(h + row * ldh + ch * 8) = pack8(o);
    }
  }
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" int vd_patchify(const float* lat, int64_t B, int64_t C, int64_t F, int64_t H, int64_t W,
                           int32_t p, int32_t dup, float in_div, void* out, int64_t kpad,
                           vd_stream_t stream) {
  VD_CHECK_ARG(lat && out && p >= 1 && H % p == 0 && W % p == 0 && (dup == 1 || dup == 2));
  VD_CHECK_ARG(kpad >= C * p * p && B > 0 && C > 0 && F > 0 && in_div != 0.f);
  const int64_t total = B * F * (H / p) * (W / p) * kpad;
  hipLaunchKernelGGL(patchify_kernel, dim3(grid_of(total)), dim3(NT), 0, (hipStream_t)stream, lat, B,
                     C, F, H, W, (int)p, (int)dup, in_div, (bf16_t*)out, kpad);
  return vd_launch_status();
}

extern "C" int vd_unpatchify(const float* src, int64_t ld_src, int64_t n_img, int64_t H, int64_t W,
                             int32_t p, int32_t C, float* dst, vd_stream_t stream) {
  VD_CHECK_ARG(src && dst && p >= 1 && H % p == 0 && W % p == 0 && ld_src >= (int64_t)p * p * C);
  hipLaunchKernelGGL(unpatchify_kernel, dim3(grid_of(n_img * H * W * C)), dim3(NT), 0,
                     (hipStream_t)stream, src, ld_src, n_img, H, W, (int)p, (int)C, dst);
  return vd_launch_status();
}

extern "C" int vd_rope_qk(void* x, int64_t ld, int64_t rows, int32_t ncols, int32_t d, int32_t mode,
                          int64_t F, int64_t Hp, int64_t Wp, float theta, vd_stream_t stream) {
  VD_CHECK_ARG(x && al16(x) && ld % 8 == 0 && rows > 0 && d > 0 && ncols % d == 0 && ncols <= ld);
  VD_CHECK_ARG(mode == 0 || mode == 1);
  VD_CHECK_ARG(mode == 0 ? d % 32 == 0 : d % 16 == 0);
  VD_CHECK_ARG(F > 0 && Hp > 0 && Wp > 0 && theta > 1.f);
  const int64_t total = rows * (ncols / 16);
  auto kern = total < 0x7fffffff && Hp * Wp < 0x7fffffff ? rope_kernel<uint32_t> : rope_kernel<int64_t>;
  hipLaunchKernelGGL(kern, dim3(grid_of(total)), dim3(NT), 0, (hipStream_t)stream, (bf16_t*)x,
                     ld, rows, (int)ncols, (int)d, (int)mode, F, Hp, Wp, log2f(theta));
  return vd_launch_status();
}

extern "C" int vd_res_ln_mod(const void* x, int64_t ldx, const void* y, int64_t ldy,
                             const float* gate, const float* shift, const float* scale,
                             int64_t ld_mod, int64_t rows_per_b, void* x_out, int64_t ldxo, void* h,
                             int64_t ldh, int64_t rows, int64_t C, float eps, vd_stream_t stream) {
  VD_CHECK_ARG(x && h && rows > 0 && C % 8 == 0 && C > 0 && C <= 64 * 8 * 4 && rows_per_b > 0);
  VD_CHECK_ARG(al16(x) && al16(h) && ldx % 8 == 0 && ldh % 8 == 0);
  if (y) VD_CHECK_ARG(al16(y) && ldy % 8 == 0);
  if (x_out) VD_CHECK_ARG(y && al16(x_out) && ldxo % 8 == 0);
  if (gate || shift || scale) VD_CHECK_ARG(ld_mod % 4 == 0);
  if (gate) VD_CHECK_ARG(al16(gate));
  if (shift) VD_CHECK_ARG(al16(shift));
  if (scale) VD_CHECK_ARG(al16(scale));
  const dim3 grid((unsigned)((rows + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
#define RLM(CPL)                                                                                          \
  hipLaunchKernelGGL(res_ln_mod_kernel<CPL>, grid, dim3(NT), 0, s, (const bf16_t*)x, ldx, (const bf16_t*)y, \
                     ldy, gate, shift, scale, ld_mod, rows_per_b, (bf16_t*)x_out, ldxo, (bf16_t*)h, ldh,  \
                     rows, (int)C, eps)
  if (C <= 512) RLM(1);
  else if (C <= 1024) RLM(2);
  else if (C <= 1536) RLM(3);
  else RLM(4);
#undef RLM
  return vd_launch_status();
}
