// Step glue: timestep embedding, latent layout conversion, the fused
// CFG-combine + DDIM update, and the row-block transpose used by the frame
// <-> position re-shard.  All HBM-bound elementwise kernels.
//
// vd_ddim_cfg_step fuses SURVEY.md §8a a1 (eps = e_u + g (e_c - e_u)) and a13
// (diffusers:DDIMScheduler.step, eta 0, epsilon prediction — App. A.7):
//   x0 = (x - sqrt(1-a_t) eps) / sqrt(a_t);  x <- sqrt(a_p) x0 + sqrt(1-a_p) eps
// reading the conv_out rows directly (NHWC fp32) and, optionally, writing the
// next step's packed bf16 UNet input (the CFG cat([x, x])) in the same pass.
// Coefficients come from a device table indexed by a device step counter so a
// captured hipGraph of one step can be replayed for every timestep.
#include "common.h"

namespace {

constexpr int NT = 256;

// fp32 quotient, correctly rounded (via double: 53 >= 2*24 + 2, so the second rounding is
// innocuous) — the GPU's default f32 division is a reciprocal-refinement sequence
__device__ __forceinline__ float div_rn(float a, float b) { return (float)((double)a / (double)b); }


// Step index into a device table of n entries, clamped to [0, n-1]: a graph replayed past the
// end of its schedule (run(n) beyond n_steps without reset()) keeps reading the last row
// instead of memory past the table (the host loops raise before that happens).
__device__ __forceinline__ int table_row(const int32_t* step_idx, int64_t n) {
  int st = step_idx ? *step_idx : 0;
  st = st < 0 ? 0 : st;
  return (int64_t)st < n ? st : (int)(n - 1);
}

__global__ void timestep_embed_kernel(const float* ts, int64_t n_ts, const int32_t* step_idx, int64_t B, int dim,
                                      bf16_t* out) {
  const int half = dim / 2;
  const int64_t total = B * dim;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int64_t b = i / dim;
    const int c = (int)(i - b * dim);
    const float t = step_idx ? ts[table_row(step_idx, n_ts)] : ts[b];
    const int j = c < half ? c : c - half;
    // diffusers get_timestep_embedding: exp(-ln(1e4) * j / half); flip -> [cos, sin]
    const float freq = expf(-9.210340371976184f * (float)j / (float)half);
    const float arg = t * freq;
    out[i] = f2bf(c < half ? cosf(arg) : sinf(arg));
  }
}

__global__ void pack_latents_kernel(const float* x, int64_t B, int64_t C, int64_t F, int64_t HW,
                                    int dup, bf16_t* out, int64_t cpad, float in_div) {
  // out row r = ((d*B + b)*F + f)*HW + p, channel c  <-  x[b][c][f][p] / in_div
  const int64_t rows = dup * B * F * HW;
  const int64_t total = rows * cpad;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int64_t r = i / cpad;
    const int64_t c = i - r * cpad;
    const int64_t p = r % HW;
    const int64_t f = (r / HW) % F;
    const int64_t b = (r / (HW * F)) % B;
    float val = 0.f;
    if (c < C) val = in_div == 1.f ? x[((b * C + c) * F + f) * HW + p] : div_rn(x[((b * C + c) * F + f) * HW + p], in_div);
    out[i] = f2bf(val);
  }
}

__global__ void unpack_kernel(const void* src, int src_f32, int64_t ld, int64_t B, int64_t C,
                              int64_t F, int64_t HW, float* dst) {
  const int64_t total = B * C * F * HW;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int64_t p = i % HW;
    const int64_t f = (i / HW) % F;
    const int64_t c = (i / (HW * F)) % C;
    const int64_t b = i / (HW * F * C);
    const int64_t r = (b * F + f) * HW + p;
    dst[i] = src_f32 ? ((const float*)src)[r * ld + c] : bf2f(((const bf16_t*)src)[r * ld + c]);
  }
}

// fp32 in diffusers' operation order with one rounding per operation (no contraction,
// correctly rounded division), as torch's separate fp32 ops: bit-exact vs oracle/ddim_ref.py.
__global__ void ddim_cfg_kernel(const float* eps, int64_t ld_eps, int ncfg, float g, float* lat,
                                int64_t B, int64_t C, int64_t F, int64_t HW, const float* coef,
                                int64_t n_coef, const int32_t* step_idx, float* x0_out, bf16_t* next_in,
                                int64_t cpad) {
#pragma clang fp contract(off)
  const int st = table_row(step_idx, n_coef);
  const float sat = coef[4 * st + 0], s1at = coef[4 * st + 1];
  const float sap = coef[4 * st + 2], s1ap = coef[4 * st + 3];
  const int64_t total = B * C * F * HW;
  const int64_t half_rows = B * F * HW;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int64_t p = i % HW;
    const int64_t f = (i / HW) % F;
    const int64_t c = (i / (HW * F)) % C;
    const int64_t b = i / (HW * F * C);
    const int64_t r = (b * F + f) * HW + p;
    float e = eps[r * ld_eps + c];
    if (ncfg == 2) {
      const float ec = eps[(r + half_rows) * ld_eps + c];
      e = e + g * (ec - e);
    }
    const float x = lat[i];
    const float x0 = div_rn(x - s1at * e, sat);
    const float xn = sap * x0 + s1ap * e;
    lat[i] = xn;
    if (x0_out) x0_out[i] = x0;
    if (next_in) {
      const bf16_t v = f2bf(xn);
      next_in[r * cpad + c] = v;
      if (ncfg == 2) next_in[(r + half_rows) * cpad + c] = v;
    }
  }
}

// CFG combine + diffusers:EulerDiscreteScheduler.step (s_churn = 0, epsilon
// prediction), in diffusers' fp32 operation order:
//   x0 = x - sigma*eps;  d = (x - x0) / sigma;  x <- x + d * (sigma_next - sigma)
// and the next step's UNet input = scale_model_input(x, sigma_next) = x / sqrt(sigma_next^2 + 1)
// (coef[4*st] = {sigma, sigma_next, sqrt(sigma_next^2 + 1), 0}).
__global__ void euler_cfg_kernel(const float* eps, int64_t ld_eps, int ncfg, float g, float* lat,
                                 int64_t B, int64_t C, int64_t F, int64_t HW, const float* coef,
                                 int64_t n_coef, const int32_t* step_idx, float* x0_out, bf16_t* next_in,
                                 int64_t cpad) {
#pragma clang fp contract(off)  // one rounding per operation, as torch's separate fp32 ops
  const int st = table_row(step_idx, n_coef);
  const float sig = coef[4 * st + 0], sig_n = coef[4 * st + 1], in_div = coef[4 * st + 2];
  const float dt = sig_n - sig;
  const int64_t total = B * C * F * HW;
  const int64_t half_rows = B * F * HW;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int64_t p = i % HW;
    const int64_t f = (i / HW) % F;
    const int64_t c = (i / (HW * F)) % C;
    const int64_t b = i / (HW * F * C);
    const int64_t r = (b * F + f) * HW + p;
    float e = eps[r * ld_eps + c];
    if (ncfg == 2) {
      const float ec = eps[(r + half_rows) * ld_eps + c];
      e = e + g * (ec - e);
    }
    const float x = lat[i];
    const float x0 = x - sig * e;
    const float d = div_rn(x - x0, sig);
    const float xn = x + d * dt;
    lat[i] = xn;
    if (x0_out) x0_out[i] = x0;
    if (next_in) {
      const bf16_t v = f2bf(div_rn(xn, in_div));
      next_in[r * cpad + c] = v;
      if (ncfg == 2) next_in[(r + half_rows) * cpad + c] = v;
    }
  }
}

__global__ void step_advance_kernel(int32_t* step_idx) { *step_idx += 1; }

__global__ void block_transpose_kernel(const bf16_t* src, bf16_t* dst, int64_t nb, int64_t na,
                                       int64_t nc, int64_t width) {
  // dst[((a*nb + b)*nc + c)][:] = src[((b*na + a)*nc + c)][:], 16-byte chunks
  const int64_t wch = width / 8;
  const int64_t total = nb * na * nc * wch;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int64_t ch = i % wch;
    const int64_t drow = i / wch;
    const int64_t c = drow % nc;
    const int64_t ab = drow / nc;
    const int64_t b = ab % nb, a = ab / nb;
    const int64_t srow = (b * na + a) * nc + c;
    *(uint4*)(dst + drow * width + ch * 8) = *(const uint4*)(src + srow * width + ch * 8);
  }
}

unsigned grid_for(int64_t total) {
  const int64_t b = (total + NT - 1) / NT;
  return (unsigned)(b < 16384 ? (b > 0 ? b : 1) : 16384);
}

}  // namespace

extern "C" int vd_timestep_embed(const float* ts, int64_t n_ts, const int32_t* step_idx, int64_t B,
                                 int32_t dim, void* out, vd_stream_t stream) {
  VD_CHECK_ARG(ts && out && B > 0 && dim > 0 && dim % 2 == 0 && n_ts > 0);
  if (!step_idx) VD_CHECK_ARG(n_ts >= B);
  hipLaunchKernelGGL(timestep_embed_kernel, dim3(grid_for(B * dim)), dim3(NT), 0,
                     (hipStream_t)stream, ts, n_ts, step_idx, B, dim, (bf16_t*)out);
  return vd_launch_status();
}

extern "C" int vd_pack_latents(const float* x, int64_t B, int64_t C, int64_t F, int64_t H,
                               int64_t W, int32_t dup, void* out, int64_t cpad, float in_div,
                               vd_stream_t stream) {
  VD_CHECK_ARG(x && out && B > 0 && C > 0 && F > 0 && H > 0 && W > 0 && cpad >= C && dup >= 1 && in_div > 0.f);
  const int64_t total = dup * B * F * H * W * cpad;
  hipLaunchKernelGGL(pack_latents_kernel, dim3(grid_for(total)), dim3(NT), 0, (hipStream_t)stream,
                     x, B, C, F, H * W, dup, (bf16_t*)out, cpad, in_div);
  return vd_launch_status();
}

extern "C" int vd_unpack_nhwc(const void* src, int32_t src_f32, int64_t ld, int64_t B, int64_t C,
                              int64_t F, int64_t H, int64_t W, float* dst, vd_stream_t stream) {
  VD_CHECK_ARG(src && dst && ld >= C && B > 0 && C > 0 && F > 0 && H > 0 && W > 0);
  hipLaunchKernelGGL(unpack_kernel, dim3(grid_for(B * C * F * H * W)), dim3(NT), 0,
                     (hipStream_t)stream, src, src_f32, ld, B, C, F, H * W, dst);
  return vd_launch_status();
}

extern "C" int vd_ddim_cfg_step(const float* eps, int64_t ld_eps, int32_t ncfg, float guidance,
                                float* latents, int64_t B, int64_t C, int64_t F, int64_t H,
                                int64_t W, const float* coef, int64_t n_coef, const int32_t* step_idx,
                                float* x0_out, void* next_in, int64_t cpad, vd_stream_t stream) {
  VD_CHECK_ARG(eps && latents && coef && n_coef > 0 && (ncfg == 1 || ncfg == 2) && ld_eps >= C);
  if (next_in) VD_CHECK_ARG(cpad >= C);
  hipLaunchKernelGGL(ddim_cfg_kernel, dim3(grid_for(B * C * F * H * W)), dim3(NT), 0,
                     (hipStream_t)stream, eps, ld_eps, ncfg, guidance, latents, B, C, F, H * W,
                     coef, n_coef, step_idx, x0_out, (bf16_t*)next_in, cpad);
  return vd_launch_status();
}

extern "C" int vd_euler_cfg_step(const float* eps, int64_t ld_eps, int32_t ncfg, float guidance,
                                 float* latents, int64_t B, int64_t C, int64_t F, int64_t H,
                                 int64_t W, const float* coef, int64_t n_coef, const int32_t* step_idx,
                                 float* x0_out, void* next_in, int64_t cpad, vd_stream_t stream) {
  VD_CHECK_ARG(eps && latents && coef && n_coef > 0 && (ncfg == 1 || ncfg == 2) && ld_eps >= C);
  if (next_in) VD_CHECK_ARG(cpad >= C);
  hipLaunchKernelGGL(euler_cfg_kernel, dim3(grid_for(B * C * F * H * W)), dim3(NT), 0,
                     (hipStream_t)stream, eps, ld_eps, ncfg, guidance, latents, B, C, F, H * W,
                     coef, n_coef, step_idx, x0_out, (bf16_t*)next_in, cpad);
  return vd_launch_status();
}

extern "C" int vd_step_advance(int32_t* step_idx, vd_stream_t stream) {
  VD_CHECK_ARG(step_idx);
  hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, step_idx);
  return vd_launch_status();
}

extern "C" int vd_block_transpose(const void* src, void* dst, int64_t nb, int64_t na, int64_t nc,
                                  int64_t width, vd_stream_t stream) {
  VD_CHECK_ARG(src && dst && src != dst && width % 8 == 0 && nb > 0 && na > 0 && nc > 0);
  VD_CHECK_ARG(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0);
  hipLaunchKernelGGL(block_transpose_kernel, dim3(grid_for(nb * na * nc * (width / 8))), dim3(NT), 0,
                     (hipStream_t)stream, (const bf16_t*)src, (bf16_t*)dst, nb, na, nc, width);
  return vd_launch_status();
}

extern "C" const char* vd_strerror(int code) {
  switch (code) {
    case VD_OK: return "ok";
    case VD_EINVAL: return "vdiff: invalid argument (shape/stride/alignment)";
    case VD_EUNSUPPORTED: return "vdiff: unsupported parameter (no compiled variant)";
    case VD_ERCCL: return "vdiff: RCCL call failed";
    default: return hipGetErrorString((hipError_t)code);
  }
}

extern "C" int vd_version(void) { return 6; }  // 6: vd_gn_finalize_g_ranks (round 6); 5: vd_gemm_desc rmap_* / ln_fold_*, vd_gemm_plan, vd_gn_apply_rev3, fp8 q_scale (round 5)

#ifndef VD_BUILD_HASH
#define VD_BUILD_HASH "unhashed"
#endif
// Content hash of the sources + flags this library was built from (build_ext.py);
// vdiff._lib refuses to load a library whose hash differs from the tree's sources.
extern "C" const char* vd_build_hash(void) { return VD_BUILD_HASH; }

#ifndef VD_BUILD_ARCH
#define VD_BUILD_ARCH "gfx950"
#endif
// The --offload-arch the library was compiled for (kept out of the content hash).
extern "C" const char* vd_build_arch(void) { return VD_BUILD_ARCH; }
