// Elementwise row ops over bf16 NHWC rows: the pieces of diffusers' module-level
// forward that the fused fast path never materialises — residual adds
// (`attn_output + hidden_states`, `hidden_states + residual`), the ResnetBlock2D time
// embedding broadcast (`h + temb[:, :, None, None]`), SinusoidalPositionalEmbedding
// (`x + pe[:, :S]`), `repeat_interleave(num_frames)`, `torch.cat([x, skip], 1)`
// (column slices), `nn.SiLU`, and Upsample2D's `F.interpolate(scale_factor=2,
// mode="nearest")`.  They run when a caller drives the modules one by one (the
// reference's forward-hook tracing, experiments/03_trace_forward_pass.py:105-113 via
// utils/forward_tracer.py:177-206, or a direct motion_modules[i](x, num_frames=F)
// call, 03:182) — so every module's __call__ sees diffusers-shaped tensors while
// all arithmetic stays on HIP kernels.  HBM-bound: 16-byte chunks, one per thread.
#include "common.h"

namespace {

constexpr int NT = 256;

__device__ __forceinline__ void load8_any(const void* p, int is_f32, float* f) {
  if (is_f32) {
    const float4 a = *(const float4*)p, b = *((const float4*)p + 1);
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  } else {
    unpack8(*(const uint4*)p, f);
  }
}

// op 0: out[r] = (x ? x[r] : 0) + y[(r / y_div) % y_period]     (y bf16 or fp32)
// op 1: out[r] = silu(x[r])
__global__ void rows_eltwise_kernel(int op, const bf16_t* x, int64_t ldx, const void* y, int64_t ldy, int y_f32,
                                    int64_t y_div, int64_t y_period, int64_t rows, int64_t C, bf16_t* out,
                                    int64_t ldo) {
  const int64_t cpr = C / 8;
  const int64_t total = rows * cpr;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int64_t r = i / cpr;
    const int64_t c = (i - r * cpr) * 8;
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (x) unpack8(*(const uint4*)(x + r * ldx + c), v);
    if (op == 0) {
      const int64_t yr = (r / y_div) % y_period;
      float w[8];
      load8_any(y_f32 ? (const void*)((const float*)y + yr * ldy + c) : (const void*)((const bf16_t*)y + yr * ldy + c),
                y_f32, w);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += w[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = silu_f(v[j]);
    }
    *(uint4*)(out + r * ldo + c) = pack8(v);
  }
}

// out row (n, y, x) of the 2h x 2w grid <- in row (n, y/2, x/2)
__global__ void upsample2x_kernel(const bf16_t* x, int64_t ldx, int64_t n_img, int64_t h, int64_t w, int64_t C,
                                  bf16_t* out, int64_t ldo) {
  const int64_t cpr = C / 8;
  const int64_t total = n_img * 4 * h * w * cpr;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int64_t r = i / cpr;
    const int64_t c = (i - r * cpr) * 8;
    const int64_t ox = r % (2 * w), oy = (r / (2 * w)) % (2 * h), n = r / (4 * h * w);
    const int64_t src = (n * h + oy / 2) * w + ox / 2;
    *(uint4*)(out + r * ldo + c) = *(const uint4*)(x + src * ldx + c);
  }
}

unsigned grid_for(int64_t total) {
  const int64_t b = (total + NT - 1) / NT;
  return (unsigned)(b < 16384 ? (b > 0 ? b : 1) : 16384);
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" int vd_rows_eltwise(int32_t op, const void* x, int64_t ldx, const void* y, int64_t ldy, int32_t y_f32,
                               int64_t y_div, int64_t y_period, int64_t rows, int64_t C, void* out, int64_t ldo,
                               vd_stream_t stream) {
  VD_CHECK_ARG((op == 0 || op == 1) && out && rows > 0 && C > 0 && C % 8 == 0 && ldo % 8 == 0 && ldo >= C);
  VD_CHECK_ARG(al16(out));
  if (x) VD_CHECK_ARG(al16(x) && ldx % 8 == 0 && ldx >= C);
  if (op == 0) {
    VD_CHECK_ARG(y && al16(y) && ldy >= C && ldy % (y_f32 ? 4 : 8) == 0 && y_div > 0 && y_period > 0);
  } else {
    VD_CHECK_ARG(x != nullptr);
  }
  hipLaunchKernelGGL(rows_eltwise_kernel, dim3(grid_for(rows * (C / 8))), dim3(NT), 0, (hipStream_t)stream, op,
                     (const bf16_t*)x, ldx, y, ldy, y_f32, y_div, y_period, rows, C, (bf16_t*)out, ldo);
  return vd_launch_status();
}

extern "C" int vd_upsample_nearest2x(const void* x, int64_t ldx, int64_t n_img, int64_t h, int64_t w, int64_t C,
                                     void* out, int64_t ldo, vd_stream_t stream) {
  VD_CHECK_ARG(x && out && al16(x) && al16(out) && n_img > 0 && h > 0 && w > 0 && C > 0 && C % 8 == 0);
  VD_CHECK_ARG(ldx % 8 == 0 && ldo % 8 == 0 && ldx >= C && ldo >= C);
  hipLaunchKernelGGL(upsample2x_kernel, dim3(grid_for(n_img * 4 * h * w * (C / 8))), dim3(NT), 0, (hipStream_t)stream,
                     (const bf16_t*)x, ldx, n_img, h, w, C, (bf16_t*)out, ldo);
  return vd_launch_status();
}
