// Issue rate of the transcendental exp variants on gfx950, one wave per SIMD and two:
// v_exp_f32, v_exp_f16, and v_exp_f32 interleaved with v_mfma_f32_32x32x16_bf16.
// Each thread runs 8 independent chains of ITER exps; time from s_memtime per wave.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/exp_rate tools/mb/exp_rate.hip && /tmp/exp_rate
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int ITER = 4096;

template <int MODE>
__global__ void k_exp(float* out, long long* cyc) {
  float a[8];
  _Float16 h[8];
  for (int i = 0; i < 8; ++i) { a[i] = -0.001f * (threadIdx.x + i); h[i] = (_Float16)a[i]; }
  typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
  typedef __attribute__((ext_vector_type(16))) float f32x16;
  bf16x8 x = {};
  f32x16 acc = {};
  const long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < ITER; ++it) {
    if constexpr (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = __builtin_amdgcn_exp2f(a[i]);
    } else if constexpr (MODE == 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_exp_f16 %0, %0" : "+v"(h[i]));
    } else if constexpr (MODE == 2) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, x, acc, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = __builtin_amdgcn_exp2f(a[i]);
    } else {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, x, acc, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_exp_f16 %0, %0" : "+v"(h[i]));
    }
  }
  const long long t1 = __builtin_readcyclecounter();
  float s = acc[0];
  for (int i = 0; i < 8; ++i) s += a[i] + (float)h[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float* out;
  long long* cyc;
  hipMalloc(&out, 1 << 24);
  hipMalloc(&cyc, 1 << 16);
  const char* names[4] = {"v_exp_f32 x8", "v_exp_f16 x8", "mfma32 + v_exp_f32 x8", "mfma32 + v_exp_f16 x8"};
  for (int waves_per_simd = 1; waves_per_simd <= 2; ++waves_per_simd) {
    for (int mode = 0; mode < 4; ++mode) {
      const dim3 grid(256), block(256 * waves_per_simd);
      for (int rep = 0; rep < 2; ++rep) {
        if (mode == 0) hipLaunchKernelGGL(k_exp<0>, grid, block, 0, 0, out, cyc);
        if (mode == 1) hipLaunchKernelGGL(k_exp<1>, grid, block, 0, 0, out, cyc);
        if (mode == 2) hipLaunchKernelGGL(k_exp<2>, grid, block, 0, 0, out, cyc);
        if (mode == 3) hipLaunchKernelGGL(k_exp<3>, grid, block, 0, 0, out, cyc);
      }
      hipDeviceSynchronize();
      long long h[256];
      hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
      double avg = 0;
      for (int i = 0; i < 256; ++i) avg += h[i];
      avg /= 256;
      printf("%d wave(s)/SIMD  %-24s %8.2f cycles per iteration (8 exps%s)\n", waves_per_simd, names[mode],
             avg / ITER, mode >= 2 ? " + 1 MFMA" : "");
    }
  }
  return 0;
}
