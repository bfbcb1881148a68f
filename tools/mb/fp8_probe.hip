// Probe of the block-scaled fp8 MFMA (v_mfma_scale_f32_32x32x64_f8f6f4) operand layout:
// one wave; lane l passes its 32 A bytes, 32 B bytes and E8M0 scales, and stores its 16
// accumulators.  The host (tools/mb/fp8_probe.py) checks candidate lane maps against A@B.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

__global__ void probe_kernel(const i32x8* a, const i32x8* b, float* c, int sa, int sb) {
  const int l = threadIdx.x;
  f32x16 acc = {};
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[l], b[l], acc, 0, 0, 0, sa, 0, sb);
  for (int r = 0; r < 16; ++r) c[l * 16 + r] = acc[r];
}

extern "C" int fp8_probe(const void* a, const void* b, float* c, int sa, int sb) {
  hipLaunchKernelGGL(probe_kernel, dim3(1), dim3(64), 0, 0, (const i32x8*)a, (const i32x8*)b, c, sa, sb);
  return hipDeviceSynchronize();
}
