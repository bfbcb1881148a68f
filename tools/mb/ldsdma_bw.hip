// Microbenchmark: per-CU load throughput from an L2-resident window, LDS-DMA
// (buffer_load_dwordx4 ... lds) vs register loads (buffer_load_dwordx4), by waves per
// workgroup and instructions in flight per wave.  One workgroup per CU (LDS 64 KiB).
// build: hipcc --offload-arch=gfx950 -O3 -o mb_ldsdma tools/mb/ldsdma_bw.hip
// (round 4: also MALL / HBM-sized windows; results in profiles/r04_ldsdma_fill.txt)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef __attribute__((address_space(3))) void lds_void;

template <int DEPTH, bool DMA>
__global__ void kern(const char* src, uint32_t window, int iters, float* sink) {
  __shared__ __attribute__((aligned(1024))) char smem[65536];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // all workgroups of one XCD (b % 8) share one window -> L2 hits after the first pass
  const char* base = src + (size_t)(blockIdx.x % 8) * window;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, window, 0x00020000);
  uint32_t off = (uint32_t)((blockIdx.x * 7919 + wid * 1024) % (window / 1024)) * 1024 + lane * 16;
  float acc = 0.f;
  char* l = smem + (wid % 16) * 4096;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < DEPTH; ++j) {
      if constexpr (DMA) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)(l + (j & 3) * 1024), 16, off, 0, 0, 0);
      } else {
        uint4 v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
        acc += __uint_as_float(v.x ^ v.w);
      }
      off += nw * 1024;
      if (off >= window) off -= window;
    }
    if constexpr (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (acc == 12345.f) sink[0] = acc;
}

template <int DEPTH, bool DMA>
void run(const char* src, uint32_t window, int wg_threads, int cus, float* sink) {
  const int iters = 2000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  kern<DEPTH, DMA><<<cus, wg_threads>>>(src, window, 10, sink);
  hipEventRecord(e0);
  kern<DEPTH, DMA><<<cus, wg_threads>>>(src, window, iters, sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double bytes = (double)cus * (wg_threads / 64) * iters * DEPTH * 1024.0;
  printf("%-4s waves/CU=%2d depth=%2d  %8.1f GB/s chip  %6.1f GB/s/CU  %5.2f B/cyc/CU@2.2GHz\n", DMA ? "dma" : "reg",
         wg_threads / 64, DEPTH, bytes / ms / 1e6, bytes / ms / 1e6 / cus, bytes / ms / 1e6 / cus / 2.2);
}

int main() {
  int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float* sink; hipMalloc(&sink, 4);
  // per-XCD windows: 2 MiB (L2-resident), 64 MiB (512 MiB in all: beyond the 256 MiB MALL... per
  // XCD it streams from MALL/HBM), 256 MiB (2 GiB in all: HBM streaming)
  for (uint32_t window : {2u << 20, 64u << 20, 256u << 20}) {
    char* src; hipMalloc(&src, 8 * (size_t)window); hipMemset(src, 1, 8 * (size_t)window);
    printf("window %u MiB per XCD\n", window >> 20);
    for (int wt : {256, 512}) {
      run<2, true>(src, window, wt, cus, sink);
      run<4, true>(src, window, wt, cus, sink);
      run<8, true>(src, window, wt, cus, sink);
      run<16, true>(src, window, wt, cus, sink);
      run<4, false>(src, window, wt, cus, sink);
      run<8, false>(src, window, wt, cus, sink);
    }
    hipFree(src);
  }
  return 0;
}
