// Temporal-consistency metrics of decoded videos: the integer
// cores of experiments/06_measure_grid_search.py's compute_mse over consecutive frames
// (:209-211, :320-326) and compute_flicker_index (:221-235), for a whole batch of
// videos in one HBM pass.
//
// Input: uint8 RGB frames, video-major [videos][frames][bytes_per_frame] (the PNG decode
// of load_frames, before its /255).  Output, exact and deterministic (integer atomics):
//   sse[v][f] = sum (x[f+1] - x[f])^2            f < frames - 1
//   sad[v][f] = sum |x[f] - 2 x[f+1] + x[f+2]|   f < frames - 2
// from which the host forms mse = sse / (255^2 n), psnr, and the flicker index.
// Layout: one thread owns a 16-byte column of the frame and walks it through time with
// a two-frame register window, so every byte is read once (HBM-bound); bytes are split
// into 16-bit lanes (v_pk_* i16 math) and squared/summed with v_dot2 (2 values per op).
#include "common.h"

namespace {

constexpr int NT = 256;
constexpr int MAXF = 32;

typedef short __attribute__((ext_vector_type(2))) s16x2;
typedef unsigned short __attribute__((ext_vector_type(2))) u16x2;
typedef unsigned int __attribute__((ext_vector_type(4))) u32x4;

__device__ __forceinline__ s16x2 lane16(uint32_t w) { return __builtin_bit_cast(s16x2, w); }

// bytes of a uint4 as 8 x (2 x i16): even bytes then odd bytes of each dword
__device__ __forceinline__ void split(const u32x4& u, s16x2 (&o)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = lane16(w[i] & 0x00ff00ffu);
    o[2 * i + 1] = lane16((w[i] >> 8) & 0x00ff00ffu);
  }
}

__global__ __launch_bounds__(NT) void frame_metrics_kernel(const uint8_t* __restrict__ x, int frames,
                                                           int64_t chunks, int64_t bytes_per_frame,
                                                           int blocks_per_video, unsigned long long* sse,
                                                           unsigned long long* sad) {
  const int v = blockIdx.x / blocks_per_video;
  const int blk = blockIdx.x % blocks_per_video;
  const uint8_t* base = x + (int64_t)v * frames * bytes_per_frame;
  uint32_t acc_e[MAXF], acc_a[MAXF];
#pragma unroll
  for (int f = 0; f < MAXF; ++f) acc_e[f] = acc_a[f] = 0u;
  const u16x2 one = {1, 1};
  for (int64_t c = (int64_t)blk * NT + threadIdx.x; c < chunks; c += (int64_t)blocks_per_video * NT) {
    // window: the previous frame p1 and the previous first difference dp = p1 - p2, so the
    // second difference is d - dp (d = cur - p1, already formed for the squared error)
    s16x2 p1[8], dp[8];
    const uint32_t col = (uint32_t)(c * 16);  // < frames * bytes_per_frame < 2^32 (host check)
#pragma unroll
    for (int f0 = 0; f0 < MAXF; f0 += 8) {
      if (f0 < frames) {
        // 8 frames' loads in flight before any of them is consumed
        u32x4 u[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (f0 + j < frames)
            u[j] = __builtin_nontemporal_load((const u32x4*)(base + col + (uint32_t)(f0 + j) * (uint32_t)bytes_per_frame));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int f = f0 + j;
          if (f < frames) {
            s16x2 cur[8];
            split(u[j], cur);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              if (f >= 1) {
                const s16x2 d = cur[i] - p1[i];
                acc_e[f - 1] = (uint32_t)__builtin_amdgcn_sdot2(d, d, (int)acc_e[f - 1], false);
                if (f >= 2) {
                  const s16x2 e = d - dp[i];
                  const s16x2 ae = __builtin_elementwise_max(e, -e);
                  acc_a[f - 2] = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, ae), one, acc_a[f - 2], false);
                }
                dp[i] = d;
              }
              p1[i] = cur[i];
            }
          }
        }
      }
    }
  }
  // per-thread sums stay < 2^32: <= 16 * 65025 per chunk, and a thread sees at most
  // ceil(chunks / (blocks_per_video * NT)) chunks (host keeps that <= 4096)
#pragma unroll
  for (int f = 0; f < MAXF - 1; ++f) {
    if (f < frames - 1) {
      const unsigned long long e = wave_sum((unsigned long long)acc_e[f]);
      if ((threadIdx.x & 63) == 0 && e) atomicAdd(sse + (int64_t)v * (frames - 1) + f, e);
    }
    if (f < frames - 2) {
      const unsigned long long a = wave_sum((unsigned long long)acc_a[f]);
      if ((threadIdx.x & 63) == 0 && a) atomicAdd(sad + (int64_t)v * (frames - 2) + f, a);
    }
  }
}

}  // namespace

extern "C" int vd_frame_metrics(const void* frames_u8, int64_t videos, int32_t frames, int64_t bytes_per_frame,
                                uint64_t* sse, uint64_t* sad, vd_stream_t stream) {
  VD_CHECK_ARG(frames_u8 && sse && videos > 0 && frames >= 2 && frames <= MAXF);
  VD_CHECK_ARG(bytes_per_frame > 0 && bytes_per_frame % 16 == 0 && ((uintptr_t)frames_u8 & 15) == 0);
  if (frames >= 3) VD_CHECK_ARG(sad != nullptr);
  const int64_t chunks = bytes_per_frame / 16;
  int64_t bpv = (chunks + 4 * NT - 1) / (4 * NT);            // ~4 chunks per thread
  const int64_t min_bpv = (chunks + 4096LL * NT - 1) / (4096LL * NT);  // keeps per-thread sums < 2^32
  bpv = bpv < min_bpv ? min_bpv : bpv;
  VD_CHECK_ARG(videos * bpv < 0x7fffffff && frames * bytes_per_frame < 0xffffffffLL);
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(sse, 0, (size_t)videos * (frames - 1) * 8, s) != hipSuccess) return vd_launch_status();
  if (frames >= 3 && hipMemsetAsync(sad, 0, (size_t)videos * (frames - 2) * 8, s) != hipSuccess)
    return vd_launch_status();
  hipLaunchKernelGGL(frame_metrics_kernel, dim3((unsigned)(videos * bpv)), dim3(NT), 0, s, (const uint8_t*)frames_u8,
                     (int)frames, chunks, bytes_per_frame, (int)bpv, (unsigned long long*)sse,
                     (unsigned long long*)sad);
  return vd_launch_status();
}
