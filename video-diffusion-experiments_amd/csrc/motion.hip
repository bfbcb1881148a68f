// Motion-module temporal attention with its Q/K/V projection fused (a8/a9).
//
// diffusers' AnimateDiffTransformer3D runs, per temporal self-attention of its
// BasicTransformerBlock, q/k/v = to_q/k/v(norm(h)) over the (B*H*W, F, C) tokens and then
// SDPA over the F frames of every position (experiments/03_trace_forward_pass.py:160-169).
// The unfused path writes the [rows][3C] QKV projection to HBM and the attention kernel
// reads it back (at level 1: 252 MB each way per layer, 10 layers per step).  Here one
// workgroup owns P positions (x PW per wave) x all 16 frames of one video (P*16 NHWC rows, read
// from their row stride H*W): each wave holds its own positions' 16 token rows of the normed
// activations as register fragments, and for every head h that head's 3d rows of the fused QKV
// weight stream through an LDS-DMA ring; Q_h|K_h|V_h of the wave's 16 tokens accumulate on
// 16x16x32 MFMAs (C^T = W.A^T as in gemm.hip: lane (fr, fq) ends with frame fr, channels
// 16a + 4fq + j), are rounded to bf16 into a per-wave scratch, and the 16-frame attention of
// that position and head runs exactly as temporal_mfma_kernel does (S^T = K.Q^T, softmax in log2
// units, O^T = V^T.P^T with V's ones column giving the row sum).  Only the normed rows are read
// and O is written: the QKV round trip and one launch per attention disappear.
//
// The projection's k order (32-wide MFMA steps, ascending) and the attention arithmetic
// are those of the unfused v5 GEMM + temporal_mfma_kernel, so the output is bit-identical
// to that path (tests/test_gpu_kernels.py::test_motion_qkv_attention).
#include "common.h"

namespace {

constexpr int MF = 16;  // frames of the window (the UNet's 16-frame videos)
// staging registers as ext_vector (HIP's uint4 struct arrays stayed on the scratch stack)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int D>
struct MqCfg {
  static_assert(D == 40, "motion_qkv: d = 40 (the level-1 motion modules)");
  static constexpr int C = 8 * D;                  // 8 heads
  static constexpr int P = 8;                      // positions per workgroup = waves
  static constexpr int NT = 64 * P;
  static constexpr int ROWS = P * MF;              // staged token rows
  static constexpr int KC = 64;                    // k-chunk of the weight ring (elements)
  static constexpr int NCH = C / KC;               // chunks per head
  static constexpr int NBLK = (3 * D + 15) / 16;   // 16-channel output blocks: q | k | v (+ pad)
  static constexpr int NWP = NBLK * 16;            // ring rows (pad rows stay zero)
  static constexpr int KSTEPS = (D + 31) / 32;     // attention d-steps
  static constexpr int DPAD = KSTEPS * 32;         // Q/K scratch row (elements)
  static constexpr int DB = (D + 1 + 15) / 16;     // O^T row blocks incl. the ones row
  static constexpr int VS = 16 * (DB | 1);         // V image row (elements), conflict-free tr reads
  static constexpr int A_ELEMS = ROWS * C;
  static constexpr int W_ELEMS = NWP * KC;         // one ring slot
  static constexpr int S_ELEMS = 2 * MF * DPAD + MF * VS;  // per-wave scratch: Q, K, V image
  static constexpr int LDS_BYTES = 2 * (A_ELEMS + 2 * W_ELEMS + P * S_ELEMS);
  static constexpr int ACH = ROWS * C / 8;         // 16-byte chunks of the token tile
  static constexpr int WCH = 3 * D * KC / 8;       // 16-byte chunks of one weight chunk
  static constexpr int AREG = (ACH + NT - 1) / NT;
  static constexpr int WREG = (WCH + NT - 1) / NT;
  static_assert(LDS_BYTES <= 160 * 1024, "LDS");
  static_assert(C % KC == 0 && D % 4 == 0, "shape");
};

// element offset inside a [rows][64] block, 16-byte chunks XOR-swizzled by (row & 7) so the
// 16x16x32 fragment reads (ds_read_b128) are conflict-free (gemm.hip's lds_off)
__device__ __forceinline__ int sw64(int row, int chunk) { return row * 64 + ((chunk ^ (row & 7)) << 3); }

// ---------------------------------------------------------------- the kernel (round 3)
// Round 2's form staged the token rows in an 80 KiB LDS tile and streamed register-staged weight
// chunks one step ahead (an L2 round trip exposed per 256 cycles of MFMA).  Here a wave only ever
// reads ITS OWN 16 token rows, so their A fragments live in registers (40 VGPRs: all 10 32-deep
// k-steps, loaded once), and the LDS holds the weight stream: a 6-slot ring of 16 KiB chunks
// (128 ring rows x 64 k) filled by LDS-DMA (16 x 1 KiB pieces per chunk, two per wave, the sw64
// swizzle applied on the source address, pad rows zero-filled by the buffer range check), five
// chunks in flight behind counted vmcnt waits: 212.5 -> 157.3 us per level-1 layer, bit-identical
// (profiles/r03k_motion_qkv_v2.txt).
constexpr int MQ2_S = 6;  // ring slots

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4m;

__device__ __forceinline__ u32x4m mq_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  u32x4m r;
  r[0] = __builtin_amdgcn_readfirstlane((uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) & 0xffffu;  // stride 0
  r[2] = __builtin_amdgcn_readfirstlane(bytes);                          // num_records: range check
  r[3] = 0x00020000u;
  return r;
}
// one 1 KiB LDS-DMA piece (lane l's 16 bytes at voff land at LDS byte lds + 16 l); inline asm so
// hipcc neither counts it in vmcnt nor drains it before the ring's LDS reads
__device__ __forceinline__ void mq_dma(u32x4m rs_, uint32_t lds, uint32_t voff) {
  u32x4m rs;
#pragma unroll
  for (int i = 0; i < 4; ++i) rs[i] = __builtin_amdgcn_readfirstlane(rs_[i]);
  uint32_t keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
               "buffer_load_dwordx4 %2, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(voff), "s"(rs) : "memory");
}
template <int N>
__device__ __forceinline__ void mq_wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
}

template <int D>
struct Mq2Cfg {
  using B = MqCfg<D>;
  static constexpr int W_BYTES = B::NWP * B::KC * 2;               // 16 KiB ring slot
  static constexpr int S_BYTES = B::S_ELEMS * 2;                   // per-wave scratch
  static constexpr int TAB_BYTES = 8192;                           // LNF: one head's s | P' table
  static constexpr int STAT_BYTES = 2 * MF * 8;                     // LNF: per wave (-mean, rstd) of 2 x 16 rows
  static constexpr int LDS_BYTES = MQ2_S * W_BYTES + B::P * S_BYTES + 2 * TAB_BYTES + B::P * STAT_BYTES;
  static_assert(B::NWP == 128 && B::KC == 64, "16 pieces of 8 ring rows x 128 B per chunk");
  static_assert(8 * 1024 == TAB_BYTES && 3 * B::C / 8 * (1 + MF) <= TAB_BYTES / 4, "table: one KiB piece per wave");
  static_assert(LDS_BYTES <= 160 * 1024, "LDS");
};

// PW (round 3, second pass): positions per wave.  Every wave reads the whole 16 KiB weight chunk
// from LDS per chunk (8 waves: 128 KiB per chunk) for 16 MFMAs per position: at PW = 1 that is
// ~250 B/clk per CU, the LDS read port's limit, so the kernel was LDS-bound.  PW = 2 gives each
// weight fragment two positions' MFMAs (half the LDS bytes per MFMA, half the weight stream per
// token) for 40 more VGPRs of token fragments and 32 of accumulators; the heads' attention runs
// position by position through the same per-wave scratch.
// LNF (round 5): the motion block's norm1 / norm2 (+ the sinusoidal PE by frame) folded in, as
// gemm.hip's v8 LNF: x holds the UN-normalised rows, w = W_qkv∘gamma, and `tab` per head h the
// 120 fp32 column sums s of w's rows of that head (q | k | v, 40 each) then, per frame f < 16,
// the 120 values P[f] = W·(beta + pe[f]) — an 8 KiB table that rides the weight ring as one 1 KiB
// LDS-DMA piece per wave with the head's first chunk (double-buffered in LDS).  Each wave's token
// rows (16 frames of a position) get mean / rstd from two extra MFMAs per k-step over the
// fragments it already holds; the head epilogue writes rstd (acc - mean s) + P[frame] to the scratch.
template <int D, int PW = 1, bool LNF = false>
__global__ __launch_bounds__(MqCfg<D>::NT, 1) void motion_qkv_attn2_kernel(
    const bf16_t* __restrict__ x, int64_t ldx, const bf16_t* __restrict__ w, int64_t ldw, bf16_t* __restrict__ o,
    int64_t ldo, int64_t batch, int64_t positions, float c, const float* __restrict__ tab, float eps) {
  using Cf = MqCfg<D>;
  using C2 = Mq2Cfg<D>;
  constexpr int PWG = Cf::P * PW;  // positions per workgroup
  extern __shared__ __attribute__((aligned(1024))) char lds2[];
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds2;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  bf16_t* s_l = (bf16_t*)(lds2 + MQ2_S * C2::W_BYTES + wave * C2::S_BYTES);
  bf16_t* q_s = s_l;                                     // [16][DPAD]
  bf16_t* k_s = s_l + MF * Cf::DPAD;                     // [16][DPAD]
  bf16_t* v_s = s_l + 2 * MF * Cf::DPAD;                 // V image [16][VS]
  const uint32_t tab0 = (uint32_t)(MQ2_S * C2::W_BYTES + Cf::P * C2::S_BYTES);  // LNF tables (byte offset)
  // LNF: this wave's row statistics, parked in LDS between the prologue and the head epilogues (in
  // VGPRs the kernel spilled: it sits at the 256-register limit)
  float2* const st_l = (float2*)(lds2 + tab0 + 2 * C2::TAB_BYTES + wave * C2::STAT_BYTES);

  const int64_t nblk_p = (positions + PWG - 1) / PWG;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t b = lid / nblk_p;
  const int64_t p0 = (lid - b * nblk_p) * PWG;  // this wave's positions: p0 + PW * wave + pw

  // ---- weight-chunk DMA: chunk t = (head h, k-chunk kc) -> slot t % S; wave w moves pieces 2w,
  // 2w + 1 = ring rows 8g .. 8g + 7; ring row n < 3D is W row (n / D) * C + h * D + n % D
  const u32x4m rw = mq_rsrc(w, (uint32_t)(3 * Cf::C * ldw * 2));
  const uint32_t rsub = (uint32_t)lane >> 3, pch = (uint32_t)lane & 7;  // row in the piece, physical chunk
  const u32x4m rt = mq_rsrc(LNF ? (const void*)tab : (const void*)w, LNF ? 8u * C2::TAB_BYTES : 0u);
  auto issue = [&](int t) {
    const int h = t / Cf::NCH, kc = t % Cf::NCH;
    const uint32_t slot = lds0 + (uint32_t)(t % MQ2_S) * C2::W_BYTES;
    if (LNF && kc == 0)  // head h's table: this wave's KiB, with the head's first chunk
      mq_dma(rt, lds0 + tab0 + (uint32_t)(h & 1) * C2::TAB_BYTES + (uint32_t)wave * 1024,
             (uint32_t)h * C2::TAB_BYTES + (uint32_t)wave * 1024 + (uint32_t)lane * 16);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int g = 2 * wave + i;
      const uint32_t r = (uint32_t)(8 * g) + rsub;                      // ring row
      const uint32_t lc = pch ^ (r & 7);                                 // logical chunk (sw64)
      const uint32_t n = (r / D) * Cf::C + (uint32_t)h * D + r % D;      // W row
      const uint32_t off = r < 3 * D ? n * (uint32_t)ldw * 2 + (uint32_t)kc * (Cf::KC * 2) + lc * 16 : 0x80000000u;
      mq_dma(rw, slot + (uint32_t)g * 1024, off);
    }
  };
  constexpr int T = 8 * Cf::NCH;
#pragma unroll
  for (int t = 0; t < MQ2_S - 1; ++t) issue(t);

  // ---- scratch padding (written once; the heads only write columns < D): Q/K columns
  // [D, DPAD) zero; the V image zero except column D = 1.0 (the row-sum column)
  for (int i = lane; i < Cf::S_ELEMS / 8; i += 64) *(uint4*)(s_l + i * 8) = make_uint4(0, 0, 0, 0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane < MF) v_s[lane * Cf::VS + D] = (bf16_t)0x3F80;

  // ---- this wave's A fragments: token (frame fr, position p0 + PW wave + pw), k = 32 kk + 8 fq .. +7
  bf16x8 xf[PW][Cf::C / 32];
#pragma unroll
  for (int pw = 0; pw < PW; ++pw) {
    int64_t p = p0 + PW * wave + pw;
    p = p < positions ? p : positions - 1;
    const bf16_t* xr = x + ((b * MF + fr) * positions + p) * ldx + 8 * fq;
#pragma unroll
    for (int kk = 0; kk < Cf::C / 32; ++kk) xf[pw][kk] = __builtin_bit_cast(bf16x8, *(const u32x4*)(xr + 32 * kk));
  }
  // LNF: each token row's mean and rstd (lane (fr, fq) holds row fr's channels 32 kk + 8 fq ..):
  // ones·x gives the row sum in every entry, x·x^T the Gram block whose diagonal (fr, fr) sits in
  // lane fr + 16 (fr >> 2), register fr & 3
#pragma unroll
  for (int pw = 0; pw < PW; ++pw) {
    if constexpr (LNF) {
      const bf16x8 ones = __builtin_bit_cast(bf16x8, make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u));
      f32x4 sacc = f32x4{0.f, 0.f, 0.f, 0.f}, gacc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < Cf::C / 32; ++kk) {
        sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, xf[pw][kk], sacc, 0, 0, 0);
        gacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[pw][kk], xf[pw][kk], gacc, 0, 0, 0);
      }
      const int j3 = fr & 3;
      const float gd = j3 == 0 ? gacc[0] : j3 == 1 ? gacc[1] : j3 == 2 ? gacc[2] : gacc[3];
      const float sxx = __shfl(gd, fr + 16 * (fr >> 2), 64);
      constexpr float RK = 1.0f / (float)Cf::C;
      const float mean = sacc[0] * RK;
      const float var = row_var_guarded<Cf::C / 32>(xf[pw], mean, fmaf(sxx, RK, -mean * mean), RK);
      if (fq == 0) st_l[pw * MF + fr] = make_float2(-mean, rsqrtf(var + eps));
    }
  }

  const bool unitc = c == 1.0f;
  const int vtr = (4 * fq + (fr >> 2)) * Cf::VS + 4 * (fr & 3);  // tr-read lane offset (temporal_mfma_kernel)
  f32x4 acc[PW][Cf::NBLK];
#pragma unroll
  for (int pw = 0; pw < PW; ++pw)
#pragma unroll
    for (int a = 0; a < Cf::NBLK; ++a) acc[pw][a] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int h = 0; h < 8; ++h) {
#pragma unroll
   for (int kc = 0; kc < Cf::NCH; ++kc) {  // unrolled: the A fragment index 2 kc + ks is static
    const int t = h * Cf::NCH + kc;
    // this wave's pieces of chunk t landed: the younger ones are chunks t+1 .. min(t+S-2, T-1)
    const int ahead = (T - 1 - t) < (MQ2_S - 2) ? (T - 1 - t) : (MQ2_S - 2);
    // LNF: + one table piece for every head-first chunk among them.  With the full window (4 chunks
    // ahead, every chunk but the last head's tail) that is one piece exactly when kc >= 1 — a
    // compile-time count in this unrolled loop; the tail (head 7, kc >= 1) has no younger table piece.
    // (A run-time count through a 10-way switch cost the kernel 18 %: 156.5 vs 132.7 us per launch.)
    static_assert(MQ2_S - 2 == 4 && Cf::NCH == 5, "the static table-piece count below");
    if (LNF && ahead >= 4) {
      if (kc == 0) mq_wait_vm<8>();
      else mq_wait_vm<9>();
    } else if (ahead >= 4) mq_wait_vm<8>();
    else if (ahead == 3) mq_wait_vm<6>();
    else if (ahead == 2) mq_wait_vm<4>();
    else if (ahead == 1) mq_wait_vm<2>();
    else mq_wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's pieces of chunk t landed; slot (t-1) % S free
    asm volatile("" ::: "memory");
    if (t + MQ2_S - 1 < T) issue(t + MQ2_S - 1);
    const bf16_t* ws = (const bf16_t*)(lds2 + (t % MQ2_S) * C2::W_BYTES);
    if constexpr (PW == 1) {
      // all 16 weight fragments of the chunk read ahead of its 16 MFMAs (counted lgkmcnt waits)
      bf16x8 wf[2][Cf::NBLK];
#pragma unroll
      for (int ks = 0; ks < Cf::KC / 32; ++ks)
#pragma unroll
        for (int a = 0; a < Cf::NBLK; ++a) wf[ks][a] = *(const bf16x8*)(ws + sw64(a * 16 + fr, ks * 4 + fq));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < Cf::KC / 32; ++ks)
#pragma unroll
        for (int a = 0; a < Cf::NBLK; ++a)
          acc[0][a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ks][a], xf[0][2 * kc + ks], acc[0][a], 0, 0, 0);
    } else {
      // one k-step's 8 fragments at a time (32 VGPRs: the second position's tokens and
      // accumulators take the rest), each feeding PW MFMAs
#pragma unroll
      for (int ks = 0; ks < Cf::KC / 32; ++ks) {
        bf16x8 wf[Cf::NBLK];
#pragma unroll
        for (int a = 0; a < Cf::NBLK; ++a) wf[a] = *(const bf16x8*)(ws + sw64(a * 16 + fr, ks * 4 + fq));
#pragma unroll
        for (int a = 0; a < Cf::NBLK; ++a)
#pragma unroll
          for (int pw = 0; pw < PW; ++pw)
            acc[pw][a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[a], xf[pw][2 * kc + ks], acc[pw][a], 0, 0, 0);
      }
    }
   }
#pragma unroll
    for (int pw = 0; pw < PW; ++pw) {  // ---- head h done: attention of (position p0 + PW wave + pw, head h)
      const bool pok = p0 + PW * wave + pw < positions;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the previous head's / position's scratch reads
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int a = 0; a < Cf::NBLK; ++a) {
        const int ch = a * 16 + 4 * fq;
        if (ch < 3 * D) {
          const int part = ch / D, cd = ch - part * D;
          bf16_t* dst = part == 0 ? q_s + fr * Cf::DPAD + cd : (part == 1 ? k_s + fr * Cf::DPAD + cd : v_s + fr * Cf::VS + cd);
          f32x4 v = acc[pw][a];
          if constexpr (LNF) {
            const float* tb = (const float*)(lds2 + tab0 + (h & 1) * C2::TAB_BYTES);
            const float4 sv = *(const float4*)(tb + ch), pv = *(const float4*)(tb + 3 * D + fr * 3 * D + ch);
            const float2 st = st_l[pw * MF + fr];  // (-mean, rstd) of row fr
            v[0] = fmaf(st.y, fmaf(st.x, sv.x, v[0]), pv.x);
            v[1] = fmaf(st.y, fmaf(st.x, sv.y, v[1]), pv.y);
            v[2] = fmaf(st.y, fmaf(st.x, sv.z, v[2]), pv.z);
            v[3] = fmaf(st.y, fmaf(st.x, sv.w, v[3]), pv.w);
          }
          *(uint2*)dst = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        }
        acc[pw][a] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < Cf::KSTEPS; ++ks) {
        const bf16x8 kq = *(const bf16x8*)(k_s + fr * Cf::DPAD + ks * 32 + 8 * fq);
        const bf16x8 qq = *(const bf16x8*)(q_s + fr * Cf::DPAD + ks * 32 + 8 * fq);
        s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kq, qq, s, 0, 0, 0);
      }
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (!unitc) s[j] *= c;
        mx = fmaxf(mx, s[j]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      bf16x8 pf;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pf[j] = (__bf16)__builtin_amdgcn_exp2f(s[j] - mx);
        pf[4 + j] = (__bf16)0.0f;
      }
      f32x4 ot[Cf::DB];
#pragma unroll
      for (int a = 0; a < Cf::DB; ++a) {
        const bf16x4 tv = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (bf16x4 __attribute__((address_space(3)))*)(v_s + vtr + 16 * a));
        const bf16x8 vf = {tv[0], tv[1], tv[2], tv[3], (__bf16)0.0f, (__bf16)0.0f, (__bf16)0.0f, (__bf16)0.0f};
        ot[a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      }
      const float l = __shfl(ot[D / 16][(D % 16) % 4], ((D % 16) / 4) * 16 + fr, 64);
      const float inv = __builtin_amdgcn_rcpf(l);
      if (pok) {
        bf16_t* orow = o + ((b * MF + fr) * positions + p0 + PW * wave + pw) * ldo + (int64_t)h * D;
#pragma unroll
        for (int a = 0; a < Cf::DB; ++a) {
          const int dd = 16 * a + 4 * fq;
          if (dd + 4 <= D)
            *(uint2*)(orow + dd) =
                make_uint2(pack2(ot[a][0] * inv, ot[a][1] * inv), pack2(ot[a][2] * inv, ot[a][3] * inv));
        }
      }
    }
  }
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

namespace {
// the shapes the fused kernel takes: frames 16, 8 heads, d 40, and at least one round of the chip
// (one workgroup per CU: below it the unfused GEMM + attention is faster — tools/motion_qkv_bench.py:
// 2-frame rank, 128 workgroups: v2 39.1 vs unfused 34.8 us; 4-frame rank, 256: v2 42.4 vs 56.8 us;
// the full step, 1024: v2 157 vs 250)
bool mq_takes(int64_t batch, int32_t frames, int64_t positions, int32_t heads, int32_t d) {
  if (frames != MF || heads != 8 || d != 40 || batch <= 0 || positions <= 0) return false;
  const int64_t nwg = batch * ((positions + MqCfg<40>::P - 1) / MqCfg<40>::P);
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess &&
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  return nwg >= (int64_t)cus;
}

template <int PW, bool LNF>
int mq_launch(const void* x, int64_t ldx, const void* wqkv, int64_t ldw, void* o, int64_t ldo, int64_t batch,
              int64_t positions, float scale, const float* tab, float eps, int64_t nwg, hipStream_t stream) {
  using C2 = Mq2Cfg<40>;
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void*)motion_qkv_attn2_kernel<40, PW, LNF>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, C2::LDS_BYTES) != hipSuccess)
      return vd_launch_status();
    attr_set = true;
  }
  hipLaunchKernelGGL((motion_qkv_attn2_kernel<40, PW, LNF>), dim3((unsigned)nwg), dim3(MqCfg<40>::NT), C2::LDS_BYTES,
                     stream, (const bf16_t*)x, ldx, (const bf16_t*)wqkv, ldw, (bf16_t*)o, ldo, batch, positions,
                     scale * 1.4426950408889634f, tab, eps);
  return vd_launch_status();
}
}  // namespace

extern "C" int vd_motion_qkv_attention_takes(int64_t batch, int32_t frames, int64_t positions, int32_t heads,
                                             int32_t d) {
  return mq_takes(batch, frames, positions, heads, d) ? 1 : 0;
}

extern "C" int vd_motion_qkv_attention(const void* x, int64_t ldx, const void* wqkv, int64_t ldw, void* o,
                                       int64_t ldo, int64_t batch, int32_t frames, int64_t positions,
                                       int32_t heads, int32_t d, float scale, const float* ln_fold_tab,
                                       float ln_fold_eps, vd_stream_t stream) {
  VD_CHECK_ARG(x && wqkv && o && al16(x) && al16(wqkv) && ((uintptr_t)o & 7) == 0);
  VD_CHECK_ARG(ldx % 8 == 0 && ldw % 8 == 0 && ldo % 4 == 0 && batch > 0 && positions > 0);
  if (ln_fold_tab) VD_CHECK_ARG(al16(ln_fold_tab) && ln_fold_eps >= 0.f);
  if (!mq_takes(batch, frames, positions, heads, d)) return VD_EUNSUPPORTED;
  using Cf = MqCfg<40>;
  VD_CHECK_ARG(ldx >= Cf::C && ldw >= Cf::C && ldo >= Cf::C);
  const int64_t nwg = batch * ((positions + Cf::P - 1) / Cf::P);
  VD_CHECK_ARG(nwg < 0x7fffffff && batch * MF * positions < 0x7fffffff);
  hipStream_t s = (hipStream_t)stream;
  // two positions per wave where that still gives one round of the chip (156 -> 128 us per
  // level-1 layer, profiles/r03s_motion_pw2.txt)
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess &&
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  const int64_t nwg2 = batch * ((positions + 2 * Cf::P - 1) / (2 * Cf::P));
  if (nwg2 >= (int64_t)cus)
    return ln_fold_tab ? mq_launch<2, true>(x, ldx, wqkv, ldw, o, ldo, batch, positions, scale, ln_fold_tab, ln_fold_eps, nwg2, s)
                       : mq_launch<2, false>(x, ldx, wqkv, ldw, o, ldo, batch, positions, scale, nullptr, 0.f, nwg2, s);
  return ln_fold_tab ? mq_launch<1, true>(x, ldx, wqkv, ldw, o, ldo, batch, positions, scale, ln_fold_tab, ln_fold_eps, nwg, s)
                     : mq_launch<1, false>(x, ldx, wqkv, ldw, o, ldo, batch, positions, scale, nullptr, 0.f, nwg, s);
}
