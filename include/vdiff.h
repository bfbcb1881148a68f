/*
 * vdiff.h — C ABI of libvdiff_hip.so, the MI355X (gfx950) kernels behind the
 * video-diffusion denoising step.
 *
 * The reference has no native code: every op below replaces a stock
 * torch/cuDNN/cuBLAS/SDPA call that diffusers issues inside
 * `UNetMotionModel.forward` (called at
 * /root/reference/experiments/03_trace_forward_pass.py:109-113) and
 * `DDIMScheduler.step` (configured at
 * /root/reference/experiments/05_grid_search_ablation.py:136-141, stepped
 * inside the pipe(...) call at :158-167).  Per-entry citations name the
 * diffusers op replaced.
 *
 * Conventions:
 *  - plain device pointers + explicit int64 sizes/strides (in ELEMENTS);
 *  - activations bf16 ("bf16" = raw 16-bit storage), statistics and
 *    latents fp32, weights bf16 packed [N][K] (K contiguous);
 *  - every call takes the hipStream_t to launch on, never allocates, never
 *    synchronises, never retains a pointer: all calls are hipGraph-capturable;
 *  - returns 0 (VD_OK) or a vd_status / hipError_t code; vd_strerror() names it.
 *  - activation layout is NHWC rows: pixel/token m of image n at row
 *    n*H*W + h*W + w; video b, frame f -> image n = b*F + f.
 */
#ifndef VDIFF_H
#define VDIFF_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* vd_stream_t; /* hipStream_t */

enum vd_status {
  VD_OK = 0,
  VD_EINVAL = 1000,       /* bad shape / alignment / unsupported parameter */
  VD_EUNSUPPORTED = 1001, /* valid request outside the compiled variants    */
  VD_ERCCL = 1002         /* RCCL call failed                                */
};

const char* vd_strerror(int code);
int vd_version(void);  /* 6 */
/* Content hash (16 hex digits) of the sources and compile flags the library was built from
 * (video-diffusion-experiments_amd/build_ext.py); the Python loader compares it with the tree. */
const char* vd_build_hash(void);
/* The --offload-arch the library's code objects were compiled for ("gfx950" unless the build
 * set VDIFF_ARCH); not part of the content hash above. */
const char* vd_build_arch(void);

/* ---------------------------------------------------------------- GEMM / conv
 * out[m, n] = epi( sum_k A[m, k] * W[n, k] )          (bf16 MFMA, fp32 accumulate)
 *
 * a_mode VD_A_DENSE : A[m, k] = a0[m*lda0 + k]              for k <  k0
 *                              a1[m*lda1 + (k - k0)]       for k >= k0  (channel concat)
 * a_mode VD_A_CONV3X3: implicit-GEMM 3x3 conv, pad 1, over NHWC images (or a kt x 3 x 3
 *   conv over the frames of each video, see kt below); the
 *   K index is tap*(Cin) + ci with Cin = k0 + (channels of a1); channels
 *   [0,k0) come from a0 (pixel stride lda0), the rest from a1 (pixel stride
 *   lda1) — this is the up-block torch.cat([x, skip], 1) without materialising
 *   it.  stride 2 = Downsample2D; upsample 1 = Upsample2D (nearest x2 of the
 *   h_in x w_in input, then conv).  M = n_img*h_out*w_out.
 *   Replaces torch conv2d in ResnetBlock2D.conv1/conv2, Down/Upsample2D.conv,
 *   conv_in/conv_out and nn.Linear / 1x1 convs (a5, a8, a10).
 * epilogue, in order: + bias[n] (fp32) ; + rowbias[(m / rb_div) * ld_rb + n]
 *   (fp32, the ResnetBlock2D time_emb_proj broadcast) ; act ; + res[m*ld_res + n]
 *   (bf16) ; store bf16 (or fp32 if out_f32).
 * act VD_ACT_GEGLU: W rows are packed in 16-row blocks alternating (hidden,
 *   gate); out has N/2 columns: h * gelu_erf(g)  (diffusers GEGLU, a10).
 */
enum { VD_A_DENSE = 0, VD_A_CONV3X3 = 1 };
enum { VD_ACT_NONE = 0, VD_ACT_SILU = 1, VD_ACT_GEGLU = 2, VD_ACT_GELU = 3 };
/* VD_ACT_GELU: pointwise gelu (erf form) — the DiT MLP (build-defined, §8f rank 3). */

typedef struct vd_gemm_desc {
  const void* a0; int64_t lda0; int64_t k0;
  const void* a1; int64_t lda1;
  int32_t a_mode;
  int32_t n_img, h_in, w_in, h_out, w_out, stride, upsample;
  const void* w; int64_t ldw;
  int64_t M, N, K;
  const float* bias;
  const float* rowbias; int64_t ld_rb; int64_t rb_div;
  const void* res; int64_t ld_res;
  int32_t act;
  void* out; int64_t ldc; int32_t out_f32;
  /* split-K workspace (fp32 partial slabs); size from vd_gemm_ws_bytes(), may be
   * NULL when that returns 0. */
  void* ws; int64_t ws_bytes;
  /* 3-D / (2+1)D conv (VD_A_CONV3X3 only): a kt x ks x ks kernel over the frames of each
   * video — kt temporal taps (1 or 3; 0 means 1), ks spatial (3, or 1 for the temporal half
   * of a (2+1)D conv; 0 means 3; pad ks/2).  K index = (dt*ks*ks + tap)*Cin + ci.  Output
   * image n = b*frames_out + f reads, at temporal tap dt, input image
   * b*frames_in + f + t_off + dt - kt/2, zero outside [0, frames_in) (the conv's temporal
   * zero padding; a frame-sharded rank passes its halo'd frames with frames_in =
   * frames_out + 2, t_off = 1).  n_img counts OUTPUT images. */
  int32_t kt, ks, frames_in, frames_out, t_off;
  /* Fused LayerNorm of the output rows (BasicTransformerBlock norm1/2/3 after the GEMM that
   * produces the residual stream: proj_in, attn out-proj + residual): when ln_out != NULL,
   * also ln_out[m] = (out[m] - mean) * rstd * ln_gamma + ln_beta
   * (+ ln_pe[((m / ln_pe_div) % ln_pe_period) * N .. ], the motion block's sinusoidal PE),
   * statistics over the N bf16-rounded outputs of row m (vd_layernorm's arithmetic).  Fused
   * into the 256 x 320 GEMM's epilogue when N == 320 (one tile owns whole rows); otherwise
   * vd_gemm runs vd_layernorm on the output after the GEMM.  bf16 outputs only. */
  const float* ln_gamma; const float* ln_beta; float ln_eps;
  const float* ln_pe; int64_t ln_pe_div; int64_t ln_pe_period;
  void* ln_out; int64_t ld_ln;
  /* Per-call plan controls (the library keeps no mutable selector state; zero = the product
   * plan).  path: 0 = automatic; 1 = v1 (register-staged, any shape), 2 = v2 (256 x {128,160}
   * persistent LDS-DMA), 3 = v3 (256 x 256 ping-pong, dense A), 5 = v5 (256 x 320, BK 32),
   * 6 = v6 (64 x 64, split K toward 2 workgroups per CU), 8 = v8 (weight-stationary, dense
   * K = 320, M >= 4096; automatic at M >= 16384), 9 = v9 (M <= 16 rows: one wave per 16
   * columns streaming W, v1's arithmetic; never automatic since round 6) — forced wherever that kernel takes the
   * shape, else the automatic choice; every path computes the same arithmetic for an
   * unsplit K (the K order of each output is fixed), the parity tests run each one.
   * plan_m > 0: choose kernel, split-K and LayerNorm fusion as if M were plan_m, launch over
   * all M rows — an unsharded run planned with a frame shard's M reproduces the shard's
   * summation order bit for bit (tests/test_gpu_dist2.py). */
  int32_t path;
  int64_t plan_m;
  /* Output-row permutation (round 5; 0 = none): with rmap_inner > 0 the epilogue writes row m
   * of the product — and reads its residual — at row rev3(m), where
   *   m = ((i0*rmap_n1 + i1)*rmap_n2 + i2)*rmap_inner + j  ->  ((i2*rmap_n1 + i1)*n0 + i0)*rmap_inner + j,
   * n0 = M / (rmap_n1*rmap_n2*rmap_inner).  The frame-sharded motion module's proj_out takes the
   * rows of the returning all-to-all, (position chunk, frame, video, position) on a rank, and writes
   * them straight into the rank's (video, frame, position) layout with the residual added
   * (vdiff.dist.FrameShard.return_perm) — no separate re-shard transpose.  Not with ln_out, GEGLU
   * or a row bias. */
  int32_t rmap_n1, rmap_n2, rmap_inner;
  /* LayerNorm folded into the consuming GEMM (round 5; NULL = none).  With ln_fold_s != NULL
   * the A rows are the UN-normalised LayerNorm input x (K = its row length), w = W∘gamma (each
   * column k of the Linear's W scaled by gamma[k], rounded to bf16 once), bias = b + W·beta
   * (fp32), and ln_fold_s[n] = Σ_k w[n][k] in fp32 (of the bf16 w).  The kernel takes each row's
   * mean and rstd = 1/sqrt(var + ln_fold_eps) from A itself (Σx and Σx² over the A fragments it
   * holds: two extra MFMAs per X fragment, on v8 and v6) and its epilogue forms
   *   rstd·(Σ_k w[n][k] x[m][k] − mean·ln_fold_s[n]) + bias[n]   (then act / GEGLU as usual)
   * = Linear(LayerNorm(x)) without the normalised rows being written or read.  Only the
   * weight-stationary v8 path (K = 320) and an unsplit v6 (levels 2-4 of a rank) carry it (dense, no
   * residual / rmap; a row bias — the motion block's positional encoding W·pe[frame] — is added
   * after the fold on v6): vd_gemm_plan reports kernel 0 and vd_gemm returns
   * VD_EUNSUPPORTED for any other plan. */
  const float* ln_fold_s; float ln_fold_eps;
} vd_gemm_desc;

int vd_gemm(const vd_gemm_desc* d, vd_stream_t stream);
/* The plan vd_gemm would run for this descriptor (its path / plan_m controls included):
 * *kernel = 1, 2, 3, 5, 6 or 8 (v1 .. v8; 0: no kernel takes it, vd_gemm would refuse it) and
 * *split = its K slices.  Lets a caller choose between a folded and an unfolded form (ln_fold_s)
 * and lets tools label their timings; no launch, no state. */
int vd_gemm_plan(const vd_gemm_desc* d, int32_t* kernel, int32_t* split);
/* Workspace bytes vd_gemm needs for this descriptor (0 = none): shapes with too
 * few output tiles to fill 256 CUs are split along K into fp32 slabs that a
 * second kernel reduces (deterministic, no atomics) while applying the epilogue. */
int64_t vd_gemm_ws_bytes(const vd_gemm_desc* d);
/* ---------------------------------------------------------------- GroupNorm
 * torch GroupNorm over NHWC rows, for ResnetBlock2D.norm1/2 (eps 1e-5, +SiLU),
 * Transformer2DModel.norm (eps 1e-6) and the motion-module norm whose
 * statistics span (C/G, F, H, W) (eps 1e-6) — SURVEY.md §8a a11.
 * An "instance" is a run of pix_per_inst consecutive NHWC rows sharing
 * statistics (one image, or all F frames of a video).  Channels [0,c0) come
 * from x0 (row stride ldx0), [c0,C) from x1 (row stride ldx1).
 *   vd_gn_partial : per (inst, split, channel) {count, mean, M2, 0} -> ws
 *                   ws has n_inst*n_split*C float4 entries.
 *   vd_gn_finalize: combines n_split_total partial splits (Chan), groups of
 *                   C/groups channels, -> scale_shift[inst][C] float2 {a, b}
 *                   with y = x*a + b = (x-mean)*rstd*gamma + beta.
 *   vd_gn_apply   : y = x*a + b (then SiLU if silu) -> bf16 rows (ldy).
 */
int vd_gn_partial(const void* x0, int64_t ldx0, int64_t c0, const void* x1, int64_t ldx1,
                  int64_t C, int64_t n_inst, int64_t pix_per_inst, int32_t n_split,
                  float* ws, vd_stream_t stream);
int vd_gn_finalize(const float* ws, int64_t n_inst, int32_t n_split_total, int64_t C,
                   int32_t groups, float eps, const float* gamma, const float* beta,
                   float* scale_shift, vd_stream_t stream);
int vd_gn_apply(const void* x0, int64_t ldx0, int64_t c0, const void* x1, int64_t ldx1,
                int64_t C, int64_t n_inst, int64_t pix_per_inst, const float* scale_shift,
                int32_t silu, void* y, int64_t ldy, vd_stream_t stream);
/* vd_gn_apply writing input row m to output row rev3(m) (the vd_gemm_desc.rmap_* map: rows
 * ((i0*n1 + i1)*n2 + i2)*inner + j -> ((i2*n1 + i1)*n0 + i0)*inner + j; n1, n2, inner powers of
 * two, inner = 0 the identity): the frame-sharded motion module's norm writes its rows straight
 * into the all-to-all's send order (round 5, vdiff.dist.FrameShard.send_perm). */
int vd_gn_apply_rev3(const void* x0, int64_t ldx0, int64_t c0, const void* x1, int64_t ldx1,
                     int64_t C, int64_t n_inst, int64_t pix_per_inst, const float* scale_shift,
                     int32_t silu, void* y, int64_t ldy, int64_t n1, int64_t n2, int64_t inner,
                     vd_stream_t stream);
/* Two-launch GroupNorm for image instances (ResnetBlock2D / Transformer2DModel / VAE
 * norms): vd_gn_partial_g writes ONE {n, mean, M2} record per (instance, split, group)
 * (ws: n_inst*n_split*groups float4; C <= 2560, 256 % groups == 0), and vd_gn_apply_g
 * finalizes those records itself (prologue, per workgroup of rows_per_blk rows) before
 * applying y = (x-mean)*rstd*gamma + beta (+SiLU) — no finalize launch. */
int vd_gn_partial_g(const void* x0, int64_t ldx0, int64_t c0, const void* x1, int64_t ldx1,
                    int64_t C, int64_t n_inst, int64_t pix_per_inst, int32_t n_split,
                    int32_t groups, float* ws, vd_stream_t stream);
int vd_gn_apply_g(const void* x0, int64_t ldx0, int64_t c0, const void* x1, int64_t ldx1,
                  int64_t C, int64_t n_inst, int64_t pix_per_inst, const float* ws,
                  int32_t n_split_total, int32_t groups, float eps, const float* gamma,
                  const float* beta, int32_t silu, void* y, int64_t ldy, int64_t rows_per_blk,
                  vd_stream_t stream);
/* One-launch GroupNorm (+SiLU) for small image instances (round 5): one workgroup per (instance,
 * chunk of whole groups) holding its rows in registers, exact two-pass statistics, then the apply.
 * Taken when C / groups is a multiple of 8 and a chunk's rows fit 16 pieces of 8 channels per
 * thread (the UNet's levels 3-4 and mid block: pix <= 256); otherwise VD_EUNSUPPORTED, decided
 * from (pix_per_inst, C, groups) before any operand is read — callers may probe with null pointers
 * (vdiff.ops.gn_small_chunk mirrors the rule). */
int vd_gn_small(const void* x0, int64_t ldx0, int64_t c0, const void* x1, int64_t ldx1, int64_t C,
                int64_t n_inst, int64_t pix_per_inst, int32_t groups, float eps, const float* gamma,
                const float* beta, int32_t silu, void* y, int64_t ldy, vd_stream_t stream);
/* vd_gn_finalize over vd_gn_partial_g's per-group records (ws: n_inst*n_split_total*groups
 * float4, e.g. all-gathered from frame-sharded ranks) -> scale_shift[inst][C] {a, b}: the
 * motion-module norm, whose video instances need more records than vd_gn_apply_g's prologue
 * merges (round 5: C/groups times fewer records than vd_gn_partial's per-channel ones). */
int vd_gn_finalize_g(const float* ws, int64_t n_inst, int32_t n_split_total, int64_t C,
                     int32_t groups, float eps, const float* gamma, const float* beta,
                     float* scale_shift, vd_stream_t stream);
/* vd_gn_finalize_g over RANK-MAJOR records: ws = [n_ranks][n_inst][n_split_per_rank][groups]
 * float4, the frame-sharded ranks' all-gather output as it lands (round 6: no transpose copy into
 * vd_gn_finalize_g's [n_inst][n_ranks * n_split_per_rank][groups] order).  Split s of an instance
 * is rank s / n_split_per_rank's split s % n_split_per_rank, merged in vd_gn_finalize_g's order:
 * the result equals vd_gn_finalize_g on the transposed records bit for bit. */
int vd_gn_finalize_g_ranks(const float* ws, int64_t n_inst, int32_t n_ranks, int32_t n_split_per_rank,
                           int64_t C, int32_t groups, float eps, const float* gamma, const float* beta,
                           float* scale_shift, vd_stream_t stream);

/* ---------------------------------------------------------------- LayerNorm
 * BasicTransformerBlock.norm1/2/3 (eps 1e-5) over the last dim of bf16 rows,
 * optionally + pe[(row / pe_div) % pe_period][c] (fp32; the motion block's
 * SinusoidalPositionalEmbedding, applied after norm1 and norm2 — App. A.4).
 */
int vd_layernorm(const void* x, int64_t ldx, int64_t rows, int64_t C, const float* gamma,
                 const float* beta, float eps, const float* pe, int64_t pe_div,
                 int64_t pe_period, void* y, int64_t ldy, vd_stream_t stream);

/* ---------------------------------------------------------------- attention
 * softmax(q k^T * scale) v per (batch b, head h): replaces
 * F.scaled_dot_product_attention in Attention/AttnProcessor2_0 (a6 spatial
 * self-attention, a7 cross-attention).  Row (b, s) of q at q + (b*sq + s)*ldq,
 * head h at column h*d.  K/V batch index = b / kv_div (cross-attention reads the
 * un-repeated encoder_hidden_states projection once per video).
 * d in {32, 40, 64, 80, 128, 160, 512}; flash (online softmax) with bf16 MFMA.  d = 512
 * (round 3) is the VAE decoder's single-head mid-block Attention (diffusers AttnProcessor2_0
 * over the 64x64 latent pixels of each frame): flash512_kernel,
 * o 16-byte aligned with ldo % 8 == 0 (bf16) / % 4 == 0 (fp32).
 */
int vd_attention(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v,
                 int64_t ldv, void* o, int64_t ldo, int64_t batch, int32_t heads, int64_t sq,
                 int64_t skv, int32_t d, int64_t kv_div, float scale, vd_stream_t stream);
/* vd_attention with the output O in fp32 (o: float rows, ldo in floats, 16-byte aligned):
 * the same kernels and arithmetic, minus the final bf16 rounding of O — the parity tests
 * hold it to rtol 1e-3 / atol 1e-4 against an fp64 reference. */
int vd_attention_f32(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v,
                     int64_t ldv, float* o, int64_t ldo, int64_t batch, int32_t heads,
                     int64_t sq, int64_t skv, int32_t d, int64_t kv_div, float scale, vd_stream_t stream);
/* vd_attention / vd_attention_f32 with an explicit kernel choice per call (the library keeps no
 * selector state): kernel 0 = the automatic choice (what vd_attention runs: d = 40 -> flash40
 * from 4 key tiles, flash32 below; d = 80 -> flash80 from 4 key tiles (round 6); other d -> the
 * 16x16x32 flash kernel), 1 = the 16x16x32 flash kernel for any d, 2 = flash32 (d = 40),
 * 3 = flash40 / flash80 wherever they apply (d = 40 / 80, >= 2 key tiles); a kernel that does not
 * take the shape falls through to the next one down.  All of
 * them compute softmax(q k^T * scale) v; flash40 is bit-identical to flash32 (the parity tests
 * run each).  out_f32 as vd_attention_f32. */
int vd_attention_ex(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                    void* o, int64_t ldo, int64_t batch, int32_t heads, int64_t sq, int64_t skv, int32_t d,
                    int64_t kv_div, float scale, int32_t out_f32, int32_t kernel, vd_stream_t stream);

/* Temporal (motion-module) self-attention over frames (a9): token (b, f, p) is
 * row (b*frames + f)*positions + p of q/k/v/o (the NHWC layout, no permute);
 * frames <= 32. */
int vd_temporal_attention(const void* q, const void* k, const void* v, int64_t ld,
                          void* o, int64_t ldo, int64_t batch, int32_t frames,
                          int64_t positions, int32_t heads, int32_t d, float scale,
                          vd_stream_t stream);
/* Temporal attention of a frame-sharded rank under the K/V all-gather layout (SURVEY.md §8e,
 * the north star's "RCCL all-gather for the temporal-attention window"): the rank's own
 * qframes query frames, rows (b*qframes + f)*positions + p of q (stride ldq) and o (stride
 * ldo), against all kframes key frames gathered from every rank, rows
 * (b*kframes + f)*positions + p of k and v (stride ldkv).  Replaces, for the rank's frames,
 * the rows of diffusers' temporal Attention (motion_module.py: attention over the
 * (B*H*W, F, C) sequence; 03_trace_forward_pass.py:160-169).  qframes <= kframes <= 16;
 * d in {32, 40, 64, 80, 160} (else VD_EUNSUPPORTED). */
int vd_temporal_attention_kv(const void* q, int64_t ldq, const void* k, const void* v, int64_t ldkv,
                             void* o, int64_t ldo, int64_t batch, int32_t qframes, int32_t kframes,
                             int64_t positions, int32_t heads, int32_t d, float scale,
                             vd_stream_t stream);
/* The motion module's temporal self-attention WITH its Q/K/V projection (round 2): x = the
 * normed rows (b, f, p) [row stride ldx] of one BasicTransformerBlock attention
 * (AnimateDiffTransformer3D, a8/a9), wqkv = the fused [3C][C] to_q|to_k|to_v weight (the
 * softmax scale folded into to_q as vdiff's Attention.prepare does, or passed as `scale`),
 * o = the attention output rows [row stride ldo], before to_out.  Equal bit for bit to
 * vd_gemm(x, wqkv) followed by vd_temporal_attention; the [rows][3C] projection never
 * reaches HBM.  Implemented for the level-1 shape (frames 16, 8 heads, d 40) with at least
 * two workgroups (8 positions of one video each) per CU; else VD_EUNSUPPORTED — callers run
 * the two-launch path. */
int vd_motion_qkv_attention(const void* x, int64_t ldx, const void* wqkv, int64_t ldw, void* o, int64_t ldo,
                            int64_t batch, int32_t frames, int64_t positions, int32_t heads, int32_t d,
                            float scale, const float* ln_fold_tab, float ln_fold_eps, vd_stream_t stream);
/* ln_fold_tab != NULL (round 5): the block's LayerNorm (+ the sinusoidal PE by frame) folded in,
 * as vd_gemm_desc.ln_fold_s: x holds the UN-normalised rows, wqkv = W_qkv∘gamma (bf16), and
 * ln_fold_tab is [8 heads][2048] fp32: per head h, the 120 row sums of wqkv's rows of that head
 * (q | k | v, 40 each, in that order), then for each frame f < 16 the 120 values
 * W·(beta + pe[f]) of the same rows (W the unfolded fp32 weight), zero-padded to 2048.
 * vd_motion_qkv_attention_takes: 1 when the fused kernel takes the shape (else the call
 * returns VD_EUNSUPPORTED and the caller runs GEMM + vd_temporal_attention); no launch. */
int vd_motion_qkv_attention_takes(int64_t batch, int32_t frames, int64_t positions, int32_t heads, int32_t d);
/* vd_temporal_attention for the DiT's temporal blocks (d = 64, 17..32 frames) with the 1-D
 * temporal RoPE (vd_rope_qk mode 1, angle by frame) applied to q/k inside the kernel as they
 * are loaded; q and k are read un-rotated and left unchanged. */
int vd_temporal_attention_rope(const void* q, const void* k, const void* v, int64_t ld, void* o,
                               int64_t ldo, int64_t batch, int32_t frames, int64_t positions,
                               int32_t heads, int32_t d, float scale, float theta,
                               vd_stream_t stream);
/* vd_temporal_attention on the VALU kernel for every shape (vd_temporal_attention takes the
 * MFMA kernel for frames <= 16 and d in {32, 40, 64, 80, 160}, frames 17..32 and d in {40, 64, 80,
 * 160}, and this one otherwise): the same arguments and result; the parity tests run both. */
int vd_temporal_attention_valu(const void* q, const void* k, const void* v, int64_t ld, void* o,
                               int64_t ldo, int64_t batch, int32_t frames, int64_t positions,
                               int32_t heads, int32_t d, float scale, vd_stream_t stream);

/* Row softmax over fp32 scores in log2 units (p = exp2(s - max) / sum, bf16 out): round 2's
 * materialised-score form of the VAE mid-block attention (now vd_attention with d = 512;
 * kept for tools/vae_attn_ab.py's A/B and as a general row softmax).
 * rows x cols, cols % 4 == 0, row strides ld_s / ld_p in elements. */
int vd_softmax_rows(const float* s, int64_t ld_s, int64_t rows, int64_t cols, void* p,
                    int64_t ld_p, vd_stream_t stream);

/* Temporal-consistency metric cores (experiments/
 * 06_measure_grid_search.py compute_mse :209-211 over consecutive frames and
 * compute_flicker_index :221-235) for a batch of uint8 videos [videos][frames][bytes]
 * (bytes_per_frame = H*W*3, multiple of 16, base 16-byte aligned), exact integers:
 *   sse[v][f] = sum (x[f+1]-x[f])^2 (f < frames-1); sad[v][f] = sum |x[f]-2x[f+1]+x[f+2]|
 * (f < frames-2; sad may be NULL when frames == 2).  2 <= frames <= 32. */
int vd_frame_metrics(const void* frames_u8, int64_t videos, int32_t frames, int64_t bytes_per_frame,
                     uint64_t* sse, uint64_t* sad, vd_stream_t stream);

/* Dense optical flow of every consecutive frame pair (replaces
 * OpticalFlowEstimator.compute_flow, experiments/06_measure_grid_search.py:163-188 =
 * cv2.calcOpticalFlowFarneback(grey_f, grey_f+1, None, pyr_scale, levels, winsize,
 * iterations, poly_n, poly_sigma, flags=0) with grey = uint8(mean_c(x/255)*255), :173).
 * frames_u8: [videos][frames][H][W][3] uint8; flow out: fp32 [videos][frames-1][H][W][2]
 * (dx, dy); poly_n 5 or 7; workspace: at least the byte count vd_farneback_workspace
 * returns for the same sizes (-1 on bad sizes), device memory. */
int64_t vd_farneback_workspace(int64_t videos, int32_t frames, int32_t H, int32_t W);
int vd_farneback_flow(const void* frames_u8, int64_t videos, int32_t frames, int32_t H, int32_t W,
                      double pyr_scale, int32_t levels, int32_t winsize, int32_t iterations,
                      int32_t poly_n, double poly_sigma, float* flow, void* workspace,
                      int64_t workspace_bytes, vd_stream_t stream);

/* Flow magnitude moments and warp error per pair (06:190-199 compute_flow_stats,
 * :259-284 warp_frame, :336-337): stats [videos*(frames-1)][3] fp64 =
 * { sum |flow|, sum |flow|^2 over H*W, sum over 3*H*W of (warp(frame_f, flow) - frame_f+1)^2 }
 * with frames as u8/255, warp = grid_sample(bilinear, border, align_corners=True) at
 * (x + dx, y + dy).  Deterministic (fixed-order partials in the workspace: at least the
 * byte count vd_flow_warp_workspace returns). */
int64_t vd_flow_warp_workspace(int64_t videos, int32_t frames);
int vd_flow_warp_stats(const void* frames_u8, const float* flow, int64_t videos, int32_t frames,
                       int32_t H, int32_t W, double* stats, void* workspace, int64_t workspace_bytes,
                       vd_stream_t stream);

/* ---------------------------------------------------------------- step glue
 * vd_timestep_embed: diffusers Timesteps(dim, flip_sin_to_cos=True, shift 0)
 *   (a12) -> bf16 [B][dim].  Timestep = ts[*step_idx] if step_idx else ts[b]; ts holds
 *   n_ts entries (the device step index is clamped to [0, n_ts - 1]; without step_idx
 *   n_ts >= B).
 * vd_pack_latents: x (B,C,F,H,W) fp32 / in_div -> NHWC bf16 rows [(dup*B*F*H*W)][cpad],
 *   channels >= C zero; dup = 2 repeats the batch (the CFG cat([x, x])); in_div is
 *   the scheduler's scale_model_input divisor (1 for DDIM, sqrt(sigma^2+1) for Euler).
 * vd_unpack_nhwc: NHWC rows (fp32 if src_f32 else bf16, row stride ld) ->
 *   (B,C,F,H,W) fp32.
 * vd_ddim_cfg_step: eps rows NHWC fp32 [(ncfg*B*F*H*W)][ld_eps]; if ncfg == 2
 *   eps = e_u + g*(e_c - e_u) (uncond first); DDIM eta=0 epsilon update of
 *   latents (B,C,F,H,W) fp32 in place with coef[4*step] = {sqrt(a_t),
 *   sqrt(1-a_t), sqrt(a_prev), sqrt(1-a_prev)}, step = *step_idx (or 0 if
 *   NULL) clamped to the n_coef rows of the table; fp32 in diffusers' operation
 *   order, one rounding per op (bit-exact vs torch); optional x0_out (B,C,F,H,W) fp32; optional next_in = the packed
 *   bf16 UNet input of the next step (dup = ncfg) — a1 + a13 fused.
 * vd_euler_cfg_step: as vd_ddim_cfg_step, with the EulerDiscreteScheduler.step
 *   update (s_churn 0, epsilon; diffusers' fp32 order x0 = x - s*eps,
 *   d = (x - x0)/s, x += d*(s_next - s)) and coef[4*step] = {sigma, sigma_next,
 *   sqrt(sigma_next^2 + 1), 0}; next_in = the next step's scale_model_input(x)
 *   packed to bf16 — §8f rank 2 (experiments/01_baseline_generation.py:76-80).
 * vd_step_advance: ++*step_idx (one thread; the last node of a captured step).
 */
int vd_timestep_embed(const float* ts, int64_t n_ts, const int32_t* step_idx, int64_t B,
                      int32_t dim, void* out, vd_stream_t stream);
int vd_pack_latents(const float* x, int64_t B, int64_t C, int64_t F, int64_t H, int64_t W,
                    int32_t dup, void* out, int64_t cpad, float in_div, vd_stream_t stream);
int vd_unpack_nhwc(const void* src, int32_t src_f32, int64_t ld, int64_t B, int64_t C,
                   int64_t F, int64_t H, int64_t W, float* dst, vd_stream_t stream);
int vd_ddim_cfg_step(const float* eps, int64_t ld_eps, int32_t ncfg, float guidance,
                     float* latents, int64_t B, int64_t C, int64_t F, int64_t H, int64_t W,
                     const float* coef, int64_t n_coef, const int32_t* step_idx, float* x0_out,
                     void* next_in, int64_t cpad, vd_stream_t stream);
int vd_euler_cfg_step(const float* eps, int64_t ld_eps, int32_t ncfg, float guidance,
                      float* latents, int64_t B, int64_t C, int64_t F, int64_t H, int64_t W,
                      const float* coef, int64_t n_coef, const int32_t* step_idx, float* x0_out,
                      void* next_in, int64_t cpad, vd_stream_t stream);
int vd_step_advance(int32_t* step_idx, vd_stream_t stream);

/* Row-block permute for the frame<->position re-shard around motion modules:
 * dst[(a*nb + b)*nc + c] = src[(b*na + a)*nc + c] for bf16 rows of `width`
 * elements (a transpose of the [nb][na] grid of row blocks, nc rows each). */
int vd_block_transpose(const void* src, void* dst, int64_t nb, int64_t na, int64_t nc,
                       int64_t width, vd_stream_t stream);

/* ---- module-level (diffusers-layout) path: csrc/rows.hip ----
 * Elementwise ops a caller driving the modules one by one needs between HIP GEMM / norm /
 * attention calls (forward-hook tracing, experiments/03_trace_forward_pass.py:105-113; a
 * direct motion_modules[i](x, num_frames=F) call, 03:182).  bf16 rows, C % 8 == 0, 16-B
 * aligned bases, row strides in elements.
 * vd_rows_eltwise: op 0: out[r] = (x ? x[r] : 0) + y[(r / y_div) % y_period] (y bf16, or fp32
 *   if y_f32) — residual adds, the ResnetBlock2D time-embedding broadcast, the sinusoidal
 *   positional embedding, repeat_interleave, channel concat into column slices;
 *   op 1: out[r] = silu(x[r]) (nn.SiLU).
 * vd_upsample_nearest2x: rows of n_img h x w images -> rows of their nearest x2 upsample
 *   (Upsample2D's F.interpolate(scale_factor=2.0, mode="nearest")). */
int vd_rows_eltwise(int32_t op, const void* x, int64_t ldx, const void* y, int64_t ldy, int32_t y_f32,
                    int64_t y_div, int64_t y_period, int64_t rows, int64_t C, void* out, int64_t ldo,
                    vd_stream_t stream);
int vd_upsample_nearest2x(const void* x, int64_t ldx, int64_t n_img, int64_t h, int64_t w, int64_t C,
                          void* out, int64_t ldo, vd_stream_t stream);

/* ---- DiT-style denoiser (BASELINE config 5; build-defined model,
 * no reference counterpart — oracle/dit_ref.py is its restatement) ----
 * vd_patchify: latents fp32 (B,C,F,H,W) / in_div -> token rows bf16 [(b,f,hp,wp)][kpad],
 *   k = (c*p + ph)*p + pw (Conv3d (1,p,p) patch-embed flattening), zero-padded; dup = 2
 *   writes the CFG copy after the first B*F*(H/p)*(W/p) rows.
 * vd_unpatchify: token rows fp32 [(n,hp,wp)][(ph,pw,c)] -> NHWC pixel rows fp32 [(n,h,w)][c].
 * vd_rope_qk: rotary embedding (rotate-half pairs) in place on columns [0, ncols) of token
 *   rows, head width d; mode 0 = spatial 2-D (first d/2 dims by row h, last d/2 by column
 *   w), mode 1 = temporal 1-D (frame f); token r = ((b*F + f)*Hp + h)*Wp + w.
 * vd_res_ln_mod: per row (b = row / rows_per_b): xn = x + gate[b]*y (y, gate optional),
 *   x_out = xn (optional, may alias x), h = LN(xn, eps; no affine)*(1 + scale[b]) + shift[b]
 *   (shift/scale optional); C <= 2048, C % 8 == 0; gate/shift/scale fp32 rows of ld_mod. */
int vd_patchify(const float* lat, int64_t B, int64_t C, int64_t F, int64_t H, int64_t W,
                int32_t p, int32_t dup, float in_div, void* out, int64_t kpad, vd_stream_t stream);
int vd_unpatchify(const float* src, int64_t ld_src, int64_t n_img, int64_t H, int64_t W,
                  int32_t p, int32_t C, float* dst, vd_stream_t stream);
int vd_rope_qk(void* x, int64_t ld, int64_t rows, int32_t ncols, int32_t d, int32_t mode,
               int64_t F, int64_t Hp, int64_t Wp, float theta, vd_stream_t stream);
int vd_res_ln_mod(const void* x, int64_t ldx, const void* y, int64_t ldy, const float* gate,
                  const float* shift, const float* scale, int64_t ld_mod, int64_t rows_per_b,
                  void* x_out, int64_t ldxo, void* h, int64_t ldh, int64_t rows, int64_t C,
                  float eps, vd_stream_t stream);

/* fp8 spatial self-attention, d = 64 (BASELINE config 5 "fp8 MFMA QK^T/PV"; the DiT's
 * spatial blocks): block-scaled v_mfma_scale_f32_32x32x64_f8f6f4, OCP e4m3 operands.
 * vd_attention_fp8_quant: q/k/v bf16 rows (column slices of the fused QKV buffer) ->
 *   q8/k8 fp8 rows [batch*s][ld8] (ld8 >= heads*64, % 16) with one E8M0 scale byte per
 *   (row, head) in qs/ks [batch*s][heads]; vt8 = V^T fp8 [batch*heads][64][skv] with the keys
 *   of every 64-key tile in the MFMA's k-slot order, vs = one E8M0 per (image, head, tile).
 *   q_scale multiplies q before it is quantized (round 5): pass scale * log2(e) and call
 *   vd_attention_fp8 with scale = 1 / log2(e) to fold the softmax scale into q8 (the kernel then
 *   applies no per-score multiply and takes its exp2 argument straight from the MFMA); 1.0 keeps q.
 * vd_attention_fp8: softmax(scale * Q K^T) V from those operands (Q the dequantized q8) ->
 *   bf16 rows o (column h*64 of head h).  sq % 32 == 0, skv % 64 == 0.
 * vd_attention_fp8_quant_rope: vd_attention_fp8_quant for the DiT's spatial blocks with
 *   vd_rope_qk mode 0 (s = Hp*Wp tokens per image) applied to q and k in fp32 inside the
 *   quantization pass (q/k are read un-rotated and left unchanged). */
int vd_attention_fp8_quant(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v,
                           int64_t ldv, int64_t batch, int32_t heads, int64_t sq, int64_t skv,
                           int32_t d, void* q8, void* k8, int64_t ld8, void* vt8, void* qs, void* ks,
                           void* vs, float q_scale, vd_stream_t stream);
int vd_attention_fp8_quant_rope(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v,
                                int64_t ldv, int64_t batch, int32_t heads, int64_t s, int32_t d,
                                int64_t Hp, int64_t Wp, float theta, void* q8, void* k8, int64_t ld8,
                                void* vt8, void* qs, void* ks, void* vs, float q_scale,
                                vd_stream_t stream);
int vd_attention_fp8(const void* q8, const void* k8, int64_t ld8, const void* qs, const void* ks,
                     const void* vt8, const void* vs, void* o, int64_t ldo, int64_t batch,
                     int32_t heads, int64_t sq, int64_t skv, int32_t d, float scale,
                     vd_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* VDIFF_H */
