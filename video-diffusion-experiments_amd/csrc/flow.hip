// Dense optical flow and warp error of generated videos: the
// OpticalFlowEstimator / warp_frame half of experiments/06_measure_grid_search.py
// (:163-199 compute_flow + compute_flow_stats, :259-284 warp_frame, :330-338 per pair),
// i.e. cv2.calcOpticalFlowFarneback(grey1, grey2, None, 0.5, 3, 15, 3, 5, 1.2, 0) over every
// consecutive frame pair of a batch of uint8 videos, then the flow-magnitude moments and the
// MSE of frame i warped by the flow against frame i+1.
//
// The algorithm is Farneback's polynomial-expansion flow as OpenCV implements it
// (optflowgf.cpp; restated step by step in oracle/flow_ref.py, which agrees with the
// reference's own per-pair records to ~1e-6): per pyramid level, from the coarsest,
//   grey  = uint8(mean_c(x / 255) * 255)                      (06:173, torch fp32 ops)
//   I     = resize_linear(GaussianBlur(grey, smooth, sigma))  (full-res blur per level)
//   R     = PolyExp(I)       5 coefficients / pixel: fp32 vertical, fp64 horizontal pass
//   flow  = 2 * resize_linear(flow of the coarser level)      (zeros at the top)
//   M     = UpdateMatrices(R_prev, R_next, flow)              5 products / pixel, fp32
//   3 x { flow = solve(box_{w x w}(M) / w^2);  M = UpdateMatrices(...) }   (box in fp64)
// Every stage is a gather over a small window (HBM / L2-bound, no GEMM shape): one thread
// per output value, planar [plane][h][w] buffers so a wave's 64 lanes read 64 consecutive
// floats of a row, and all frames / pairs of the batch in one launch per stage.  Arithmetic
// follows the oracle's operation order with fp contraction off, so every stage up to the
// box sums reproduces it bit for bit; the box sums are direct (the oracle uses running sums,
// as OpenCV does) — the only source of last-bit differences.
#include "common.h"

#pragma clang fp contract(off)

namespace {

constexpr int NT = 256;
constexpr int MAXTAP = 63;  // Gaussian smoothing taps (level sigma 3.5 -> 19)
constexpr int MAXPOLY = 15;  // 2 poly_n + 1, poly_n <= 7

struct Taps {
  float k[MAXTAP];
  int n;
};
struct PolyCoef {
  float g[MAXPOLY], xg[MAXPOLY], xxg[MAXPOLY];
  double ig11, ig03, ig33, ig55;
  int n;
};

__device__ __forceinline__ int reflect101(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * (n - 1) - i : i;
}
__device__ __forceinline__ int clampi(int i, int lo, int hi) { return i < lo ? lo : (i > hi ? hi : i); }

// 06:173 `(frame.mean(dim=0) * 255).numpy().astype(np.uint8)` with frame = u8 / 255:
// torch's fp32 ops in order (IEEE divides, sum of the three channels left to right).
__device__ __forceinline__ float grey_of(const uint8_t* px) {
  const float r = __fdiv_rn((float)px[0], 255.0f), g = __fdiv_rn((float)px[1], 255.0f),
              b = __fdiv_rn((float)px[2], 255.0f);
  const float m = __fdiv_rn((r + g) + b, 3.0f);
  return (float)(uint32_t)(m * 255.0f);
}

// GaussianBlur horizontal pass (reflect-101), fp32 sum from zero in tap order.  src: the
// RGB frames (grey formed on the fly) -> tmp [img][H][W].
__global__ void blur_h_kernel(const uint8_t* frames, int64_t n_img, int H, int W, Taps t, float* tmp) {
  const int64_t total = n_img * H * W;
  const int r = t.n / 2;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int x = (int)(i % W);
    const int64_t row = i / W;
    const uint8_t* src = frames + row * W * 3;
    float acc = 0.f;
    for (int k = 0; k < t.n; ++k) acc = acc + t.k[k] * grey_of(src + 3 * reflect101(x + k - r, W));
    tmp[i] = acc;
  }
}

// vertical pass over tmp -> out [img][H][W]
__global__ void blur_v_kernel(const float* tmp, int64_t n_img, int H, int W, Taps t, float* out) {
  const int64_t total = n_img * H * W;
  const int r = t.n / 2;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int x = (int)(i % W);
    const int y = (int)((i / W) % H);
    const float* src = tmp + (i / ((int64_t)W * H)) * H * W + x;
    float acc = 0.f;
    for (int k = 0; k < t.n; ++k) acc = acc + t.k[k] * src[(int64_t)reflect101(y + k - r, H) * W];
    out[i] = acc;
  }
}

// resize(INTER_LINEAR) source coordinate and weights (OpenCV's half-pixel mapping, clamped)
struct Lin {
  int i0, i1;
  float a0, a1;
};
__device__ __forceinline__ Lin lin_coeff(int d, int dsize, int ssize) {
  const double scale = (double)ssize / (double)dsize;
  float f = (float)(((double)d + 0.5) * scale - 0.5);
  int s = (int)floorf(f);
  f = f - (float)s;
  if (s < 0) { f = 0.f; s = 0; }
  if (s >= ssize - 1) { f = 0.f; s = ssize - 1; }
  Lin l;
  l.i0 = s;
  l.i1 = s + 1 < ssize ? s + 1 : ssize - 1;
  l.a0 = 1.0f - f;
  l.a1 = f;
  return l;
}

// planes [p][sh][sw] -> [p][h][w] (horizontal then vertical, as the oracle), times `mul`
// (2 for the flow carried down a level).  interleave2: source and output are [p][y][x][2].
__global__ void resize_kernel(const float* src, int64_t planes, int sh, int sw, int h, int w, int interleave2,
                              float mul, float* out) {
  const int c2 = interleave2 ? 2 : 1;
  const int64_t total = planes * h * w * c2;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int c = (int)(i % c2);
    const int x = (int)((i / c2) % w);
    const int y = (int)((i / c2 / w) % h);
    const int64_t p = i / c2 / w / h;
    const Lin lx = lin_coeff(x, w, sw), ly = lin_coeff(y, h, sh);
    const float* s = src + p * sh * sw * c2 + c;
    const float r0 = s[((int64_t)ly.i0 * sw + lx.i0) * c2] * lx.a0 + s[((int64_t)ly.i0 * sw + lx.i1) * c2] * lx.a1;
    const float r1 = s[((int64_t)ly.i1 * sw + lx.i0) * c2] * lx.a0 + s[((int64_t)ly.i1 * sw + lx.i1) * c2] * lx.a1;
    const float v = r0 * ly.a0 + r1 * ly.a1;
    out[i] = v * mul;
  }
}

// FarnebackPolyExp, vertical part (fp32, rows clamped): I [img][h][w] -> rv [img][3][h][w]
__global__ void poly_v_kernel(const float* I, int64_t n_img, int h, int w, PolyCoef pc, float* rv) {
  const int64_t hw = (int64_t)h * w, total = n_img * hw;
  const int n = pc.n;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int64_t img = i / hw;
    const int y = (int)((i % hw) / w), x = (int)(i % w);
    const float* s = I + img * hw + x;
    float r0 = s[(int64_t)y * w] * pc.g[n], r1 = 0.f, r2 = 0.f;
    for (int k = 1; k <= n; ++k) {
      const float s0 = s[(int64_t)(y - k < 0 ? 0 : y - k) * w];
      const float s1 = s[(int64_t)(y + k > h - 1 ? h - 1 : y + k) * w];
      const float p = s0 + s1;
      r0 = r0 + pc.g[n + k] * p;
      r1 = r1 + pc.xg[n + k] * (s1 - s0);
      r2 = r2 + pc.xxg[n + k] * p;
    }
    float* o = rv + img * 3 * hw + (i % hw);
    o[0] = r0;
    o[hw] = r1;
    o[2 * hw] = r2;
  }
}

// horizontal part (fp64 accumulators, columns replicated): rv -> R [img][5][h][w]
// (plane order as OpenCV stores it: 0 y-linear, 1 x-linear, 2 yy, 3 xx, 4 xy)
__global__ void poly_h_kernel(const float* rv, int64_t n_img, int h, int w, PolyCoef pc, float* R) {
  const int64_t hw = (int64_t)h * w, total = n_img * hw;
  const int n = pc.n;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int64_t img = i / hw;
    const int x = (int)(i % w);
    const float* row0 = rv + img * 3 * hw + (i % hw) - x;
    const float* row1 = row0 + hw;
    const float* row2 = row0 + 2 * hw;
    const double gc = (double)pc.g[n];
    double b1 = (double)row0[x] * gc, b3 = (double)row1[x] * gc, b5 = (double)row2[x] * gc;
    double b2 = 0.0, b4 = 0.0, b6 = 0.0;
    for (int k = 1; k <= n; ++k) {
      const int xp = x + k > w - 1 ? w - 1 : x + k, xm = x - k < 0 ? 0 : x - k;
      const double gk = (double)pc.g[n + k], xgk = (double)pc.xg[n + k], xxgk = (double)pc.xxg[n + k];
      const double p0 = row0[xp], m0 = row0[xm], p1 = row1[xp], m1 = row1[xm], p2 = row2[xp], m2 = row2[xm];
      const double tg = p0 + m0;
      b1 = b1 + tg * gk;
      b4 = b4 + tg * xxgk;
      b2 = b2 + (p0 - m0) * xgk;
      b3 = b3 + (p1 + m1) * gk;
      b6 = b6 + (p1 - m1) * xgk;
      b5 = b5 + (p2 + m2) * gk;
    }
    float* o = R + img * 5 * hw + (i % hw);
    o[hw] = (float)(b2 * pc.ig11);
    o[0] = (float)(b3 * pc.ig11);
    o[3 * hw] = (float)(b1 * pc.ig03 + b4 * pc.ig33);
    o[2 * hw] = (float)(b1 * pc.ig03 + b5 * pc.ig33);
    o[4 * hw] = (float)(b6 * pc.ig55);
  }
}

__device__ __forceinline__ float border_w(int i, int n) {
  // FarnebackUpdateMatrices' border attenuation over the outer 5 rows / columns
  const float B[5] = {0.14f, 0.14f, 0.4472f, 0.4472f, 0.4472f};
  float s = 1.0f;
  if (i < 5) s = s * B[i];
  if (i >= n - 5) s = s * B[n - 1 - i];
  return s;
}

// FarnebackUpdateMatrices for every pair pixel: R of the pair's frames (prev = frame f,
// next = f + 1 of the same video), flow [pair][h][w][2] -> M [pair][5][h][w]
__global__ void update_matrices_kernel(const float* R, int frames, int64_t pairs, int h, int w, const float* flow,
                                       float* M) {
  const int64_t hw = (int64_t)h * w, total = pairs * hw;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int64_t pair = i / hw;
    const int64_t pix = i % hw;
    const int y = (int)(pix / w), x = (int)(pix % w);
    const int64_t prev = pair / (frames - 1) * frames + pair % (frames - 1);
    const float* R0 = R + prev * 5 * hw;
    const float* R1 = R0 + 5 * hw;
    const float dx = flow[i * 2], dy = flow[i * 2 + 1];
    float fx = (float)x + dx, fy = (float)y + dy;
    const float flx = floorf(fx), fly = floorf(fy);
    const int x1 = (int)flx, y1 = (int)fly;
    fx = fx - flx;
    fy = fy - fly;
    const bool inside = x1 >= 0 && x1 < w - 1 && y1 >= 0 && y1 < h - 1;
    const int xc = clampi(x1, 0, w - 2), yc = clampi(y1, 0, h - 2);
    const float a00 = (1.0f - fx) * (1.0f - fy), a01 = fx * (1.0f - fy), a10 = (1.0f - fx) * fy, a11 = fx * fy;
    float r[5];
#pragma unroll
    for (int c = 0; c < 5; ++c) {
      const float* p = R1 + c * hw + (int64_t)yc * w + xc;
      r[c] = ((a00 * p[0] + a01 * p[1]) + a10 * p[w]) + a11 * p[w + 1];
    }
    const float q0 = R0[pix], q1 = R0[hw + pix], q2 = R0[2 * hw + pix], q3 = R0[3 * hw + pix],
                q4 = R0[4 * hw + pix];
    float r4 = inside ? (q2 + r[2]) * 0.5f : q2;
    float r5 = inside ? (q3 + r[3]) * 0.5f : q3;
    float r6 = inside ? (q4 + r[4]) * 0.25f : q4 * 0.5f;
    float r2 = inside ? r[0] : 0.f;
    float r3 = inside ? r[1] : 0.f;
    r2 = (q0 - r2) * 0.5f;
    r3 = (q1 - r3) * 0.5f;
    r2 = (r2 + r4 * dy) + r6 * dx;
    r3 = (r3 + r6 * dy) + r5 * dx;
    const float sc = border_w(y, h) * border_w(x, w);
    r2 = r2 * sc;
    r3 = r3 * sc;
    r4 = r4 * sc;
    r5 = r5 * sc;
    r6 = r6 * sc;
    float* o = M + pair * 5 * hw + pix;
    o[0] = r4 * r4 + r6 * r6;
    o[hw] = (r4 + r5) * r6;
    o[2 * hw] = r5 * r5 + r6 * r6;
    o[3 * hw] = r4 * r2 + r6 * r3;
    o[4 * hw] = r6 * r2 + r5 * r3;
  }
}

// FarnebackUpdateFlow_Blur, vertical box sums (fp64, rows replicated): M -> V [pair][5][h][w]
__global__ void box_v_kernel(const float* M, int64_t planes, int h, int w, int win, double* V) {
  const int64_t hw = (int64_t)h * w, total = planes * hw;
  const int m = win / 2;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int y = (int)((i % hw) / w), x = (int)(i % w);
    const float* s = M + (i / hw) * hw + x;
    double acc = 0.0;
    for (int k = -m; k <= m; ++k) acc += (double)s[(int64_t)clampi(y + k, 0, h - 1) * w];
    V[i] = acc;
  }
}

// horizontal box sums, / win^2, and the 2x2 solve -> flow [pair][h][w][2]
__global__ void box_h_solve_kernel(const double* V, int64_t pairs, int h, int w, int win, float* flow) {
  const int64_t hw = (int64_t)h * w, total = pairs * hw;
  const int m = win / 2;
  const double inv = 1.0 / (double)(win * win);
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
    const int x = (int)(i % w);
    const double* row = V + (i / hw) * 5 * hw + (i % hw) - x;
    double s[5];
#pragma unroll
    for (int c = 0; c < 5; ++c) {
      double acc = 0.0;
      for (int k = -m; k <= m; ++k) acc += row[c * hw + clampi(x + k, 0, w - 1)];
      s[c] = acc * inv;
    }
    const double g11 = s[0], g12 = s[1], g22 = s[2], h1 = s[3], h2 = s[4];
    const double idet = 1.0 / ((g11 * g22 - g12 * g12) + 1e-3);
    flow[i * 2] = (float)((g11 * h2 - g12 * h1) * idet);
    flow[i * 2 + 1] = (float)((g22 * h1 - g12 * h2) * idet);
  }
}

// Per pair: sum |flow|, sum |flow|^2 (|flow| = sqrt(fx^2 + fy^2) in fp32 as numpy) and
// sum over C*H*W of (warp_frame(frame_f, flow) - frame_{f+1})^2, where warp_frame is 06's
// grid_sample(bilinear, border, align_corners=True) at (x + fx, y + fy).  Fixed-order
// per-block partials [pair][blocks][3] (deterministic); flow_stats_finalize sums them.
constexpr int WB = 64;  // blocks per pair
__global__ void warp_stats_kernel(const uint8_t* frames, const float* flow, int frames_per_video, int H, int W,
                                  double* partial) {
  const int64_t pair = blockIdx.y;
  const int64_t f1 = pair / (frames_per_video - 1) * frames_per_video + pair % (frames_per_video - 1);
  const uint8_t* a = frames + f1 * (int64_t)H * W * 3;
  const uint8_t* b = a + (int64_t)H * W * 3;
  const float* fl = flow + pair * (int64_t)H * W * 2;
  const int64_t hw = (int64_t)H * W;
  const float sxs = (float)(W - 1) * 0.5f, sys = (float)(H - 1) * 0.5f;
  double sm = 0.0, sm2 = 0.0, se = 0.0;
  for (int64_t p = (int64_t)blockIdx.x * NT + threadIdx.x; p < hw; p += (int64_t)WB * NT) {
    const int x = (int)(p % W), y = (int)(p / W);
    const float fx = fl[p * 2], fy = fl[p * 2 + 1];
    const float mag = __fsqrt_rn(fx * fx + fy * fy);
    sm += (double)mag;
    sm2 += (double)mag * (double)mag;
    // 06:263-269 in numpy fp32, then grid_sample's align_corners unnormalise and border clip
    const float gx = __fdiv_rn(2.0f * ((float)x + fx), (float)(W - 1)) - 1.0f;
    const float gy = __fdiv_rn(2.0f * ((float)y + fy), (float)(H - 1)) - 1.0f;
    float ix = (gx + 1.0f) * sxs, iy = (gy + 1.0f) * sys;
    ix = fminf(fmaxf(ix, 0.f), (float)(W - 1));
    iy = fminf(fmaxf(iy, 0.f), (float)(H - 1));
    const float x0f = floorf(ix), y0f = floorf(iy);
    const int x0 = (int)x0f, y0 = (int)y0f;
    const int x1 = x0 + 1 < W ? x0 + 1 : W - 1, y1 = y0 + 1 < H ? y0 + 1 : H - 1;
    const float tx = ix - x0f, ty = iy - y0f;
    const float wnw = (1.0f - tx) * (1.0f - ty), wne = tx * (1.0f - ty), wsw = (1.0f - tx) * ty, wse = tx * ty;
    for (int c = 0; c < 3; ++c) {
      const float v00 = __fdiv_rn((float)a[((int64_t)y0 * W + x0) * 3 + c], 255.0f);
      const float v01 = __fdiv_rn((float)a[((int64_t)y0 * W + x1) * 3 + c], 255.0f);
      const float v10 = __fdiv_rn((float)a[((int64_t)y1 * W + x0) * 3 + c], 255.0f);
      const float v11 = __fdiv_rn((float)a[((int64_t)y1 * W + x1) * 3 + c], 255.0f);
      const float wv = ((v00 * wnw + v01 * wne) + v10 * wsw) + v11 * wse;
      const float d = wv - __fdiv_rn((float)b[p * 3 + c], 255.0f);
      se += (double)d * (double)d;
    }
  }
  __shared__ double red[3][NT];
  red[0][threadIdx.x] = sm;
  red[1][threadIdx.x] = sm2;
  red[2][threadIdx.x] = se;
  __syncthreads();
  for (int s = NT / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s)
      for (int k = 0; k < 3; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x < 3) partial[(pair * WB + blockIdx.x) * 3 + threadIdx.x] = red[threadIdx.x][0];
}

__global__ void warp_stats_finalize(const double* partial, int64_t pairs, double* stats) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= pairs * 3) return;
  const int64_t pair = i / 3;
  const int k = (int)(i % 3);
  double acc = 0.0;
  for (int b = 0; b < WB; ++b) acc += partial[(pair * WB + b) * 3 + k];
  stats[i] = acc;
}

unsigned grid_for(int64_t total) {
  const int64_t b = (total + NT - 1) / NT;
  return (unsigned)(b < 65536 ? (b > 0 ? b : 1) : 65536);
}

// ---------------------------------------------------------------- host-side coefficients
// getGaussianKernel(n, sigma, CV_32F) (sigma <= 0: OpenCV's fixed small-kernel tables)
bool gaussian_taps(int n, double sigma, Taps& t) {
  if (n < 1 || n > MAXTAP || n % 2 == 0) return false;
  static const float small[4][7] = {{1.f},
                                    {0.25f, 0.5f, 0.25f},
                                    {0.0625f, 0.25f, 0.375f, 0.25f, 0.0625f},
                                    {0.03125f, 0.109375f, 0.21875f, 0.28125f, 0.21875f, 0.109375f, 0.03125f}};
  const bool fixed = sigma <= 0 && n <= 7;
  const double sx = sigma > 0 ? sigma : ((n - 1) * 0.5 - 1) * 0.3 + 0.8;
  const double scale2 = -0.5 / (sx * sx);
  float cf[MAXTAP];
  double s = 0.0;
  for (int i = 0; i < n; ++i) {
    const double x = i - (n - 1) * 0.5;
    const double v = fixed ? (double)small[n / 2][i] : exp(scale2 * x * x);
    cf[i] = (float)v;
    s += (double)cf[i];
  }
  s = 1.0 / s;
  for (int i = 0; i < n; ++i) t.k[i] = (float)((double)cf[i] * s);
  t.n = n;
  return true;
}

// numpy's pairwise float64 sum for short arrays (8 partial sums, then the tail)
double np_sum(const double* a, int n) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  double r[8];
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - n % 8; i += 8)
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}

// FarnebackPrepareGaussian: g, xg, xxg and the four entries of G^-1 PolyExp uses
bool poly_coef(int n, double sigma, PolyCoef& pc) {
  if (n < 1 || 2 * n + 1 > MAXPOLY) return false;
  if (sigma < 1.1920928955078125e-07) sigma = n * 0.3;
  double gd[MAXPOLY];
  for (int i = 0; i <= 2 * n; ++i) {
    const double x = i - n;
    gd[i] = (double)(float)exp(-x * x / (2 * sigma * sigma));
  }
  const double s = 1.0 / np_sum(gd, 2 * n + 1);
  for (int i = 0; i <= 2 * n; ++i) {
    const double x = i - n;
    pc.g[i] = (float)(gd[i] * s);
    pc.xg[i] = (float)(x * (double)pc.g[i]);
    pc.xxg[i] = (float)(x * x * (double)pc.g[i]);
  }
  double G[6][6] = {};
  for (int yi = 0; yi <= 2 * n; ++yi)
    for (int xi = 0; xi <= 2 * n; ++xi) {
      const double y = yi - n, x = xi - n;
      const double w = (double)pc.g[yi] * (double)pc.g[xi];
      G[0][0] += w;
      G[1][1] += w * x * x;
      G[3][3] += w * x * x * x * x;
      G[5][5] += w * x * x * y * y;
    }
  G[2][2] = G[0][3] = G[0][4] = G[3][0] = G[4][0] = G[1][1];
  G[4][4] = G[3][3];
  G[3][4] = G[4][3] = G[5][5];
  // Gauss-Jordan with partial pivoting
  double A[6][12];
  for (int r = 0; r < 6; ++r)
    for (int c = 0; c < 12; ++c) A[r][c] = c < 6 ? G[r][c] : (c - 6 == r ? 1.0 : 0.0);
  for (int c = 0; c < 6; ++c) {
    int piv = c;
    for (int r = c + 1; r < 6; ++r)
      if (fabs(A[r][c]) > fabs(A[piv][c])) piv = r;
    if (A[piv][c] == 0.0) return false;
    for (int k = 0; k < 12; ++k) {
      const double t = A[c][k];
      A[c][k] = A[piv][k];
      A[piv][k] = t;
    }
    const double d = A[c][c];
    for (int k = 0; k < 12; ++k) A[c][k] /= d;
    for (int r = 0; r < 6; ++r)
      if (r != c) {
        const double f = A[r][c];
        for (int k = 0; k < 12; ++k) A[r][k] -= f * A[c][k];
      }
  }
  pc.ig11 = A[1][7];
  pc.ig03 = A[0][9];
  pc.ig33 = A[3][9];
  pc.ig55 = A[5][11];
  pc.n = n;
  return true;
}

struct Plan {
  int levels;
  int h[16], w[16];
  Taps blur[16];
};

bool make_plan(int H, int W, double pyr_scale, int levels, Plan& p) {
  if (!(pyr_scale > 0 && pyr_scale < 1) || levels < 0 || levels > 15) return false;
  double scale = 1.0;
  int k = 0;
  for (; k < levels; ++k) {
    scale *= pyr_scale;
    if (W * scale < 32 || H * scale < 32) break;
  }
  p.levels = k;
  for (int l = 0; l <= k; ++l) {
    double s = 1.0;
    for (int j = 0; j < l; ++j) s *= pyr_scale;
    const double sigma = (1.0 / s - 1) * 0.5;
    int smooth = ((int)nearbyint(sigma * 5)) | 1;
    if (smooth < 3) smooth = 3;
    p.w[l] = (int)nearbyint(W * s);
    p.h[l] = (int)nearbyint(H * s);
    if (!gaussian_taps(smooth, sigma, p.blur[l])) return false;
  }
  return true;
}

struct WsLayout {
  int64_t tmp, blurred, lvl, rv, R, M, V, flow_a, bytes;
};
WsLayout ws_layout(int64_t n_img, int64_t pairs, int64_t H, int64_t W) {
  const int64_t hw = H * W;
  auto al = [](int64_t b) { return (b + 255) / 256 * 256; };
  WsLayout l;
  int64_t o = 0;
  l.tmp = o; o += al(n_img * hw * 4);
  l.blurred = o; o += al(n_img * hw * 4);
  l.lvl = o; o += al(n_img * hw * 4);
  l.rv = o; o += al(n_img * 3 * hw * 4);
  l.R = o; o += al(n_img * 5 * hw * 4);
  l.M = o; o += al(pairs * 5 * hw * 4);
  l.V = o; o += al(pairs * 5 * hw * 8);
  l.flow_a = o; o += al(pairs * hw * 2 * 4);
  l.bytes = o;
  return l;
}

}  // namespace

extern "C" int64_t vd_farneback_workspace(int64_t videos, int32_t frames, int32_t H, int32_t W) {
  if (videos <= 0 || frames < 2 || H <= 0 || W <= 0) return -1;
  return ws_layout(videos * frames, videos * (frames - 1), H, W).bytes;
}

extern "C" int vd_farneback_flow(const void* frames_u8, int64_t videos, int32_t frames, int32_t H, int32_t W,
                                 double pyr_scale, int32_t levels, int32_t winsize, int32_t iterations,
                                 int32_t poly_n, double poly_sigma, float* flow, void* workspace,
                                 int64_t workspace_bytes, vd_stream_t stream) {
  VD_CHECK_ARG(frames_u8 && flow && workspace && videos > 0 && frames >= 2 && H >= 8 && W >= 8);
  VD_CHECK_ARG(winsize >= 1 && winsize % 2 == 1 && iterations >= 1 && (poly_n == 5 || poly_n == 7));
  const int64_t n_img = videos * frames, pairs = videos * (frames - 1);
  const WsLayout L = ws_layout(n_img, pairs, H, W);
  VD_CHECK_ARG(workspace_bytes >= L.bytes);
  Plan plan;
  PolyCoef pc;
  VD_CHECK_ARG(make_plan(H, W, pyr_scale, levels, plan) && poly_coef(poly_n, poly_sigma, pc));
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)workspace;
  float* tmp = (float*)(ws + L.tmp);
  float* blurred = (float*)(ws + L.blurred);
  float* lvl = (float*)(ws + L.lvl);
  float* rv = (float*)(ws + L.rv);
  float* R = (float*)(ws + L.R);
  float* M = (float*)(ws + L.M);
  double* V = (double*)(ws + L.V);
  float* fa = (float*)(ws + L.flow_a);
  const uint8_t* fr = (const uint8_t*)frames_u8;
  const int64_t full = n_img * H * W;
  // the levels alternate their flow between the workspace and the output so that level 0
  // lands in `flow`
  float* cur = nullptr;
  int ph = 0, pw = 0;
  for (int k = plan.levels; k >= 0; --k) {
    const int h = plan.h[k], w = plan.w[k];
    const int64_t hw = (int64_t)h * w;
    float* fl = (k % 2 == 0) ? flow : fa;
    hipLaunchKernelGGL(blur_h_kernel, dim3(grid_for(full)), dim3(NT), 0, s, fr, n_img, H, W, plan.blur[k], tmp);
    hipLaunchKernelGGL(blur_v_kernel, dim3(grid_for(full)), dim3(NT), 0, s, tmp, n_img, H, W, plan.blur[k], blurred);
    hipLaunchKernelGGL(resize_kernel, dim3(grid_for(n_img * hw)), dim3(NT), 0, s, blurred, n_img, H, W, h, w, 0, 1.0f,
                       lvl);
    hipLaunchKernelGGL(poly_v_kernel, dim3(grid_for(n_img * hw)), dim3(NT), 0, s, lvl, n_img, h, w, pc, rv);
    hipLaunchKernelGGL(poly_h_kernel, dim3(grid_for(n_img * hw)), dim3(NT), 0, s, rv, n_img, h, w, pc, R);
    if (cur == nullptr) {
      (void)hipMemsetAsync(fl, 0, pairs * hw * 2 * sizeof(float), s);
    } else {
      hipLaunchKernelGGL(resize_kernel, dim3(grid_for(pairs * hw * 2)), dim3(NT), 0, s, cur, pairs, ph, pw, h, w, 1,
                         (float)(1.0 / pyr_scale), fl);
    }
    hipLaunchKernelGGL(update_matrices_kernel, dim3(grid_for(pairs * hw)), dim3(NT), 0, s, R, frames, pairs, h, w, fl,
                       M);
    for (int it = 0; it < iterations; ++it) {
      hipLaunchKernelGGL(box_v_kernel, dim3(grid_for(pairs * 5 * hw)), dim3(NT), 0, s, M, pairs * 5, h, w, winsize, V);
      hipLaunchKernelGGL(box_h_solve_kernel, dim3(grid_for(pairs * hw)), dim3(NT), 0, s, V, pairs, h, w, winsize, fl);
      if (it < iterations - 1)
        hipLaunchKernelGGL(update_matrices_kernel, dim3(grid_for(pairs * hw)), dim3(NT), 0, s, R, frames, pairs, h, w,
                           fl, M);
    }
    cur = fl;
    ph = h;
    pw = w;
  }
  return vd_launch_status();
}

extern "C" int64_t vd_flow_warp_workspace(int64_t videos, int32_t frames) {
  if (videos <= 0 || frames < 2) return -1;
  return videos * (frames - 1) * WB * 3 * (int64_t)sizeof(double);
}

extern "C" int vd_flow_warp_stats(const void* frames_u8, const float* flow, int64_t videos, int32_t frames, int32_t H,
                                  int32_t W, double* stats, void* workspace, int64_t workspace_bytes,
                                  vd_stream_t stream) {
  VD_CHECK_ARG(frames_u8 && flow && stats && workspace && videos > 0 && frames >= 2 && H >= 2 && W >= 2);
  const int64_t pairs = videos * (frames - 1);
  VD_CHECK_ARG(pairs <= 65535 && workspace_bytes >= pairs * WB * 3 * (int64_t)sizeof(double));
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(warp_stats_kernel, dim3(WB, (unsigned)pairs), dim3(NT), 0, s, (const uint8_t*)frames_u8, flow,
                     frames, H, W, (double*)workspace);
  hipLaunchKernelGGL(warp_stats_finalize, dim3(grid_for(pairs * 3)), dim3(NT), 0, s, (const double*)workspace, pairs,
                     stats);
  return vd_launch_status();
}
