// Support layers needed to run LeNet / CIFAR / AlexNet / GoogLeNet end to end
// (SURVEY.md §2.1 "minimal correct support kernels").  Semantics follow the
// reference layers (file:line cited per kernel); none of these is on the
// fault path, so they are plain coalesced elementwise / per-column kernels.
#include <float.h>
#include <math.h>

#include <stdlib.h>

#include "rram_common.hpp"

namespace rram {
namespace {

// a^b for a > 0 via the native v_log_f32 / v_exp_f32 (powf's special-case
// handling is not needed for LRN scales, which are >= k > 0)
__device__ __forceinline__ float pow_pos(float a, float b) { return exp2f(b * log2f(a)); }
// unsigned division by a runtime constant for in-plane indices (x < 2^31)
struct FastDivI {
  uint32_t d, m, s;
};
static FastDivI make_fastdivi(uint32_t d) {
  FastDivI f{d, 0, 0};
  if (d <= 1) return f;
  uint32_t sh = 0;
  while ((1ull << sh) < d) ++sh;
  f.s = sh;
  f.m = static_cast<uint32_t>(((1ull << 32) * ((1ull << sh) - d)) / d + 1);
  return f;
}
__device__ __forceinline__ uint32_t fdivi(uint32_t x, const FastDivI& f) { return (__umulhi(x, f.m) + x) >> f.s; }

// 32-bit index arithmetic (64-bit division is a long software sequence on
// the VALU); every host wrapper checks that its element count is < 2^31.
#define GRID_LOOP(i, n)                                                                    \
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < static_cast<int>(n); \
       i += gridDim.x * blockDim.x)
#define RRAM_REQUIRE_I32(total, what) \
  RRAM_REQUIRE((int64_t)(total) < 2147483647ll, what ": more than 2^31 elements is not supported")

// relu_layer.cu:9-15 / :35-44
__global__ void k_relu_fwd(const float* __restrict__ x, float* __restrict__ y, int64_t n, float slope) {
  GRID_LOOP(i, n) {
    const float v = x[i];
    y[i] = v > 0.0f ? v : v * slope;
  }
}
__global__ void k_relu_bwd(const float* __restrict__ x, const float* __restrict__ dy,
                           float* __restrict__ dx, int64_t n, float slope) {
  GRID_LOOP(i, n) dx[i] = dy[i] * ((x[i] > 0.0f) + (x[i] <= 0.0f) * slope);
}

// pooling_layer.cu MaxPoolForward / AvePoolForward
// relu != 0: the in-place ReLU that follows (rram_pool_relu_fwd), k_relu_fwd's expression
__device__ __forceinline__ float pool_out(float v, int relu, float slope) {
  return relu ? (v > 0.0f ? v : v * slope) : v;
}
__global__ void k_pool_fwd(const float* __restrict__ x, float* __restrict__ y, int* __restrict__ mask,
                           int num, int C, int H, int W, int PH, int PW, int kh, int kw, int sh,
                           int sw, int ph, int pw, int method, int relu, float slope) {
  const int64_t total = (int64_t)num * C * PH * PW;
  GRID_LOOP(idx, total) {
    const int pwi = idx % PW;
    const int phi = (idx / PW) % PH;
    const int64_t nc = idx / PW / PH;
    const float* xs = x + nc * H * W;
    int hs = phi * sh - ph, ws = pwi * sw - pw;
    if (method == RRAM_POOL_MAX) {
      const int he = min(hs + kh, H), we = min(ws + kw, W);
      hs = max(hs, 0);
      ws = max(ws, 0);
      float mv = -FLT_MAX;
      int mi = -1;
      for (int h = hs; h < he; ++h)
        for (int w = ws; w < we; ++w)
          if (xs[h * W + w] > mv) {
            mi = h * W + w;
            mv = xs[mi];
          }
      y[idx] = pool_out(mv, relu, slope);
      if (mask) mask[idx] = mi;
    } else {
      int he = min(hs + kh, H + ph), we = min(ws + kw, W + pw);
      const int psize = (he - hs) * (we - ws);
      hs = max(hs, 0);
      ws = max(ws, 0);
      he = min(he, H);
      we = min(we, W);
      float s = 0.0f;
      for (int h = hs; h < he; ++h)
        for (int w = ws; w < we; ++w) s += xs[h * W + w];
      y[idx] = pool_out(s / psize, relu, slope);
    }
  }
}

// MAX pooling with a compile-time window (AlexNet/CaffeNet/GoogLeNet 3x3, LeNet
// 2x2): all K*K guarded loads are issued before the compares, same strict-">"
// first-argmax rule and -FLT_MAX start as MaxPoolForward (pooling_layer.cu).
template <int K>
__global__ void __launch_bounds__(256) k_pool_max_fixed(const float* __restrict__ x, float* __restrict__ y,
                                                        int* __restrict__ mask, int num, int C, int H, int W,
                                                        int PH, int PW, int sh, int sw, int ph, int pw,
                                                        int relu, float slope) {
  const int total = num * C * PH * PW;
  GRID_LOOP(idx, total) {
    const int pwi = idx % PW;
    const int phi = (idx / PW) % PH;
    const int nc = idx / PW / PH;
    const float* xs = x + (int64_t)nc * H * W;
    const int hs = phi * sh - ph, ws = pwi * sw - pw;
    float v[K * K];
    bool ok[K * K];
#pragma unroll
    for (int a = 0; a < K; ++a)
#pragma unroll
      for (int b = 0; b < K; ++b) {
        const int h = hs + a, w = ws + b;
        ok[a * K + b] = static_cast<unsigned>(h) < static_cast<unsigned>(H) &&
                        static_cast<unsigned>(w) < static_cast<unsigned>(W);
        v[a * K + b] = ok[a * K + b] ? xs[h * W + w] : 0.0f;
      }
    float mv = -FLT_MAX;
    int mi = -1;
#pragma unroll
    for (int a = 0; a < K; ++a)
#pragma unroll
      for (int b = 0; b < K; ++b)
        if (ok[a * K + b] && v[a * K + b] > mv) {
          mv = v[a * K + b];
          mi = (hs + a) * W + (ws + b);
        }
    y[idx] = pool_out(mv, relu, slope);
    if (mask) mask[idx] = mi;
  }
}

// Pooling of small planes (H*W <= kPlaneMax): a block stages whole (n, c)
// planes - contiguous in NCHW - in LDS, then computes every output of those
// planes from LDS, so each input is read from HBM once and the window re-reads
// stay on-chip.  The staging issues kStageU 16-byte raw buffer loads per
// thread before the first LDS store (any 4-byte alignment; the per-dword range
// check zeroes the tail), so a block keeps ~kStageU KB per wave in flight.
// Outputs are written contiguously.  K = 2, 3: MAX with that square window
// (k_pool_max_fixed's loop); K = 0: any window, MAX or AVE, with k_pool_fwd's
// loops - the same window, summation order, divisor, tie rule and argmax.
constexpr int kPlaneTile = 4096;   // floats: planes per block fill this much LDS
constexpr int kPlaneMax = 16384;   // larger planes (64 KB) take one block each
constexpr int kStageU = 8;
// floor(a / b) for 0 <= a < 2^22, b >= 1 via the float reciprocal: (a + 0.5) / b
// is >= 0.5 / b away from an integer, and the product's relative error
// (<= 2^-23) is smaller than that while a + 0.5 < 4e6.
__device__ __forceinline__ int div_small(int a, float inv_b) {
  return static_cast<int>((static_cast<float>(a) + 0.5f) * inv_b);
}
template <int K>
__global__ void __launch_bounds__(256) k_pool_planes(const float* __restrict__ x, float* __restrict__ y,
                                                     int* __restrict__ mask, int planes, int H, int W, int PH,
                                                     int PW, int kh, int kw, int sh, int sw, int ph, int pw,
                                                     int method, int ppb, float inv_phw, float inv_pw, int relu,
                                                     float slope) {
  extern __shared__ __attribute__((aligned(16))) float tile[];
  const int HW = H * W, PHW = PH * PW;
  const int p0 = blockIdx.x * ppb;
  const int np = min(ppb, planes - p0);
  const int n_in = np * HW;
  const int n4 = (n_in + 3) >> 2;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(x + (int64_t)p0 * HW), 0, n_in * 4, 0x00020000);
  for (int i0 = threadIdx.x; i0 < n4; i0 += 256 * kStageU) {
    float4 r[kStageU];
#pragma unroll
    for (int u = 0; u < kStageU; ++u) {
      const int i = min(i0 + 256 * u, n4);  // i == n4: past the range, loads zeros
      r[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * i, 0, 0));
    }
#pragma unroll
    for (int u = 0; u < kStageU; ++u)
      if (i0 + 256 * u < n4) reinterpret_cast<float4*>(tile)[i0 + 256 * u] = r[u];
  }
  __syncthreads();
  const int n_out = np * PHW;
  float* dst = y + (int64_t)p0 * PHW;
  for (int o = threadIdx.x; o < n_out; o += 256) {
    const int pl = div_small(o, inv_phw), r = o - pl * PHW;
    const int phi = div_small(r, inv_pw), pwi = r - phi * PW;
    int hs = phi * sh - ph, ws = pwi * sw - pw;
    const float* t = tile + pl * HW;
    float mv = -FLT_MAX;
    int mi = -1;
    if constexpr (K > 0) {
#pragma unroll
      for (int a = 0; a < K; ++a)
#pragma unroll
        for (int b = 0; b < K; ++b) {
          const int h = hs + a, w = ws + b;
          const bool ok = static_cast<unsigned>(h) < static_cast<unsigned>(H) &&
                          static_cast<unsigned>(w) < static_cast<unsigned>(W);
          const float v = t[ok ? h * W + w : 0];
          if (ok && v > mv) {
            mv = v;
            mi = h * W + w;
          }
        }
    } else if (method == RRAM_POOL_MAX) {
      const int he = min(hs + kh, H), we = min(ws + kw, W);
      hs = max(hs, 0);
      ws = max(ws, 0);
      for (int h = hs; h < he; ++h)
        for (int w = ws; w < we; ++w)
          if (t[h * W + w] > mv) {
            mi = h * W + w;
            mv = t[mi];
          }
    } else {
      int he = min(hs + kh, H + ph), we = min(ws + kw, W + pw);
      const int psize = (he - hs) * (we - ws);
      hs = max(hs, 0);
      ws = max(ws, 0);
      he = min(he, H);
      we = min(we, W);
      float s = 0.0f;
      for (int h = hs; h < he; ++h)
        for (int w = ws; w < we; ++w) s += t[h * W + w];
      mv = s / psize;
    }
    dst[o] = pool_out(mv, relu, slope);
    if (mask) mask[(int64_t)p0 * PHW + o] = mi;
  }
}

// MAX pooling of small planes with a 3 x 3 window, stride 1, no argmax (the
// TEST-phase pools of GoogLeNet's inception branches).  Planes staged in LDS
// as in k_pool_planes; the window is separable: a work item (plane, output
// column, segment of kSepRows output rows) walks the input rows of its
// segment once, each row's 3-column maximum formed once and kept in a 3-row
// ring, so an output costs one new row maximum (3 LDS reads) instead of 9
// guarded taps.
// The same strict-">" scan from -FLT_MAX as MaxPoolForward (pooling_layer.cu),
// row by row: the first maximum in row-major order wins, so the value (its
// sign of zero included) is the one k_pool_planes picks; taps outside the
// image are skipped (here: -FLT_MAX, which no ">" replaces).
constexpr int kSepRows = 8;
__global__ void __launch_bounds__(256) k_pool_planes_sep3(const float* __restrict__ x, float* __restrict__ y, int planes,
                                                          int H, int W, int PH, int PW, int ph, int pw, int ppb,
                                                          int nseg, float inv_pw, float inv_nseg, int relu,
                                                          float slope) {
  extern __shared__ __attribute__((aligned(16))) float tile[];
  const int HW = H * W, PHW = PH * PW;
  const int p0 = blockIdx.x * ppb;
  const int np = min(ppb, planes - p0);
  const int n_in = np * HW;
  const int n4 = (n_in + 3) >> 2;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(x + (int64_t)p0 * HW), 0, n_in * 4, 0x00020000);
  for (int i0 = threadIdx.x; i0 < n4; i0 += 256 * kStageU) {
    float4 r[kStageU];
#pragma unroll
    for (int u = 0; u < kStageU; ++u) {
      const int i = min(i0 + 256 * u, n4);  // i == n4: past the range, loads zeros
      r[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * i, 0, 0));
    }
#pragma unroll
    for (int u = 0; u < kStageU; ++u)
      if (i0 + 256 * u < n4) reinterpret_cast<float4*>(tile)[i0 + 256 * u] = r[u];
  }
  __syncthreads();
  const int items = np * nseg * PW;
  float* dst = y + (int64_t)p0 * PHW;
  for (int it = threadIdx.x; it < items; it += 256) {
    const int rest = div_small(it, inv_pw), ow = it - rest * PW;
    const int pl = div_small(rest, inv_nseg), sg = rest - pl * nseg;
    const float* t = tile + pl * HW;
    const int c0 = ow - pw;
    const bool ok0 = static_cast<unsigned>(c0) < static_cast<unsigned>(W);
    const bool ok1 = static_cast<unsigned>(c0 + 1) < static_cast<unsigned>(W);
    const bool ok2 = static_cast<unsigned>(c0 + 2) < static_cast<unsigned>(W);
    const int ca = ok0 ? c0 : 0, cb = ok1 ? c0 + 1 : 0, cc = ok2 ? c0 + 2 : 0;
    const int oh0 = sg * kSepRows, nout = min(kSepRows, PH - oh0);
    const int r0 = oh0 - ph;
    auto rowmax = [&](int r) __attribute__((always_inline)) {
      float m = -FLT_MAX;
      if (static_cast<unsigned>(r) < static_cast<unsigned>(H)) {
        const float* tr = t + r * W;
        const float va = tr[ca], vb = tr[cb], vc = tr[cc];
        if (ok0 && va > m) m = va;
        if (ok1 && vb > m) m = vb;
        if (ok2 && vc > m) m = vc;
      }
      return m;
    };
    float q0 = rowmax(r0), q1 = rowmax(r0 + 1);
    float* out = dst + (int64_t)pl * PHW + oh0 * PW + ow;
    for (int o = 0; o < nout; ++o) {
      const float q2 = rowmax(r0 + o + 2);
      float m = q0;  // rows top to bottom: the first row holding the maximum wins
      if (q1 > m) m = q1;
      if (q2 > m) m = q2;
      out[o * PW] = pool_out(m, relu, slope);
      q0 = q1;  // next window: rows r0 + o + 1 .. r0 + o + 3
      q1 = q2;
    }
  }
}

// pooling_layer.cu MaxPoolBackward / AvePoolBackward
// ry != nullptr: times the backward factor of the in-place ReLU whose output
// ry is (rram_pool_relu_bwd; k_relu_bwd's expression)
__global__ void k_pool_bwd(const float* __restrict__ dy, const int* __restrict__ mask,
                           float* __restrict__ dx, int num, int C, int H, int W, int PH, int PW,
                           int kh, int kw, int sh, int sw, int ph, int pw, int method,
                           const float* __restrict__ ry, float slope) {
  const int64_t total = (int64_t)num * C * H * W;
  GRID_LOOP(idx, total) {
    const int w = idx % W;
    const int h = (idx / W) % H;
    const int64_t nc = idx / W / H;
    const float* d = dy + nc * PH * PW;
    float g = 0.0f;
    if (method == RRAM_POOL_MAX) {
      const int* m = mask + nc * PH * PW;
      const int phs = (h + ph < kh) ? 0 : (h + ph - kh) / sh + 1;
      const int phe = min((h + ph) / sh + 1, PH);
      const int pws = (w + pw < kw) ? 0 : (w + pw - kw) / sw + 1;
      const int pwe = min((w + pw) / sw + 1, PW);
      for (int a = phs; a < phe; ++a)
        for (int b = pws; b < pwe; ++b)
          if (m[a * PW + b] == h * W + w) g += d[a * PW + b];
    } else {
      const int hh = h + ph, ww = w + pw;
      const int phs = (hh < kh) ? 0 : (hh - kh) / sh + 1;
      const int phe = min(hh / sh + 1, PH);
      const int pws = (ww < kw) ? 0 : (ww - kw) / sw + 1;
      const int pwe = min(ww / sw + 1, PW);
      for (int a = phs; a < phe; ++a)
        for (int b = pws; b < pwe; ++b) {
          const int hs = a * sh - ph, ws = b * sw - pw;
          const int he = min(hs + kh, H + ph), we = min(ws + kw, W + pw);
          g += d[a * PW + b] / ((he - hs) * (we - ws));
        }
    }
    if (ry != nullptr) g = g * ((ry[idx] > 0.0f) + (ry[idx] <= 0.0f) * slope);
    dx[idx] = g;
  }
}

// lrn_layer.cu LRNFillScale + LRNComputeOutput.  The window sum is evaluated
// directly, the squares added in channel order (lrn_sq_add), not by the
// reference's add-entering / subtract-leaving slide: every scale is then a
// function of its own SIZE inputs only (no cancellation carried along the
// channel walk), so a kernel may start the walk at any channel (the chunked
// LRN + pool fusion, fused.hip) and still produce these bits.
__global__ void k_lrn_fwd(const float* __restrict__ x, float* __restrict__ y, float* __restrict__ scale,
                          int num, int C, int HW, int size, float alpha_over_size, float beta,
                          float k) {
  const int64_t total = (int64_t)num * C * HW;
  const int pre = (size - 1) / 2;
  GRID_LOOP(idx, total) {
    const int s = idx % HW;
    const int c = (idx / HW) % C;
    const int64_t n = idx / HW / C;
    const float* xc = x + n * C * HW + s;
    float acc = 0.0f;
    const int c0 = max(c - pre, 0), c1 = min(c - pre + size, C);
    for (int j = c0; j < c1; ++j) acc = lrn_sq_add(acc, xc[(int64_t)j * HW]);
    const float sc = lrn_scale(acc, alpha_over_size, k);
    if (scale) scale[idx] = sc;
    y[idx] = lrn_out(x[idx], sc, beta);
  }
}

// The same arithmetic for SIZE 3 / 5: one thread per (n, h, w) column walks
// the channels with the window in registers, so x is read once and y written
// once.
template <int SIZE>
__global__ void __launch_bounds__(256) k_lrn_fwd_slide(const float* __restrict__ x, float* __restrict__ y,
                                                       float* __restrict__ scale, int num, int C, int HW,
                                                       float alpha_over_size, float beta, float k) {
  constexpr int PRE = (SIZE - 1) / 2, POST = SIZE - PRE - 1;
  constexpr int D = 8;  // channels prefetched per step: D independent loads in flight per thread
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // one (image, pixel) column per thread
  if (idx >= num * HW) return;
  const int s = idx % HW;
  const int64_t base = (int64_t)(idx / HW) * C * HW + s;
  const float* xc = x + base;
  float* yc = y + base;
  // ring of the SIZE channels centred on c, plus D channels read ahead
  float win[SIZE + D];
#pragma unroll
  for (int j = 0; j < SIZE; ++j) {
    const int cc = j - PRE;
    win[j] = (cc >= 0 && cc < C) ? xc[(int64_t)cc * HW] : 0.0f;
  }
  for (int c0 = 0; c0 < C; c0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int cn = c0 + d + POST + 1;
      win[SIZE + d] = cn < C ? xc[(int64_t)cn * HW] : 0.0f;
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int c = c0 + d;
      if (c < C) {
        float acc = 0.0f;  // channels c - PRE .. c + POST in order (zeros outside [0, C) add nothing)
#pragma unroll
        for (int j = 0; j < SIZE; ++j) acc = lrn_sq_add(acc, win[d + j]);
        const float sc = lrn_scale(acc, alpha_over_size, k);
        if (scale) scale[base + (int64_t)c * HW] = sc;
        yc[(int64_t)c * HW] = lrn_out(win[d + PRE], sc, beta);
      }
    }
#pragma unroll
    for (int j = 0; j < SIZE; ++j) win[j] = win[j + D];
  }
}

// lrn_layer.cu LRNComputeDiff
__global__ void k_lrn_bwd(const float* __restrict__ x, const float* __restrict__ y,
                          const float* __restrict__ scale, const float* __restrict__ dy,
                          float* __restrict__ dx, int num, int C, int HW, int size,
                          float cache_ratio, float beta) {
  const int64_t total = (int64_t)num * C * HW;
  const int pre = (size - 1) / 2;
  const int post = size - pre - 1;
  GRID_LOOP(idx, total) {
    const int s = idx % HW;
    const int c = (idx / HW) % C;
    const int64_t base = (idx / HW / C) * C * HW + s;
    // channels j whose window contains c: j in [c - post, c + pre]
    float ratio = 0.0f;
    const int j0 = max(c - post, 0), j1 = min(c + pre + 1, C);
    for (int j = j0; j < j1; ++j) {
      const int64_t o = base + (int64_t)j * HW;
      ratio += dy[o] * y[o] / scale[o];
    }
    dx[idx] = dy[idx] * pow_pos(scale[idx], -beta) - cache_ratio * x[idx] * ratio;
  }
}

// LRN WITHIN_CHANNEL (lrn_layer.cpp WithinChannelForward: square -> AVE pool
// (k = size, pad = (size-1)/2, stride 1, Caffe's pool_size rule) -> (1 + alpha*.)^-beta -> product)
__device__ __forceinline__ int within_psize(int p, int pre, int size, int L) {
  const int s = p - pre;
  const int e = min(s + size, L + pre);
  return e - s;
}
__global__ void k_lrn_within_fwd(const float* __restrict__ x, float* __restrict__ y, float* __restrict__ scale,
                                 int64_t planes, int H, int W, int size, float alpha, float beta) {
  const int64_t total = planes * H * W;
  const int pre = (size - 1) / 2;
  GRID_LOOP(idx, total) {
    const int w = idx % W;
    const int h = (idx / W) % H;
    const float* xp = x + (idx / W / H) * H * W;
    const int hs = max(h - pre, 0), he = min(h - pre + size, H);
    const int ws = max(w - pre, 0), we = min(w - pre + size, W);
    float s = 0.0f;
    for (int a = hs; a < he; ++a)
      for (int b = ws; b < we; ++b) {
        const float v = xp[a * W + b];
        s += v * v;
      }
    const float n = static_cast<float>(within_psize(h, pre, size, H) * within_psize(w, pre, size, W));
    const float sc = 1.0f + alpha * (s / n);
    if (scale) scale[idx] = sc;
    y[idx] = x[idx] * pow_pos(sc, -beta);
  }
}
// relu != 0: times the backward factor of the in-place ReLU whose output x is
// (rram_lrn_within_relu_bwd; k_relu_bwd's expression)
__global__ void k_lrn_within_bwd(const float* __restrict__ x, const float* __restrict__ scale,
                                 const float* __restrict__ dy, float* __restrict__ dx, int64_t planes, int H,
                                 int W, int size, float alpha, float beta, int relu, float slope) {
  const int64_t total = planes * H * W;
  const int pre = (size - 1) / 2;
  GRID_LOOP(idx, total) {
    const int w = idx % W;
    const int h = (idx / W) % H;
    const int64_t base = (idx / W / H) * H * W;
    // windows p containing r: p - pre <= r <= p - pre + size - 1
    const int ps = max(h + pre - size + 1, 0), pe = min(h + pre, H - 1);
    const int qs = max(w + pre - size + 1, 0), qe = min(w + pre, W - 1);
    float acc = 0.0f;
    for (int a = ps; a <= pe; ++a)
      for (int b = qs; b <= qe; ++b) {
        const int64_t o = base + a * W + b;
        const float n = static_cast<float>(within_psize(a, pre, size, H) * within_psize(b, pre, size, W));
        acc += dy[o] * x[o] * pow_pos(scale[o], -beta - 1.0f) / n;
      }
    float g = dy[idx] * pow_pos(scale[idx], -beta) - 2.0f * alpha * beta * x[idx] * acc;
    if (relu) g = g * ((x[idx] > 0.0f) + (x[idx] <= 0.0f) * slope);
    dx[idx] = g;
  }
}

// k_lrn_within_bwd with one plane per block (H * W <= kBwdPlaneMax): every
// element's window term dy x scale^(-beta-1) / n is formed once into LDS (the
// per-element kernel formed it once per window holding the element: 9x the
// pow for local_size 3) and summed from there in the same (a, b) order, so
// each dx is the same bits.
constexpr int kBwdPlaneMax = 4096;
__global__ void __launch_bounds__(256) k_lrn_within_bwd_plane(const float* __restrict__ x,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ dy, float* __restrict__ dx,
                                                              int H, int W, FastDivI wdiv, int size, float alpha,
                                                              float beta, int relu, float slope) {
  __shared__ float tl[kBwdPlaneMax];
  const int HW = H * W, pre = (size - 1) / 2;
  const int64_t base = (int64_t)blockIdx.x * HW;
  for (int e = threadIdx.x; e < HW; e += blockDim.x) {
    const int a = static_cast<int>(fdivi(static_cast<uint32_t>(e), wdiv)), b = e - a * W;
    const float n = static_cast<float>(within_psize(a, pre, size, H) * within_psize(b, pre, size, W));
    tl[e] = dy[base + e] * x[base + e] * pow_pos(scale[base + e], -beta - 1.0f) / n;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < HW; e += blockDim.x) {
    const int h = static_cast<int>(fdivi(static_cast<uint32_t>(e), wdiv)), w = e - h * W;
    const int ps = max(h + pre - size + 1, 0), pe = min(h + pre, H - 1);
    const int qs = max(w + pre - size + 1, 0), qe = min(w + pre, W - 1);
    float acc = 0.0f;
    for (int a = ps; a <= pe; ++a)
      for (int b = qs; b <= qe; ++b) acc += tl[a * W + b];
    const int64_t idx = base + e;
    float g = dy[idx] * pow_pos(scale[idx], -beta) - 2.0f * alpha * beta * x[idx] * acc;
    if (relu) g = g * ((x[idx] > 0.0f) + (x[idx] <= 0.0f) * slope);
    dx[idx] = g;
  }
}

// k_pool_bwd (MAX, mask) with one plane per block (H * W <= kBwdPlaneMax,
// PH * PW <= 1024): the pooled gradients and argmax indices of the plane in
// LDS, each input element gathering from them in k_pool_bwd's (a, b) order
// (same bits), with no 64-bit index arithmetic
__global__ void __launch_bounds__(256) k_pool_bwd_plane(const float* __restrict__ dy, const int* __restrict__ mask,
                                                        float* __restrict__ dx, int H, int W, int PH, int PW,
                                                        FastDivI wdiv, int kh, int kw, int sh, int sw, int ph,
                                                        int pw, const float* __restrict__ ry, float slope) {
  __shared__ float dl[1024];
  __shared__ int ml[1024];
  const int HW = H * W, PHW = PH * PW;
  const int64_t pb = (int64_t)blockIdx.x * PHW, xb = (int64_t)blockIdx.x * HW;
  for (int e = threadIdx.x; e < PHW; e += blockDim.x) {
    dl[e] = dy[pb + e];
    ml[e] = mask[pb + e];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < HW; e += blockDim.x) {
    const int h = static_cast<int>(fdivi(static_cast<uint32_t>(e), wdiv)), w = e - h * W;
    const int phs = (h + ph < kh) ? 0 : (h + ph - kh) / sh + 1;
    const int phe = min((h + ph) / sh + 1, PH);
    const int pws = (w + pw < kw) ? 0 : (w + pw - kw) / sw + 1;
    const int pwe = min((w + pw) / sw + 1, PW);
    float g = 0.0f;
    for (int a = phs; a < phe; ++a)
      for (int b = pws; b < pwe; ++b)
        if (ml[a * PW + b] == e) g += dl[a * PW + b];
    if (ry != nullptr) g = g * ((ry[xb + e] > 0.0f) + (ry[xb + e] <= 0.0f) * slope);
    dx[xb + e] = g;
  }
}

// softmax_layer.cu: one wave per (outer, inner) column
__global__ void __launch_bounds__(256) k_softmax(const float* __restrict__ x, float* __restrict__ y,
                                                 int outer, int C, int inner) {
  const int lane = threadIdx.x & 63;
  const int64_t cols = (int64_t)outer * inner;
  for (int64_t col = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; col < cols;
       col += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    const int64_t o = col / inner, q = col - o * inner;
    const float* xs = x + o * C * inner + q;
    float* ys = y + o * C * inner + q;
    float m = -FLT_MAX;
    for (int c = lane; c < C; c += 64) m = fmaxf(m, xs[(int64_t)c * inner]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    float s = 0.0f;
    for (int c = lane; c < C; c += 64) {
      const float e = expf(xs[(int64_t)c * inner] - m);
      ys[(int64_t)c * inner] = e;
      s += e;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    for (int c = lane; c < C; c += 64) ys[(int64_t)c * inner] /= s;
  }
}

// k_softmax with the column held in registers (C <= 64 R): one load pass and
// one store pass instead of three loads; the same per-lane partial order and
// shuffle trees, so the results are k_softmax's bit for bit.
template <int R>
__global__ void __launch_bounds__(256) k_softmax_reg(const float* __restrict__ x, float* __restrict__ y, int outer,
                                                     int C, int inner) {
  const int lane = threadIdx.x & 63;
  const int64_t cols = (int64_t)outer * inner;
  for (int64_t col = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; col < cols;
       col += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    const int64_t o = col / inner, q = col - o * inner;
    const float* xs = x + o * C * inner + q;
    float* ys = y + o * C * inner + q;
    float v[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int c = lane + 64 * i;
      v[i] = c < C ? xs[(int64_t)c * inner] : -FLT_MAX;
    }
    float m = -FLT_MAX;
#pragma unroll
    for (int i = 0; i < R; ++i)
      if (lane + 64 * i < C) m = fmaxf(m, v[i]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < R; ++i)
      if (lane + 64 * i < C) {
        v[i] = expf(v[i] - m);
        s += v[i];
      }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
#pragma unroll
    for (int i = 0; i < R; ++i)
      if (lane + 64 * i < C) ys[(int64_t)(lane + 64 * i) * inner] = v[i] / s;
  }
}

// softmax_loss_layer.cpp:95-112 (single block, deterministic)
// acc_sum / acc_row (nullable): the MonteCarlo statistics of this output
// (k_mc_accumulate's sum += v, row = v) written by the thread that stores v
__global__ void __launch_bounds__(1024) k_softmax_loss_fwd(const float* __restrict__ prob,
                                                           const float* __restrict__ label,
                                                           float* out, int outer, int C, int inner,
                                                           int ignore, float* acc_sum, float* acc_row) {
  __shared__ float sl[16], sc[16];
  float loss = 0.0f, cnt = 0.0f;
  const int64_t cols = (int64_t)outer * inner;
  for (int64_t col = threadIdx.x; col < cols; col += blockDim.x) {
    const int64_t o = col / inner, q = col - o * inner;
    const int lv = static_cast<int>(label[col]);
    if (ignore >= 0 && lv == ignore) continue;
    loss -= logf(fmaxf(prob[(o * C + lv) * inner + q], FLT_MIN));
    cnt += 1.0f;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    loss += __shfl_xor(loss, off, 64);
    cnt += __shfl_xor(cnt, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    sl[threadIdx.x >> 6] = loss;
    sc[threadIdx.x >> 6] = cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float L = 0.0f, N = 0.0f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
      L += sl[i];
      N += sc[i];
    }
    const float v = L / fmaxf(N, 1.0f);
    out[0] = v;
    if (acc_sum) *acc_sum += v;
    if (acc_row) *acc_row = v;
  }
}

// k_softmax_loss_fwd + k_softmax_loss_bwd in one block (TRAIN phase, small
// heads): the loss in k_softmax_loss_fwd's order, then dx with
// k_softmax_loss_bwd's expression; scale = scale_all (host: loss_weight /
// (outer * inner)) without an ignore label, else loss_weight / max(#valid, 1)
// as rram_softmax_loss_bwd forms it from k_count_valid's exact count
__global__ void __launch_bounds__(1024) k_softmax_loss_fwd_bwd(const float* __restrict__ prob,
                                                               const float* __restrict__ label, float* out,
                                                               float* __restrict__ dx, int outer, int C, int inner,
                                                               int ignore, float loss_weight, float scale_all) {
  __shared__ float sl[16], sc[16], sscale;
  float loss = 0.0f, cnt = 0.0f;
  const int64_t cols = (int64_t)outer * inner;
  for (int64_t col = threadIdx.x; col < cols; col += blockDim.x) {
    const int64_t o = col / inner, q = col - o * inner;
    const int lv = static_cast<int>(label[col]);
    if (ignore >= 0 && lv == ignore) continue;
    loss -= logf(fmaxf(prob[(o * C + lv) * inner + q], FLT_MIN));
    cnt += 1.0f;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    loss += __shfl_xor(loss, off, 64);
    cnt += __shfl_xor(cnt, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    sl[threadIdx.x >> 6] = loss;
    sc[threadIdx.x >> 6] = cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float L = 0.0f, N = 0.0f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
      L += sl[i];
      N += sc[i];
    }
    out[0] = L / fmaxf(N, 1.0f);
    sscale = ignore >= 0 ? loss_weight / fmaxf(N, 1.0f) : scale_all;
  }
  __syncthreads();
  const float scale_valid = sscale;
  const int64_t total = cols * C;
  for (int64_t idx = threadIdx.x; idx < total; idx += blockDim.x) {
    const int64_t q = idx % inner;
    const int c = static_cast<int>((idx / inner) % C);
    const int64_t o = idx / inner / C;
    const int lv = static_cast<int>(label[o * inner + q]);
    if (ignore >= 0 && lv == ignore) {
      dx[idx] = 0.0f;
    } else {
      dx[idx] = (prob[idx] - (c == lv ? 1.0f : 0.0f)) * scale_valid;
    }
  }
}

__global__ void k_softmax_loss_bwd(const float* __restrict__ prob, const float* __restrict__ label,
                                   float* __restrict__ dx, int outer, int C, int inner, int ignore,
                                   float scale_valid) {
  const int64_t total = (int64_t)outer * C * inner;
  GRID_LOOP(idx, total) {
    const int64_t q = idx % inner;
    const int c = static_cast<int>((idx / inner) % C);
    const int64_t o = idx / inner / C;
    const int lv = static_cast<int>(label[o * inner + q]);
    if (ignore >= 0 && lv == ignore) {
      dx[idx] = 0.0f;
    } else {
      dx[idx] = (prob[idx] - (c == lv ? 1.0f : 0.0f)) * scale_valid;
    }
  }
}

constexpr int kLossFusedMax = 65536;  // rram_softmax_loss_fwd_bwd: one block writes every dx
__global__ void k_count_valid(const float* __restrict__ label, int64_t n, int ignore, float* out) {
  __shared__ float part[16];
  float c = 0.0f;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x)
    c += (ignore >= 0 && static_cast<int>(label[i]) == ignore) ? 0.0f : 1.0f;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.0f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += part[i];
    out[0] = s;
  }
}

// accuracy_layer.cpp:48-90 for one (outer, inner) column xs (stride inner),
// lanes over classes: hit = the label's (value, index) pair is within the
// top_k of the descending pair order, cnt = the label is not ignored.  For
// C <= 1024 the class values are loaded 16 per lane before the label (a
// strided loop waited one memory latency per 64 classes, and the label's own
// value one more behind the label: 10 us for a 256 x 1000 head) and the
// label's value is taken from the lane holding it; integer counts, so the
// result is the loop's whatever the order.
__device__ __forceinline__ void label_hit(const float* __restrict__ xs, int64_t inner, int C,
                                          const float* __restrict__ lab, int ignore, int top_k, int lane, int& hit,
                                          int& cnt) {
  constexpr int R = 16;
  int rank = 0;
  if (C <= 64 * R) {
    float u[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int c = lane + 64 * i;
      u[i] = c < C ? xs[(int64_t)c * inner] : 0.0f;
    }
    const int lv = static_cast<int>(*lab);
    if (ignore >= 0 && lv == ignore) return;
    float mine = 0.0f;  // lv is wave-uniform
#pragma unroll
    for (int i = 0; i < R; ++i)
      if (i == (lv >> 6)) mine = u[i];
    const float v = (lv >= 0 && lv < C) ? __shfl(mine, lv & 63, 64) : xs[(int64_t)lv * inner];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int c = lane + 64 * i;
      rank += c < C && ((u[i] > v) || (u[i] == v && c > lv));
    }
  } else {
    const int lv = static_cast<int>(*lab);
    if (ignore >= 0 && lv == ignore) return;
    const float v = xs[(int64_t)lv * inner];
    for (int c = lane; c < C; c += 64) {
      const float u = xs[(int64_t)c * inner];
      rank += (u > v) || (u == v && c > lv);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) rank += __shfl_xor(rank, off, 64);
  hit = rank < top_k;
  cnt = 1;
}

// accuracy_layer.cpp:48-90: label counted correct when its (value, index)
// pair is within the top_k of the descending pair order.  One wave per
// (outer, inner) column (lanes over classes), many blocks; the per-block
// counts are integers, so float atomics on them are exact and order-independent.
__global__ void __launch_bounds__(256) k_accuracy(const float* __restrict__ x, const float* __restrict__ label,
                                                  float* correct, float* count, int outer, int C, int inner,
                                                  int top_k, int ignore) {
  __shared__ int sa[4], sc[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t cols = (int64_t)outer * inner;
  const int64_t col = (int64_t)blockIdx.x * 4 + wave;
  int hit = 0, cnt = 0;
  if (col < cols) {
    const int64_t o = col / inner, q = col - o * inner;
    label_hit(x + o * C * inner + q, inner, C, label + col, ignore, top_k, lane, hit, cnt);
  }
  if (lane == 0) {
    sa[wave] = hit;
    sc[wave] = cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int A = sa[0] + sa[1] + sa[2] + sa[3], N = sc[0] + sc[1] + sc[2] + sc[3];
    if (A) atomicAdd(correct, static_cast<float>(A));
    if (N) atomicAdd(count, static_cast<float>(N));
  }
}
// Single-launch form for the large heads (AlexNet / GoogLeNet: 256 x 1000):
// k_accuracy's per-block counts go to a per-block slot instead of atomics on
// zeroed outputs; the last block to finish (a device-scope ticket) sums the
// slots in block order and writes correct / count / ratio, then re-arms the
// ticket — no memsets, no second launch.  Launches on one stream are ordered;
// the slots are a single per-device set, so concurrent accuracy launches on
// different streams are not supported (the host runs them on its one stream).
constexpr int kAccFusedBlocks = 4096;
__device__ int g_acc_part[2 * kAccFusedBlocks];
__device__ unsigned g_acc_ticket;
__global__ void __launch_bounds__(256) k_accuracy_fused(const float* __restrict__ x, const float* __restrict__ label,
                                                        float* correct, float* count, float* ratio, int outer, int C,
                                                        int inner, int top_k, int ignore, float* acc_sum,
                                                        float* acc_row) {
  __shared__ int sa[4], sc[4];
  __shared__ bool last;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t cols = (int64_t)outer * inner;
  const int64_t col = (int64_t)blockIdx.x * 4 + wave;
  int hit = 0, cnt = 0;
  if (col < cols) {
    const int64_t o = col / inner, q = col - o * inner;
    label_hit(x + o * C * inner + q, inner, C, label + col, ignore, top_k, lane, hit, cnt);
  }
  if (lane == 0) {
    sa[wave] = hit;
    sc[wave] = cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    g_acc_part[2 * blockIdx.x] = sa[0] + sa[1] + sa[2] + sa[3];
    g_acc_part[2 * blockIdx.x + 1] = sc[0] + sc[1] + sc[2] + sc[3];
    __threadfence();
    last = atomicAdd(&g_acc_ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  // integer sums: exact in any order (< 2^24, host check), written as floats;
  // the slots are read by all 256 threads at once (one memory latency, not
  // one per block) and reduced through the waves
  int A = 0, N = 0;
  for (unsigned b = threadIdx.x; b < gridDim.x; b += 256) {
    A += __hip_atomic_load(&g_acc_part[2 * b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    N += __hip_atomic_load(&g_acc_part[2 * b + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    A += __shfl_xor(A, off, 64);
    N += __shfl_xor(N, off, 64);
  }
  __syncthreads();  // every wave is past its reads of sa / sc
  if (lane == 0) {
    sa[wave] = A;
    sc[wave] = N;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    A = sa[0] + sa[1] + sa[2] + sa[3];
    N = sc[0] + sc[1] + sc[2] + sc[3];
    *correct = static_cast<float>(A);
    *count = static_cast<float>(N);
    const float v = static_cast<float>(A) / static_cast<float>(N > 0 ? N : 1);
    if (ratio) *ratio = v;
    if (acc_sum) *acc_sum += v;
    if (acc_row) *acc_row = v;
    g_acc_ticket = 0u;
  }
}
// Single-launch form for small heads (columns x classes <= kAccSmall, classes
// <= 64: the configs' TEST batches of CIFAR / LeNet): one block, a thread per
// column looping over the classes (independent loads, so one memory latency),
// block reduction, then correct / count / ratio written directly — no memsets,
// no atomics, no second launch.
constexpr int kAccSmall = 1 << 16;
__global__ void __launch_bounds__(1024) k_accuracy_small(const float* __restrict__ x, const float* __restrict__ label,
                                                         float* correct, float* count, float* ratio, int outer, int C,
                                                         int inner, int top_k, int ignore, float* acc_sum, float* acc_row) {
  __shared__ int sa[16], sc[16];
  const int cols = outer * inner;
  int hits = 0, cnt = 0;
  for (int col = threadIdx.x; col < cols; col += 1024) {
    const int o = col / inner, q = col - o * inner;
    const int lv = static_cast<int>(label[col]);
    if (ignore >= 0 && lv == ignore) continue;
    const float* xs = x + (int64_t)o * C * inner + q;
    const float v = xs[(int64_t)lv * inner];
    int rank = 0;  // #classes ahead of the label in Caffe's (value, index) descending order
    for (int c = 0; c < C; ++c) {
      const float u = xs[(int64_t)c * inner];
      rank += (u > v) || (u == v && c > lv);
    }
    hits += rank < top_k;
    cnt += 1;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    hits += __shfl_xor(hits, off, 64);
    cnt += __shfl_xor(cnt, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    sa[threadIdx.x >> 6] = hits;
    sc[threadIdx.x >> 6] = cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int A = 0, N = 0;
    for (int w = 0; w < 16; ++w) {
      A += sa[w];
      N += sc[w];
    }
    correct[0] = static_cast<float>(A);
    count[0] = static_cast<float>(N);
    const float v = static_cast<float>(A) / fmaxf(static_cast<float>(N), 1.0f);
    if (ratio) ratio[0] = v;
    if (acc_sum) *acc_sum += v;
    if (acc_row) *acc_row = v;
  }
}

__global__ void k_accuracy_ratio(const float* correct, const float* count, float* ratio, float* acc_sum,
                                 float* acc_row) {
  const float v = correct[0] / fmaxf(count[0], 1.0f);
  ratio[0] = v;
  if (acc_sum) *acc_sum += v;
  if (acc_row) *acc_row = v;
}

// concat_layer.cu Concat kernel (axis 1)
__global__ void k_concat(const float* __restrict__ src, float* __restrict__ dst, int num, int sci,
                         int dci, int off, int backward) {
  const int64_t total = (int64_t)num * sci;
  GRID_LOOP(idx, total) {
    const int64_t n = idx / sci, j = idx - n * sci;
    const int64_t d = n * dci + off + j;
    if (backward) const_cast<float*>(src)[idx] = dst[d];
    else dst[d] = src[idx];
  }
}

// euclidean_loss_layer.cu:9-20: diff = a - b; loss = dot(diff, diff) / num / 2
// (one block: loss layers see one blob, the summation order is fixed)
__global__ void __launch_bounds__(1024) k_euclidean_fwd(const float* __restrict__ a, const float* __restrict__ b,
                                                      float* __restrict__ diff, float* __restrict__ loss,
                                                      int64_t n, int num) {
  __shared__ float part[16];
  float acc = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const float d = a[i] - b[i];
    diff[i] = d;
    acc += d * d;
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += part[w];
    loss[0] = t / static_cast<float>(num) / 2.0f;
  }
}

__global__ void k_i32_to_f32(const int* __restrict__ x, float* __restrict__ y, int64_t n) {
  GRID_LOOP(i, n) y[i] = static_cast<float>(x[i]);
}

// euclidean_loss_layer.cu:23-38: dx = alpha * diff (caffe_gpu_axpby with beta 0)
__global__ void k_scale_copy(const float* __restrict__ x, float* __restrict__ y, int64_t n, float alpha) {
  GRID_LOOP(i, n) y[i] = alpha * x[i];
}

}  // namespace
}  // namespace rram

namespace rram {
namespace {
int rram_lrn_within_relu_bwd_core(const float* x, const float* scale, const float* dy, float* dx, int num, int C,
                                  int H, int W, int size, float alpha, float beta, int relu, float slope,
                                  rram_stream_t s);
}  // namespace
}  // namespace rram

using namespace rram;

extern "C" {

int rram_relu_fwd(const float* x, float* y, int64_t n, float slope, rram_stream_t s) {
  RRAM_REQUIRE(n >= 0, "relu: n < 0");
  RRAM_REQUIRE_I32(n, "relu");
  if (n == 0) return RRAM_OK;
  RRAM_REQUIRE(x && y, "relu: NULL");
  hipLaunchKernelGGL(k_relu_fwd, dim3(stream_blocks(n)), dim3(kThreads), 0, as_stream(s), x, y, n, slope);
  return launch_status("relu_fwd");
}
int rram_relu_bwd(const float* x, const float* dy, float* dx, int64_t n, float slope, rram_stream_t s) {
  RRAM_REQUIRE(n >= 0, "relu: n < 0");
  RRAM_REQUIRE_I32(n, "relu");
  if (n == 0) return RRAM_OK;
  RRAM_REQUIRE(x && dy && dx, "relu: NULL");
  hipLaunchKernelGGL(k_relu_bwd, dim3(stream_blocks(n)), dim3(kThreads), 0, as_stream(s), x, dy, dx, n, slope);
  return launch_status("relu_bwd");
}

}  // extern "C"
namespace rram {
namespace {
int pool_fwd_core(const float* x, float* y, int* mask, int num, int C, int H, int W, int PH, int PW, int kh, int kw,
                  int sh, int sw, int ph, int pw, int method, int relu, float slope, hipStream_t s) {
  RRAM_REQUIRE(num >= 0 && C > 0 && H > 0 && W > 0 && PH > 0 && PW > 0 && kh > 0 && kw > 0 &&
                   sh > 0 && sw > 0 && ph >= 0 && pw >= 0,
               "pool_fwd: bad geometry");
  RRAM_REQUIRE(method == RRAM_POOL_MAX || method == RRAM_POOL_AVE, "pool_fwd: bad method");
  const int64_t total = (int64_t)num * C * PH * PW;
  RRAM_REQUIRE_I32(total, "layer kernel");
  if (total == 0) return RRAM_OK;
  RRAM_REQUIRE(x && y, "pool_fwd: NULL");
  const int planes = num * C;
  if (H * W <= kPlaneMax) {
    // planes per block: fill the LDS tile, but keep >= 2048 blocks when possible
    int ppb = H * W <= kPlaneTile ? kPlaneTile / (H * W) : 1;
    while (ppb > 1 && (planes + ppb - 1) / ppb < 2048) --ppb;
    const dim3 grid(static_cast<unsigned>((planes + ppb - 1) / ppb));
    const size_t lds = (static_cast<size_t>(ppb) * H * W + 3) / 4 * 16;
    const float inv_phw = 1.0f / static_cast<float>(PH * PW), inv_pw = 1.0f / static_cast<float>(PW);
    if (mask == nullptr && method == RRAM_POOL_MAX && kh == 3 && kw == 3 && sh == 1 && sw == 1 &&
        H * W <= kPlaneTile) {
      // separable 3 x 3 / 1 window (no argmax to record): k_pool_planes_sep3.
      // GoogLeNet b256 (profiles/r06_ab_pool_sep3.txt): the nine inception
      // pools 554 -> 391 us per map; its stride-2 form (two new row maxima
      // per output) ran slower than k_pool_planes on pool1 / pool3 / pool4
      const int nseg = (PH + kSepRows - 1) / kSepRows;
      hipLaunchKernelGGL(k_pool_planes_sep3, grid, dim3(kThreads), lds, s, x, y, planes, H, W, PH, PW, ph, pw, ppb,
                         nseg, 1.0f / static_cast<float>(PW), 1.0f / static_cast<float>(nseg), relu, slope);
      return launch_status("pool_fwd");
    }
    const int k = method == RRAM_POOL_MAX && kh == kw && (kh == 3 || kh == 2) ? kh : 0;
    auto kern = k == 3 ? k_pool_planes<3> : k == 2 ? k_pool_planes<2> : k_pool_planes<0>;
    hipLaunchKernelGGL(kern, grid, dim3(kThreads), lds, s, x, y, mask, planes, H, W, PH, PW, kh, kw, sh, sw, ph, pw,
                       method, ppb, inv_phw, inv_pw, relu, slope);
  } else if (method == RRAM_POOL_MAX && kh == kw && kh == 3)
    hipLaunchKernelGGL(k_pool_max_fixed<3>, dim3(stream_blocks(total)), dim3(kThreads), 0, s, x, y, mask, num, C, H,
                       W, PH, PW, sh, sw, ph, pw, relu, slope);
  else if (method == RRAM_POOL_MAX && kh == kw && kh == 2)
    hipLaunchKernelGGL(k_pool_max_fixed<2>, dim3(stream_blocks(total)), dim3(kThreads), 0, s, x, y, mask, num, C, H,
                       W, PH, PW, sh, sw, ph, pw, relu, slope);
  else
    hipLaunchKernelGGL(k_pool_fwd, dim3(stream_blocks(total)), dim3(kThreads), 0, s, x, y, mask, num, C, H, W, PH,
                       PW, kh, kw, sh, sw, ph, pw, method, relu, slope);
  return launch_status("pool_fwd");
}
}  // namespace
}  // namespace rram

extern "C" {

int rram_pool_fwd(const float* x, float* y, int* mask, int num, int C, int H, int W, int PH, int PW,
                  int kh, int kw, int sh, int sw, int ph, int pw, int method, rram_stream_t s) {
  return pool_fwd_core(x, y, mask, num, C, H, W, PH, PW, kh, kw, sh, sw, ph, pw, method, 0, 0.0f, as_stream(s));
}
int rram_pool_relu_fwd(const float* x, float* y, int* mask, int num, int C, int H, int W, int PH, int PW, int kh,
                       int kw, int sh, int sw, int ph, int pw, int method, float relu_slope, rram_stream_t s) {
  return pool_fwd_core(x, y, mask, num, C, H, W, PH, PW, kh, kw, sh, sw, ph, pw, method, 1, relu_slope,
                       as_stream(s));
}
int rram_pool_bwd(const float* dy, const int* mask, float* dx, int num, int C, int H, int W, int PH,
                  int PW, int kh, int kw, int sh, int sw, int ph, int pw, int method, rram_stream_t s) {
  return rram_pool_relu_bwd(dy, mask, dx, num, C, H, W, PH, PW, kh, kw, sh, sw, ph, pw, method, nullptr, 0.0f, s);
}
int rram_pool_relu_bwd(const float* dy, const int* mask, float* dx, int num, int C, int H, int W, int PH,
                       int PW, int kh, int kw, int sh, int sw, int ph, int pw, int method, const float* relu_y,
                       float relu_slope, rram_stream_t s) {
  RRAM_REQUIRE(num >= 0 && C > 0 && H > 0 && W > 0 && PH > 0 && PW > 0 && sh > 0 && sw > 0,
               "pool_bwd: bad geometry");
  RRAM_REQUIRE(method != RRAM_POOL_MAX || mask != nullptr, "pool_bwd: MAX needs mask");
  const int64_t total = (int64_t)num * C * H * W;
  RRAM_REQUIRE_I32(total, "layer kernel");
  if (total == 0) return RRAM_OK;
  RRAM_REQUIRE(dy && dx, "pool_bwd: NULL");
  // plane path: one 256-thread block per (n, c) plane; the grid's work-item
  // count (num * C * 256) must stay a 32-bit value, else the grid-stride form
  if (method == RRAM_POOL_MAX && H * W <= kBwdPlaneMax && PH * PW <= 1024 && (int64_t)num * C <= (1ll << 24)) {
    hipLaunchKernelGGL(k_pool_bwd_plane, dim3(static_cast<unsigned>(num * C)), dim3(256), 0, as_stream(s), dy, mask,
                       dx, H, W, PH, PW, make_fastdivi(W), kh, kw, sh, sw, ph, pw, relu_y, relu_slope);
    return launch_status("pool_bwd");
  }
  hipLaunchKernelGGL(k_pool_bwd, dim3(stream_blocks(total)), dim3(kThreads), 0, as_stream(s), dy,
                     mask, dx, num, C, H, W, PH, PW, kh, kw, sh, sw, ph, pw, method, relu_y, relu_slope);
  return launch_status("pool_bwd");
}

int rram_lrn_fwd(const float* x, float* y, float* scale, int num, int C, int H, int W, int size,
                 float alpha, float beta, float k, rram_stream_t s) {
  RRAM_REQUIRE(num >= 0 && C > 0 && H > 0 && W > 0 && size > 0 && (size & 1),
               "lrn_fwd: bad geometry (local_size must be odd)");
  const int64_t total = (int64_t)num * C * H * W;
  RRAM_REQUIRE_I32(total, "layer kernel");
  if (total == 0) return RRAM_OK;
  RRAM_REQUIRE(x && y, "lrn_fwd: NULL");
  const int cols = num * H * W;
  if (size == 5)
    hipLaunchKernelGGL(k_lrn_fwd_slide<5>, dim3((cols + kThreads - 1) / kThreads), dim3(kThreads), 0, as_stream(s), x, y,
                       scale, num, C, H * W, alpha / size, beta, k);
  else if (size == 3)
    hipLaunchKernelGGL(k_lrn_fwd_slide<3>, dim3((cols + kThreads - 1) / kThreads), dim3(kThreads), 0, as_stream(s), x, y,
                       scale, num, C, H * W, alpha / size, beta, k);
  else
    hipLaunchKernelGGL(k_lrn_fwd, dim3(stream_blocks(total)), dim3(kThreads), 0, as_stream(s), x, y,
                       scale, num, C, H * W, size, alpha / size, beta, k);
  return launch_status("lrn_fwd");
}
int rram_lrn_bwd(const float* x, const float* y, const float* scale, const float* dy, float* dx,
                 int num, int C, int H, int W, int size, float alpha, float beta, rram_stream_t s) {
  RRAM_REQUIRE(num >= 0 && C > 0 && H > 0 && W > 0 && size > 0 && (size & 1),
               "lrn_bwd: bad geometry");
  const int64_t total = (int64_t)num * C * H * W;
  RRAM_REQUIRE_I32(total, "layer kernel");
  if (total == 0) return RRAM_OK;
  RRAM_REQUIRE(x && y && scale && dy && dx, "lrn_bwd: NULL");
  hipLaunchKernelGGL(k_lrn_bwd, dim3(stream_blocks(total)), dim3(kThreads), 0, as_stream(s), x, y,
                     scale, dy, dx, num, C, H * W, size, 2.0f * alpha * beta / size, beta);
  return launch_status("lrn_bwd");
}

int rram_lrn_within_fwd(const float* x, float* y, float* scale, int num, int C, int H, int W, int size,
                        float alpha, float beta, rram_stream_t s) {
  RRAM_REQUIRE(num >= 0 && C > 0 && H > 0 && W > 0 && size > 0 && (size & 1), "lrn_within_fwd: bad geometry");
  const int64_t total = (int64_t)num * C * H * W;
  RRAM_REQUIRE_I32(total, "layer kernel");
  if (total == 0) return RRAM_OK;
  RRAM_REQUIRE(x && y, "lrn_within_fwd: NULL");
  hipLaunchKernelGGL(k_lrn_within_fwd, dim3(stream_blocks(total)), dim3(kThreads), 0, as_stream(s), x, y,
                     scale, (int64_t)num * C, H, W, size, alpha, beta);
  return launch_status("lrn_within_fwd");
}
int rram_lrn_within_bwd(const float* x, const float* scale, const float* dy, float* dx, int num, int C, int H,
                        int W, int size, float alpha, float beta, rram_stream_t s) {
  return rram_lrn_within_relu_bwd_core(x, scale, dy, dx, num, C, H, W, size, alpha, beta, 0, 0.0f, s);
}
int rram_lrn_within_relu_bwd(const float* x, const float* scale, const float* dy, float* dx, int num, int C, int H,
                             int W, int size, float alpha, float beta, float relu_slope, rram_stream_t s) {
  return rram_lrn_within_relu_bwd_core(x, scale, dy, dx, num, C, H, W, size, alpha, beta, 1, relu_slope, s);
}
}  // extern "C"
namespace rram {
namespace {
int rram_lrn_within_relu_bwd_core(const float* x, const float* scale, const float* dy, float* dx, int num, int C,
                                  int H, int W, int size, float alpha, float beta, int relu, float slope,
                                  rram_stream_t s) {
  RRAM_REQUIRE(num >= 0 && C > 0 && H > 0 && W > 0 && size > 0 && (size & 1), "lrn_within_bwd: bad geometry");
  const int64_t total = (int64_t)num * C * H * W;
  RRAM_REQUIRE_I32(total, "layer kernel");
  if (total == 0) return RRAM_OK;
  RRAM_REQUIRE(x && scale && dy && dx, "lrn_within_bwd: NULL");
  if (H * W <= kBwdPlaneMax && (int64_t)num * C <= (1ll << 24)) {  // num * C * 256 work-items fit 32 bits
    hipLaunchKernelGGL(k_lrn_within_bwd_plane, dim3(static_cast<unsigned>(num * C)), dim3(256), 0, as_stream(s), x,
                       scale, dy, dx, H, W, make_fastdivi(W), size, alpha, beta, relu, slope);
    return launch_status("lrn_within_bwd");
  }
  hipLaunchKernelGGL(k_lrn_within_bwd, dim3(stream_blocks(total)), dim3(kThreads), 0, as_stream(s), x, scale,
                     dy, dx, (int64_t)num * C, H, W, size, alpha, beta, relu, slope);
  return launch_status("lrn_within_bwd");
}
}  // namespace
}  // namespace rram
extern "C" {

int rram_softmax_fwd(const float* x, float* y, int outer, int C, int inner, rram_stream_t s) {
  RRAM_REQUIRE(outer >= 0 && C > 0 && inner > 0, "softmax: bad shape");
  const int64_t cols = (int64_t)outer * inner;
  if (cols == 0) return RRAM_OK;
  RRAM_REQUIRE(x && y, "softmax: NULL");
  int blocks = static_cast<int>((cols + 3) / 4);
  if (blocks > 2048) blocks = 2048;
  if (C <= 64 * 16)
    hipLaunchKernelGGL(k_softmax_reg<16>, dim3(blocks), dim3(256), 0, as_stream(s), x, y, outer, C, inner);
  else
    hipLaunchKernelGGL(k_softmax, dim3(blocks), dim3(256), 0, as_stream(s), x, y, outer, C, inner);
  return launch_status("softmax");
}

int rram_softmax_loss_fwd(const float* prob, const float* label, float* out, int outer, int C,
                          int inner, int ignore, rram_stream_t s) {
  return rram_softmax_loss_fwd_acc(prob, label, out, outer, C, inner, ignore, nullptr, nullptr, s);
}
int rram_softmax_loss_fwd_acc(const float* prob, const float* label, float* out, int outer, int C, int inner,
                              int ignore, float* acc_sum, float* acc_row, rram_stream_t s) {
  RRAM_REQUIRE(outer >= 0 && C > 0 && inner > 0 && out, "softmax_loss_fwd: bad args");
  RRAM_REQUIRE(outer == 0 || (prob && label), "softmax_loss_fwd: NULL");
  RRAM_REQUIRE(acc_row == nullptr || acc_sum != nullptr, "softmax_loss_fwd: acc_row without acc_sum");
  hipLaunchKernelGGL(k_softmax_loss_fwd, dim3(1), dim3(1024), 0, as_stream(s), prob, label, out,
                     outer, C, inner, ignore, acc_sum, acc_row);
  return launch_status("softmax_loss_fwd");
}

int rram_softmax_loss_fwd_bwd(const float* prob, const float* label, float* out, float* dx, int outer, int C,
                              int inner, int ignore, float loss_weight, rram_stream_t s) {
  RRAM_REQUIRE(outer >= 0 && C > 0 && inner > 0 && out, "softmax_loss_fwd_bwd: bad args");
  const int64_t total = (int64_t)outer * C * inner;
  RRAM_REQUIRE(total <= kLossFusedMax, "softmax_loss_fwd_bwd: more than %d elements", kLossFusedMax);
  RRAM_REQUIRE(outer == 0 || (prob && label && dx), "softmax_loss_fwd_bwd: NULL");
  const float scale_all = loss_weight / static_cast<float>((int64_t)outer * inner);
  hipLaunchKernelGGL(k_softmax_loss_fwd_bwd, dim3(1), dim3(1024), 0, as_stream(s), prob, label, out, dx, outer, C,
                     inner, ignore, loss_weight, scale_all);
  return launch_status("softmax_loss_fwd_bwd");
}

int rram_softmax_loss_bwd(const float* prob, const float* label, float* dx, int outer, int C,
                          int inner, int ignore, float loss_weight, rram_stream_t s) {
  RRAM_REQUIRE(outer >= 0 && C > 0 && inner > 0, "softmax_loss_bwd: bad shape");
  const int64_t total = (int64_t)outer * C * inner;
  RRAM_REQUIRE_I32(total, "layer kernel");
  if (total == 0) return RRAM_OK;
  RRAM_REQUIRE(prob && label && dx, "softmax_loss_bwd: NULL");
  // normalizer = #valid labels; computed on host for the common no-ignore case
  float scale = loss_weight / static_cast<float>((int64_t)outer * inner);
  if (ignore >= 0) {
    float* dcount = nullptr;
    RRAM_HIP_RET(hipMallocAsync(reinterpret_cast<void**>(&dcount), sizeof(float), as_stream(s)));
    hipLaunchKernelGGL(k_count_valid, dim3(1), dim3(1024), 0, as_stream(s), label,
                       (int64_t)outer * inner, ignore, dcount);
    float hc = 0.f;
    RRAM_HIP_RET(hipMemcpyAsync(&hc, dcount, sizeof(float), hipMemcpyDeviceToHost, as_stream(s)));
    RRAM_HIP_RET(hipStreamSynchronize(as_stream(s)));
    RRAM_HIP_RET(hipFreeAsync(dcount, as_stream(s)));
    scale = loss_weight / fmaxf(hc, 1.0f);
  }
  hipLaunchKernelGGL(k_softmax_loss_bwd, dim3(stream_blocks(total)), dim3(kThreads), 0,
                     as_stream(s), prob, label, dx, outer, C, inner, ignore, scale);
  return launch_status("softmax_loss_bwd");
}

int rram_accuracy(const float* x, const float* label, float* correct, float* count, float* ratio,
                  int outer, int C, int inner, int top_k, int ignore, rram_stream_t s) {
  return rram_accuracy_acc(x, label, correct, count, ratio, outer, C, inner, top_k, ignore, nullptr, nullptr, s);
}
int rram_accuracy_acc(const float* x, const float* label, float* correct, float* count, float* ratio, int outer,
                      int C, int inner, int top_k, int ignore, float* acc_sum, float* acc_row, rram_stream_t s) {
  RRAM_REQUIRE(acc_row == nullptr || acc_sum != nullptr, "accuracy: acc_row without acc_sum");
  RRAM_REQUIRE(acc_sum == nullptr || ratio != nullptr, "accuracy: acc_sum needs the ratio output");
  RRAM_REQUIRE(outer >= 0 && C > 0 && inner > 0 && top_k >= 1 && correct && count,
               "accuracy: bad args");
  RRAM_REQUIRE(outer == 0 || (x && label), "accuracy: NULL");
  const int64_t cols = (int64_t)outer * inner;
  RRAM_REQUIRE(cols < (1ll << 24), "accuracy: more than 2^24 samples (float counts would round)");
  if (cols * C <= kAccSmall && C <= 64) {
    hipLaunchKernelGGL(k_accuracy_small, dim3(1), dim3(1024), 0, as_stream(s), x, label, correct, count, ratio,
                       outer, C, inner, top_k, ignore, acc_sum, acc_row);
    return launch_status("accuracy");
  }
  if (cols > 0 && (cols + 3) / 4 <= kAccFusedBlocks) {
    hipLaunchKernelGGL(k_accuracy_fused, dim3(static_cast<unsigned>((cols + 3) / 4)), dim3(256), 0, as_stream(s), x,
                       label, correct, count, ratio, outer, C, inner, top_k, ignore, acc_sum, acc_row);
    return launch_status("accuracy");
  }
  RRAM_HIP_RET(hipMemsetAsync(correct, 0, sizeof(float), as_stream(s)));
  RRAM_HIP_RET(hipMemsetAsync(count, 0, sizeof(float), as_stream(s)));
  if (cols > 0)
    hipLaunchKernelGGL(k_accuracy, dim3(static_cast<unsigned>((cols + 3) / 4)), dim3(256), 0, as_stream(s), x,
                       label, correct, count, outer, C, inner, top_k, ignore);
  if (ratio)
    hipLaunchKernelGGL(k_accuracy_ratio, dim3(1), dim3(1), 0, as_stream(s), correct, count, ratio, acc_sum, acc_row);
  return launch_status("accuracy");
}

int rram_i32_to_f32(const int* x, float* y, int64_t n, rram_stream_t s) {
  RRAM_REQUIRE(n >= 0, "i32_to_f32: n < 0");
  RRAM_REQUIRE_I32(n, "i32_to_f32");
  if (n == 0) return RRAM_OK;
  RRAM_REQUIRE(x && y, "i32_to_f32: NULL");
  hipLaunchKernelGGL(k_i32_to_f32, dim3(stream_blocks(n)), dim3(kThreads), 0, as_stream(s), x, y, n);
  return launch_status("i32_to_f32");
}

int rram_euclidean_loss_fwd(const float* a, const float* b, float* diff, float* loss_out, int64_t n, int num,
                            rram_stream_t s) {
  RRAM_REQUIRE(n >= 0 && num > 0 && loss_out, "euclidean_loss_fwd: bad args");
  RRAM_REQUIRE(n == 0 || (a && b && diff), "euclidean_loss_fwd: NULL");
  hipLaunchKernelGGL(k_euclidean_fwd, dim3(1), dim3(1024), 0, as_stream(s), a, b, diff, loss_out, n, num);
  return launch_status("euclidean_loss_fwd");
}

int rram_euclidean_loss_bwd(const float* diff, float* dx, int64_t n, float alpha, rram_stream_t s) {
  RRAM_REQUIRE(n >= 0, "euclidean_loss_bwd: n < 0");
  RRAM_REQUIRE_I32(n, "euclidean_loss_bwd");
  if (n == 0) return RRAM_OK;
  RRAM_REQUIRE(diff && dx, "euclidean_loss_bwd: NULL");
  hipLaunchKernelGGL(k_scale_copy, dim3(stream_blocks(n)), dim3(kThreads), 0, as_stream(s), diff, dx, n, alpha);
  return launch_status("euclidean_loss_bwd");
}

int rram_concat_copy(const float* src, float* dst, int num, int sci, int dci, int off, int backward,
                     rram_stream_t s) {
  RRAM_REQUIRE(num >= 0 && sci >= 0 && dci >= sci && off >= 0 && off + sci <= dci,
               "concat: bad geometry");
  const int64_t total = (int64_t)num * sci;
  RRAM_REQUIRE_I32(total, "layer kernel");
  if (total == 0) return RRAM_OK;
  RRAM_REQUIRE(src && dst, "concat: NULL");
  hipLaunchKernelGGL(k_concat, dim3(stream_blocks(total)), dim3(kThreads), 0, as_stream(s), src, dst,
                     num, sci, dci, off, backward);
  return launch_status("concat");
}

}  // extern "C"
