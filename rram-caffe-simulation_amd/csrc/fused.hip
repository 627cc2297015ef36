// Inference-time layer fusions (TEST phase).  A fusion here never changes
// the arithmetic of the layers it merges: every intermediate value is the one
// the unfused kernels produce, only its round trip through HBM disappears.
#include <float.h>
#include <math.h>

#include "rram_common.hpp"

namespace rram {
namespace {

// LRN ACROSS_CHANNELS followed by MAX pooling with a K x K window.
//
// One thread per pooled (n, ph, pw) walks the channels.  For each of the K*K
// input positions of its window it keeps the SIZE-channel ring of x and the
// running sum of squares, updated exactly as k_lrn_fwd_slide / LRNFillScale
// (lrn_layer.cu:9-51: add the channel entering the window, then subtract the
// one leaving it), so each LRN value x * (k + alpha/size * sum)^-beta
// (lrn_layer.cu:72-78) is the unfused kernel's bit for bit.  The max over the
// window follows MaxPoolForward (pooling_layer.cu:11-47): window clipped to
// the image, -FLT_MAX start, strict ">" in row-major order.
// HBM traffic: x read once (neighbouring windows overlap in L2), y written once;
// the LRN output (the pool's bottom) is never materialised.
template <int K, int SIZE>
__global__ void __launch_bounds__(256)
    k_lrn_maxpool(const float* __restrict__ x, float* __restrict__ y, int num, int C, int H, int W,
                  int PH, int PW, int sh, int sw, int ph, int pw, float alpha_over_size, float beta,
                  float k) {
  constexpr int PRE = (SIZE - 1) / 2, POST = SIZE - PRE - 1;
  constexpr int P = K * K;
  constexpr int D = 4;  // channels loaded ahead per step (D * P loads in flight)
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= num * PH * PW) return;
  const int pwi = idx % PW;
  const int phi = (idx / PW) % PH;
  const int n = idx / (PW * PH);
  const int hs = phi * sh - ph, ws = pwi * sw - pw;
  const int HW = H * W;
  const float* xn = x + (int64_t)n * C * HW;
  float* yn = y + (int64_t)n * C * PH * PW + phi * PW + pwi;
  int off[P];
  bool ok[P];
#pragma unroll
  for (int a = 0; a < K; ++a)
#pragma unroll
    for (int b = 0; b < K; ++b) {
      const int h = hs + a, w = ws + b;
      ok[a * K + b] = static_cast<unsigned>(h) < static_cast<unsigned>(H) &&
                      static_cast<unsigned>(w) < static_cast<unsigned>(W);
      off[a * K + b] = ok[a * K + b] ? h * W + w : 0;
    }
  // win[p][j] = x at channel (c - PRE + j), zero outside [0, C)
  float win[P][SIZE + D];
  float acc[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
#pragma unroll
    for (int j = 0; j < SIZE; ++j) {
      const int cc = j - PRE;
      win[p][j] = (cc >= 0 && cc < C && ok[p]) ? xn[(int64_t)cc * HW + off[p]] : 0.0f;
    }
    acc[p] = 0.0f;
#pragma unroll
    for (int j = PRE; j < SIZE; ++j) acc[p] = lrn_sq_add(acc[p], win[p][j]);
  }
  for (int c0 = 0; c0 < C; c0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int cn = c0 + d + POST + 1;
#pragma unroll
      for (int p = 0; p < P; ++p)
        win[p][SIZE + d] = (cn < C && ok[p]) ? xn[(int64_t)cn * HW + off[p]] : 0.0f;
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int c = c0 + d;
      if (c < C) {
        float mv = -FLT_MAX;
#pragma unroll
        for (int p = 0; p < P; ++p) {
          // the helpers k_lrn_fwd_slide uses, in the same order
          const float v = lrn_out(win[p][d + PRE], lrn_scale(acc[p], alpha_over_size, k), beta);
          if (ok[p] && v > mv) mv = v;
          acc[p] = lrn_slide(acc[p], win[p][d + SIZE], win[p][d]);
        }
        yn[(int64_t)c * PH * PW] = mv;
      }
    }
#pragma unroll
    for (int p = 0; p < P; ++p)
#pragma unroll
      for (int j = 0; j < SIZE; ++j) win[p][j] = win[p][j + D];
  }
}

}  // namespace
}  // namespace rram

using namespace rram;

extern "C" {

int rram_lrn_maxpool_fwd(const float* x, float* y, int num, int C, int H, int W, int PH, int PW,
                         int kernel, int sh, int sw, int ph, int pw, int size, float alpha, float beta,
                         float k, rram_stream_t s) {
  RRAM_REQUIRE(num >= 0 && C > 0 && H > 0 && W > 0 && PH > 0 && PW > 0 && sh > 0 && sw > 0 && ph >= 0 &&
                   pw >= 0,
               "lrn_maxpool_fwd: bad geometry");
  RRAM_REQUIRE((kernel == 2 || kernel == 3) && (size == 3 || size == 5),
               "lrn_maxpool_fwd: supports kernel 2/3 and local_size 3/5 (got %d, %d)", kernel, size);
  RRAM_REQUIRE(ph < kernel && pw < kernel, "lrn_maxpool_fwd: pad must be < kernel");
  const int64_t cols = (int64_t)num * PH * PW;
  RRAM_REQUIRE((int64_t)num * C * H * W < 2147483647ll && cols * C < 2147483647ll,
               "lrn_maxpool_fwd: more than 2^31 elements is not supported");
  if (cols == 0) return RRAM_OK;
  RRAM_REQUIRE(x && y, "lrn_maxpool_fwd: NULL");
  const dim3 grid(static_cast<unsigned>((cols + kThreads - 1) / kThreads));
  const float aos = alpha / size;
#define RRAM_LP(K_, S_)                                                                                   \
  if (kernel == K_ && size == S_)                                                                         \
    hipLaunchKernelGGL((k_lrn_maxpool<K_, S_>), grid, dim3(kThreads), 0, as_stream(s), x, y, num, C, H, W, \
                       PH, PW, sh, sw, ph, pw, aos, beta, k);
  RRAM_LP(3, 5)
  else RRAM_LP(3, 3) else RRAM_LP(2, 5) else RRAM_LP(2, 3)
#undef RRAM_LP
  return launch_status("lrn_maxpool_fwd");
}

}  // extern "C"
