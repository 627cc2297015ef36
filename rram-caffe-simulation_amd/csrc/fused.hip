// Inference-time layer fusions (TEST phase).  A fusion here never changes
// the arithmetic of the layers it merges: every intermediate value is the one
// the unfused kernels produce, only its round trip through HBM disappears.
#include <float.h>
#include <math.h>
#include <stdlib.h>

#include "rram_common.hpp"
#include "split3.hpp"

namespace rram {
namespace {

// LRN ACROSS_CHANNELS followed by MAX pooling with a K x K window.
//
// Block = one image x a band of RB pooled rows x a chunk of CC channels
// (blockIdx.z): the chunks give the grid several block waves (one image x
// band per block, walking all channels, left AlexNet's norm2 at 512 blocks,
// latency-bound).  Per channel, every thread produces the LRN value of up to
// PPT input pixels of the band (the band's input rows are contiguous in
// memory, so the loads are coalesced), from a register ring of the SIZE
// channels around it: scale = k + alpha/size * sum of the SIZE squares in
// channel order (lrn_sq_add, the unfused k_lrn_fwd_slide's sum, so each LRN
// value x * scale^-beta (lrn_layer.cu:72-78) is the unfused kernel's bit for
// bit, whatever chunk it falls in).  A chunk reads its PRE / POST halo
// channels too (AlexNet: 4 of 36 per chunk, mostly L2 / MALL hits).  The
// values go to an LDS plane (double-buffered: one barrier per group of G
// channels) from which the band's pooled outputs take the max over their
// window exactly as MaxPoolForward (pooling_layer.cu:11-47): window clipped to
// the image, -FLT_MAX start, strict ">" in row-major order.
// HBM traffic: x read once (plus the shared input row between adjacent bands
// and the chunk halos), y written once; the LRN output never leaves the CU.
constexpr int kBandPix = 512;  // input pixels per band (PPT = 2 per thread)
// target grid of the LRN + pool band kernel: several block waves of 256 CUs
constexpr int kLrnBlocks = 4096;

// G channels per barrier; the loads run one group ahead.  Measured on MI355X
// (AlexNet b256): G = 2 for norm1 (55 x 55 planes), G = 4 for norm2 (27 x 27).
// OCT: also write y's channel-octet companion yo (the next convolution's
// pre-split input, x6.hip k_pack_octets_x6 layout [num][C/8][PH][PW][3][8]
// bf16): the pooled values of 8 channels are gathered in an LDS plane and
// split by the band's output threads (C % 8 == 0 and CC % 8 == 0; G divides 8).
// WT > 0: the plane width W is WT (AlexNet's 55 / 27), so a window that lies
// wholly inside the image reads its K x K taps at immediate LDS offsets with
// no per-tap mask (3 instructions a tap instead of ~6; every AlexNet window
// is such, the ceil rule clips none); WT = 0: any W.
template <int K, int SIZE, int G, bool OCT, int WT = 0>
__global__ void __launch_bounds__(256)
    k_lrn_maxpool_band(const float* __restrict__ x, float* __restrict__ y, char* __restrict__ yo, int C, int H, int W,
                       int PH, int PW, int sh, int sw, int ph, int pw, int RB, int CC, float alpha_over_size,
                       float beta, float k) {
  static_assert(!OCT || (8 % (2 * G) == 0), "the octet walk needs G in {2, 4}");
  constexpr int PRE = (SIZE - 1) / 2;
  constexpr int D = G;
  constexpr int PPT = kBandPix / 256;
  __shared__ float ybuf[2][D][kBandPix];
  __shared__ float obuf[OCT ? 8 : 1][OCT ? 256 : 1];
  const int n = blockIdx.y;
  const int cb = blockIdx.z * CC;
  const int ce = min(C, cb + CC);
  const int pr0 = blockIdx.x * RB;
  const int pr1 = min(PH, pr0 + RB);
  const int h0 = max(0, pr0 * sh - ph);
  const int h1 = min(H, (pr1 - 1) * sh - ph + K);  // exclusive
  const int NP = (h1 - h0) * W;
  const int HW = H * W;
  const float* xb = x + (int64_t)n * C * HW + (int64_t)h0 * W;
  int pix[PPT];
  bool own[PPT];
#pragma unroll
  for (int q = 0; q < PPT; ++q) {
    pix[q] = threadIdx.x + q * 256;
    own[q] = pix[q] < NP;
  }
  // buffer loads with 32-bit offsets from the band's first row (one image is
  // < 2 GiB: host check); a channel outside [0, C) or a pixel outside the band
  // reads past the range, i.e. zero
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(xb), 0, static_cast<int>(((int64_t)C * HW - (int64_t)h0 * W) * 4), 0x00020000);
  auto ld = [&](int q, int cc) {
    const uint32_t off = (cc >= 0 && cc < C && own[q]) ? static_cast<uint32_t>((cc * HW + pix[q]) * 4) : 0x80000000u;
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xrs, static_cast<int>(off), 0, 0));
  };
  // win[q][j] = x at channel (c0 - PRE + j) of pixel q, zero outside [0, C).
  // The entering channels of group g + 2 are loaded at the top of group g
  // into one of two staging arrays (st0 / st1, alternating by group parity so
  // the registers are named statically) and moved into the ring at the bottom
  // of group g + 1: two groups of loads stay in flight across the LDS / pool
  // work, instead of one group whose loads the ring shift waits for.
  float win[PPT][SIZE + D];
  float st0[D][PPT], st1[D][PPT];
#pragma unroll
  for (int q = 0; q < PPT; ++q)
#pragma unroll
    for (int j = 0; j < SIZE + D; ++j) win[q][j] = ld(q, cb + j - PRE);
#pragma unroll
  for (int d = 0; d < D; ++d)
#pragma unroll
    for (int q = 0; q < PPT; ++q) st1[d][q] = ld(q, cb + SIZE + D - PRE + d);  // group 1's entering channels
  const int NO = (pr1 - pr0) * PW;  // pooled outputs of the band per channel
  const int64_t PHW = (int64_t)PH * PW;
  float* yn = y + (int64_t)n * C * PHW;
  // pooling items of a group: (channel d, output o), consecutive outputs of
  // one channel on consecutive lanes (coalesced stores); each thread's items
  // and their windows are fixed for the whole channel walk, so they are
  // decoded once here: LDS base of the window, tap validity (the window
  // clipped to the image), output offset
  constexpr int MAXI = D;  // D * NO <= D * 256 items
  int it_d[MAXI], it_l[MAXI], it_out[MAXI];
  uint32_t it_ok[MAXI];
#pragma unroll
  for (int i = 0; i < MAXI; ++i) {
    const int it = threadIdx.x + i * 256;
    const int d = it / max(NO, 1), o = it - d * NO;
    const int prl = o / PW, pwi = o - prl * PW;
    const int hr = (pr0 + prl) * sh - ph, wr = pwi * sw - pw;
    uint32_t ok = 0;
#pragma unroll
    for (int a = 0; a < K; ++a)
#pragma unroll
      for (int b = 0; b < K; ++b)
        ok |= static_cast<uint32_t>(static_cast<unsigned>(hr + a) < static_cast<unsigned>(H) &&
                                    static_cast<unsigned>(wr + b) < static_cast<unsigned>(W))
              << (a * K + b);
    it_d[i] = it < D * NO ? d : D;  // D = no item
    it_l[i] = (hr - h0) * W + wr;
    it_out[i] = (pr0 + prl) * PW + pwi;
    it_ok[i] = ok;
  }
  // one channel group: c0 = its first channel, yb = its LDS plane buffer
  auto group = [&](int c0, float (*yb)[kBandPix], float (&load_into)[D][PPT], const float (&fill_from)[D][PPT]) {
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int q = 0; q < PPT; ++q) load_into[d][q] = ld(q, c0 - PRE + SIZE + 2 * D + d);
#pragma unroll
    for (int d = 0; d < D; ++d) {
#pragma unroll
      for (int q = 0; q < PPT; ++q) {
        // the helpers k_lrn_fwd_slide uses, in the same order
        float acc = 0.0f;
#pragma unroll
        for (int j = 0; j < SIZE; ++j) acc = lrn_sq_add(acc, win[q][d + j]);
        const float v = lrn_out(win[q][d + PRE], lrn_scale(acc, alpha_over_size, k), beta);
        if (own[q]) yb[d][pix[q]] = v;
      }
    }
    __syncthreads();
    // pool the group's D channels (MaxPoolForward: -FLT_MAX start, strict ">"
    // in row-major window order over the taps inside the image)
    const int nd = min(D, ce - c0);
#pragma unroll
    for (int i = 0; i < MAXI; ++i) {
      const int d = it_d[i];
      if (d < nd) {
        const float* yl = yb[d] + it_l[i];
        float mv = -FLT_MAX;
        if (WT > 0 && it_ok[i] == (1u << (K * K)) - 1u) {
#pragma unroll
          for (int a = 0; a < K; ++a)
#pragma unroll
            for (int b = 0; b < K; ++b) {
              const float v = yl[a * WT + b];
              mv = v > mv ? v : mv;
            }
        } else {
#pragma unroll
          for (int a = 0; a < K; ++a)
#pragma unroll
            for (int b = 0; b < K; ++b) {
              const bool ok = (it_ok[i] >> (a * K + b)) & 1u;
              const float v = yl[ok ? a * W + b : -it_l[i]];  // masked taps read element 0
              if (ok && v > mv) mv = v;
            }
        }
        yn[(int64_t)(c0 + d) * PHW + it_out[i]] = mv;
        if (OCT) obuf[(c0 + d) & 7][it_out[i] - pr0 * PW] = mv;
      }
    }
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
#pragma unroll
      for (int j = 0; j < SIZE; ++j) win[q][j] = win[q][j + D];
#pragma unroll
      for (int d = 0; d < D; ++d) win[q][SIZE + d] = fill_from[d][q];
    }
  };
  if (!OCT) {
    for (int c0 = cb; c0 < ce; c0 += 2 * D) {
      group(c0, ybuf[0], st0, st1);
      if (c0 + D < ce) group(c0 + D, ybuf[1], st1, st0);
    }
    return;
  }
  // OCT: 8 channels per step (an even number of groups), then the octet
  char* yon = yo + (int64_t)n * (C / 8) * PHW * 48;
  for (int c0 = cb; c0 < ce; c0 += 8) {
#pragma unroll
    for (int g = 0; g < 8; g += 2 * D) {
      group(c0 + g, ybuf[0], st0, st1);
      group(c0 + g + D, ybuf[1], st1, st0);
    }
    __syncthreads();  // obuf complete (the next group's barrier orders its rewrite)
    const int o = threadIdx.x;
    if (o < NO) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = obuf[e][o];
      const int prl = o / PW;
      const int64_t out = (int64_t)(pr0 + prl) * PW + (o - prl * PW);
      x6::store_terms8(v, yon + ((int64_t)(c0 / 8) * PHW + out) * 48);
    }
  }
}

}  // namespace
}  // namespace rram

using namespace rram;

extern "C" {

int rram_lrn_maxpool_fwd(const float* x, float* y, int num, int C, int H, int W, int PH, int PW,
                         int kernel, int sh, int sw, int ph, int pw, int size, float alpha, float beta,
                         float k, rram_stream_t s) {
  return rram_lrn_maxpool_fwd_octets(x, y, nullptr, num, C, H, W, PH, PW, kernel, sh, sw, ph, pw, size, alpha, beta,
                                     k, s);
}

int rram_lrn_maxpool_fwd_octets(const float* x, float* y, void* y_oct, int num, int C, int H, int W, int PH, int PW,
                                int kernel, int sh, int sw, int ph, int pw, int size, float alpha, float beta,
                                float k, rram_stream_t s) {
  RRAM_REQUIRE(y_oct == nullptr || C % 8 == 0, "lrn_maxpool_fwd_octets: octets need channels %% 8 == 0");
  RRAM_REQUIRE(num >= 0 && C > 0 && H > 0 && W > 0 && PH > 0 && PW > 0 && sh > 0 && sw > 0 && ph >= 0 &&
                   pw >= 0,
               "lrn_maxpool_fwd: bad geometry");
  RRAM_REQUIRE((kernel == 2 || kernel == 3) && (size == 3 || size == 5),
               "lrn_maxpool_fwd: supports kernel 2/3 and local_size 3/5 (got %d, %d)", kernel, size);
  RRAM_REQUIRE(ph < kernel && pw < kernel, "lrn_maxpool_fwd: pad must be < kernel");
  RRAM_REQUIRE((int64_t)num * C * H * W < 2147483647ll && (int64_t)num * C * PH * PW < 2147483647ll,
               "lrn_maxpool_fwd: more than 2^31 elements is not supported");
  RRAM_REQUIRE((int64_t)C * H * W * 4 < 2147483647ll, "lrn_maxpool_fwd: one image must be < 2 GiB");
  if (num == 0) return RRAM_OK;
  RRAM_REQUIRE(x && y, "lrn_maxpool_fwd: NULL");
  // band height: input rows of RB pooled rows must fit the block's pixel
  // budget and RB * PW outputs its threads
  auto fits = [&](int rb) {
    const int rows = min(H, (rb - 1) * sh + kernel);
    return rb * PW <= kThreads && rows * W <= kBandPix;
  };
  RRAM_REQUIRE(fits(1), "lrn_maxpool_fwd: a pooled row needs more than %d input pixels", kBandPix);
  int rb = 1;
  while (rb < PH && fits(rb + 1)) ++rb;
  // channels per barrier: measured G = 2 for 55 x 55 planes, 4 for 27 x 27
  const int gsel = H * W >= 1024 ? 2 : 4;
  // channel chunks: as few as give >= kLrnBlocks blocks (each chunk re-reads
  // SIZE - 1 halo channels), equal sizes in multiples of 8 (2 * G without octets)
  const int step = y_oct ? 8 : 2 * gsel;
  const int64_t bands = (PH + rb - 1) / rb;
  const int64_t tiles = (int64_t)num * bands;  // > 0
  const int64_t want = ((int64_t)kLrnBlocks + tiles - 1) / tiles;
  const int64_t most = (C + step - 1) / step;
  const int chunks = static_cast<int>(want < 1 ? 1 : (want > most ? most : want));
  const int cc = ((C + chunks - 1) / chunks + step - 1) / step * step;
  const dim3 grid(static_cast<unsigned>(bands), static_cast<unsigned>(num), static_cast<unsigned>((C + cc - 1) / cc));
  const float aos = alpha / size;
  char* yo = static_cast<char*>(y_oct);
#define RRAM_LP3(K_, S_, G_, WT_)                                                                             \
  if (yo)                                                                                                     \
    hipLaunchKernelGGL((k_lrn_maxpool_band<K_, S_, G_, true, WT_>), grid, dim3(kThreads), 0, as_stream(s), x, y, \
                       yo, C, H, W, PH, PW, sh, sw, ph, pw, rb, cc, aos, beta, k);                            \
  else                                                                                                        \
    hipLaunchKernelGGL((k_lrn_maxpool_band<K_, S_, G_, false, WT_>), grid, dim3(kThreads), 0, as_stream(s), x, \
                       y, yo, C, H, W, PH, PW, sh, sw, ph, pw, rb, cc, aos, beta, k);
#define RRAM_LP2(K_, S_, G_)                               \
  if (K_ == 3 && S_ == 5 && W == 55) {                     \
    RRAM_LP3(K_, S_, G_, (K_ == 3 && S_ == 5 ? 55 : 0))    \
  } else if (K_ == 3 && S_ == 5 && W == 27) {              \
    RRAM_LP3(K_, S_, G_, (K_ == 3 && S_ == 5 ? 27 : 0))    \
  } else {                                                 \
    RRAM_LP3(K_, S_, G_, 0)                                \
  }
#define RRAM_LP(K_, S_)          \
  if (kernel == K_ && size == S_) { \
    if (gsel == 2) {             \
      RRAM_LP2(K_, S_, 2)        \
    } else {                     \
      RRAM_LP2(K_, S_, 4)        \
    }                            \
  }
  RRAM_LP(3, 5)
  else RRAM_LP(3, 3) else RRAM_LP(2, 5) else RRAM_LP(2, 3)
#undef RRAM_LP
#undef RRAM_LP2
#undef RRAM_LP3
  return launch_status("lrn_maxpool_fwd");
}

}  // extern "C"
