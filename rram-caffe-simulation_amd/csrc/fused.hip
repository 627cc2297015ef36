// Inference-time layer fusions (TEST phase).  A fusion here never changes
// the arithmetic of the layers it merges: every intermediate value is the one
// the unfused kernels produce, only its round trip through HBM disappears.
#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdlib.h>

#include <type_traits>

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
// memory, so the loads are coalesced), from a register ring of 16 channels
// (the SIZE around it and the loads of the next NS groups in flight): scale = k + alpha/size * sum of the SIZE squares in
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
// y == nullptr (with a companion): only the companion is written (the host's
// pooled-output fold, Net::Net: its one reader takes the companion).
constexpr int kBandPix = 512;  // input pixels per band (PPT = 2 per thread)
// target grid of the LRN + pool band kernel: several block waves of 256 CUs
#ifndef RRAM_LRN_BLOCKS
#define RRAM_LRN_BLOCKS 4096
#endif
#ifndef RRAM_LRN_ALT
#define RRAM_LRN_ALT 0
#endif
#ifndef RRAM_LRN_BAL  // even band heights (A/B builds: 0 = the tallest bands first)
#define RRAM_LRN_BAL 1
#endif
#ifndef RRAM_LRN_YNT  // cache policy of the pooled y stores (A/B builds: 2 = nontemporal)
#define RRAM_LRN_YNT 0
#endif
#ifndef RRAM_LRN_DIAG
#define RRAM_LRN_DIAG 0
#endif
#ifndef RRAM_LRN_XCD
#define RRAM_LRN_XCD 1
#endif
constexpr int kLrnBlocks = RRAM_LRN_BLOCKS;
constexpr int kLrnG = 2;

// G channels per barrier (kLrnG = 2: measured on MI355X for both AlexNet
// planes once the loads run 8 channels ahead; G = 4 spilled SGPRs).
// OCT: also write y's channel-octet companion yo (the next convolution's
// pre-split input, x6.hip k_pack_octets_x6 layout [num][C/8][PH][PW][3][8]
// bf16): the pooled values of 8 channels are gathered in an LDS plane and
// split by the band's output threads (C % 8 == 0 and CC % 8 == 0; G divides 8).
// WT > 0: the plane width W is WT (AlexNet's 55 / 27) and the window stride
// is 2 with no column padding (host check), so a window that lies wholly
// inside the image reads its K x K taps at immediate LDS offsets with no
// per-tap mask (every AlexNet window is such, the ceil rule clips none), and
// each plane row is stored de-interleaved, even input columns then odd ones
// (column c at (c & 1) * HWC + (c >> 1)): the taps of consecutive pooled
// outputs (input columns 2 o + b) then sit on consecutive words, where the
// plain row had consecutive lanes two words apart (2-way LDS bank conflicts
// on every tap: 46-48 % of the LDS-active cycles in round 3).  WT = 0: any W,
// plain rows.
// CCT > 0: every chunk is exactly CCT channels (host check; AlexNet b256:
// 32-channel chunks of both planes): the channel walk is straight-line code
// (the looped walk's back edge made the compiler drain every load in flight
// at each trip top).  Round 5, norm2 / norm1 per launch: 84.6 / 112.1 us ->
// 80.5 / 109.0 (ring, straight line) -> 73.8 / 102.1 (coalesced companion
// stores), profiles/r05_ab_lrn_walk.txt.
__device__ __forceinline__ float max3f(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

template <int K, int SIZE, int G, bool OCT, int WT = 0, int CCT = 0>
__global__ void __launch_bounds__(256)
    k_lrn_maxpool_band(const float* __restrict__ x, float* __restrict__ y, char* __restrict__ yo, int C, int H, int W,
                       int PH, int PW, int sh, int sw, int ph, int pw, int RB, int CC, int bands, int chunks,
                       float alpha_over_size, float beta, float k) {
  static_assert(!OCT || (8 % (2 * G) == 0), "the octet walk needs G in {2, 4}");
  static_assert(CCT % 16 == 0, "straight-line walks cover whole ring trips");
  static_assert(kBandPix == 2 * 256, "two pixels per thread: the packed LRN pair");
  constexpr int PRE = (SIZE - 1) / 2;
  constexpr int D = G;
  // WT rows: input row i at rowbase(i) = (i / 2) R2 + (i % 2) WT, R2 >= 2 WT with
  // R2 = PWT (mod 32), PWT the pooled width: a pooled row (two input rows
  // down) then starts PWT banks after the previous one, so the 32 consecutive
  // outputs of a ds_read_b32 lane group sit on 32 distinct banks even across a
  // row wrap (a plain pitch put 2 addresses on some bank of almost every read:
  // 40-46 % of the LDS-active cycles were conflicts in round 4)
  constexpr int PWT = WT > 0 ? (WT - K + 1) / 2 + 1 : 1;
  constexpr int R2 = WT > 0 ? 2 * WT + (((PWT - 2 * WT) % 32) + 32) % 32 : 0;
  constexpr int YBS = WT > 0 ? ((kBandPix / WT - 1) / 2 * R2 + ((kBandPix / WT - 1) % 2) * WT + WT + 3) / 4 * 4
                             : kBandPix;
  auto rowbase = [](int i) { return (i >> 1) * R2 + (i & 1) * WT; };
  __shared__ float ybuf[2][D][YBS];
  __shared__ float obuf[OCT ? 8 : 1][OCT ? 256 : 1];
  // XCD-aware tile order: consecutive workgroups go to the 8 XCDs in turn, so
  // workgroup L runs on XCD L % 8 as that XCD's (L / 8)-th; each XCD gets a
  // contiguous range of tiles in (image, chunk, band) order, band fastest.
  // Tiles that read the same input rows (adjacent bands share a row, adjacent
  // chunks share the LRN halo channels) then run on one XCD close in time, and
  // the second read can hit that XCD's L2 instead of going to HBM.
  const int total = bands * chunks * static_cast<int>(gridDim.y);  // gridDim.y = images
  const int L = blockIdx.x + static_cast<int>(gridDim.x) * blockIdx.y;
  const int xq = total / 8, xr = total % 8, xcd = L % 8, xk = L / 8;
  const int tile = !RRAM_LRN_XCD ? L : xcd < xr ? xcd * (xq + 1) + xk : xr * (xq + 1) + (xcd - xr) * xq + xk;
  const int band = tile % bands, rest = tile / bands;
  const int n = rest / chunks;
  const int cb = (rest - n * chunks) * CC;
  const int ce = min(C, cb + CC);
  const int pr0 = band * RB;
  const int pr1 = min(PH, pr0 + RB);
  const int h0 = max(0, pr0 * sh - ph);
  const int h1 = min(H, (pr1 - 1) * sh - ph + K);  // exclusive
  const int NP = (h1 - h0) * W;
  const int HW = H * W;
  // the thread's two pixels of the band: threadIdx.x and threadIdx.x + 256
  const int pix0 = threadIdx.x, pix1 = threadIdx.x + 256;
  const bool own0 = pix0 < NP, own1 = pix1 < NP;
  // LDS slots of the two pixels (WT: de-interleaved rows)
  constexpr int HWC = (WT + 1) / 2;
  auto slot = [&](int pix) {
    if constexpr (WT > 0) {
      const int r = pix / WT, c = pix - r * WT;
      return rowbase(r) + (c & 1) * HWC + (c >> 1);
    } else {
      return pix;
    }
  };
  const int sl0 = slot(pix0), sl1 = slot(pix1);
  // one buffer resource over image n (range C H W floats) and a lane offset
  // per channel: channel cc at (h0 W + pix + cc H W) * 4, one VALU add per
  // pixel (a resource per channel cost ~10 scalar instructions a load: SALU
  // above VALU in round 3).  A pixel outside the band starts at 2^31 and a
  // channel outside [0, C) lands past the range (cc < 0 wraps above 2^31):
  // zero either way
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x + (int64_t)n * C * HW), 0, C * HW * 4, 0x00020000);
  const uint32_t vo0 = own0 ? static_cast<uint32_t>(h0 * W + pix0) * 4u : 0x80000000u;
  const uint32_t vo1 = own1 ? static_cast<uint32_t>(h0 * W + pix1) * 4u : 0x80000000u;
  auto ld = [&](int cc) {
    const uint32_t co = static_cast<uint32_t>(cc) * static_cast<uint32_t>(HW * 4);  // mod 2^32
    return f32x2{__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xrs, static_cast<int>(vo0 + co), 0, 0)),
                 __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xrs, static_cast<int>(vo1 + co), 0, 0))};
  };
  // The channel walk keeps both pixels of a ring of RL = 16 consecutive
  // channels in registers: ring[r & 15] holds the channel at walk position r
  // (UP: channel base + r, base = cb - PRE; DN: channel base - r, base = the
  // top group's window end), so the walk, unrolled over 16 channels (8 groups
  // of D = 2) per loop trip, names every register statically with no copy at
  // the loop latch.  (Round 4's window + staging arrays rotated by copies:
  // the compiler moved the freshly loaded staging registers at the latch,
  // behind a vmcnt(0), which drained every load in flight once per octet.)
  // Group g's window is positions 2 g .. 2 g + SIZE + D - 1; it loads the
  // positions its NS-th successor enters with, 2 g + SIZE + NS D + {0 .. D-1},
  // so NS groups of loads stay in flight across the LDS / pool work.
  constexpr int RL = 16;
  constexpr int NS = (RL - SIZE - D) / D;  // 4 (SIZE 5) / 5 (SIZE 3) groups ahead
  // the live positions at a group (its window up to the entering channels of
  // its NS-th successor, loaded before the window is read) span SIZE + NS D + D
  static_assert(SIZE + NS * D + D <= RL && D == 2, "ring span");
  f32x2 ring[RL];
  const int NO = (pr1 - pr0) * PW;  // pooled outputs of the band per channel
  const int PHW = PH * PW;
  // y of image n through a buffer resource too (one image < 2 GiB: host check)
  // (y == nullptr: the pooled fp32 output is not materialised, only its
  // octet companion -- the host's pooled-output fold; the range-0 resource
  // then drops the stores)
  const bool ys = y != nullptr;
  const __amdgpu_buffer_rsrc_t yrs =
      __builtin_amdgcn_make_buffer_rsrc(ys ? y + (int64_t)n * C * PHW : y, 0, ys ? C * PHW * 4 : 0, 0x00020000);
  // pooling items of a group: (channel d, output o), consecutive outputs of
  // one channel on consecutive lanes (coalesced stores); each thread's items
  // and their windows are fixed for the whole channel walk, so they are
  // decoded once here: LDS base of the window, tap validity (the window
  // clipped to the image), output byte offset from the group's first channel
  constexpr int MAXI = D;  // D * NO <= D * 256 items
  int it_d[MAXI], it_l[MAXI], it_out[MAXI], it_vo[MAXI];
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
    // WT: wr is even (stride 2, no column pad) and hr - h0 too (stride 2, no row pad)
    it_l[i] = WT > 0 ? rowbase(hr - h0) + (wr >> 1) : (hr - h0) * W + wr;
    it_out[i] = (pr0 + prl) * PW + pwi;
    it_vo[i] = (d * PHW + it_out[i]) * 4;
    it_ok[i] = ok;
  }
  // one channel group: c0 = its first channel, g = its place in the loop trip
  // (static: ring slots and LDS plane buffer g & 1), DN = the walk's direction
  auto group = [&](int c0, auto gi, auto dn) {
    constexpr int GG = decltype(gi)::value;
    constexpr bool DN = decltype(dn)::value;
    // entering channels of group g + NS: positions 2 g + SIZE + NS D + d
#pragma unroll
    for (int d = 0; d < D; ++d) {
      constexpr int P0 = 2 * GG + SIZE + NS * D;
      ring[(P0 + d) & (RL - 1)] = ld(DN ? c0 - PRE + D - 1 - NS * D - d : c0 - PRE + SIZE + NS * D + d);
    }
    // the window in channel order: w[j] = channel c0 - PRE + j (UP: position
    // 2 g + j; DN: position 2 g + SIZE + D - 1 - j)
    f32x2 w[SIZE + D];
#pragma unroll
    for (int j = 0; j < SIZE + D; ++j) w[j] = ring[(DN ? 2 * GG + SIZE + D - 1 - j : 2 * GG + j) & (RL - 1)];
    float(*yb)[YBS] = ybuf[GG & 1];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      // lrn_sq_add / lrn_scale / lrn_out (the unfused kernels' arithmetic) on
      // both pixels at once
#if RRAM_LRN_DIAG == 1  // diagnostic builds only: no LRN arithmetic
      const f32x2 v = w[d + PRE];
#else
      const f32x2 v = lrn_value2<SIZE>(w + d, alpha_over_size, beta, k);
#endif
      if (own0) yb[d][sl0] = v.x;
      if (own1) yb[d][sl1] = v.y;
    }
#if RRAM_LRN_DIAG != 3  // diagnostic builds only: no barrier (garbage values)
    __syncthreads();
#endif
    // pool the group's D channels (MaxPoolForward: -FLT_MAX start, strict ">"
    // in row-major window order over the taps inside the image)
    const int nd = RRAM_LRN_DIAG == 2 ? 0 : min(D, ce - c0);  // DIAG 2: no pooling
#pragma unroll
    for (int i = 0; i < MAXI; ++i) {
      const int d = it_d[i];
      if (d < nd) {
        const float* yl = yb[d] + it_l[i];
        float mv = -FLT_MAX;
        if (WT > 0 && it_ok[i] == (1u << (K * K)) - 1u) {
          float t[K * K];
#pragma unroll
          for (int a = 0; a < K; ++a)
#pragma unroll
            for (int b = 0; b < K; ++b)  // DIAG 5: no tap reads
              t[a * K + b] = RRAM_LRN_DIAG == 5 ? __builtin_bit_cast(float, it_l[i] + a + b) : yl[rowbase(a) + (b & 1) * HWC + (b >> 1)];
          // v_max3 over the taps: the strict-">" walk's value whenever the
          // maximum is not zero (a quiet NaN loses to any number in both; the
          // plane holds products, never a signalling NaN); for a zero maximum
          // the walk keeps the FIRST zero's sign where v_max takes +0 over
          // -0, so such a window is walked again in order
#pragma unroll
          for (int j = 0; j < K * K; j += 2) mv = max3f(mv, t[j], t[j + 1 < K * K ? j + 1 : j]);
          if (RRAM_LRN_DIAG != 6 && mv == 0.0f) {  // DIAG 6: no in-order re-walk
            mv = -FLT_MAX;
#pragma unroll
            for (int j = 0; j < K * K; ++j) mv = t[j] > mv ? t[j] : mv;
          }
        } else {
#pragma unroll
          for (int a = 0; a < K; ++a)
#pragma unroll
            for (int b = 0; b < K; ++b) {
              const bool ok = (it_ok[i] >> (a * K + b)) & 1u;
              const int tap = WT > 0 ? rowbase(a) + (b & 1) * HWC + (b >> 1) : a * W + b;
              const float v = yl[ok ? tap : -it_l[i]];  // masked taps read element 0
              if (ok && v > mv) mv = v;
            }
        }
        if (RRAM_LRN_DIAG != 4 && ys)  // DIAG 4: no y store
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, mv), yrs, it_vo[i], c0 * PHW * 4,
                                                RRAM_LRN_YNT);
        if (OCT) obuf[(c0 + d) & 7][it_out[i] - pr0 * PW] = mv;
      }
    }
  };
  // OCT: after each 8 channels (4 groups) the octet's companion
  char* yon = OCT ? yo + (int64_t)n * (C / 8) * PHW * 48 : nullptr;
  auto octet_out = [&](int c8) {
    __syncthreads();  // obuf complete (the next group's barrier orders its rewrite)
    // the band's outputs are consecutive (pr0 PW + o), so the octet's
    // companion run is NO x 48 contiguous bytes: thread p stores 16-byte piece
    // p (output p / 3, term p % 3), consecutive lanes on consecutive pieces
    // (one thread per output storing its three terms left each store
    // instruction 16 bytes per lane at a 48-byte stride)
    char* run = yon + ((int64_t)(c8 / 8) * PHW + (int64_t)pr0 * PW) * 48;
    for (int p = threadIdx.x; p < 3 * NO; p += kThreads) {
      const int o = p / 3, tt = p - 3 * o;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = obuf[e][o];
      x6::Parts t;
      x6::split8_safe(v, t);
      *reinterpret_cast<x6::bf16x8*>(run + p * 16) = tt == 0 ? t.h : tt == 1 ? t.m : t.l;
    }
  };
  // the walk: prime the window of group 0 and the entering channels of groups
  // 1 .. NS - 1 (positions 0 .. SIZE + NS D - 1), then 16 channels per trip
  auto walk = [&](auto dn) {
    constexpr bool DN = decltype(dn)::value;
    // UP: groups at cb, cb + 2, ...; DN: at top, top - 2, ... (top = the
    // highest group start; octets: ce - 2)
    const int top = OCT ? ce - D : cb + (ce - cb - 1) / D * D;
    const int first = DN ? top : cb;
    const int base = DN ? top - PRE + SIZE + D - 1 : cb - PRE;
#pragma unroll
    for (int r = 0; r < SIZE + NS * D; ++r) ring[r] = ld(DN ? base - r : base + r);
    if constexpr (CCT > 0) {
      // a chunk of exactly CCT channels (host check): the whole walk straight
      // line, no loop and no per-group branch, so the compiler's wait counts
      // stay exact (each group waits only for its own window's loads, NS
      // groups old; the loop form's back edge made it drain every load in
      // flight at the trip top and behind each group's loads)
      auto step = [&](auto gi) {
        constexpr int GG = decltype(gi)::value;
        const int cg = DN ? first - GG * D : first + GG * D;
        group(cg, gi, dn);
        if constexpr (OCT && (GG & 3) == 3) octet_out(DN ? cg : cg - 6);
      };
      [&]<int... I>(std::integer_sequence<int, I...>) {
        (step(std::integral_constant<int, I>{}), ...);
      }(std::make_integer_sequence<int, CCT / D>{});
      return;
    }
    for (int t0 = 0;; t0 += RL) {
      const int c0 = DN ? first - t0 : first + t0;  // group 0 of the trip
      auto live = [&](int c) { return DN ? c >= cb : c < ce; };
      if (!live(c0)) break;
      auto step = [&](auto gi) {
        constexpr int GG = decltype(gi)::value;
        const int cg = DN ? c0 - GG * D : c0 + GG * D;
        if (live(cg)) {
          group(cg, gi, dn);
          // the octet ends with the group at its top (UP) / bottom (DN)
          if constexpr (OCT && (GG & 3) == 3) octet_out(DN ? cg : cg - 6);
        }
      };
      step(std::integral_constant<int, 0>{});
      step(std::integral_constant<int, 1>{});
      step(std::integral_constant<int, 2>{});
      step(std::integral_constant<int, 3>{});
      step(std::integral_constant<int, 4>{});
      step(std::integral_constant<int, 5>{});
      step(std::integral_constant<int, 6>{});
      step(std::integral_constant<int, 7>{});
    }
  };
  // Odd channel chunks walk down (RRAM_LRN_ALT): chunk i's last halo channels
  // and chunk i + 1's first ones are then the same channels read at the same
  // time (both at the chunks' shared boundary, start or end of the walk), so
  // the second read can merge in the XCD's L2 instead of going to memory
  if (RRAM_LRN_ALT && (((rest - n * chunks) & 1) != 0))
    walk(std::true_type{});
  else
    walk(std::false_type{});
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
  RRAM_REQUIRE((int64_t)C * H * W * 4 < 2147483647ll && (int64_t)C * PH * PW * 4 < 2147483647ll,
               "lrn_maxpool_fwd: one image must be < 2 GiB");
  if (num == 0) return RRAM_OK;
  RRAM_REQUIRE(x && (y || y_oct), "lrn_maxpool_fwd: NULL (y may be NULL only with a companion)");
  // band height: input rows of RB pooled rows must fit the block's pixel
  // budget and RB * PW outputs its threads
  auto fits = [&](int rb) {
    const int rows = min(H, (rb - 1) * sh + kernel);
    return rb * PW <= kThreads && rows * W <= kBandPix;
  };
  RRAM_REQUIRE(fits(1), "lrn_maxpool_fwd: a pooled row needs more than %d input pixels", kBandPix);
  int rb = 1;
  while (rb < PH && fits(rb + 1)) ++rb;
  // the fewest bands at that height, then their rows evened out (AlexNet
  // norm2: 7 + 6 pooled rows, not 8 + 5, so no block carries 1.5x another's
  // pixels)
  if (RRAM_LRN_BAL) rb = (PH + (PH + rb - 1) / rb - 1) / ((PH + rb - 1) / rb);
  // channel chunks: as few as give >= kLrnBlocks blocks (each chunk re-reads
  // SIZE - 1 halo channels), equal sizes in multiples of 8 (2 * G without octets)
  const int step = y_oct ? 8 : 2 * kLrnG;
  const int bands = (PH + rb - 1) / rb;
  const int64_t tiles = (int64_t)num * bands;  // > 0
  // (targets of 1024 / 2048 / 4096 blocks measured within noise, AlexNet b256)
  const int64_t want = (kLrnBlocks + tiles - 1) / tiles;
  const int64_t most = (C + step - 1) / step;
  const int chunks = static_cast<int>(want < 1 ? 1 : (want > most ? most : want));
  const int cc = ((C + chunks - 1) / chunks + step - 1) / step * step;
  const int nchunks = (C + cc - 1) / cc;
  RRAM_REQUIRE((int64_t)bands * nchunks * num < 2147483647ll && num < 65536, "lrn_maxpool_fwd: grid too large");
  // (bands x chunks, images): the kernel maps the linear workgroup id to an
  // XCD-local tile order itself
  const dim3 grid(static_cast<unsigned>(bands * nchunks), static_cast<unsigned>(num));
  const float aos = alpha / size;
  char* yo = static_cast<char*>(y_oct);
#define RRAM_LP4(K_, S_, WT_, CCT_)                                                                             \
  if (yo)                                                                                                       \
    hipLaunchKernelGGL((k_lrn_maxpool_band<K_, S_, kLrnG, true, WT_, CCT_>), grid, dim3(kThreads), 0,          \
                       as_stream(s), x, y, yo, C, H, W, PH, PW, sh, sw, ph, pw, rb, cc, bands, nchunks, aos, beta, \
                       k);                                                                                      \
  else                                                                                                          \
    hipLaunchKernelGGL((k_lrn_maxpool_band<K_, S_, kLrnG, false, WT_, CCT_>), grid, dim3(kThreads), 0,         \
                       as_stream(s), x, y, yo, C, H, W, PH, PW, sh, sw, ph, pw, rb, cc, bands, nchunks, aos, beta, \
                       k);
  // AlexNet's planes (WT > 0) in whole 32-channel chunks take the
  // straight-line walk
#define RRAM_LP3(K_, S_, WT_)                          \
  if (WT_ > 0 && cc == 32 && C % 32 == 0) {            \
    RRAM_LP4(K_, S_, WT_, (WT_ > 0 ? 32 : 0))          \
  } else {                                             \
    RRAM_LP4(K_, S_, WT_, 0)                           \
  }
  // the WT plane rows are de-interleaved by a window stride of 2 and paired
  // two rows per pitch (a pooled row = two input rows down, from an even row)
  const bool wt_ok = sw == 2 && pw == 0 && sh == 2 && ph == 0;
#define RRAM_LP(K_, S_)                                  \
  if (kernel == K_ && size == S_) {                      \
    if (K_ == 3 && S_ == 5 && W == 55 && wt_ok) {        \
      RRAM_LP3(K_, S_, (K_ == 3 && S_ == 5 ? 55 : 0))    \
    } else if (K_ == 3 && S_ == 5 && W == 27 && wt_ok) { \
      RRAM_LP3(K_, S_, (K_ == 3 && S_ == 5 ? 27 : 0))    \
    } else {                                             \
      RRAM_LP3(K_, S_, 0)                                \
    }                                                    \
  }
  RRAM_LP(3, 5)
  else RRAM_LP(3, 3) else RRAM_LP(2, 5) else RRAM_LP(2, 3)
#undef RRAM_LP
#undef RRAM_LP3
#undef RRAM_LP4
  return launch_status("lrn_maxpool_fwd");
}

}  // extern "C"
