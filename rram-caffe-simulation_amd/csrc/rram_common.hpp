// Shared helpers for the gfx950 kernels: status plumbing, launch geometry and
// the counter-based RNG (Philox4x32-10) used by every random draw.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "rram_kernels.h"

namespace rram {

// ---------------------------------------------------------------------------
// Status plumbing: every C-ABI entry returns an int and records a message.
// ---------------------------------------------------------------------------
void set_error(const char* fmt, ...);
void clear_error();

#define RRAM_REQUIRE(cond, ...)                 \
  do {                                          \
    if (!(cond)) {                              \
      ::rram::set_error(__VA_ARGS__);           \
      return RRAM_EINVAL;                       \
    }                                           \
  } while (0)

#define RRAM_HIP_RET(expr)                                                   \
  do {                                                                       \
    hipError_t e_ = (expr);                                                  \
    if (e_ != hipSuccess) {                                                  \
      ::rram::set_error("%s: %s", #expr, hipGetErrorString(e_));             \
      return RRAM_EHIP;                                                      \
    }                                                                        \
  } while (0)

// Check the launch just issued (hipGetLastError) and return its status.
int launch_status(const char* what);

inline hipStream_t as_stream(rram_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// Streaming-kernel geometry: 256 threads, at most 8 blocks per CU x 256 CUs,
// grid-stride beyond that (cdna_hip_programming.md Guideline 11).
constexpr int kThreads = 256;
constexpr int kMaxStreamBlocks = 2048;
inline int stream_blocks(int64_t work_items) {
  int64_t b = (work_items + kThreads - 1) / kThreads;
  if (b < 1) b = 1;
  if (b > kMaxStreamBlocks) b = kMaxStreamBlocks;
  return static_cast<int>(b);
}

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11), host + device.  Counter layout used by
// the fault draws: {index_lo, index_hi, map_id, (layer_id << 4) | purpose},
// key = {seed_lo, seed_hi}.
// ---------------------------------------------------------------------------
struct U32x4 {
  uint32_t x, y, z, w;
};

// a ^ b ^ c; one v_bitop3_b32 (gfx950) on the device
__host__ __device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

__host__ __device__ __forceinline__ U32x4 philox4x32_10(U32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = static_cast<uint64_t>(0xD2511F53u) * c.x;
    const uint64_t p1 = static_cast<uint64_t>(0xCD9E8D57u) * c.z;
    const uint32_t hi0 = static_cast<uint32_t>(p0 >> 32), lo0 = static_cast<uint32_t>(p0);
    const uint32_t hi1 = static_cast<uint32_t>(p1 >> 32), lo1 = static_cast<uint32_t>(p1);
    c = U32x4{xor3(hi1, c.y, k0), lo1, xor3(hi0, c.w, k1), lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

enum Purpose : uint32_t {
  kPurposeFault = 0,     // broken / stuck-value words
  kPurposeVariation = 1, // Box-Muller words for lognormal variation
  kPurposePairFault = 2, // differential-pair cell faults
  kPurposePairVar = 3,   // differential-pair variation
  kPurposeEndurance = 4, // endurance normal draw (fault_init)
  kPurposeFill = 5,      // fillers
  kPurposeDropout = 6,
};

__host__ __device__ __forceinline__ U32x4 draw(uint64_t seed, uint64_t index, uint32_t map_id,
                                               uint32_t layer_id, uint32_t purpose) {
  U32x4 c{static_cast<uint32_t>(index), static_cast<uint32_t>(index >> 32), map_id,
          (layer_id << 4) | (purpose & 15u)};
  return philox4x32_10(c, static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32));
}

// LRN ACROSS_CHANNELS arithmetic (lrn_layer.cu:9-78), shared by the unfused
// kernel (layers.hip) and the LRN+pool fusion (fused.hip) so both produce the
// same bits: explicit fmaf leaves nothing to the compiler's contraction choice.
__device__ __forceinline__ float lrn_sq_add(float acc, float v) { return fmaf(v, v, acc); }
__device__ __forceinline__ float lrn_scale(float acc, float alpha_over_size, float k) {
  return fmaf(acc, alpha_over_size, k);
}
// x * scale^-beta via the raw v_log_f32 / v_exp_f32 (scale >= k > 0).  The
// libm-style log2f / exp2f wrap each in denormal range scaling (two
// v_ldexp + compares + selects per call); neither applies here: scale >= k
// is normal for any LRN k >= 2^-126, and scale^-beta >= FLT_MAX^-beta is
// normal for beta < 1 (Caffe's 0.75), with exp2 of a tinier argument
// flushing to 0 as powf's would round to a denormal.
__device__ __forceinline__ float lrn_out(float x, float scale, float beta) {
  return x * __builtin_amdgcn_exp2f(-beta * __builtin_amdgcn_logf(scale));
}
// The same three steps on two pixels at once: v_pk_fma_f32 / v_pk_mul_f32 are
// two IEEE fmas / multiplies per instruction (half the issue of two scalar
// ones), so each component is the scalar helpers' value bit for bit.
// win[j] = the SIZE channels' values of the two pixels in channel order.
typedef float f32x2 __attribute__((ext_vector_type(2)));
template <int SIZE>
__device__ __forceinline__ f32x2 lrn_value2(const f32x2* win, float alpha_over_size, float beta, float k) {
  f32x2 acc = {0.0f, 0.0f};
#pragma unroll
  for (int j = 0; j < SIZE; ++j) acc = __builtin_elementwise_fma(win[j], win[j], acc);
  const f32x2 sc = __builtin_elementwise_fma(acc, f32x2{alpha_over_size, alpha_over_size}, f32x2{k, k});
  const f32x2 e = f32x2{-beta, -beta} * f32x2{__builtin_amdgcn_logf(sc.x), __builtin_amdgcn_logf(sc.y)};
  return win[(SIZE - 1) / 2] * f32x2{__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)};
}

// 32-bit word -> uniform in (0, 1] (never 0: safe for log) and [0, 1).
__host__ __device__ __forceinline__ float u01_open0(uint32_t r) {
  return (static_cast<float>(r >> 8) + 1.0f) * (1.0f / 16777216.0f);
}
__host__ __device__ __forceinline__ float u01(uint32_t r) {
  return static_cast<float>(r >> 8) * (1.0f / 16777216.0f);
}

// Call options of the bf16x6 convolution forward.  The packed-weight
// companion (rram_conv2d_fwd_cached): the engine's pre-split fragment form of
// w in a caller-owned buffer that outlives the call, so weights that do not
// change between calls (Monte-Carlo inference: only the faultable blobs are
// rewritten) are split once.  y_img: the output's image stride in floats
// (rram_conv2d_fwd_strided: y inside a larger NCHW tensor, e.g. a Concat top
// at a channel offset); 0 = dense (num_output * Ho * Wo).
struct WPack {
  void* p = nullptr;         // caller's buffer (nullptr: the per-stream scratch buffer)
  bool valid = false;        // p already holds this shape's pack of w: launch no pack kernel
  size_t* query = nullptr;   // set: report the pack bytes of the engine that would run, launch nothing
  int64_t y_img = 0;
};
int conv_x6_fwd(const rram_conv_desc* d, const float* x, const void* x_oct, const float* w, const float* bias,
                float* y, void* y_oct, int relu, hipStream_t s, const WPack& wk = WPack{});
}  // namespace rram
