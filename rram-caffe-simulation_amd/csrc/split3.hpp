// The exact three-term bf16 split of fp32 operands shared by the bf16x6
// kernels (x6.hip) and the producers that write a tensor's pre-split
// channel-octet companion (fused.hip): x = xh + xm + xl, each term the
// round-to-nearest-even bf16 of the remainder (the remainders are exact in
// fp32 and the third term holds the last 8 significand bits).
#pragma once
#include <stdint.h>

namespace rram {
namespace {
namespace x6 {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float float2v __attribute__((ext_vector_type(2)));
struct Parts {
  bf16x8 h, m, l;
};
// The plain split (each term = bf16 round-to-nearest-even of the remainder)
// is exact for every finite |x| up to the largest bf16
// (BF16_MAX = 0x1.fep127); past it the high term rounds to Inf, and an Inf
// operand gives Inf - Inf = NaN in the middle term where the fp32 product the
// reference forms is +-Inf.  The safe form clamps each term's input to
// [-BF16_MAX, BF16_MAX] before rounding (two v_med3 per element, nothing else):
//   |x| <= BF16_MAX            the same terms as split8 (bit for bit);
//   BF16_MAX < |x| <= FLT_MAX  high = +-BF16_MAX, the remainder split exactly;
//   x = +-Inf                  (+-BF16_MAX, +-BF16_MAX, +-Inf): every product
//                              with a nonzero operand is +-Inf, with 0 NaN, as in fp32;
//   NaN                        NaN reaches the low term.
// Every split of the engine uses it (the pack kernels, the conv1 staging and
// the in-loop splits of k_conv_patch_x6 / k_gemm_x6), so the engine's
// products of non-finite or > BF16_MAX operands follow fp32's.
constexpr float kBf16Max = 0x1.fep127f;
__device__ __forceinline__ float2v clamp_bf16(float2v v) {
  return float2v{__builtin_amdgcn_fmed3f(v[0], -kBf16Max, kBf16Max), __builtin_amdgcn_fmed3f(v[1], -kBf16Max, kBf16Max)};
}
__device__ __forceinline__ float2v bf16_high_safe(float2v v, bf16x2& h) {
  h = __builtin_convertvector(clamp_bf16(v), bf16x2);
  return v - __builtin_convertvector(h, float2v);
}
__device__ __forceinline__ void split8_safe(const float (&x)[8], Parts& r) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4 hw, mw, lw;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float2v v = {x[2 * p], x[2 * p + 1]};
    bf16x2 h;
    const float2v r1 = bf16_high_safe(v, h);
    const bf16x2 m = __builtin_convertvector(clamp_bf16(r1), bf16x2);
    const float2v r2 = r1 - __builtin_convertvector(m, float2v);
    const bf16x2 l = __builtin_convertvector(r2, bf16x2);
    hw[p] = __builtin_bit_cast(uint32_t, h);
    mw[p] = __builtin_bit_cast(uint32_t, m);
    lw[p] = __builtin_bit_cast(uint32_t, l);
  }
  r.h = __builtin_bit_cast(bf16x8, hw);
  r.m = __builtin_bit_cast(bf16x8, mw);
  r.l = __builtin_bit_cast(bf16x8, lw);
}
// term p (0 = high, 1 = middle, 2 = low) of the split of v, as bf16 bits
__device__ __forceinline__ uint16_t split_term(float v, int p) {
  bf16x2 h;
  const float2v r1 = bf16_high_safe(float2v{v, 0.0f}, h);
  const __bf16 m = static_cast<__bf16>(__builtin_amdgcn_fmed3f(r1[0], -kBf16Max, kBf16Max));
  const __bf16 l = static_cast<__bf16>(r1[0] - static_cast<float>(m));
  const uint32_t hb = __builtin_bit_cast(uint32_t, h) & 0xFFFFu;
  return p == 0 ? static_cast<uint16_t>(hb) : __builtin_bit_cast(uint16_t, p == 1 ? m : l);
}
// the three bf16 terms of 8 floats as 3 x 16 bytes at dst (16-byte aligned)
__device__ __forceinline__ void store_terms8(const float (&v)[8], char* dst) {
  Parts t;
  split8_safe(v, t);
  *reinterpret_cast<bf16x8*>(dst) = t.h;
  *reinterpret_cast<bf16x8*>(dst + 16) = t.m;
  *reinterpret_cast<bf16x8*>(dst + 32) = t.l;
}
}  // namespace x6
}  // namespace
}  // namespace rram
