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
// exact three-term split of 8 floats (round to nearest even at each step)
__device__ __forceinline__ void split8(const float (&x)[8], Parts& r) {
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float2v v = {x[2 * p], x[2 * p + 1]};
    const bf16x2 h = __builtin_convertvector(v, bf16x2);
    const float2v r1 = v - __builtin_convertvector(h, float2v);
    const bf16x2 m = __builtin_convertvector(r1, bf16x2);
    const float2v r2 = r1 - __builtin_convertvector(m, float2v);
    const bf16x2 l = __builtin_convertvector(r2, bf16x2);
    r.h[2 * p] = h[0];
    r.h[2 * p + 1] = h[1];
    r.m[2 * p] = m[0];
    r.m[2 * p + 1] = m[1];
    r.l[2 * p] = l[0];
    r.l[2 * p + 1] = l[1];
  }
}
// term p (0 = high, 1 = middle, 2 = low) of the split of v, as bf16 bits
__device__ __forceinline__ uint16_t split_term(float v, int p) {
  const __bf16 h = static_cast<__bf16>(v);
  const float r1 = v - static_cast<float>(h);
  const __bf16 m = static_cast<__bf16>(r1);
  const __bf16 l = static_cast<__bf16>(r1 - static_cast<float>(m));
  const __bf16 t = p == 0 ? h : p == 1 ? m : l;
  return __builtin_bit_cast(uint16_t, t);
}
// the three bf16 terms of 8 floats as 3 x 16 bytes at dst (16-byte aligned)
__device__ __forceinline__ void store_terms8(const float (&v)[8], char* dst) {
  Parts t;
  split8(v, t);
  *reinterpret_cast<bf16x8*>(dst) = t.h;
  *reinterpret_cast<bf16x8*>(dst + 16) = t.m;
  *reinterpret_cast<bf16x8*>(dst + 32) = t.l;
}
}  // namespace x6
}  // namespace
}  // namespace rram
