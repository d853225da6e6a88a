// Exact 32-bit modulo forms of the uniform reservoir (rowwise_sampling.cu:85-92 draws
// `curand(&rng) % (idx + 1)`): fp32-estimated quotients with integer corrections, each exact on
// its stated range.  Shared by csrc/sample.hip and the exhaustive checker tools/modfuzz.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace dgs {

// x mod d, exact for 2^12 <= d < 2^30 (kU24: d < 2^24).  x/d < 2^20, and the fp32 estimate
// x * rcp(d) carries a relative error <= 2^-22 (x and d conversions 2^-24 each, v_rcp_f32 1
// ulp), i.e. <= 0.25 absolute; the fma's own rounding adds <= 2^-4.  Biased by -0.5, the
// estimate lies in [x/d - 0.8125, x/d - 0.1875], so its truncation q is floor(x/d) or one less:
// r = x - q*d is in [0, 2d) and one conditional subtract finishes (the generic % spends four
// quarter-rate multiplies).  With d < 2^24 both factors of q*d fit 24 bits and the product is
// the full-rate v_mul_u32_u24 instead of the quarter-rate v_mul_lo_u32.
// tools/modfuzz.hip: every x for ~1K divisors + 2^34 random pairs, 0 mismatches.
constexpr uint32_t kModBigMin = 4096;
// Low 32 bits of the product of two values below 2^24, on the full-rate 24-bit multiplier
// (the compiler lowers __umul24's masks to v_mul_lo_u32 when it cannot bound the operands).
__device__ __forceinline__ uint32_t umul24(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
template <bool kU24>
__device__ __forceinline__ uint32_t mod_big(uint32_t x, uint32_t d) {
  const float rcp = __builtin_amdgcn_rcpf((float)d);
  const uint32_t q = (uint32_t)(int32_t)__builtin_fmaf((float)x, rcp, -0.5f);
  const uint32_t r = x - (kU24 ? umul24(q, d) : q * d);
  return r >= d ? r - d : r;
}

// x mod d, exact for 1 <= d <= kModMidMax (kU24: 257 <= d <= kModMidMax).  Step 1: q1 =
// trunc(x * rcp(d)) is within 1024/d + 1 of x/d (relative error <= 2^-22 on x/d < 2^32/d), so
// r1 = x - q1*d (wrapping 32-bit arithmetic) is an exact int32 with |r1| <= 1024 + d.  Step 2:
// r1 * rcp(d) has absolute error <= (1024/d + 1) * 2^-22.4, below the 1/d distance of any
// non-integer r1/d from the next integer, so floor() is exact unless r1/d is an integer, where it
// may be one low; r2 = r1 - q2*d is then exact in fp32 (an fma of integers below 2^24) and lies
// in [0, d]: one compare finishes.  kU24: q1 < 2^32/257 + 1 < 2^24, so q1*d is v_mul_u32_u24.
// One quarter-rate op (the rcp) + one mul (kU24: full rate) against the generic %'s five.
// tools/modfuzz.hip: every (x, d) with x < 2^32 and d <= kModMidMax, 0 mismatches.
constexpr uint32_t kModMidMax = 8192;
template <bool kU24>
__device__ __forceinline__ uint32_t mod_mid(uint32_t x, uint32_t d) {
  const float df = (float)d;
  const float rcp = __builtin_amdgcn_rcpf(df);
  const uint32_t q1 = (uint32_t)((float)x * rcp);
  const int32_t r1 = (int32_t)(x - (kU24 ? umul24(q1, d) : q1 * d));
  const float r1f = (float)r1;
  const float q2 = __builtin_floorf(r1f * rcp);
  const uint32_t r = (uint32_t)(int32_t)__builtin_fmaf(-q2, df, r1f);
  return r >= d ? r - d : r;
}

}  // namespace dgs
