// dgs_lane.cuh -- cross-lane moves inside the 32-lane halves of a wave64 without the LDS
// crossbar.  HIP's __shfl_xor / __shfl_up / __shfl lower to ds_bpermute_b32, an LDS-unit round
// trip (address VGPR, then tens of cycles of latency) on every compare-exchange of the half-wave
// top-k networks, which run at one or two waves per SIMD where nothing hides that latency.
// The fixed patterns those networks use map onto VALU data-parallel-primitive (DPP) moves and
// gfx950's v_permlane16_swap_b32:
//   xor 1, 2    quad_perm [1,0,3,2] / [2,3,0,1]
//   xor 4       row_shl:4 into banks 0, 2 and row_shr:4 into banks 1, 3 (a bank = 4 lanes of a
//               16-lane row; lanes with bit 2 clear read lane + 4, the others lane - 4)
//   xor 8       row_ror:8 (a rotation by half a 16-lane row)
//   xor 16      v_permlane16_swap_b32 (swaps odd 16-lane rows of one operand with the even rows
//               of the other: with both operands x, row 2j reads row 2j + 1 from the second
//               result and row 2j + 1 reads row 2j from the first)
//   31 - l      row_mirror (15 - l inside each row), then xor 16
//   l - 1       row_shr:1 inside each row; lane 16 of each half takes lane 15 from the reversal
//               (branch-free: a select between readlanes of lanes 15 and 47 compiles to a branch)
// Every helper reads lanes of the caller's own half only, so it is safe when the two halves of a
// wave follow different control flow, but each half must be wholly active: a DPP move that reads
// a lane whose exec bit is clear does not see that lane's value.
// tools/lane_ops_test.hip checks each helper against the __shfl form on the GPU.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace dgs {

template <int kCtrl, int kBanks = 0xF>
__device__ __forceinline__ int32_t dpp_keep(int32_t old, int32_t x) {
  return __builtin_amdgcn_update_dpp(old, x, kCtrl, 0xF, kBanks, false);
}

// x of lane l ^ M (M in {1, 2, 4, 8, 16}; other masks fall back to the bpermute form).
template <int M>
__device__ __forceinline__ int32_t lane_xor32(int32_t x) {
  if constexpr (M == 1) {
    return dpp_keep<0xB1>(x, x);  // quad_perm [1,0,3,2]
  } else if constexpr (M == 2) {
    return dpp_keep<0x4E>(x, x);  // quad_perm [2,3,0,1]
  } else if constexpr (M == 4) {
    const int32_t t = dpp_keep<0x104, 0x5>(x, x);  // row_shl:4 -> banks 0, 2
    return dpp_keep<0x114, 0xA>(t, x);             // row_shr:4 -> banks 1, 3
  } else if constexpr (M == 8) {
    return dpp_keep<0x128>(x, x);  // row_ror:8
  } else if constexpr (M == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return (threadIdx.x & 16) ? (int32_t)r[0] : (int32_t)r[1];
  } else {
    return __shfl_xor(x, M, 32);
  }
}
template <int M>
__device__ __forceinline__ float lane_xor32(float x) {
  return __int_as_float(lane_xor32<M>(__float_as_int(x)));
}

// lane_xor32<m>(x) for a mask that is a constant once the caller's loop is unrolled.
template <typename T>
__device__ __forceinline__ T lane_xor32v(T x, int m) {
  switch (m) {
    case 1: return lane_xor32<1>(x);
    case 2: return lane_xor32<2>(x);
    case 4: return lane_xor32<4>(x);
    case 8: return lane_xor32<8>(x);
    case 16: return lane_xor32<16>(x);
    default: return __shfl_xor(x, m, 32);
  }
}

// x of lane 31 - l of this half.
__device__ __forceinline__ int32_t lane_rev32(int32_t x) {
  return lane_xor32<16>(dpp_keep<0x140>(x, x));  // row_mirror, then swap the two rows
}
__device__ __forceinline__ float lane_rev32(float x) {
  return __int_as_float(lane_rev32(__float_as_int(x)));
}

// x of lane l - 1 of this half (lane 0 of the half: its own x; callers ignore it).
__device__ __forceinline__ int32_t lane_up1_32(int32_t x) {
  const int32_t t = dpp_keep<0x111>(x, x);  // row_shr:1 (lane 0 of a row keeps x)
  const int32_t b = lane_rev32(x);           // at lane 16: lane 15
  return (threadIdx.x & 31) == 16 ? b : t;
}
__device__ __forceinline__ float lane_up1_32(float x) {
  return __int_as_float(lane_up1_32(__float_as_int(x)));
}

// x of lane q of this half, q the same on every lane of the wave (two scalar reads).
__device__ __forceinline__ int32_t half_bcast(int32_t x, int q) {
  const int32_t lo = __builtin_amdgcn_readlane(x, q);
  const int32_t hi = __builtin_amdgcn_readlane(x, q + 32);
  return (threadIdx.x & 32) ? hi : lo;
}
__device__ __forceinline__ float half_bcast(float x, int q) {
  return __int_as_float(half_bcast(__float_as_int(x), q));
}

}  // namespace dgs
