// dgs_block.cuh -- wave64 / workgroup primitives (device only).
#pragma once

#include "dgs_common.h"

namespace dgs {

// Inclusive scan across the 64 lanes of a wave.
template <typename T>
__device__ __forceinline__ T wave_inclusive_scan(T x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  return x;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

// Workgroup exclusive scan of one value per thread (THREADS a multiple of 64, <= 4096).
// `lds` must hold THREADS/64 values.  Returns the exclusive prefix; *total = sum.
template <int THREADS, typename T>
__device__ __forceinline__ T block_exclusive_scan(T v, T *total, T *lds) {
  constexpr int W = THREADS / 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  T x = wave_inclusive_scan(v);
  if (lane == 63) lds[wid] = x;
  __syncthreads();
  if (wid == 0) {
    T w = lane < W ? lds[lane] : T(0);
    w = wave_inclusive_scan(w);
    if (lane < W) lds[lane] = w;
  }
  __syncthreads();
  const T wave_prefix = wid ? lds[wid - 1] : T(0);
  *total = lds[W - 1];
  __syncthreads();
  return wave_prefix + x - v;
}

template <int THREADS, typename T>
__device__ __forceinline__ T block_sum(T v, T *lds) {
  constexpr int W = THREADS / 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  T x = wave_sum(v);
  if (lane == 0) lds[wid] = x;
  __syncthreads();
  T t = T(0);
#pragma unroll
  for (int i = 0; i < W; ++i) t += lds[i];
  __syncthreads();
  return t;
}

// out[i] = carry + exclusive prefix of in[0..n) for one workgroup; each thread owns ITEMS
// contiguous elements per pass (one block scan per THREADS * ITEMS elements).  Returns the
// total.  `in` may be null (reads as zeros).  Call from every thread of the workgroup.
template <int THREADS, int ITEMS, typename T>
__device__ __forceinline__ T block_scan_range(const T *in, int64_t n, T *out, T *lds) {
  T carry = T(0);
  for (int64_t base = 0; base < n; base += (int64_t)THREADS * ITEMS) {
    const int64_t b = base + (int64_t)threadIdx.x * ITEMS;
    T v[ITEMS];
    T s = T(0);
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      v[j] = (b + j < n) ? in[b + j] : T(0);
      s += v[j];
    }
    T tot;
    T ex = block_exclusive_scan<THREADS>(s, &tot, lds) + carry;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      if (b + j < n) out[b + j] = ex;
      ex += v[j];
    }
    carry += tot;
  }
  return carry;
}

}  // namespace dgs
