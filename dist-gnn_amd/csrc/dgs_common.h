// dgs_common.h -- shared host/device utilities for the DGS-AMD HIP library (gfx950).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

namespace dgs {

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define DGS_HIP(call)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (call);                                                             \
    if (e_ != hipSuccess)                                                               \
      throw ::dgs::Error(std::string(#call) + " failed: " + hipGetErrorString(e_) +     \
                         " (" + __FILE__ + ":" + std::to_string(__LINE__) + ")");       \
  } while (0)

#define DGS_CHECK(cond, msg)                                                            \
  do {                                                                                  \
    if (!(cond)) throw ::dgs::Error(std::string("DGS check failed: ") + (msg));         \
  } while (0)

// Launch-error check after a kernel launch (no sync).
#define DGS_LAUNCH_CHECK() DGS_HIP(hipGetLastError())

constexpr int kWave = 64;

// Grow-only device scratch buffer owned by a service object.
struct DevBuf {
  void *p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  // Returns true when (re)allocated (contents undefined).
  bool ensure(size_t need) {
    if (need <= bytes && p) return false;
    release();
    size_t n = need < 256 ? 256 : need;
    DGS_HIP(hipMalloc(&p, n));
    bytes = n;
    return true;
  }
  template <typename T>
  T *as() const {
    return reinterpret_cast<T *>(p);
  }
};

// Temporary device buffer of a setup-time or synchronous call: hipMalloc now; on scope exit the
// stream is synchronised, then hipFree.  (The library keeps away from the stream-ordered
// allocator, hipMallocAsync / hipFreeAsync: see DESIGN.md section 3.)
struct TmpBuf {
  void *p = nullptr;
  hipStream_t st = nullptr;
  TmpBuf(size_t bytes, hipStream_t s) : st(s) { DGS_HIP(hipMalloc(&p, bytes ? bytes : 1)); }
  TmpBuf(const TmpBuf &) = delete;
  TmpBuf &operator=(const TmpBuf &) = delete;
  ~TmpBuf() {
    if (p) {
      (void)hipStreamSynchronize(st);
      (void)hipFree(p);
    }
  }
  template <typename T>
  T *as() const {
    return reinterpret_cast<T *>(p);
  }
};

// Pinned host staging for small D2H size reads.
struct HostPinned {
  void *p = nullptr;
  size_t bytes = 0;
  unsigned flags = hipHostMallocDefault;
  ~HostPinned() {
    if (p) (void)hipHostFree(p);
  }
  void ensure(size_t need) {
    if (need <= bytes && p) return;
    if (p) (void)hipHostFree(p);
    DGS_HIP(hipHostMalloc(&p, need, flags));
    bytes = need;
  }
  template <typename T>
  T *as() const {
    return reinterpret_cast<T *>(p);
  }
};

// Sizes a kernel publishes to the host without a copy or a stream synchronisation: `n` device
// words are written to coherent pinned host memory host[1..n], then host[0] = seq with a
// system-scope release (HostSizes{} = nothing to publish).
struct HostSizes {
  const int64_t *dev = nullptr;
  int64_t n = 0;
  int64_t *host = nullptr;  // device-visible address of the pinned block
  uint64_t seq = 0;
};

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline uint64_t next_pow2(uint64_t x) {
  uint64_t c = 1;
  while (c < x) c <<= 1;
  return c;
}

// ---------------------------------------------------------------------------------
// Node-location encoding used by the graph shard context and the feature table.
// A location is 0..kMaxDevices-1 (a GPU rank of the communicator) or kLocHost.
constexpr int kMaxDevices = 8;
constexpr int kLocHost = kMaxDevices;  // index into pointer tables
constexpr int kLocShift = 56;
constexpr int64_t kOffMask = (int64_t(1) << kLocShift) - 1;

// Per-location base pointers, passed by value in kernel arguments (no device-side
// pointer table indirection).
struct PtrTable {
  const void *p[kMaxDevices + 1];
};

// Graph node table entry (16 B, one load per seed):
//   ptr = absolute (device-accessible) address of the node's first neighbour id in whichever
//         location holds its row (local HBM cache, a peer's IPC-mapped cache, mapped host),
//   dl  = degree | (location << 56)  (the location only selects the probs array).
struct NodeEntry {
  const int64_t *ptr;
  int64_t dl;
};

// A count that is either known on the host (p == nullptr) or produced on the device by an
// earlier kernel of the same stream (then `v` is only an upper bound used to size grids and
// buffers).  Lets a whole multi-hop sample run without host synchronisation.
struct Count {
  int64_t v;
  const int64_t *p;
#ifdef __HIPCC__
  __device__ __forceinline__ int64_t get() const { return p ? *p : v; }
#endif
};

// ---------------------------------------------------------------------------------
// Device helpers
#ifdef __HIPCC__
// Global-address-space view of a pointer that came from memory (a node-table entry, a hub
// record): loads through it are global_load, not flat_load.  Flat loads count on lgkmcnt as
// well as vmcnt and complete out of order, so every LDS / shuffle / scalar-load wait would also
// wait for them and no wait could be counted.
template <typename T>
using global_ptr = const __attribute__((address_space(1))) T *;
template <typename T>
__device__ __forceinline__ global_ptr<T> as_global(const T *p) {
  return (global_ptr<T>)(uintptr_t)p;
}

// a ^ b ^ c in one gfx950 v_bitop3_b32 (truth table 0x96) instead of two v_xor_b32
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Philox4x32-10 (curand / Random123 layout).  Each 32x32 product is one 64-bit multiply
// (v_mad_u64_u32, a quarter-rate instruction: 4.4 v_fma_f32 issue slots measured,
// tools/valu_bench.hip) instead of a mul_lo + mul_hi pair; each round's two 3-input XORs are one
// v_bitop3_b32 each.  Round 0 keeps plain XORs: its inputs are often wave-uniform (counter word
// 0 and the key), and scalar instructions do that round for free.
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k.x += 0x9E3779B9u;
      k.y += 0xBB67AE85u;
    }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    if (r == 0)
      c = make_uint4((uint32_t)(p1 >> 32) ^ c.y ^ k.x, (uint32_t)p1,
                     (uint32_t)(p0 >> 32) ^ c.w ^ k.y, (uint32_t)p0);
    else
      c = make_uint4(xor3((uint32_t)(p1 >> 32), c.y, k.x), (uint32_t)p1,
                     xor3((uint32_t)(p0 >> 32), c.w, k.y), (uint32_t)p0);
  }
  return c;
}

// The ten round keys of philox4x32_10 (for a loop over many blocks under one key: the schedule's
// additions once, not per block).
struct PhiloxKeys {
  uint32_t x[10], y[10];
};
__device__ __forceinline__ PhiloxKeys philox_keys(uint2 k) {
  PhiloxKeys K;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    K.x[r] = k.x + (uint32_t)r * 0x9E3779B9u;
    K.y[r] = k.y + (uint32_t)r * 0xBB67AE85u;
  }
  return K;
}
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, const PhiloxKeys &K) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    if (r == 0)
      c = make_uint4((uint32_t)(p1 >> 32) ^ c.y ^ K.x[0], (uint32_t)p1,
                     (uint32_t)(p0 >> 32) ^ c.w ^ K.y[0], (uint32_t)p0);
    else
      c = make_uint4(xor3((uint32_t)(p1 >> 32), c.y, K.x[r]), (uint32_t)p1,
                     xor3((uint32_t)(p0 >> 32), c.w, K.y[r]), (uint32_t)p0);
  }
  return c;
}

// Issue priority of the latency-bound per-hop kernels (prep, row sampling, compaction,
// relabel) over co-resident waves of the throughput-bound hub kernels of other batches in
// flight (s_setprio; 0 = the hardware default).
#ifndef DGS_LAT_PRIO
#define DGS_LAT_PRIO 1
#endif
__device__ __forceinline__ void latency_prio() {
#if DGS_LAT_PRIO
  __builtin_amdgcn_s_setprio(DGS_LAT_PRIO);
#endif
}

// Wave-uniform 64-bit value -> scalar registers.
__device__ __forceinline__ uint64_t wave_uniform(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t u4_get(const uint4 &v, int w) {
  return w == 0 ? v.x : (w == 1 ? v.y : (w == 2 ? v.z : v.w));
}

// curand_uniform(): x * 2^-32 + 2^-33.  The product of the (rounded) float x with a power of
// two is exact, so the reference's multiply-then-add rounds once, in the add: one fma gives
// the same bits.
__device__ __forceinline__ float curand_uniform_from(uint32_t x) {
  return __builtin_fmaf((float)x, 2.3283064365386963e-10f, 1.1641532182693481e-10f);
}
#endif

}  // namespace dgs
