// gather.hip -- row gather kernels (feature server, index_select).
//
// Reference: feature_ops.cu:12-73 (_IndexP2PCacheKernel: one 128-thread block per row,
// 4-byte scalar loads, separate hashmap-lookup pass K18) and :140-171 (_IndexKernel).
//
// MI355X design: the output [n, row_bytes] is treated as one flat stream of V-byte chunks
// (V = 16 whenever alignment allows).  Consecutive lanes own consecutive output chunks, so
// every store instruction writes 64 * V contiguous bytes and every row read is a run of
// contiguous 16-byte lane loads; no lane idles for row sizes that are not a multiple of the
// wave width (d = 100 floats = 25 chunks).  Each thread keeps U independent row reads in
// flight before its stores.  For the feature server the node -> (location, row) lookup is
// fused into the same kernel (one 8-byte table load per row instead of a hash probe chain
// plus a second pass).
#include "dgs_common.h"
#include "dgs_ops.h"

namespace dgs {
namespace {

template <int V>
struct VecT;
template <>
struct VecT<16> {
  using T = uint4;
};
template <>
struct VecT<8> {
  using T = uint2;
};
template <>
struct VecT<4> {
  using T = uint32_t;
};
template <>
struct VecT<2> {
  using T = uint16_t;
};
template <>
struct VecT<1> {
  using T = uint8_t;
};

// x / d for 32-bit x via multiply-high (Granlund-Montgomery).
struct FastDivU32 {
  uint32_t d, m, s;
  static FastDivU32 make(uint32_t d) {
    FastDivU32 f;
    f.d = d;
    uint32_t s = 0;
    while ((uint64_t(1) << s) < d) ++s;
    f.s = s;
    f.m = (uint32_t)(((uint64_t(1) << 32) * ((uint64_t(1) << s) - d)) / d + 1);
    return f;
  }
  __device__ __forceinline__ uint32_t div(uint32_t x) const {
    return (uint32_t)(((uint64_t)__umulhi(x, m) + x) >> s);
  }
};

template <typename IdT>
struct PlainSrc {
  const char *data;
  const IdT *nid;
  int64_t row_bytes;
  int64_t row_base;
  __device__ __forceinline__ const char *row(uint32_t r) const {
    return data + (int64_t)nid[row_base + r] * row_bytes;
  }
};

struct TableSrc {
  const int64_t *ftab;
  const int64_t *nid;
  PtrTable bases;
  int64_t row_bytes;
  int64_t row_base;
  __device__ __forceinline__ const char *row(uint32_t r) const {
    const int64_t v = nid[row_base + r];
    const int64_t e = ftab[v];
    const int loc = (int)((uint64_t)e >> kLocShift);
    const int64_t idx = e & kOffMask;
    return reinterpret_cast<const char *>(bases.p[loc]) + idx * row_bytes;
  }
};

constexpr int kGatherThreads = 256;
constexpr int kGatherUnroll = 4;

template <int V, typename Src>
__global__ __launch_bounds__(kGatherThreads) void k_gather(Src src, uint32_t nchunks,
                                                           uint32_t cpr, FastDivU32 fd,
                                                           char *__restrict__ out) {
  using T = typename VecT<V>::T;
  const uint32_t base = blockIdx.x * (uint32_t)(kGatherThreads * kGatherUnroll) + threadIdx.x;
  T v[kGatherUnroll];
#pragma unroll
  for (int u = 0; u < kGatherUnroll; ++u) {
    const uint32_t g = base + u * kGatherThreads;
    if (g < nchunks) {
      const uint32_t r = fd.div(g);
      const uint32_t c = g - r * cpr;
      v[u] = *reinterpret_cast<const T *>(src.row(r) + (size_t)c * V);
    }
  }
#pragma unroll
  for (int u = 0; u < kGatherUnroll; ++u) {
    const uint32_t g = base + u * kGatherThreads;
    if (g < nchunks) *reinterpret_cast<T *>(out + (size_t)g * V) = v[u];
  }
}

template <typename Src>
void launch_gather_v(int V, Src src, int64_t n, int64_t row_bytes, char *out, hipStream_t st) {
  const int64_t cpr = row_bytes / V;
  DGS_CHECK(cpr > 0 && cpr < (int64_t(1) << 30), "gather: unsupported row size");
  const int64_t max_rows = ((int64_t(1) << 31) - kGatherThreads * kGatherUnroll) / cpr;
  const FastDivU32 fd = FastDivU32::make((uint32_t)cpr);
  for (int64_t r0 = 0; r0 < n; r0 += max_rows) {
    const int64_t rows = n - r0 < max_rows ? n - r0 : max_rows;
    Src s = src;
    s.row_base = r0;
    const uint32_t nchunks = (uint32_t)(rows * cpr);
    const dim3 grid((unsigned)ceil_div(nchunks, kGatherThreads * kGatherUnroll));
    char *o = out + r0 * row_bytes;
    switch (V) {
      case 16: hipLaunchKernelGGL((k_gather<16, Src>), grid, dim3(kGatherThreads), 0, st, s, nchunks, (uint32_t)cpr, fd, o); break;
      case 8: hipLaunchKernelGGL((k_gather<8, Src>), grid, dim3(kGatherThreads), 0, st, s, nchunks, (uint32_t)cpr, fd, o); break;
      case 4: hipLaunchKernelGGL((k_gather<4, Src>), grid, dim3(kGatherThreads), 0, st, s, nchunks, (uint32_t)cpr, fd, o); break;
      case 2: hipLaunchKernelGGL((k_gather<2, Src>), grid, dim3(kGatherThreads), 0, st, s, nchunks, (uint32_t)cpr, fd, o); break;
      default: hipLaunchKernelGGL((k_gather<1, Src>), grid, dim3(kGatherThreads), 0, st, s, nchunks, (uint32_t)cpr, fd, o); break;
    }
    DGS_LAUNCH_CHECK();
  }
}

int pick_vec(int64_t row_bytes, uintptr_t align_or) {
  for (int V = 16; V > 1; V >>= 1)
    if (row_bytes % V == 0 && (align_or % V) == 0) return V;
  return 1;
}

__global__ void k_ftab_init_host(int64_t *ftab, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ftab[i] = ((int64_t)kLocHost << kLocShift) | i;
}

__global__ void k_ftab_assign(int64_t *ftab, const int64_t *nids, int64_t n, int64_t loc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ftab[nids[i]] = (loc << kLocShift) | i;
}

}  // namespace

void gather_plain(const void *data, int64_t row_bytes, const void *nid, int nid_bytes,
                  int64_t n, void *out, hipStream_t st) {
  if (n <= 0 || row_bytes <= 0) return;
  const int V = pick_vec(row_bytes, (uintptr_t)data | (uintptr_t)out);
  profile_begin(st, 0);
  if (nid_bytes == 8) {
    PlainSrc<int64_t> s{(const char *)data, (const int64_t *)nid, row_bytes, 0};
    launch_gather_v(V, s, n, row_bytes, (char *)out, st);
  } else {
    DGS_CHECK(nid_bytes == 4, "index ids must be int32 or int64");
    PlainSrc<int32_t> s{(const char *)data, (const int32_t *)nid, row_bytes, 0};
    launch_gather_v(V, s, n, row_bytes, (char *)out, st);
  }
  profile_end(st, 0);
}

void gather_table(const int64_t *ftab, PtrTable bases, int64_t row_bytes, const int64_t *nids,
                  int64_t n, void *out, hipStream_t st) {
  if (n <= 0 || row_bytes <= 0) return;
  uintptr_t a = (uintptr_t)out;
  for (int i = 0; i <= kMaxDevices; ++i) a |= (uintptr_t)bases.p[i];
  const int V = pick_vec(row_bytes, a);
  TableSrc s{ftab, nids, bases, row_bytes, 0};
  profile_begin(st, 0);
  launch_gather_v(V, s, n, row_bytes, (char *)out, st);
  profile_end(st, 0);
}

void ftab_init_host(int64_t *ftab, int64_t n, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_ftab_init_host, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, ftab,
                     n);
  DGS_LAUNCH_CHECK();
}

void ftab_assign(int64_t *ftab, const int64_t *nids, int64_t n, int loc, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_ftab_assign, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, ftab,
                     nids, n, (int64_t)loc);
  DGS_LAUNCH_CHECK();
}

}  // namespace dgs
