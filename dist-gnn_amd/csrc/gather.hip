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
// flight before its stores, and the stores are non-temporal.  For the feature server the
// node -> (location, row) lookup is fused into the same kernel: computed outright when every
// node is cached in an identity / v-mod-W layout (StridedSrc), otherwise one 8-byte address
// table load per row (TableSrc) instead of a hash probe chain plus a second pass.
#include <hip/hip_ext.h>

#include "context.h"
#include "dgs_common.h"
#include "dgs_ops.h"

namespace dgs {
namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
template <int V>
struct VecT;
// Global-address-space pointer: row addresses come from memory, so without this the
// compiler emits flat loads (counted on both vmcnt and lgkmcnt).
template <typename T>
using gptr = const __attribute__((address_space(1))) T *;
template <typename T>
__device__ __forceinline__ gptr<T> to_global(const void *p) {
  return (gptr<T>)(uintptr_t)p;
}

// Pins a loaded value in registers at this point: keeps the compiler from sinking the load
// into the (conditional) store branch, which would serialise the unrolled chunks again.
__device__ __forceinline__ void keep(const u32x4 &v) { asm volatile("" ::"v"(v)); }
__device__ __forceinline__ void keep(const u32x2 &v) { asm volatile("" ::"v"(v)); }
__device__ __forceinline__ void keep(uint32_t v) { asm volatile("" ::"v"(v)); }
__device__ __forceinline__ void keep(uint16_t v) { asm volatile("" ::"v"((uint32_t)v)); }
__device__ __forceinline__ void keep(uint8_t v) { asm volatile("" ::"v"((uint32_t)v)); }
template <>
struct VecT<16> {
  using T = u32x4;
};
template <>
struct VecT<8> {
  using T = u32x2;
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

// Row sources.  row_ptr(r) = address of output row r's source row.  Each is split in two
// stages (id load, then address) so the kernel can batch the loads of its U chunks.
template <typename IdT>
struct PlainSrc {
  const char *data;
  const IdT *nid;
  int64_t row_bytes;
  int64_t row_base;
  using Key = int64_t;
  __device__ __forceinline__ Key key(uint32_t r) const { return (int64_t)nid[row_base + r]; }
  __device__ __forceinline__ const char *addr(Key k) const { return data + k * row_bytes; }
};

// Feature-server source: ftab[nid] holds the absolute address of the node's row (local HBM
// cache, a peer GPU's IPC-mapped cache, or mapped host memory), so the fused lookup is one
// 8-byte load per row with no per-location base indexing.
struct TableSrc {
  const int64_t *ftab;
  const int64_t *nid;
  int64_t row_bytes;  // unused (kept for a uniform launcher)
  int64_t row_base;
  using Key = int64_t;
  __device__ __forceinline__ Key key(uint32_t r) const { return nid[row_base + r]; }
  __device__ __forceinline__ const char *addr(Key k) const {
    return reinterpret_cast<const char *>(to_global<int64_t>(ftab)[k]);
  }
};

// Strided source (see gather_strided): loc = v & (W - 1), row = v >> wshift; the base is
// picked with a select chain (a dynamically indexed kernel argument would go to scratch).
template <bool Strided>
struct StridedSrc {
  const int64_t *nid;
  const char *b0, *b1, *b2, *b3, *b4, *b5, *b6, *b7;
  int64_t row_bytes;
  int64_t row_base;
  uint32_t wshift;
  using Key = int64_t;
  __device__ __forceinline__ Key key(uint32_t r) const { return nid[row_base + r]; }
  __device__ __forceinline__ const char *addr(Key k) const {
    if (!Strided) return b0 + k * row_bytes;
    const uint32_t loc = (uint32_t)k & ((1u << wshift) - 1u);
    const char *b = b0;
    b = loc == 1 ? b1 : b;
    b = loc == 2 ? b2 : b;
    b = loc == 3 ? b3 : b;
    b = loc == 4 ? b4 : b;
    b = loc == 5 ? b5 : b;
    b = loc == 6 ? b6 : b;
    b = loc == 7 ? b7 : b;
    return b + (k >> wshift) * row_bytes;
  }
};

#ifndef DGS_GATHER_PRIO
#define DGS_GATHER_PRIO 1
#endif
#ifndef DGS_GATHER_UNROLL
#define DGS_GATHER_UNROLL 4
#endif
// One-wave workgroups: inside the pipeline the gather's workgroups wait for free slots on CUs
// the sampling kernels of the other batches hold, and a one-wave workgroup fits where a
// four-wave one does not (dispatch spread 24.5 -> 19.6 us, in-pipeline fraction 0.46 -> 0.50;
// alone unchanged)
#ifndef DGS_GATHER_THREADS
#define DGS_GATHER_THREADS 64
#endif
constexpr int kGatherThreads = DGS_GATHER_THREADS;
constexpr int kGatherUnroll = DGS_GATHER_UNROLL;
// Large 16-byte-chunk gathers take 8 chunks per lane (half the workgroups to dispatch: inside
// the pipeline the gather's span is mostly the dispatch of its one-wave workgroups).  Round 5,
// same box, 5 rounds: products-like uniform (3.2 M chunks per launch) gather 0.441 -> 0.455 of
// 8 TB/s, +0.5 % pipelined; the small biased gathers (0.3-0.9 M chunks) lose with 8 (0.223 ->
// 0.211) and keep 4 (profiles/r05_ab_gather_unroll.txt).
constexpr int kGatherUnrollBig = 8;
constexpr int64_t kGatherBigChunks = int64_t(2) << 20;

// Stores the first out-of-range id a launch met into the process's async error words
// (context.h): id, row count and call tag first, then the kind with a system-scope release.
__device__ __attribute__((noinline)) void report_bad_id(int64_t *err, int64_t kind, int64_t id,
                                                        uint64_t rows, int64_t tag) {
  __hip_atomic_store(err + 1, id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(err + 2, (int64_t)rows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(err + 3, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(err, kind, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int V, int U, typename Src>
__global__ __launch_bounds__(kGatherThreads) void k_gather(Src src, uint32_t nchunks,
                                                           uint32_t cpr, FastDivU32 fd,
                                                           char *__restrict__ out,
                                                           uint64_t *stamp, LabelTail lt,
                                                           GatherGuard gd) {
  using T = typename VecT<V>::T;
#if DGS_GATHER_PRIO
  // issue priority over co-resident waves of other kernels (the sampler's VALU-bound waves
  // share the SIMDs in the pipeline): this wave's loads and stores go out first
  __builtin_amdgcn_s_setprio(DGS_GATHER_PRIO);
#endif
  if (blockIdx.x >= lt.blk0) {  // fused label rows (uniform branch), one per lane
    const uint32_t i = (blockIdx.x - lt.blk0) * (uint32_t)kGatherThreads + threadIdx.x;
    if (i < lt.n) {
      const int64_t raw = lt.ids[i];
      // range guard: an id outside [0, label rows) reads row 0 and is reported
      const bool bad = (uint64_t)raw >= lt.nrows;
      const int64_t id = bad ? 0 : raw;
      if (lt.row_bytes == 8)
        reinterpret_cast<uint64_t *>(lt.out)[i] =
            *to_global<uint64_t>(lt.data + (size_t)id * 8);
      else
        reinterpret_cast<uint32_t *>(lt.out)[i] =
            *to_global<uint32_t>(lt.data + (size_t)id * 4);
      if (bad) report_bad_id(gd.err, kAsyncErrLabel, raw, lt.nrows, gd.tag);
    }
    return;
  }
  // profiling only (stamp != nullptr, a kernel argument: uniform branch)
  if (stamp && threadIdx.x == 0) stamp[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  const uint32_t base = blockIdx.x * (uint32_t)(kGatherThreads * U) + threadIdx.x;
  // Branch-free: out-of-range chunks re-read the last chunk and skip only the store, so the
  // U independent id -> address -> row load chains issue back to back (3 waits, not 3U).
  uint32_t r[U], c[U];
  typename Src::Key key[U];
  const char *a[U];
  T v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    uint32_t g = base + u * kGatherThreads;
    g = g < nchunks ? g : nchunks - 1;
    r[u] = fd.div(g);
    c[u] = g - r[u] * cpr;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) key[u] = src.key(r[u]);
  // Range guard (one unsigned compare per id): an id outside [0, nrows) would address memory
  // outside the source (a GPU fault); it reads row 0 instead and the launch reports it.
  bool bad = false;
  int64_t bad_id = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool b = (uint64_t)key[u] >= gd.nrows;
    bad_id = b ? (int64_t)key[u] : bad_id;
    bad |= b;
    key[u] = b ? 0 : key[u];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) a[u] = src.addr(key[u]);
#pragma unroll
  for (int u = 0; u < U; ++u)
    v[u] = *to_global<T>(a[u] + (size_t)c[u] * V);
#pragma unroll
  for (int u = 0; u < U; ++u) keep(v[u]);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t g = base + u * kGatherThreads;
    // non-temporal: the output is consumed by the next kernel, not re-read here, so it
    // streams past L2 instead of evicting the rows other waves are fetching
    if (g < nchunks) __builtin_nontemporal_store(v[u], reinterpret_cast<T *>(out + (size_t)g * V));
  }
  if (bad) report_bad_id(gd.err, gd.kind, bad_id, gd.nrows, gd.tag);
  if (stamp) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores have landed
    __syncthreads();
    if (threadIdx.x == 0) stamp[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

template <typename Src>
void launch_gather_v(int V, Src src, int64_t n, int64_t row_bytes, char *out, hipStream_t st,
                     int which, GatherGuard gd, const LabelTail *tail = nullptr) {
  const int64_t cpr = row_bytes / V;
  DGS_CHECK(cpr > 0 && cpr < (int64_t(1) << 30), "gather: unsupported row size");
  const int64_t max_rows = ((int64_t(1) << 31) - kGatherThreads * kGatherUnrollBig) / cpr;
  const FastDivU32 fd = FastDivU32::make((uint32_t)cpr);
  for (int64_t r0 = 0; r0 < n; r0 += max_rows) {
    const int64_t rows = n - r0 < max_rows ? n - r0 : max_rows;
    Src s = src;
    s.row_base = r0;
    const uint32_t nchunks = (uint32_t)(rows * cpr);
    const bool big = V == 16 && (int64_t)nchunks >= kGatherBigChunks;
    const int U = big ? kGatherUnrollBig : kGatherUnroll;
    dim3 grid((unsigned)ceil_div(nchunks, kGatherThreads * U));
    char *o = out + r0 * row_bytes;
    // stamps cover the feature workgroups only (the label workgroups return before stamping)
    uint64_t *stamp = profile_stamps(which, (int64_t)grid.x);
    LabelTail lt;
    if (tail && r0 == 0 && tail->n > 0) {
      lt = *tail;
      lt.blk0 = grid.x;
      grid.x += (unsigned)ceil_div((int64_t)lt.n, kGatherThreads);
    }
    const dim3 block(kGatherThreads);
    const uint32_t c32 = (uint32_t)cpr;
    constexpr int U4 = kGatherUnroll, U8 = kGatherUnrollBig;
    switch (V) {
      case 16:
        if (big)
          hipLaunchKernelGGL((k_gather<16, U8, Src>), grid, block, 0, st, s, nchunks, c32, fd, o, stamp, lt, gd);
        else
          hipLaunchKernelGGL((k_gather<16, U4, Src>), grid, block, 0, st, s, nchunks, c32, fd, o, stamp, lt, gd);
        break;
      case 8: hipLaunchKernelGGL((k_gather<8, U4, Src>), grid, block, 0, st, s, nchunks, c32, fd, o, stamp, lt, gd); break;
      case 4: hipLaunchKernelGGL((k_gather<4, U4, Src>), grid, block, 0, st, s, nchunks, c32, fd, o, stamp, lt, gd); break;
      case 2: hipLaunchKernelGGL((k_gather<2, U4, Src>), grid, block, 0, st, s, nchunks, c32, fd, o, stamp, lt, gd); break;
      default: hipLaunchKernelGGL((k_gather<1, U4, Src>), grid, block, 0, st, s, nchunks, c32, fd, o, stamp, lt, gd); break;
    }
    DGS_LAUNCH_CHECK();
  }
}

int pick_vec(int64_t row_bytes, uintptr_t align_or) {
  for (int V = 16; V > 1; V >>= 1)
    if (row_bytes % V == 0 && (align_or % V) == 0) return V;
  return 1;
}

__global__ void k_ftab_init(int64_t *ftab, int64_t n, const char *base, int64_t row_bytes) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ftab[i] = (int64_t)(base + i * row_bytes);
}

// (cache lists are range-checked by the services before this runs; the guard keeps a list
// that slipped through from writing outside the table)
__global__ void k_ftab_assign(int64_t *ftab, int64_t num_rows, const int64_t *nids, int64_t n,
                              const char *base, int64_t row_bytes) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int64_t v = nids[i];
    if ((uint64_t)v < (uint64_t)num_rows) ftab[v] = (int64_t)(base + i * row_bytes);
  }
}

}  // namespace

// Guard of one gather call: ids are checked against nrows (kind says which op reports).
static GatherGuard make_guard(int64_t nrows, int64_t kind) {
  DGS_CHECK(nrows > 0, "gather: ids into a source with no rows (every id is out of range)");
  GatherGuard gd;
  gd.nrows = (uint64_t)nrows;
  gd.err = async_err_dev();
  gd.tag = (int64_t)async_err_next_tag();
  gd.kind = kind;
  return gd;
}

static const LabelTail *checked_tail(const LabelTail *tail) {
  if (tail && tail->n > 0)
    DGS_CHECK(tail->nrows > 0, "label gather: seeds into a label array with no rows");
  return tail;
}

void gather_plain(const void *data, int64_t nrows, int64_t row_bytes, const void *nid,
                  int nid_bytes, int64_t n, void *out, hipStream_t st) {
  if (n <= 0 || row_bytes <= 0) return;
  const GatherGuard gd = make_guard(nrows, kAsyncErrSelect);
  const int V = pick_vec(row_bytes, (uintptr_t)data | (uintptr_t)out);
  if (nid_bytes == 8) {
    PlainSrc<int64_t> s{(const char *)data, (const int64_t *)nid, row_bytes, 0};
    launch_gather_v(V, s, n, row_bytes, (char *)out, st, 2, gd);
  } else {
    DGS_CHECK(nid_bytes == 4, "index ids must be int32 or int64");
    PlainSrc<int32_t> s{(const char *)data, (const int32_t *)nid, row_bytes, 0};
    launch_gather_v(V, s, n, row_bytes, (char *)out, st, 2, gd);
  }
}

void gather_table(const int64_t *ftab, int64_t nrows, uintptr_t align_or, int64_t row_bytes,
                  const int64_t *nids, int64_t n, void *out, hipStream_t st,
                  const LabelTail *tail) {
  if (n <= 0 || row_bytes <= 0) return;
  const GatherGuard gd = make_guard(nrows, kAsyncErrFeature);
  const int V = pick_vec(row_bytes, align_or | (uintptr_t)out);
  TableSrc s{ftab, nids, row_bytes, 0};
  launch_gather_v(V, s, n, row_bytes, (char *)out, st, 0, gd, checked_tail(tail));
}

void gather_strided(const void *const *bases, int wshift, int64_t nrows, int64_t row_bytes,
                    const int64_t *nids, int64_t n, void *out, hipStream_t st,
                    const LabelTail *tail) {
  if (n <= 0 || row_bytes <= 0) return;
  DGS_CHECK(wshift >= 0 && wshift <= 3, "strided gather: at most 8 locations");
  const GatherGuard gd = make_guard(nrows, kAsyncErrFeature);
  const int W = 1 << wshift;
  const char *b[8];
  uintptr_t align_or = (uintptr_t)out;
  for (int d = 0; d < 8; ++d) {
    b[d] = (const char *)bases[d < W ? d : 0];
    align_or |= (uintptr_t)b[d];
  }
  const int V = pick_vec(row_bytes, align_or);
  if (wshift == 0) {
    StridedSrc<false> s{nids, b[0], b[1], b[2], b[3], b[4], b[5], b[6], b[7], row_bytes, 0, 0};
    launch_gather_v(V, s, n, row_bytes, (char *)out, st, 0, gd, checked_tail(tail));
  } else {
    StridedSrc<true> s{nids, b[0], b[1], b[2], b[3], b[4], b[5], b[6], b[7], row_bytes, 0,
                       (uint32_t)wshift};
    launch_gather_v(V, s, n, row_bytes, (char *)out, st, 0, gd, checked_tail(tail));
  }
}

namespace {
__global__ void k_stride_mismatch(const int64_t *list, int64_t n, int64_t start, int64_t stride,
                                  unsigned long long *bad) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool miss = i < n && list[i] != start + i * stride;
  const unsigned long long c = __popcll(__ballot(miss));
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(bad, c);
}

__global__ void k_out_of_range(const int64_t *list, int64_t n, int64_t num_rows,
                               unsigned long long *bad) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool miss = i < n && (uint64_t)list[i] >= (uint64_t)num_rows;
  const unsigned long long c = __popcll(__ballot(miss));
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(bad, c);
}

// rows of an address table that point into [lo, hi) (a feature table's host rows)
__global__ void k_count_in_range(const int64_t *tab, int64_t n, uint64_t lo, uint64_t hi,
                                 unsigned long long *cnt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = i < n && (uint64_t)tab[i] - lo < hi - lo;
  const unsigned long long c = __popcll(__ballot(in));
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(cnt, c);
}

// node-table entries whose row lives at location `loc` (a sampler's host rows)
__global__ void k_count_loc(const NodeEntry *tab, int64_t n, int loc, unsigned long long *cnt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = i < n && (int)((uint64_t)tab[i].dl >> kLocShift) == loc;
  const unsigned long long c = __popcll(__ballot(in));
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(cnt, c);
}

// ids of a list, marked in a byte per row (ids outside [0, num_rows) are skipped)
__global__ void k_mark_ids(const int64_t *list, int64_t n, int64_t num_rows, uint8_t *mark) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t v = list[i];
  if ((uint64_t)v < (uint64_t)num_rows) mark[v] = 1;
}

__global__ void k_count_unmarked(const uint8_t *mark, int64_t n, unsigned long long *cnt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool un = i < n && mark[i] == 0;
  const unsigned long long c = __popcll(__ballot(un));
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(cnt, c);
}

// A count made on the device and read back (setup-time checks).  Every error is raised: the
// callers take 0 as the permissive answer (a cache list accepted, a host array released), so a
// failed launch, copy or synchronisation must not read as 0.  The counter is a TmpBuf (freed
// after a stream synchronisation also when this throws).
template <typename K, typename... A>
int64_t count_on_device(K kernel, int64_t n, hipStream_t st, A... args) {
  if (n <= 0) return 0;
  TmpBuf bad(sizeof(unsigned long long), st);
  unsigned long long h = 0;
  DGS_HIP(hipMemsetAsync(bad.p, 0, sizeof(h), st));
  hipLaunchKernelGGL(kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, args...,
                     bad.as<unsigned long long>());
  DGS_LAUNCH_CHECK();
  DGS_HIP(hipMemcpyAsync(&h, bad.p, sizeof(h), hipMemcpyDeviceToHost, st));
  DGS_HIP(hipStreamSynchronize(st));
  return (int64_t)h;
}
}  // namespace

int64_t count_uncovered(const int64_t *const *lists, const int64_t *counts, int nlists,
                        int64_t num_rows, hipStream_t st) {
  if (num_rows <= 0) return 0;
  TmpBuf mark((size_t)num_rows, st);
  DGS_HIP(hipMemsetAsync(mark.p, 0, (size_t)num_rows, st));
  for (int l = 0; l < nlists; ++l) {
    if (counts[l] <= 0) continue;
    hipLaunchKernelGGL(k_mark_ids, dim3((unsigned)ceil_div(counts[l], 256)), dim3(256), 0, st,
                       lists[l], counts[l], num_rows, mark.as<uint8_t>());
    DGS_LAUNCH_CHECK();
  }
  return count_on_device(k_count_unmarked, num_rows, st, mark.as<const uint8_t>(), num_rows);
}

int64_t count_stride_mismatch(const int64_t *list, int64_t n, int64_t start, int64_t stride,
                              hipStream_t st) {
  return count_on_device(k_stride_mismatch, n, st, list, n, start, stride);
}

int64_t count_out_of_range(const int64_t *list, int64_t n, int64_t num_rows, hipStream_t st) {
  return count_on_device(k_out_of_range, n, st, list, n, num_rows);
}

int64_t count_in_range(const int64_t *tab, int64_t n, const void *lo, int64_t bytes,
                       hipStream_t st) {
  if (!lo || bytes <= 0) return 0;
  return count_on_device(k_count_in_range, n, st, tab, n, (uint64_t)(uintptr_t)lo,
                         (uint64_t)(uintptr_t)lo + (uint64_t)bytes);
}

int64_t count_loc(const NodeEntry *tab, int64_t n, int loc, hipStream_t st) {
  return count_on_device(k_count_loc, n, st, tab, n, loc);
}

void ftab_init(int64_t *ftab, int64_t n, const void *base, int64_t row_bytes, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_ftab_init, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, ftab, n,
                     (const char *)base, row_bytes);
  DGS_LAUNCH_CHECK();
}

void ftab_assign(int64_t *ftab, int64_t num_rows, const int64_t *nids, int64_t n,
                 const void *base, int64_t row_bytes, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_ftab_assign, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, ftab,
                     num_rows, nids, n, (const char *)base, row_bytes);
  DGS_LAUNCH_CHECK();
}

}  // namespace dgs
