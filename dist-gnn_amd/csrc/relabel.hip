// relabel.hip -- unique + relabel (frontier construction) for a sampling hop.
//
// Reference: tensor_relabel.cu:11-205.  unique = ids of cat(seeds, coo_col) in first-occurrence
// order (open-addressing table keeping the minimum position per key, :17-29); relabel maps
// every id to its position in unique.  The reference re-probes the table in each of its
// passes (insert, count, scatter, relabel) and uses an identity hash at load factor ~1.
//
// MI355X design: one probe per element.  The insert pass records each element's slot
// (slot_of[i]); the flag / scatter / relabel passes only index by slot.  64-bit keys, fmix64
// hash, linear probing at load factor <= 0.5 in a table sized for this hop (it stays in the
// L2 / Infinity Cache at the benchmark sizes).  The table is persistent and is cleaned by
// the relabel pass itself (only the slots this hop touched), so no per-hop memset.
#include "dgs_block.cuh"
#include "dgs_ops.h"
#include "dgs_table.cuh"

namespace dgs {
namespace {

constexpr int kThreads = 256;
constexpr int64_t kEmpty = kTableEmpty;
constexpr int32_t kNoPos = kTableNoPos;

// element i of cat(a[na], b[*nb_ptr])
__device__ __forceinline__ int64_t elem(const int64_t *a, int64_t na, const int64_t *b,
                                       int64_t i) {
  return i < na ? a[i] : b[i - na];
}

__global__ __launch_bounds__(kThreads) void k_insert(const int64_t *a, Count nac,
                                                     const int64_t *b, const int64_t *d_nb,
                                                     int64_t nb_fixed, Table t) {
  const int64_t na = nac.get();
  const int64_t n = na + (d_nb ? *d_nb : nb_fixed);
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  t.slot_of[i] = table_insert(t, elem(a, na, b, i), (int32_t)i);
}

__global__ __launch_bounds__(kThreads) void k_flag_count(Count nac, const int64_t *d_nb,
                                                         int64_t nb_fixed, Table t,
                                                         const uint32_t *slot_of, int64_t *bcnt) {
  __shared__ int64_t lds[kThreads / 64];
  const int64_t n = nac.get() + (d_nb ? *d_nb : nb_fixed);
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const int64_t f = (i < n && t.val[slot_of[i]] == (int32_t)i) ? 1 : 0;
  const int64_t s = block_sum<kThreads>(f, lds);
  if (threadIdx.x == 0) bcnt[blockIdx.x] = s;
}

__global__ __launch_bounds__(kThreads) void k_scatter(const int64_t *a, Count nac,
                                                      const int64_t *b, const int64_t *d_nb,
                                                      int64_t nb_fixed, Table t,
                                                      const uint32_t *slot_of,
                                                      const int64_t *boff, int64_t nblocks,
                                                      int64_t *unique, int64_t *d_nunique,
                                                      HostSizes pub) {
  __shared__ int64_t lds[kThreads / 64];
  const int64_t na = nac.get();
  const int64_t n = na + (d_nb ? *d_nb : nb_fixed);
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  uint32_t sl = 0;
  int64_t f = 0;
  if (i < n) {
    sl = slot_of[i];
    f = t.val[sl] == (int32_t)i ? 1 : 0;
  }
  int64_t tot;
  const int64_t ex = block_exclusive_scan<kThreads>(f, &tot, lds);
  if (f) {
    const int64_t pos = boff[blockIdx.x] + ex;
    unique[pos] = elem(a, na, b, i);
    t.lab[sl] = (int32_t)pos;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (d_nunique) *d_nunique = boff[nblocks];
    if (pub.host) {
      // every size of the call is final here (earlier hops' by earlier kernels, this hop's U
      // just above): publish them so the host need not wait for the relabel pass
      for (int64_t j = 0; j < pub.n; ++j)
        __hip_atomic_store(pub.host + 1 + j, pub.dev[j], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(pub.host, (int64_t)pub.seq, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// Hop relabel: out_col[e] = lab(slot_of[na + e]); out_row[e] holds the seed row r of edge e
// (written by the sampling kernel) and becomes lab(slot_of[r]) -- only needed when the seeds
// may repeat (the first hop): later hops' seeds are the previous unique frontier, so seed r's
// first occurrence is position r and its label is r.  Then the touched slots are emptied.
__global__ __launch_bounds__(kThreads) void k_relabel_hop(Count nac, const int64_t *d_nb,
                                                          Table t, const uint32_t *slot_of,
                                                          int remap_rows, int64_t *out_row,
                                                          int64_t *out_col) {
  const int64_t na = nac.get();
  const int64_t nb = *d_nb;
  const int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (e < nb) {
    const uint32_t sc = slot_of[na + e];
    out_col[e] = t.lab[sc];
    if (remap_rows) out_row[e] = t.lab[slot_of[out_row[e]]];
    t.key[sc] = kEmpty;
    t.val[sc] = kNoPos;
  }
  if (e < na) {
    const uint32_t ss = slot_of[e];
    t.key[ss] = kEmpty;
    t.val[ss] = kNoPos;
  }
}

// ---- direct layout (sampler hops): val / lab indexed by node id
// First occurrences, two passes over 1024-element tiles (4 contiguous elements per thread):
// element i of cat(seeds, col) is a first occurrence iff val[x] == i, and its label is its rank
// among first occurrences.  Pass 1 counts per tile; pass 2 sums the counts of all earlier tiles
// directly (a few hundred L2-resident words) instead of a separate scan launch, then scatters.
constexpr int kCompactItems = 4;
constexpr int64_t kCompactTile = (int64_t)kThreads * kCompactItems;

__device__ __forceinline__ void publish_sizes(const HostSizes &pub) {
  if (!pub.host) return;
  for (int64_t j = 0; j < pub.n; ++j)
    __hip_atomic_store(pub.host + 1 + j, pub.dev[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(pub.host, (int64_t)pub.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Branch-free flags of this thread's elements: out-of-range ones are clamped to the last
// element and dropped, so all id loads issue back to back, then all val loads.
__device__ __forceinline__ int64_t first_flags(const int64_t *a, int64_t na, const int64_t *b,
                                               int64_t n, const Table &t, int64_t i0,
                                               int64_t (&x)[kCompactItems],
                                               bool (&f)[kCompactItems]) {
  int32_t pv[kCompactItems];
#pragma unroll
  for (int j = 0; j < kCompactItems; ++j) {
    const int64_t i = i0 + j < n ? i0 + j : n - 1;
    const int64_t *src = i < na ? a + i : b + (i - na);
    x[j] = *src;
  }
#pragma unroll
  for (int j = 0; j < kCompactItems; ++j)
    pv[j] = (uint64_t)x[j] < (uint64_t)t.n ? *dval(t, x[j]) : kNoPos;
  int64_t cnt = 0;
#pragma unroll
  for (int j = 0; j < kCompactItems; ++j) {
    f[j] = i0 + j < n && pv[j] == (int32_t)(i0 + j);
    cnt += f[j];
  }
  return cnt;
}

// Pass 1 also leaves each thread's flags (one byte, bit j = element i0 + j) for pass 2, which
// then needs no second round of random table reads.
// It also range-checks the hop's sampled ids (and, at the first hop, each edge's seed row)
// before the sizes are published, so a call sees its own out-of-range id (IdCheck).
__global__ __launch_bounds__(kThreads) void k_dcount(const int64_t *a, Count nac,
                                                     const int64_t *b, const int64_t *d_nb,
                                                     Table t, int64_t *tcnt, uint8_t *flags,
                                                     IdCheck chk, const int64_t *rows) {
  latency_prio();
  __shared__ int64_t lds[kThreads / 64];
  const int64_t na = nac.get();
  const int64_t n = na + *d_nb;
  const int64_t i0 = (int64_t)blockIdx.x * kCompactTile + (int64_t)threadIdx.x * kCompactItems;
  if ((int64_t)blockIdx.x * kCompactTile >= n) return;
  int64_t x[kCompactItems];
  bool f[kCompactItems];
  const int64_t cnt = first_flags(a, na, b, n, t, i0, x, f);
  if (chk.bad) {
#pragma unroll
    for (int j = 0; j < kCompactItems; ++j) {
      const int64_t i = i0 + j;
      if (i < na || i >= n) continue;
      const int64_t row = rows ? rows[i - na] : 0;
      if ((uint64_t)x[j] >= (uint64_t)t.n || (uint64_t)row >= (uint64_t)na)
        report_bad_id(chk, i - na, x[j], n - na, rows ? row : -1);
    }
  }
  uint32_t fb = 0;
#pragma unroll
  for (int j = 0; j < kCompactItems; ++j) fb |= (uint32_t)f[j] << j;
  flags[(int64_t)blockIdx.x * kThreads + threadIdx.x] = (uint8_t)fb;
  const int64_t s = block_sum<kThreads>(cnt, lds);
  if (threadIdx.x == 0) tcnt[blockIdx.x] = s;
}

__global__ __launch_bounds__(kThreads) void k_dscatter(const int64_t *a, Count nac,
                                                       const int64_t *b, const int64_t *d_nb,
                                                       Table t, const int64_t *tcnt,
                                                       const uint8_t *flags, int64_t *unique,
                                                       int64_t *d_nunique, HostSizes pub) {
  latency_prio();
  __shared__ int64_t lds[kThreads / 64];
  const int64_t na = nac.get();
  const int64_t n = na + *d_nb;
  const int64_t tile = blockIdx.x;
  if (n == 0) {
    // an empty call (no seeds): the count and the publication still happen, from tile 0
    if (tile == 0 && threadIdx.x == 0) {
      *d_nunique = 0;
      publish_sizes(pub);
    }
    return;
  }
  const int64_t ntiles = (n + kCompactTile - 1) / kCompactTile;
  if (tile >= ntiles) return;
  // this tile's offset: sum of the earlier tiles' counts (issued before the element loads)
  int64_t pre = 0;
  for (int64_t j = threadIdx.x; j < tile; j += kThreads) pre += tcnt[j];
  const int64_t i0 = tile * kCompactTile + (int64_t)threadIdx.x * kCompactItems;
  const uint32_t fb = flags[tile * kThreads + threadIdx.x];
  int64_t x[kCompactItems];
  bool f[kCompactItems];
#pragma unroll
  for (int j = 0; j < kCompactItems; ++j) {
    const int64_t i = i0 + j < n ? i0 + j : n - 1;
    x[j] = i < na ? a[i] : b[i - na];
    f[j] = (fb >> j) & 1u;
  }
  const int64_t cnt = __builtin_popcount(fb);
  const int64_t base = block_sum<kThreads>(pre, lds);
  int64_t tot;
  int64_t ex = base + block_exclusive_scan<kThreads>(cnt, &tot, lds);
#pragma unroll
  for (int j = 0; j < kCompactItems; ++j) {
    if (f[j]) {
      unique[ex] = x[j];
      *dlab(t, x[j]) = (int32_t)ex;
      ++ex;
    }
  }
  if (tile == ntiles - 1 && threadIdx.x == 0) {
    *d_nunique = base + tot;
    publish_sizes(pub);
  }
}

__global__ __launch_bounds__(kThreads) void k_drelabel_hop(RelabelTail r) {
  latency_prio();
  relabel_tail_block(r, blockIdx.x);
}

__global__ void k_fill_i32(int32_t *p, int64_t n, int32_t v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// Generic relabel: req lookups (absent -> -1, tensor_relabel.cu:47-61).
__global__ __launch_bounds__(kThreads) void k_relabel_req(Table t, const int64_t *req,
                                                          int64_t nr, int64_t *out) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= nr) return;
  const int64_t h = table_find(t, req[i]);
  out[i] = h < 0 ? -1 : (int64_t)t.lab[h];
}

__global__ __launch_bounds__(kThreads) void k_clear_slots(Table t, const uint32_t *slot_of,
                                                          int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = slot_of[i];
  t.key[s] = kEmpty;
  t.val[s] = kNoPos;
}

__global__ void k_table_init(int64_t *key, int32_t *val, uint64_t cap) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cap) {
    key[i] = kEmpty;
    val[i] = kNoPos;
  }
}

}  // namespace

// Makes sure the persistent table has a clean region of at least 2 * n_ub slots.
Table relabel_table(HopScratch &ws, int64_t n_ub, hipStream_t st) {
  DGS_CHECK(n_ub < (int64_t(1) << 31), "relabel input too large");
  const uint64_t cap = next_pow2((uint64_t)(2 * (n_ub > 0 ? n_ub : 1)));
  DGS_CHECK(cap <= (uint64_t(1) << 32), "relabel table too large");
  if (cap > ws.table_cap || ws.table_dirty) {
    const uint64_t alloc = cap > ws.table_cap ? cap : ws.table_cap;
    ws.tkey.ensure(sizeof(int64_t) * alloc);
    ws.tval.ensure(sizeof(int32_t) * alloc);
    ws.tlab.ensure(sizeof(int32_t) * alloc);
    hipLaunchKernelGGL(k_table_init, dim3((unsigned)ceil_div((int64_t)alloc, 256)), dim3(256), 0,
                       st, ws.tkey.as<int64_t>(), ws.tval.as<int32_t>(), alloc);
    DGS_LAUNCH_CHECK();
    ws.table_cap = alloc;
    ws.table_dirty = false;
  }
  ws.slot_of.ensure(sizeof(uint32_t) * (size_t)(n_ub > 0 ? n_ub : 1));
  return Table{ws.tkey.as<int64_t>(), ws.tval.as<int32_t>(), ws.tlab.as<int32_t>(),
               ws.slot_of.as<uint32_t>(), cap - 1, false};
}

void launch_relabel_tail(const RelabelTail &tail, hipStream_t st) {
  hipLaunchKernelGGL(k_drelabel_hop, dim3((unsigned)tail.nblk), dim3(kThreads), 0, st, tail);
  DGS_LAUNCH_CHECK();
}

Table direct_table(DevBuf &pairs, int64_t num_nodes, bool *dirty, hipStream_t st) {
  const int64_t n = 2 * (num_nodes > 0 ? num_nodes : 1);  // (val, lab) per node
  const bool fresh = pairs.ensure(sizeof(int32_t) * (size_t)n);
  if (fresh || *dirty) {
    hipLaunchKernelGGL(k_fill_i32, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st,
                       pairs.as<int32_t>(), n, kNoPos);
    DGS_LAUNCH_CHECK();
    *dirty = false;
  }
  return Table{nullptr, pairs.as<int32_t>(), nullptr, nullptr, 0, true, num_nodes};
}

// The hop's seeds and sampled neighbours were already inserted by the sampling kernels
// (sample_hop with this Table); what is left is ranking the first occurrences and the COO
// rewrite.
void relabel_hop(const int64_t *seeds, Count Sc, const int64_t *col, const int64_t *d_nnz,
                 int64_t nnz_cap, bool seeds_unique, const Table &t, int64_t *unique,
                 int64_t *out_row, int64_t *out_col, int64_t *d_nunique, HopScratch &ws,
                 hipStream_t st, const HostSizes &pub, RelabelTail *defer,
                 const IdCheck &chk) {
  const int64_t n_ub = Sc.v + nnz_cap;
  const int64_t nblk = ceil_div(n_ub > 0 ? n_ub : 1, kThreads);
  ws.misc.ensure(sizeof(int64_t) * (size_t)(2 * nblk + 2));
  int64_t *bcnt = ws.misc.as<int64_t>();
  int64_t *boff = bcnt + nblk;
  if (t.direct) {
    const int64_t ntiles = ceil_div(n_ub > 0 ? n_ub : 1, kCompactTile);
    int64_t *tcnt = bcnt;  // ws.misc holds >= nblk >= ntiles words
    ws.flags.ensure((size_t)(ntiles * kThreads));
    uint8_t *flags = ws.flags.as<uint8_t>();
    hipLaunchKernelGGL(k_dcount, dim3((unsigned)ntiles), dim3(kThreads), 0, st, seeds, Sc, col,
                       d_nnz, t, tcnt, flags, chk,
                       seeds_unique ? (const int64_t *)nullptr : (const int64_t *)out_row);
    DGS_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_dscatter, dim3((unsigned)ntiles), dim3(kThreads), 0, st, seeds, Sc,
                       col, d_nnz, t, (const int64_t *)tcnt, (const uint8_t *)flags, unique,
                       d_nunique, pub);
    DGS_LAUNCH_CHECK();
    const RelabelTail tail{seeds, Sc, d_nnz, t, (int)!seeds_unique, out_row, out_col,
                           unique, d_nunique, nblk, chk};
    if (defer) {
      *defer = tail;  // the caller launches it with the next hop's prep
    } else {
      hipLaunchKernelGGL(k_drelabel_hop, dim3((unsigned)nblk), dim3(kThreads), 0, st, tail);
      DGS_LAUNCH_CHECK();
    }
    return;
  }
  hipLaunchKernelGGL(k_flag_count, dim3((unsigned)nblk), dim3(kThreads), 0, st, Sc, d_nnz,
                     (int64_t)0, t, t.slot_of, bcnt);
  DGS_LAUNCH_CHECK();
  scan_small(bcnt, nblk, boff, st);
  hipLaunchKernelGGL(k_scatter, dim3((unsigned)nblk), dim3(kThreads), 0, st, seeds, Sc, col,
                     d_nnz, (int64_t)0, t, t.slot_of, boff, nblk, unique, d_nunique, pub);
  DGS_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_relabel_hop, dim3((unsigned)nblk), dim3(kThreads), 0, st, Sc, d_nnz, t,
                     t.slot_of, (int)!seeds_unique, out_row, out_col);
  DGS_LAUNCH_CHECK();
  ws.table_dirty = false;
}

void relabel_generic(const int64_t *mapping, int64_t nm, const int64_t *req, int64_t nr,
                     int64_t *unique, int64_t *req_out, int64_t *d_nunique, HopScratch &ws,
                     hipStream_t st) {
  Table t = relabel_table(ws, nm, st);
  ws.table_dirty = true;
  const int64_t nblk = ceil_div(nm > 0 ? nm : 1, kThreads);
  ws.misc.ensure(sizeof(int64_t) * (size_t)(2 * nblk + 2));
  int64_t *bcnt = ws.misc.as<int64_t>();
  int64_t *boff = bcnt + nblk;
  const Count nmc{nm, nullptr};
  hipLaunchKernelGGL(k_insert, dim3((unsigned)nblk), dim3(kThreads), 0, st, mapping, nmc,
                     (const int64_t *)nullptr, (const int64_t *)nullptr, (int64_t)0, t);
  DGS_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_flag_count, dim3((unsigned)nblk), dim3(kThreads), 0, st, nmc,
                     (const int64_t *)nullptr, (int64_t)0, t, t.slot_of, bcnt);
  DGS_LAUNCH_CHECK();
  scan_small(bcnt, nblk, boff, st);
  hipLaunchKernelGGL(k_scatter, dim3((unsigned)nblk), dim3(kThreads), 0, st, mapping, nmc,
                     (const int64_t *)nullptr, (const int64_t *)nullptr, (int64_t)0, t, t.slot_of,
                     boff, nblk, unique, d_nunique, HostSizes{});
  DGS_LAUNCH_CHECK();
  if (nr > 0) {
    hipLaunchKernelGGL(k_relabel_req, dim3((unsigned)ceil_div(nr, kThreads)), dim3(kThreads), 0,
                       st, t, req, nr, req_out);
    DGS_LAUNCH_CHECK();
  }
  if (nm > 0) {
    hipLaunchKernelGGL(k_clear_slots, dim3((unsigned)nblk), dim3(kThreads), 0, st, t, t.slot_of,
                       nm);
    DGS_LAUNCH_CHECK();
  }
  ws.table_dirty = false;
}

}  // namespace dgs
