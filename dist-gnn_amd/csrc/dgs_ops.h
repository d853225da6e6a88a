// dgs_ops.h -- host-side launchers of the DGS-AMD HIP kernels (internal C++ interface).
#pragma once

#include <hip/hip_ext.h>

#include "dgs_common.h"
#include "dgs_table.cuh"

namespace dgs {

// ---------------------------------------------------------------- gather (gather.hip)
// A second, small gather fused into a feature gather's launch (PrefetchLoader's label gather):
// out[i] = data[ids[i]] for i < n, rows of 4 or 8 bytes, in extra workgroups after the
// feature gather's (one launch instead of two on the caller's thread).
struct LabelTail {
  const char *data = nullptr;
  const int64_t *ids = nullptr;
  char *out = nullptr;
  uint64_t nrows = 0;  // rows of `data` (ids are range-checked against it)
  uint32_t n = 0;
  uint32_t row_bytes = 0;  // 4 or 8
  uint32_t blk0 = 0xffffffffu;  // first label workgroup (set by the launcher)
};
// Range guard of one gather launch (a kernel argument): ids outside [0, nrows) read row 0 and
// are reported through the async error words (context.h) under `tag`, as error `kind`.
struct GatherGuard {
  uint64_t nrows = 0;
  int64_t *err = nullptr;
  int64_t tag = 0;
  int64_t kind = 0;
};
// Every gather below checks its ids against the source's row count (nrows > 0 is required when
// n > 0): an id outside [0, nrows) reads row 0 and the next gather entry point raises.
// out[i, :] = data[nid[i], :], a row_bytes byte copy per row.
void gather_plain(const void *data, int64_t nrows, int64_t row_bytes, const void *nid,
                  int nid_bytes, int64_t n, void *out, hipStream_t st);
// out[i, :] = *(row_bytes at ftab[nids[i]]): ftab holds the absolute (device-accessible)
// address of every node's feature row.  align_or = OR of all row base addresses.
void gather_table(const int64_t *ftab, int64_t nrows, uintptr_t align_or, int64_t row_bytes,
                  const int64_t *nids, int64_t n, void *out, hipStream_t st,
                  const LabelTail *tail = nullptr);
// Strided cache layout (every node cached, node v at row v >> wshift of GPU v & (W - 1),
// W = 1 << wshift <= 8; W = 1 is the whole-graph-in-HBM identity layout): the row address is
// computed, so the gather reads no per-node table.  bases[d] = GPU d's (IPC-mapped) block.
void gather_strided(const void *const *bases, int wshift, int64_t nrows, int64_t row_bytes,
                    const int64_t *nids, int64_t n, void *out, hipStream_t st,
                    const LabelTail *tail = nullptr);
// number of i < n with list[i] != start + i * stride (device count -> host)
int64_t count_stride_mismatch(const int64_t *list, int64_t n, int64_t start, int64_t stride,
                              hipStream_t st);
// ftab[v] = base + v * row_bytes for v < n
void ftab_init(int64_t *ftab, int64_t n, const void *base, int64_t row_bytes, hipStream_t st);
// number of i < n with list[i] outside [0, num_rows) (device count -> host)
int64_t count_out_of_range(const int64_t *list, int64_t n, int64_t num_rows, hipStream_t st);
// entries of an address table inside [lo, lo + bytes) / node-table entries at location `loc`
int64_t count_in_range(const int64_t *tab, int64_t n, const void *lo, int64_t bytes,
                       hipStream_t st);
int64_t count_loc(const NodeEntry *tab, int64_t n, int loc, hipStream_t st);
// rows of [0, num_rows) that none of the lists (device arrays, counts[l] ids each) names
int64_t count_uncovered(const int64_t *const *lists, const int64_t *counts, int nlists,
                        int64_t num_rows, hipStream_t st);
// ftab[nids[i]] = base + i * row_bytes (ids outside [0, num_rows) are skipped)
void ftab_assign(int64_t *ftab, int64_t num_rows, const int64_t *nids, int64_t n,
                 const void *base, int64_t row_bytes, hipStream_t st);

// ---------------------------------------------------------------- CSR utilities (csr.hip)
// sub_indptr[i] = sum_{j<i} deg(nids[j]), i = 0..n
void extract_indptr(const int64_t *nids, int64_t n, const int64_t *indptr, int64_t *sub_indptr,
                    hipStream_t st);
void extract_edge_data(const int64_t *nids, int64_t n, const int64_t *indptr,
                       const int64_t *sub_indptr, const void *edge_data, int64_t elem_bytes,
                       void *sub, hipStream_t st);
// node table: ntab[v] = {indices + indptr[v], deg(v) | host << 56}
void ntab_init_host(NodeEntry *ntab, const int64_t *indptr, int64_t n, const int64_t *indices,
                    hipStream_t st);
// ntab[nids[i]] = {sub_indices + sub_indptr[i], (sub_indptr[i+1]-sub_indptr[i]) | loc << 56}
// (ids outside [0, num_nodes) are skipped)
void ntab_assign(NodeEntry *ntab, int64_t num_nodes, const int64_t *nids,
                 const int64_t *sub_indptr, int64_t n, int loc, const int64_t *sub_indices,
                 hipStream_t st);
// Compacts a (loc << 56 | row) table into (nid, row, loc) triples for every node whose
// location is a GPU; *d_count receives the count.  key/idx/devid may be null (count only).
void cache_map_compact(const int64_t *tab, int64_t n, int64_t *key, int64_t *idx,
                       int64_t *devid, int64_t *d_count, hipStream_t st);
// The reference's open-addressing cache map (hashmap.cu:15-77), for its getter: capacity
// 2 * _UpPower(total) and a build from the ranks' cache lists inserted in `order` (hashmap.hip).
int64_t refmap_dir_size(int64_t total);
void refmap_build(const int64_t *const *lists, const int64_t *counts, const int *order,
                  int nlists, int id_bytes, int64_t dir, void *key, void *idx, void *dev,
                  hipStream_t st);
// frontier heat (preprocess_heat.cu); fixed_acc != nullptr: deterministic fixed-point
// accumulation in fixed_acc[num_nodes] (scratch), then written to frontier_heat as float
void heat(const int64_t *seeds, int64_t n_seeds, const int64_t *indptr, const int64_t *indices,
          const float *probs, const float *seeds_heat, int64_t num_picks, int64_t indptr_diff,
          float *frontier_heat, int64_t num_nodes, unsigned long long *fixed_acc,
          hipStream_t st);

// ---------------------------------------------------------------- scan (scan.hip)
// Single-workgroup exclusive scan of n int64 values in place into out[0..n], out[n] = total.
void scan_small(const int64_t *in, int64_t n, int64_t *out, hipStream_t st);
// Device-wide exclusive scan: out[0..n] (out[n] = total). scratch >= scan_scratch_bytes(n).
size_t scan_scratch_bytes(int64_t n);
void scan_exclusive(const int64_t *in, int64_t n, int64_t *out, void *scratch, hipStream_t st);

// ---------------------------------------------------------------- sampling (sample.hip)
struct RowSrc {
  // Node lookup: either a node table (graph shard context) or a plain CSR indptr/indices.
  const NodeEntry *ntab;   // if non-null
  const int64_t *indptr;   // else (location 0)
  const int64_t *indices;  // plain-CSR neighbour ids
  PtrTable indices_base;   // per-location neighbour-id arrays (to locate probs)
  PtrTable probs;          // per-location probabilities (biased) or all null
  // Seed validation (sampler only): a seed outside [0, num_nodes) is sampled as a degree-0
  // row, kept out of the relabel table, and reported by storing bad_tag to *bad.
  int64_t num_nodes;
  int64_t *bad;
  int64_t bad_tag;
  // Edges of the whole graph (bounds the biased hub candidate lists of one hop); 0 = unknown.
  int64_t num_edges;
};

struct HopScratch {
  DevBuf rowinfo, tpre, bsum, boff, hub, hubcount, hubslot, rowpos, slot_of, tkey, tval, tlab,
      misc, cdf, cand, flags;
  DevBuf op_tmp;  // the standalone ops' call buffers (sample_neighbors, relabel)
  HostPinned host;
  uint64_t table_cap = 0;  // capacity currently allocated and clean
  uint64_t hop_serial = 0;  // parity selects the hub counter of a hop
  bool table_dirty = false;
};

// One sampling hop over `seeds[S]` (device; S may be a device-side count, then S.v bounds it):
//   writes rowpos[e] (index of the seed row of edge e) and col[e] (neighbour nid),
//   d_nnz receives nnz (device).  Capacities: S.v * k.
// When `table.key` is set, every seed i and sampled neighbour (position S + e) is inserted
// into the relabel table by the kernels that produce them.  `tail` (the previous hop's
// deferred relabel pass, on the other table) runs in the same launch as this hop's prep.
void sample_hop(const RowSrc &src, const int64_t *seeds, Count S, int64_t k, bool replace,
                bool bias, uint64_t launch_seed, int64_t *rowpos, int64_t *col, int64_t *d_nnz,
                const Table &table, HopScratch &ws, hipStream_t st,
                const RelabelTail *tail = nullptr, bool solo = false);

// Test-only: exact A-Res keys, their lower bounds and the biased kernels' reject tests.
void test_bias_bounds(const uint32_t *x, const float *p, const float *thr, int64_t n, float *key,
                      float *key_low, uint8_t *flags, hipStream_t st);

// Clean relabel table with capacity for n_ub insertions (marks the scratch dirty until the
// hop's relabel pass has returned the touched slots to empty).
Table relabel_table(HopScratch &ws, int64_t n_ub, hipStream_t st);
// Direct-layout table over node ids [0, num_nodes) (val = empty everywhere on return; a table
// left dirty by an interrupted hop is re-filled).  The relabel pass of every hop empties the
// entries it touched, so a completed hop leaves it clean.
Table direct_table(DevBuf &pairs, int64_t num_nodes, bool *dirty, hipStream_t st);

// Relabel for the node-classification hop: mapping = cat(seeds[S], col[nnz]) where nnz is
// read from d_nnz (device); writes unique ids to `unique` (first-occurrence order),
// relabeled rows/cols to out_row/out_col (col may alias out_col), U to d_nunique.  out_row
// holds each edge's seed row r on entry (sample_hop's rowpos output) and is relabelled in
// place; seeds_unique (every hop after the first) means label(r) == r and skips the lookup.
void relabel_hop(const int64_t *seeds, Count S, const int64_t *col, const int64_t *d_nnz,
                 int64_t nnz_cap, bool seeds_unique, const Table &table, int64_t *unique,
                 int64_t *out_row, int64_t *out_col, int64_t *d_nunique, HopScratch &ws,
                 hipStream_t st, const HostSizes &pub = HostSizes{},
                 RelabelTail *defer = nullptr, const IdCheck &chk = IdCheck{});
// launches a deferred relabel tail on its own
void launch_relabel_tail(const RelabelTail &tail, hipStream_t st);

// Generic relabel (TensorRelabelCUDA): mapping[nm], req[nr] -> unique, relabeled req (-1 if
// absent), d_nunique.
void relabel_generic(const int64_t *mapping, int64_t nm, const int64_t *req, int64_t nr,
                     int64_t *unique, int64_t *req_out, int64_t *d_nunique, HopScratch &ws,
                     hipStream_t st);

// gather rows of `seeds` by rowpos (coo_row of the standalone sampler op)
void take_i64(const int64_t *src, const int64_t *idx, int64_t n, int64_t *out, hipStream_t st);

// ---------------------------------------------------------------- profiling
struct Profiler {
  bool on = false;
  int mask = 0;  // bit `which` enables that measurement
  bool wants(int which) const { return on && ((mask >> which) & 1); }
  double gather_ms = 0, sample_ms = 0, select_ms = 0;
  int64_t gather_n = 0, sample_n = 0, select_n = 0;
};
Profiler &profiler();
// which: 0 = feature-server gather kernel, 1 = multi-hop sample call (events before its
// first and after its last kernel), 2 = plain index_select gather kernel; diagnostics only
// (DGS_PROF_HUB=1 with DGS_PROF_DETAIL=1, stderr): 3 = uniform hub reservoir, 4 = biased stream.
// Kernel events: when profiling is on, returns (start, stop) events that hipExtLaunchKernelGGL
// records at the kernel's own start / end; otherwise (null, null).
struct KernelEvents {
  hipEvent_t start = nullptr, stop = nullptr;
};
KernelEvents profile_kernel(int which);
// Device-side stamps of one kernel launch: when measurement `which` is on, a device buffer of
// 2 * nblocks uint64 that the kernel fills with each workgroup's s_memrealtime at its start and
// after its last store (the launch's duration = last end - first start, the kernel's own
// execution span); nullptr otherwise.  Unlike stream events it excludes the tail of the
// previous kernel on the stream and any wait for free CUs before the first workgroup starts.
// (extra: counter words per workgroup after the 2 x nblocks stamps)
uint64_t *profile_stamps(int which, int64_t nblocks, int extra = 0);
// Stream events at both ends of a group of launches (one marker before the first and one
// after the last kernel; used around a whole sample call, where the stream is idle anyway,
// never between the kernels being measured).
void profile_begin(hipStream_t st, int which);
void profile_end(hipStream_t st, int which);
void profile_collect();
// reserves the workgroup-stamp slab (called when gather profiling is switched on)
void profile_reserve();
// cache-map helpers: tab[v] = (loc << 56) | row
void loctab_init_host(int64_t *tab, int64_t n, hipStream_t st);
void loctab_assign(int64_t *tab, int64_t num_nodes, const int64_t *nids, int64_t n, int loc,
                   hipStream_t st);

}  // namespace dgs
