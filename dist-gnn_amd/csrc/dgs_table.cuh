// dgs_table.cuh -- the relabel hash table shared by the sampling kernels (which insert the
// hop's seeds and sampled neighbours as they produce them) and relabel.hip (which ranks the
// first occurrences and rewrites the COO).  Reference semantics: tensor_relabel.cu:17-29.
#pragma once

#include "dgs_common.h"

namespace dgs {

constexpr int64_t kTableEmpty = -1;
constexpr int32_t kTableNoPos = 0x7FFFFFFF;

// Two layouts.  Hashed (key != nullptr): open addressing over arbitrary int64 ids (the
// standalone relabel op).  Direct (direct == true): the sampler's ids are graph node ids in
// [0, N), so the entry is indexed by the id itself -- one load and at most one atomicMin per
// insert, no probing, no key CAS and no slot_of bookkeeping.  A node's (val, lab) pair is one
// 8-byte word (val at 2x, lab at 2x + 1 of `val`): the scatter's val read and lab write, and
// the relabel tail's lab read and val reset, touch one cache line per node instead of two.
struct Table {
  int64_t *key;   // hashed layout: slot keys; nullptr with !direct: no table (standalone op)
  int32_t *val;   // minimum position (first occurrence), per slot; direct: the pair array
  int32_t *lab;   // label = rank among first occurrences, per slot; direct: unused
  uint32_t *slot_of;  // hashed layout: slot of every inserted position
  uint64_t mask;  // hashed layout: capacity - 1
  bool direct;
  int64_t n;      // direct layout: number of node ids (ids outside [0, n) are never recorded)
};


// Range check of a sampler call's sampled ids (an out-of-range id in the graph's indices, or
// an internal error).  The first failing element of the call stores bad_tag (-seq) to *bad,
// a word the call's sizes are published with, and records {seq, hop, edge, id, nnz, row} in
// dbg[0..5].  Tags carry the call's sequence number, so nothing needs resetting between calls
// and a later call never reports an earlier call's error.
struct IdCheck {
  int64_t *bad = nullptr;
  int64_t bad_tag = 0;
  int64_t *dbg = nullptr;
  uint64_t seq = 0;
  int64_t hop = 0;
};

// The last pass of a hop's relabel (direct layout): out_col[e] = lab[col[e]] in place,
// out_row[e] = lab[seeds[r]] when the seeds may repeat (else label(r) == r), then every touched
// node's val returns to empty.  The touched nodes are exactly the hop's unique ids, so the reset
// is one store per unique node (not one per seed and sampled edge).  Kept as a descriptor so the
// sampler can run it in the same launch as the next hop's prep (which uses the other table).
struct RelabelTail {
  const int64_t *seeds;
  Count Sc;
  const int64_t *d_nb;
  Table t;
  int remap_rows;
  int64_t *out_row;
  int64_t *out_col;
  const int64_t *unique;    // the hop's unique ids (first-occurrence order)
  const int64_t *d_nuniq;   // their count (device)
  int64_t nblk;  // 256-thread blocks covering S + nnz (upper bounds; >= nnz and >= U)
  // an id outside [0, t.n) (never produced by a correct hop) is reported here, if set; the
  // hop's count pass (k_dcount) has already checked the same ids before the sizes were
  // published, so this is the guard of the table indexing below
  IdCheck chk;
};

#ifdef __HIPCC__
// direct layout: node x's first position and label
__device__ __forceinline__ int32_t *dval(const Table &t, int64_t x) { return t.val + 2 * x; }
__device__ __forceinline__ int32_t *dlab(const Table &t, int64_t x) { return t.val + 2 * x + 1; }

__device__ __forceinline__ void report_bad_id(const IdCheck &c, int64_t e, int64_t id,
                                              int64_t nnz, int64_t row) {
  if (!c.bad) return;
  *c.bad = c.bad_tag;
  if (c.dbg && atomicMax(reinterpret_cast<unsigned long long *>(c.dbg),
                         (unsigned long long)c.seq) < (unsigned long long)c.seq) {
    c.dbg[1] = c.hop;
    c.dbg[2] = e;
    c.dbg[3] = id;
    c.dbg[4] = nnz;
    c.dbg[5] = row;
  }
}

// Ids are range-checked before they index the table (one compare each): a corrupt id yields -1
// in the output instead of an address outside the table.
__device__ __forceinline__ void relabel_tail_block(const RelabelTail &r, int64_t blk) {
  const int64_t nb = *r.d_nb;
  const int64_t nu = *r.d_nuniq;
  const int64_t e = blk * 256 + threadIdx.x;
  const uint64_t n = (uint64_t)r.t.n;
  if (e < nb) {
    const int64_t v = r.out_col[e];
    bool ok = (uint64_t)v < n;
    r.out_col[e] = ok ? *dlab(r.t, v) : -1;
    int64_t row = -1;
    if (r.remap_rows) {
      row = r.out_row[e];
      const int64_t x = (uint64_t)row < (uint64_t)r.Sc.get() ? r.seeds[row] : -1;
      ok &= (uint64_t)x < n;
      r.out_row[e] = (uint64_t)x < n ? *dlab(r.t, x) : -1;
    }
    if (!ok) report_bad_id(r.chk, e, v, nb, row);
  }
  // (the label loads above read the other word of the pair: no conflict with the resets)
  if (e < nu) {
    const int64_t u = r.unique[e];
    if ((uint64_t)u < n) *dval(r.t, u) = kTableNoPos;
  }
}

__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

// Inserts key x seen at position pos; the slot keeps min(pos).  64-bit CAS on the key, linear
// probing, load factor <= 0.5.
__device__ __forceinline__ uint32_t table_insert(const Table &t, int64_t x, int32_t pos) {
  uint64_t h = fmix64((uint64_t)x) & t.mask;
  while (true) {
    int64_t cur = t.key[h];
    if (cur == kTableEmpty) {
      cur = (int64_t)atomicCAS((unsigned long long *)(t.key + h),
                               (unsigned long long)kTableEmpty, (unsigned long long)x);
      if (cur == kTableEmpty) cur = x;
    }
    if (cur == x) break;
    h = (h + 1) & t.mask;
  }
  // val only decreases: skip the atomic when an earlier occurrence is already recorded
  // (hub nodes recur thousands of times per hop; this removes the same-address atomics).
  if (t.val[h] > pos) atomicMin(t.val + h, pos);
  return (uint32_t)h;
}

__device__ __forceinline__ void table_record(const Table &t, int64_t x, int64_t pos) {
  if (t.direct) {
    // val only decreases: skip the atomic when an earlier occurrence is already recorded.  (A
    // no-return atomic without the check measured 1.8x slower on the last hop: hot nodes
    // recur ~1000 times per hop and same-address atomics serialise.)  Ids outside [0, n) are
    // not recorded (a corrupt id must not address memory outside the table).
    if ((uint64_t)x >= (uint64_t)t.n) return;
    int32_t *v = dval(t, x);
    if (*v > (int32_t)pos) atomicMin(v, (int32_t)pos);
  } else if (t.key) {
    t.slot_of[pos] = table_insert(t, x, (int32_t)pos);
  }
}

__device__ __forceinline__ int64_t table_find(const Table &t, int64_t x) {
  uint64_t h = fmix64((uint64_t)x) & t.mask;
  while (true) {
    const int64_t cur = t.key[h];
    if (cur == x) return (int64_t)h;
    if (cur == kTableEmpty) return -1;
    h = (h + 1) & t.mask;
  }
}
#endif

}  // namespace dgs
