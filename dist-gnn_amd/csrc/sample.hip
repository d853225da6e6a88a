// sample.hip -- row-wise neighbour sampling (uniform and biased) for one hop.
//
// Reference kernels restated (bit-exact outputs for a given launch seed):
//   K1/K2/K3  rowwise_sampling.cu:16-141       (uniform, without / with replacement)
//   K4/K5/K6  rowwise_sampling_bias.cu:16-224  (A-Res without replacement, CDF with)
//   K7-K12    rowwise_sampling{,_bias}_p2p.cu   (the same over cached / peer / host rows)
//
// RNG parity.  The reference launches one 128-thread block per row (uniform) or one 32-lane
// warp per row chain of 4 rows inside 16-row blocks (biased), and draws curand Philox numbers
// per thread.  Philox is counter based, so the j-th draw of thread t is a pure function
// philox(key = seed*G + block, counter = (j/4, subsequence = t)).word[j%4]; the kernels below
// evaluate exactly those logical coordinates from whatever physical lane does the work, which
// frees the schedule for wave64:
//   * uniform: 16-lane groups own rows (4 rows per wave, 16 per workgroup in flight); rows whose
//     reservoir tail (deg - k) exceeds kHubT are split into 512-edge chunks across waves of a
//     separate kernel (any split gives the same atomicMax result);
//   * biased: one 32-lane half-wave per row; the lane's draw offset inside its (block, warp)
//     RNG chain is recomputed from the degrees of the chain's earlier rows.
// Offsets come from a reduce-then-scan over 256-row tiles (no host sync inside the hop).
#include "dgs_block.cuh"
#include "dgs_lane.cuh"
#include "dgs_mod.cuh"
#include "dgs_ops.h"
#include "dgs_table.cuh"

namespace dgs {
namespace {

constexpr int kTileRows = 256;   // rows per prep / sample workgroup
// Lanes per row in the uniform row kernel (rows per workgroup = kTileRows / lanes).  Round 5
// A/B (profiles/r05_ab_uniform_row_group.txt): wider groups shorten one call's chain (sample
// span 171.6 -> 165.7 us with 64 lanes) but cost the 3-deep pipeline 2-3 %, narrower ones lose
// both ways -- synchronous calls use kGroupSolo, a loader's calls kGroup.
constexpr int kGroup = 16;
constexpr int kGroupSolo = 64;
constexpr int kHubT = 128;       // reservoir tail length above which a row goes to the hub kernel
#ifndef DGS_BIAS_HUB_T
#define DGS_BIAS_HUB_T 1024
#endif
// biased rows above this degree go to the hub kernels (round 3, streaming scheme: 1024 and 2048
// equal pipelined, 1024 has the shorter single call; 4096 -13 %.  Round 2's chunked scheme: 2048)
constexpr int kBiasHubT = DGS_BIAS_HUB_T;
constexpr int kHubBlocks = 1536; // workgroups of the hub kernel: 6 of 8 waves per SIMD, so the
                                 // other batches in flight (feature gather) find free slots
constexpr int kMaxPicksLds = 512;
constexpr int kScanThreads = 1024;

// Workgroups of the uniform hub kernel; DGS_HUB_BLOCKS overrides (occupancy experiments).
int hub_blocks() {
  static const int n = [] {
    const char *e = getenv("DGS_HUB_BLOCKS");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : kHubBlocks;
  }();
  return n;
}

constexpr int kBiasStreamBlocks = 768;  // round 3 A/B: 512-768 best, 1024 -1.5 %, 1536 -9 %
// A synchronous call (nothing beside it) prefers more workers: round 4's grid A/B
// (profiles/r04_ab_bias_stream_grid.txt) had 1024 best for one call (+2-5 %) and 768 for the
// pipeline.
constexpr int kBiasStreamBlocksSolo = 1024;
// Workgroups of the streaming kernel; DGS_BIAS_STREAM_BLOCKS overrides both.
int bias_stream_blocks(bool solo) {
  static const int n = [] {
    const char *e = getenv("DGS_BIAS_STREAM_BLOCKS");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 0;
  }();
  return n > 0 ? n : (solo ? kBiasStreamBlocksSolo : kBiasStreamBlocks);
}

// Upper bounds on the biased boot / merge grids (the hop's S bounds both); DGS_BIAS_BOOT_BLOCKS /
// DGS_BIAS_MERGE_BLOCKS override (round 5 A/B, papers-like: 4096 / 2048 at the plateau,
// profiles/r05_ab_bias_boot_merge_grid.txt).
int env_blocks(const char *name, int dflt) {
  const char *e = getenv(name);
  const int v = e ? atoi(e) : 0;
  return v > 0 ? v : dflt;
}
int bias_boot_blocks() {
  static const int n = env_blocks("DGS_BIAS_BOOT_BLOCKS", 4096);
  return n;
}
int bias_merge_blocks() {
  static const int n = env_blocks("DGS_BIAS_MERGE_BLOCKS", 2048);
  return n;
}

using RowInfo = NodeEntry;  // {absolute neighbour-id pointer, degree | location << 56}

__device__ __forceinline__ int64_t ri_deg(const RowInfo &r) { return r.dl & kOffMask; }
__device__ __forceinline__ int ri_loc(const RowInfo &r) {
  return (int)((uint64_t)r.dl >> kLocShift);
}

__device__ __forceinline__ RowInfo lookup_row(const RowSrc &src, int64_t v) {
  if (src.ntab) return src.ntab[v];
  const int64_t b = src.indptr[v], e = src.indptr[v + 1];
  RowInfo ri;
  ri.ptr = src.indices + b;
  ri.dl = e - b;  // location 0
  return ri;
}

// Probability array of a row: same offset as its neighbour ids inside the row's location.
__device__ __forceinline__ const float *row_probs(const RowSrc &src, const RowInfo &ri) {
  const int loc = ri_loc(ri);
  const int64_t *ib = nullptr;
  const float *pb = nullptr;
#pragma unroll
  for (int d = 0; d <= kMaxDevices; ++d) {
    if (loc == d) {
      ib = reinterpret_cast<const int64_t *>(src.indices_base.p[d]);
      pb = reinterpret_cast<const float *>(src.probs.p[d]);
    }
  }
  return pb + (ri.ptr - ib);
}

__device__ __forceinline__ int64_t row_count(int64_t deg, int64_t k, bool replace) {
  return replace ? (deg == 0 ? 0 : k) : (deg < k ? deg : k);
}

// Hub bookkeeping.  `count` is one packed word, (hubs << 40) | chunks: a hub registers with a
// single atomicAdd of (1 << 40) | its chunk count, which returns its index and its first chunk
// together, so chunk offsets are increasing in the hub index with no prefix-sum pass.
// Layout inside ws.hub (int64 words): [0..8) pad, hub_row[S], hub_cptr[S], hubid[S].
constexpr int kHubShift = 40;
constexpr uint64_t kHubChunkMask = (uint64_t(1) << kHubShift) - 1;
constexpr int64_t kHubMaxRows = int64_t(1) << 23;  // hub index field: 24 bits
struct HubView {
  // thr[h] (biased hubs): the best k-th A-Res key any worker of hub h has published, in the
  // order-preserving integer form of key_order().  aux[h]: what a worker moving to hub row h
  // needs besides the row index, written by prep so that it is not a load dependent on the
  // row's node-table entry -- the degree (uniform hubs) or the probability array (biased hubs;
  // the hub kernel then needs none of the per-location base pointers)
  int64_t *count, *row, *cptr, *hubid, *thr, *aux;
  __host__ __device__ static HubView make(int64_t *base, int64_t S) {
    HubView h;
    h.count = base;
    h.row = base + 8;
    h.cptr = h.row + S;
    h.hubid = h.cptr + S;
    h.thr = h.hubid + S;
    h.aux = h.thr + S;
    return h;
  }
  static size_t bytes(int64_t S) { return sizeof(int64_t) * (size_t)(8 + 5 * S); }
};

// Largest h in [0, H) with cptr[h] <= c (cptr nondecreasing, cptr[0] <= c), by a W-ary search:
// the W lanes of a wave (W = 64) or half-wave (W = 32, c uniform per half) probe W evenly
// spaced entries per round, so a hub list of H rows costs ceil(log_W H) dependent loads instead
// of log2 H (one round for H <= W, two for H <= W^2).  Every lane of the group must be active.
template <int W>
__device__ __forceinline__ int64_t group_search(const int64_t *cptr, int64_t H, int64_t c) {
  const int lane = threadIdx.x & (W - 1);
  int64_t lo = 0, n = H;  // answer in [lo, lo + n)
  while (n > 1) {
    const int64_t step = (n + W - 1) / W;
    const int64_t idx = lo + (int64_t)lane * step;
    const bool ok = lane == 0 || (idx < lo + n && cptr[idx] <= c);
    const uint64_t b = __ballot(ok);
    const uint64_t mine = W == 64 ? b : ((threadIdx.x & 32) ? (b >> 32) : (b & 0xFFFFFFFFull));
    const int cnt = __popcll(mine);  // nondecreasing probes: the ok lanes are a prefix
    const int64_t end = lo + n;
    lo += (int64_t)(cnt - 1) * step;
    n = end - lo < step ? end - lo : step;
  }
  return lo;
}

// float -> int with the same order (negative floats have reversed magnitude bits)
__device__ __forceinline__ int32_t key_order(float f) {
  const int32_t i = __float_as_int(f);
  return i >= 0 ? i : (i ^ 0x7FFFFFFF);
}
__device__ __forceinline__ float key_from_order(int32_t m) {
  return __int_as_float(m >= 0 ? m : (m ^ 0x7FFFFFFF));
}

// Biased hub rows, streaming scheme (see k_bias_boot / k_bias_stream below): a threshold from
// a spread sample of 8 x kBiasSampleSteps 32-edge steps (4096 edges), then every edge is tested
// against it.
#ifndef DGS_BIAS_SAMPLE_STEPS
#define DGS_BIAS_SAMPLE_STEPS 16
#endif
constexpr int64_t kBiasSampleSteps = DGS_BIAS_SAMPLE_STEPS;
// Steps per streamed chunk (a chunk = 32 kStreamT edges; one new Philox block per 4 steps).
// Round 3 A/B: 8 steps +3 % over 4 (90 against 75 VGPRs, but half the row switches and
// threshold loads per edge); 12 equal, 16 -4 %.
#ifndef DGS_BIAS_STREAM_T
#define DGS_BIAS_STREAM_T 8
#endif
constexpr int kStreamT = DGS_BIAS_STREAM_T;
constexpr int kStreamChunk = 32 * kStreamT;
// Candidates k_bias_stream holds per half-wave in LDS before appending them to the rows' lists
// (a flush when more than 64 wait; a chunk adds at most kStreamChunk).
constexpr int kStreamBuf = 64 + kStreamChunk;

static_assert(kStreamT % 4 == 0, "whole Philox blocks per chunk");
// Chunks of a streamed row: its lanes' steps shifted by up to 3 (k_bias_stream aligns a lane's
// chunks to its Philox blocks), at most deg / kStreamChunk + 2.
__host__ __device__ __forceinline__ int64_t bias_stream_chunks(int64_t deg) {
  return ((deg + 31) / 32 + 3 + kStreamT - 1) / kStreamT;
}
// Candidate room of the streamed rows.  The sample threshold lets about k * deg / P of a row's
// edges through (P = min(deg, 4096) sampled edges), i.e. about k for rows the sample covers and
// k / 32 per 128-edge chunk for larger ones.  The room is linear in the row's chunk range, so it
// is addressed from the chunk offset the hub registration already returns (no second counter):
// 16 kk per hub plus kk / 4 per chunk, kk = max(k, 8): >= 8x the expectation (small k is sized
// as 8: the spread of a small order statistic is wider).  A row that overflows is recomputed
// exactly (slow, rare).
__host__ __device__ __forceinline__ int64_t bias_room_start(int64_t h, int64_t chunk, int64_t k) {
  const int64_t kk = k < 8 ? 8 : k;
  return 16 * kk * h + kk * chunk / 4;
}

// Per-hub candidate lists of the streaming scheme: hub h owns key/idx[base[h], base[h] +
// cap[h]); cnt[h] counts appends (> cap[h]: overflowed, recomputed by the merge).
struct BiasCand {
  int32_t *cnt;
  int32_t *cap;
  int64_t *base;
  float *key;
  int32_t *idx;
  int64_t limit;                // entries of key / idx
  int64_t cap_max;              // test hook (DGS_BIAS_TEST_CAP): caps every row's room
};

// ------------------------------------------------------------------------------------
// Prep: per-row lookup (one 16-byte node-table load), per-row in-tile output prefix, tile
// sums, hub detection (+ hub slot initialisation, slot s = s: rowwise_sampling.cu:80-82).
struct PrepArgs {
  RowSrc src;
  const int64_t *seeds;
  Count Sc;
  int64_t k;
  int replace;
  int use_hubs;  // 0 none, 1 uniform hubs, 2 biased hubs
  int bias_replace;
  RowInfo *rowinfo;
  int32_t *tpre;
  int32_t *tpre2;
  int64_t *bsum;
  int64_t *tsum;
  HubView hub;
  int32_t *hubslot;
  Table table;
  int64_t *next_hub_count;
  BiasCand cand;  // biased hubs: per-row candidate lists
};

__device__ __forceinline__ void prep_block(const PrepArgs &a, int64_t blk) {
  __shared__ int64_t lds[kTileRows / 64];
  const int64_t S = a.Sc.get();
  const int64_t k = a.k;
  // the next hop's counter was last used two hops ago: reset it here (no memset launch)
  if (blk == 0 && threadIdx.x == 0) *a.next_hub_count = 0;
  if (blk * kTileRows >= S) return;  // whole workgroup past the live rows
  const int64_t i = blk * kTileRows + threadIdx.x;
  int64_t cnt = 0, tdeg = 0;
  if (i < S) {
    const int64_t v = a.seeds[i];
    const bool ok = (uint64_t)v < (uint64_t)a.src.num_nodes;
    const RowInfo ri = ok ? lookup_row(a.src, v) : RowInfo{nullptr, 0};
    a.rowinfo[i] = ri;
    if (ok) {
      table_record(a.table, v, i);
    } else if (a.src.bad) {
      *a.src.bad = a.src.bad_tag;
    }
    const int64_t deg = ri_deg(ri);
    cnt = row_count(deg, k, a.replace);
    tdeg = deg;
    if (a.use_hubs) {
      int64_t h = -1;
      // 1: uniform hubs (reservoir tail > kHubT, 512-edge chunks); 2: biased hubs (degree >
      // kBiasHubT, kStreamChunk-edge chunks)
      const bool is_hub = a.use_hubs == 1 ? deg - k > kHubT : deg > kBiasHubT;
      if (is_hub) {
        const uint64_t nch = a.use_hubs == 1 ? (uint64_t)(deg - k + 511) / 512
                                             : (uint64_t)bias_stream_chunks(deg);
        const uint64_t old = atomicAdd((unsigned long long *)a.hub.count,
                                       (unsigned long long)((uint64_t(1) << kHubShift) | nch));
        h = (int64_t)(old >> kHubShift);
        a.hub.row[h] = i;
        a.hub.cptr[h] = (int64_t)(old & kHubChunkMask);
        if (a.use_hubs == 1) {
          for (int64_t s2 = 0; s2 < k; ++s2) a.hubslot[i * k + s2] = (int32_t)s2;
          a.hub.aux[h] = deg;
        } else {
          a.hub.thr[h] = key_order(-__builtin_inff());
          a.hub.aux[h] = (int64_t)row_probs(a.src, ri);
          {  // the row's candidate room, addressed from its chunk offset
            const int64_t c0 = (int64_t)(old & kHubChunkMask);
            const int64_t b = bias_room_start(h, c0, k);
            int64_t cap = bias_room_start(h + 1, c0 + (int64_t)nch, k) - b;
            if (cap > a.cand.cap_max) cap = a.cand.cap_max;
            if (b + cap > a.cand.limit) cap = 0;  // out of room: recomputed
            a.cand.base[h] = b;
            a.cand.cap[h] = (int32_t)cap;
            a.cand.cnt[h] = 0;
          }
        }
      }
      a.hub.hubid[i] = h;
    }
  }
  int64_t tot;
  const int64_t ex = block_exclusive_scan<kTileRows>(cnt, &tot, lds);
  if (i < S) a.tpre[i] = (int32_t)ex;
  if (threadIdx.x == 0) a.bsum[blk] = tot;
  if (a.bias_replace) {
    const int64_t ex2 = block_exclusive_scan<kTileRows>(tdeg, &tot, lds);
    if (i < S) a.tpre2[i] = (int32_t)ex2;
    if (threadIdx.x == 0) a.tsum[blk] = tot;
  }
}

// Prep: per-row lookup (one 16-byte node-table load), in-tile output prefix, tile sums, hub
// registration, relabel insert of the seeds.
__global__ __launch_bounds__(kTileRows) void k_prep(PrepArgs a) {
  latency_prio();
  prep_block(a, blockIdx.x);
}

// The previous hop's relabel pass (blocks [0, tail.nblk), on the other relabel table) and this
// hop's prep in one launch: both only need the previous hop's unique frontier.
__global__ __launch_bounds__(kTileRows) void k_prep_tail(PrepArgs a, RelabelTail tail) {
  latency_prio();
  if ((int64_t)blockIdx.x < tail.nblk)
    relabel_tail_block(tail, blockIdx.x);
  else
    prep_block(a, (int64_t)blockIdx.x - tail.nblk);
}

// Single workgroup: exclusive scan of tile sums (-> boff[0..nb], boff[nb] = nnz; the same for
// the CDF sizes when biased-with-replacement).
__global__ __launch_bounds__(kScanThreads) void k_scan_hop(const int64_t *bsum,
                                                          const int64_t *tsum, Count Sc,
                                                          int64_t *boff, int64_t *tboff,
                                                          int64_t *d_nnz, int64_t *d_cdf_total) {
  latency_prio();
  __shared__ int64_t lds[kScanThreads / 64];
  const int64_t nb = (Sc.get() + kTileRows - 1) / kTileRows;
  for (int pass = 0; pass < 2; ++pass) {
    const int64_t *in = pass ? tsum : bsum;
    int64_t *out = pass ? tboff : boff;
    if (!in) continue;
    const int64_t tot = block_scan_range<kScanThreads, 4>(in, nb, out, lds);
    if (threadIdx.x == 0) {
      out[nb] = tot;
      *(pass ? d_cdf_total : d_nnz) = tot;
    }
  }
}

// ------------------------------------------------------------------------------------
// Uniform sampling (rowwise_sampling.cu K2/K3).  Arguments shared by the kernels below.
struct UniformArgs {
  RowSrc src;
  Count Sc;
  int64_t k;
  uint64_t seed;
  const RowInfo *rowinfo;
  const int32_t *tpre;
  const int64_t *boff;
  HubView hub;
  int32_t *hubslot;
  int64_t *rowpos;
  int64_t *col;
  Table table;
  // a synchronous call (nothing else of ours beside it): the hub reservoir's waves lower their
  // issue priority as they progress (see hub_reservoir)
  int solo;
};

// A sampled neighbour id.  Most rows are read once per batch: non-temporal loads keep these
// reads from displacing lines other kernels reuse (same-box A/B: +0.3-1 % uniform, 6/6 rounds).
__device__ __forceinline__ int64_t nb_load(global_ptr<int64_t> nb, int64_t i) {
  return __builtin_nontemporal_load(&nb[i]);
}

// Writes the k picks of row r whose reservoir slots are `slots` (16-lane group, lane L).
template <int G>
__device__ __forceinline__ void emit_slots(const UniformArgs &a, int64_t S, int64_t r,
                                           global_ptr<int64_t> nb, int64_t out,
                                           const int32_t *slots, int L) {
  for (int64_t s2 = L; s2 < a.k; s2 += G) {
    const int64_t v = nb_load(nb, slots[s2]);
    a.rowpos[out + s2] = r;
    a.col[out + s2] = v;
    table_record(a.table, v, S + out + s2);
  }
}

// The 8 draws of one lane in one 512-edge hub chunk (idx = k + 512 q + lane + 64 tt + 128 w)
// with 32-bit indices: every idx of the chunk is below 2^30.
// kFull: the whole chunk lies inside the row (no per-draw bound test).  Each draw keeps its
// own branch: a wave enters it only when one of its 64 lanes hits (k / idx per lane); one
// branch over all 8 draws was measured slower (a wave then enters it 8 times as often).
template <bool kFull, typename Mod>
__device__ __forceinline__ void hub_chunk32(const uint4 &o4a, const uint4 &o4b, int64_t q,
                                            int64_t k, int64_t deg, int lane, int32_t *sl,
                                            Mod mod) {
  const uint32_t b0 = (uint32_t)(k + 512 * q) + (uint32_t)lane;
  const uint32_t deg32 = (uint32_t)deg, k32 = (uint32_t)k;
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const uint4 o4 = tt ? o4b : o4a;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const uint32_t idx = b0 + 64u * tt + 128u * w;
      const uint32_t num = mod(u4_get(o4, w), idx + 1u);
      if (num < k32 && (kFull || idx < deg32)) atomicMax(sl + num, (int32_t)idx);
    }
  }
}

// Hub reservoir: wave gw of nwaves takes a contiguous range of 512-edge chunks
// (idx = k + 512q + t + 128w, t < 128, w < 4 <-> one Philox block per logical thread t) of the
// hub rows and folds their picks into the rows' k global slots with atomicMax
// (rowwise_sampling.cu:85-92; any split gives the same maxima).
__device__ __forceinline__ void hub_reservoir(const UniformArgs &a, int64_t gw, int64_t nwaves) {
  const int64_t S = a.Sc.get();
  const int64_t k = a.k;
  const HubView &hub = a.hub;
  const uint64_t packed = (uint64_t)*hub.count;
  const int64_t H = (int64_t)(packed >> kHubShift);
  if (H == 0) return;
  const int64_t total = (int64_t)(packed & kHubChunkMask);
  const int lane = threadIdx.x & 63;
  // One binary search per wave, then the hub index only moves forward (a dependent search per
  // chunk would dominate the Philox work).
  const int64_t c0 = total * gw / nwaves, c1 = total * (gw + 1) / nwaves;
  if (c0 >= c1) return;
  int64_t h = group_search<64>(hub.cptr, H, c0);  // largest h with cptr[h] <= c0
  int64_t hstart = hub.cptr[h], hnext = h + 1 < H ? hub.cptr[h + 1] : total;
  // per-row values, made wave-uniform once per row (scalar key and slot address: nothing of
  // the row is recomputed per chunk)
  int64_t r = 0, deg = 0;
  uint2 kk;
  int32_t *sl = nullptr;
  auto load_row = [&]() {
    r = (int64_t)wave_uniform((uint64_t)hub.row[h]);
    deg = (int64_t)wave_uniform((uint64_t)hub.aux[h]);
    const uint64_t key = a.seed * (uint64_t)S + (uint64_t)r;
    kk = make_uint2((uint32_t)key, (uint32_t)(key >> 32));
    sl = a.hubslot + r * k;
  };
  load_row();
  // A synchronous call (a.solo): each wave lowers its issue priority as it works through its
  // share (2 in its first third, then 1, then 0).  The waves sharing a SIMD are otherwise
  // served oldest first and finish one after another; this way the youngest catch up and the
  // kernel's tail shrinks (round 5: one call's sample span 176.7 -> 171.8 us).  Inside the
  // 3-deep pipeline the same schedule cost 6 %, so a loader's calls keep the hardware order.
  int level = -1;
  for (int64_t c = c0; c < c1; ++c) {
    if (a.solo) {
      const int lv = 2 - (int)((3 * (c - c0)) / (c1 - c0));
      if (lv != level) {
        level = lv;
        if (lv >= 2)
          __builtin_amdgcn_s_setprio(2);
        else if (lv == 1)
          __builtin_amdgcn_s_setprio(1);
        else
          __builtin_amdgcn_s_setprio(0);
      }
    }
    while (c >= hnext) {
      ++h;
      hstart = hnext;
      hnext = h + 1 < H ? hub.cptr[h + 1] : total;
      load_row();
    }
    const int64_t q = c - hstart;
    const uint4 o4a = philox4x32_10(
        make_uint4((uint32_t)q, (uint32_t)((uint64_t)q >> 32), (uint32_t)lane, 0u), kk);
    const uint4 o4b = philox4x32_10(
        make_uint4((uint32_t)q, (uint32_t)((uint64_t)q >> 32), (uint32_t)(lane + 64), 0u), kk);
    // every d = idx + 1 of this chunk lies in [k + 512 q + 1, k + 512 q + 512]: the modulo
    // is chosen per chunk (wave-uniform test); the 32-bit forms are branch-free up to the (rare)
    // hit, and a chunk entirely inside the row skips the bound test
    const int64_t dmin = k + 512 * q + 1;
    const bool full = dmin + 511 <= deg;
    if (full && dmin >= (int64_t)kModBigMin && deg < (int64_t(1) << 24))
      hub_chunk32<true>(o4a, o4b, q, k, deg, lane, sl, mod_big<true>);
    else if (dmin >= (int64_t)kModBigMin && deg < (int64_t(1) << 24))
      hub_chunk32<false>(o4a, o4b, q, k, deg, lane, sl, mod_big<true>);
    else if (dmin >= (int64_t)kModBigMin && deg < (int64_t(1) << 30))
      hub_chunk32<false>(o4a, o4b, q, k, deg, lane, sl, mod_big<false>);
    else if (dmin + 511 <= (int64_t)kModMidMax && dmin >= 257)
      hub_chunk32<false>(o4a, o4b, q, k, deg, lane, sl, mod_mid<true>);
    else if (dmin + 511 <= (int64_t)kModMidMax)
      hub_chunk32<false>(o4a, o4b, q, k, deg, lane, sl, mod_mid<false>);
    else {
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const uint4 o4 = tt ? o4b : o4a;
        const int64_t base = k + lane + 64 * tt + 512 * q;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const int64_t idx = base + 128 * w;
          if (idx < deg) {
            const uint32_t num = u4_get(o4, w) % (uint32_t)(idx + 1);
            if ((int64_t)num < k) atomicMax(sl + num, (int32_t)idx);
          }
        }
      }
    }
  }
}

// Rows of one 16-row block, a 16-lane group per row.  A hub row (hubid >= 0) takes its k picks
// from the global slots k_hub_reservoir filled.
template <bool kReplace, int G>
__device__ __forceinline__ void sample_rows(const UniformArgs &a, int64_t blk, int32_t *s_slot,
                                            bool use_hubs) {
  const int64_t S = a.Sc.get();
  const int64_t k = a.k;
  const int g = threadIdx.x / G, L = threadIdx.x % G;
  const int64_t r = blk * (kTileRows / G) + g;
  if (r >= S) return;
  int32_t *sl = s_slot + g * k;
  const RowInfo ri = a.rowinfo[r];
  const int64_t deg = ri_deg(ri);
  const global_ptr<int64_t> nb = as_global(ri.ptr);
  const int64_t out = a.boff[r / kTileRows] + a.tpre[r];
  const uint64_t key = a.seed * (uint64_t)S + (uint64_t)r;
  const uint2 kk = make_uint2((uint32_t)key, (uint32_t)(key >> 32));
  if (kReplace) {
    if (deg > 0) {
      for (int64_t p = L; p < k; p += G) {
        const int64_t t = p & 127, j = p >> 7;
        const uint4 o4 = philox4x32_10(make_uint4((uint32_t)(j >> 2), 0u, (uint32_t)t, 0u), kk);
        const uint32_t x = u4_get(o4, (int)(j & 3));
        const int64_t e = (int64_t)x % deg;
        const int64_t v = nb[e];
        a.rowpos[out + p] = r;
        a.col[out + p] = v;
        table_record(a.table, v, S + out + p);
      }
    }
    return;
  }
  if (deg <= k) {
    for (int64_t p = L; p < deg; p += G) {
      const int64_t v = nb_load(nb, p);
      a.rowpos[out + p] = r;
      a.col[out + p] = v;
      table_record(a.table, v, S + out + p);
    }
    return;
  }
  // a hub row (prep's test, from the degree alone: no hub-index load) takes the slots
  // k_hub_reservoir filled; they are indexed by row
  if (use_hubs && deg - k > kHubT) {
    emit_slots<G>(a, S, r, nb, out, a.hubslot + r * k, L);
    return;
  }
  for (int64_t s2 = L; s2 < k; s2 += G) sl[s2] = (int32_t)s2;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  for (int64_t q = 0; k + 512 * q < deg; ++q) {
    for (int tt = 0; tt < 128 / G; ++tt) {
      const int t = L + G * tt;
      const int64_t base = k + t + 512 * q;
      if (base >= deg) break;
      const uint4 o4 = philox4x32_10(
          make_uint4((uint32_t)q, (uint32_t)((uint64_t)q >> 32), (uint32_t)t, 0u), kk);
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const int64_t idx = base + 128 * w;
        if (idx < deg) {
          // every row here has deg <= k + 128 when hubs are on (group-uniform test)
          const uint32_t x = u4_get(o4, w), d = (uint32_t)(idx + 1);
          const uint32_t num = deg <= (int64_t)kModMidMax ? mod_mid<false>(x, d) : x % d;
          if ((int64_t)num < k) atomicMax(sl + num, (int32_t)idx);
        }
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  emit_slots<G>(a, S, r, nb, out, sl, L);
}

// Hub kernel.  Its workgroup 0 first does the hop's tile-offset scan (k_scan_hop's job:
// boff[0..nb] from the prep tile sums, nnz), which the sampling kernel after it reads -- one
// launch fewer per hop.
__global__ __launch_bounds__(256) void k_hub_reservoir(UniformArgs a, const int64_t *bsum,
                                                       int64_t *boff, int64_t *d_nnz,
                                                       uint64_t *stamp) {
  // profiling only (DGS_PROF_HUB: stamp != nullptr, a kernel argument: uniform branch)
  if (stamp && threadIdx.x == 0) stamp[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  if (blockIdx.x == 0) {
    __shared__ int64_t lds[256 / 64];
    const int64_t nb = (a.Sc.get() + kTileRows - 1) / kTileRows;
    const int64_t tot = block_scan_range<256, 8>(bsum, nb, boff, lds);
    if (threadIdx.x == 0) {
      boff[nb] = tot;
      *d_nnz = tot;
    }
  }
  // the wave index is wave-uniform: chunk bookkeeping and the chunk index (Philox counter
  // word 0) then live in scalar registers, and so do the first round's M0 * q product and the
  // second round's M1 product of both Philox blocks of a chunk
  const int64_t gw = (int64_t)blockIdx.x * (blockDim.x >> 6) +
                     __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  hub_reservoir(a, gw, ((int64_t)gridDim.x * blockDim.x) >> 6);
  if (stamp) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) stamp[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

template <bool kReplace, int G>
__global__ __launch_bounds__(kTileRows) void k_sample_uniform(UniformArgs a, int use_hubs) {
  latency_prio();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  sample_rows<kReplace, G>(a, blockIdx.x, reinterpret_cast<int32_t *>(smem), use_hubs != 0);
}

// ------------------------------------------------------------------------------------
// Biased sampling.  A-Res key (DGS-AMD definition, see oracle/dgs_oracle.c): key = log2(u)/p
// with a fixed-operation log2; p <= 0 -> -inf.  Total order: key desc, edge index asc.
__device__ __forceinline__ float dgs_log2f(float u) {
  uint32_t b = __float_as_uint(u);
  int32_t e = (int32_t)((b >> 23) & 0xFFu) - 127;
  float m = __uint_as_float((b & 0x007FFFFFu) | 0x3F800000u);
  if (m > 1.41421356f) {
    m = __fmul_rn(m, 0.5f);
    e += 1;
  }
  const float f = __fsub_rn(m, 1.0f);
  const float s = __fdiv_rn(f, __fadd_rn(2.0f, f));
  const float s2 = __fmul_rn(s, s);
  float q = __fmaf_rn(s2, 0.11111111f, 0.14285715f);
  q = __fmaf_rn(s2, q, 0.2f);
  q = __fmaf_rn(s2, q, 0.33333334f);
  q = __fmaf_rn(s2, q, 1.0f);
  const float t = __fmul_rn(2.0f, s);
  const float ln = __fmul_rn(t, q);
  return __fmaf_rn(ln, 1.44269504f, (float)e);
}

__device__ __forceinline__ float ares_key(float u, float p) {
  if (!(p > 0.0f)) return -__builtin_inff();
  return __fdiv_rn(dgs_log2f(u), p);
}

__device__ __forceinline__ bool ares_better(float ka, int64_t ia, float kb, int64_t ib) {
  return ka > kb || (ka == kb && ia < ib);
}
__device__ __forceinline__ bool ares_better(float ka, int32_t ia, float kb, int32_t ib) {
  return ka > kb || (ka == kb && ia < ib);
}

// Cheap pre-test of the A-Res key against the current k-th best: an edge can only enter the top-k
// if key = RN(log2f(u) / p) >= thr, which needs log2f(u) >= p * thr (p > 0, rounding aside).
// The hardware log2 (v_log_f32) stands in for the fixed-operation log2 with slack (relative
// 2^-16 of p * thr plus absolute 2^-16) far above both functions' error, so a rejected edge is
// certainly not a candidate; survivors get the exact key.  Not used while thr is -inf.
// Straight-line form (round 3: the && / || chains compiled to a branch per edge), with the
// slack factor folded into the threshold once: thr_s = slack_thr(thr) = thr * (1 + 2^-16) (one
// more rounding, 2^-24 relative, far inside the 2^-16 slack).  p <= 0 fails the p > 0 test;
// thr = -inf gives a NaN or -inf bound, which the callers never test (they filter only once
// the threshold is finite).  A NaN bound lets the edge through: p = +inf with thr = 0 makes
// p * thr NaN while the edge's key (+-0) ties thr (round 3: `>=` dropped it;
// tests/test_gpu_parity.py::test_bias_filter_bounds_are_sound).
__device__ __forceinline__ float slack_thr(float thr) { return thr * 1.0000152587890625f; }
__device__ __forceinline__ bool ares_may_pass_s(float u, float p, float thr_s) {
  return (p > 0.0f) &
         !(__builtin_amdgcn_logf(u) < __builtin_fmaf(p, thr_s, -0.0000152587890625f));
}

// (a & mask) | (b & ~mask): one v_bfi_b32
__device__ __forceinline__ uint32_t bitsel(uint32_t mask, uint32_t a, uint32_t b) {
  return (a & mask) | (b & ~mask);
}

// number of edges i < d with i = l (mod 32)
__device__ __forceinline__ int64_t lane_draws(int64_t d, int l) {
  return d > l ? (d - 1 - l) / 32 + 1 : 0;
}

// 32-bit ballot of this half-wave.
__device__ __forceinline__ uint32_t half_ballot(bool p) {
  const uint64_t b = __ballot(p);
  return (threadIdx.x & 32) ? (uint32_t)(b >> 32) : (uint32_t)b;
}

template <typename T>
__device__ __forceinline__ T float_max(T a, T b) {
  return fmaxf(a, b);
}

constexpr int kBiasRowsPerBlock = kTileRows / 32;  // one 32-lane half-wave per row
#ifndef DGS_SPARSE_PUSH
#define DGS_SPARSE_PUSH 10
#endif
constexpr int kSparsePush = DGS_SPARSE_PUSH;  // candidate batches up to this size are inserted one by one

// Half-wave top-k under the total order (key desc, edge index asc): lane q holds the q-th best
// (key, idx) so far (a sorted list of 32; the first k count), thr = the k-th best.  A step's
// candidates (one per lane) that beat thr are merged in one batch: bitonic sort of the 32
// candidates, then a bitonic merge with the list (the reference's WarpSelect idea, on 32-lane
// halves of a wave64).  Once the list is full almost no step has a candidate, so the common
// cost is one compare and one ballot.
// Edge indices are row-local and 32-bit (a row holds < 2^31 - 1 edges; Sampler checks), which
// keeps every compare-exchange at two cross-lane shuffles.
struct HalfTopK {
  float bk = -__builtin_inff();
  int32_t bi = INT32_MAX;  // INT32_MAX: empty
  int cnt = 0;
  float thr_k = -__builtin_inff();
  int32_t thr_i = INT32_MAX;
  static __device__ __forceinline__ void cas(float &k, int32_t &i, int partner_mask, bool better_here) {
    const float pk = lane_xor32v(k, partner_mask);
    const int32_t pi = lane_xor32v(i, partner_mask);
    const bool pb = ares_better(pk, pi, k, i);  // partner's entry is the better one
    if (better_here ? pb : !pb) {
      k = pk;
      i = pi;
    }
  }
  // One candidate (ck, ci), the same on every lane, into the sorted list: the entries that
  // beat it are a prefix of length pos; the rest move down a lane (the 32nd drops out).
  __device__ __forceinline__ void insert_one(float ck, int32_t ci, int l) {
    const int pos = __builtin_popcount(half_ballot(ares_better(bk, bi, ck, ci)));
    const float uk = lane_up1_32(bk);
    const int32_t ui = lane_up1_32(bi);
    if (l > pos) {
      bk = uk;
      bi = ui;
    } else if (l == pos) {
      bk = ck;
      bi = ci;
    }
  }
  __device__ __forceinline__ void push(float key_i, int32_t i, bool valid, int64_t k, int l) {
    const bool cand = valid && ares_better(key_i, i, thr_k, thr_i);
    uint32_t m = half_ballot(cand);
    if (!m) return;
    if (__builtin_popcount(m) <= kSparsePush) {
      // few candidates: insert them one by one (a broadcast, a ballot and a lane shift each)
      // instead of sorting 32 lanes -- the same top-32 list either way
      do {
        const int src = __builtin_ctz(m);
        m &= m - 1;
        insert_one(__shfl(key_i, src, 32), __shfl(i, src, 32), l);
      } while (m);
      update_thr(k, l);
      return;
    }
    float ck = cand ? key_i : -__builtin_inff();
    int32_t ci = cand ? i : INT32_MAX;
    // bitonic sort of the candidates, descending
#pragma unroll
    for (int size = 2; size <= 32; size <<= 1) {
#pragma unroll
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        const bool desc = (l & size) == 0 || size == 32;
        const bool lower = (l & stride) == 0;
        cas(ck, ci, stride, desc == lower);
      }
    }
    merge_sorted(ck, ci, k, l);
  }
  // Candidates that already form a bitonic sequence over the 32 lanes -- one list sorted
  // descending (sorted=true: nothing to do), or a descending list in lanes 0-15 followed by an
  // ascending one in 16-31 (one bitonic merge) -- skip the candidate sort.  Dropping the
  // entries that do not beat thr keeps either shape.
  __device__ __forceinline__ void push_bitonic(float key_i, int32_t i, bool valid, int64_t k,
                                               int l, bool sorted) {
    const bool cand = valid && ares_better(key_i, i, thr_k, thr_i);
    if (!half_ballot(cand)) return;
    float ck = cand ? key_i : -__builtin_inff();
    int32_t ci = cand ? i : INT32_MAX;
    if (!sorted) {
#pragma unroll
      for (int stride = 16; stride > 0; stride >>= 1) cas(ck, ci, stride, (l & stride) == 0);
    }
    merge_sorted(ck, ci, k, l);
  }
  // top 32 of the list and 32 candidates sorted descending: pairwise best against the
  // reversed candidates (a bitonic sequence), then a descending bitonic merge
  __device__ __forceinline__ void merge_sorted(float ck, int32_t ci, int64_t k, int l) {
    const float rk = lane_rev32(ck);
    const int32_t ri = lane_rev32(ci);
    if (ares_better(rk, ri, bk, bi)) {
      bk = rk;
      bi = ri;
    }
#pragma unroll
    for (int stride = 16; stride > 0; stride >>= 1) cas(bk, bi, stride, (l & stride) == 0);
    update_thr(k, l);
  }
  __device__ __forceinline__ void update_thr(int64_t k, int l) {
    cnt = __builtin_popcount(half_ballot(l < k && bi != INT32_MAX));
    thr_k = half_bcast(bk, (int)(k - 1));
    thr_i = half_bcast(bi, (int)(k - 1));
  }
  // true once k entries are held and the threshold is finite (ares_may_pass is then valid)
  __device__ __forceinline__ bool filtering(int64_t k) const {
    return cnt >= k && thr_k > -__builtin_inff();
  }
};

template <bool kReplace>
__device__ __forceinline__ void sample_bias_block(
    const RowSrc &src, Count Sc, int64_t k, uint64_t seed, const RowInfo *__restrict__ rowinfo,
    const int32_t *__restrict__ tpre, const int64_t *__restrict__ boff,
    const int32_t *__restrict__ tpre2, const int64_t *__restrict__ tboff, float *cdf,
    int64_t *__restrict__ rowpos, int64_t *__restrict__ col, const Table &table,
    const int64_t *__restrict__ hubid, int64_t blk) {
  const int64_t S = Sc.get();
  const int64_t G = (S + 15) / 16;  // reference grid: ceil(S / TILE_SIZE=16)
  const int hw = threadIdx.x >> 5, l = threadIdx.x & 31;
  {
    const int64_t r = blk * kBiasRowsPerBlock + hw;
    if (r >= S) return;
    const RowInfo ri = rowinfo[r];
    const int64_t deg = ri_deg(ri);
    const global_ptr<int64_t> nb = as_global(ri.ptr);
    const global_ptr<float> pr = as_global(row_probs(src, ri));
    const int64_t out = boff[r / kTileRows] + tpre[r];
    // reference coordinates: block b = r / 16, warp w = (r % 16) % 4, chain position m
    const int64_t b = r / 16;
    const int w = (int)((r % 16) & 3), m = (int)((r % 16) >> 2);
    const uint64_t key = seed * (uint64_t)G + (uint64_t)b;
    const uint2 kk = make_uint2((uint32_t)key, (uint32_t)(key >> 32));
    const uint32_t sub = kReplace ? (uint32_t)(4 * w + l) : (uint32_t)(32 * w + l);
    // draws this lane made on the chain's earlier rows (state persists, :86-88,144)
    int64_t j = 0;
    for (int mm = 0; mm < m; ++mm) {
      const int64_t d = ri_deg(rowinfo[b * 16 + w + 4 * mm]);
      if (kReplace) {
        if (d > 0) j += lane_draws(k, l);
      } else if (d > k) {
        j += lane_draws(d, l);
      }
    }
    if (!kReplace) {
      if (deg <= k) {
        for (int64_t p = l; p < deg; p += 32) {
          const int64_t v = nb[p];
          rowpos[out + p] = r;
          col[out + p] = v;
          table_record(table, v, S + out + p);
        }
        return;
      }
      if (hubid && hubid[r] >= 0) return;  // a hub row: k_bias_boot / _stream / the merge
      HalfTopK top;
      // Step s of this lane (edge i = 32 s + l) uses draw j + s.  Steps go in groups of 4
      // over a window of two Philox blocks, one new block per group for every lane alike (the
      // lanes' offsets inside a block differ, so a per-lane lazy refill would diverge into a
      // block per step); the draw is picked with bit-select masks on the offset.
      const int64_t bl = j >> 2;
      const int off = (int)(j & 3);
      const uint32_t m2 = (off & 2) ? ~0u : 0u, m1 = (off & 1) ? ~0u : 0u;
      uint4 A = philox4x32_10(make_uint4((uint32_t)bl, (uint32_t)((uint64_t)bl >> 32), sub, 0u), kk);
      bool filter = false;
      float thr_s = -__builtin_inff();
      const int64_t nsteps = (deg + 31) / 32;
      float pn[4];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const int64_t i = 32 * s4 + l;
        pn[s4] = i < deg ? pr[i] : 0.0f;
      }
      for (int64_t g = 0; 4 * g < nsteps; ++g) {
        float p[4];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          p[s4] = pn[s4];
          const int64_t i = 128 * (g + 1) + 32 * s4 + l;  // the next group's loads go out now
          pn[s4] = i < deg ? pr[i] : 0.0f;
        }
        const uint64_t qb = (uint64_t)(bl + g + 1);
        const uint4 B = philox4x32_10(make_uint4((uint32_t)qb, (uint32_t)(qb >> 32), sub, 0u), kk);
        const uint32_t wv[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
        uint32_t w2[5];
#pragma unroll
        for (int e = 0; e < 5; ++e) w2[e] = bitsel(m2, wv[e + 2], wv[e]);
        float u[4];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) u[s4] = curand_uniform_from(bitsel(m1, w2[s4 + 1], w2[s4]));
        if (!filter) {
          // No threshold yet (a row's first group): every edge is a candidate.  The lane's 4
          // exact keys are sorted in registers and pushed best first, so only the first push is
          // a full 32-candidate merge and the later ones meet the threshold it set (mostly
          // sparse inserts) -- the same list as any order.
          float kq[4];
          int32_t iq[4];
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            const int32_t i = (int32_t)(128 * g + 32 * s4 + l);
            const bool valid = i < deg;
            kq[s4] = valid ? ares_key(u[s4], p[s4]) : -__builtin_inff();
            iq[s4] = valid ? i : INT32_MAX;
          }
          auto cswap = [&](int x, int y) {
            if (ares_better(kq[y], iq[y], kq[x], iq[x])) {
              const float tk = kq[x];
              const int32_t ti = iq[x];
              kq[x] = kq[y];
              iq[x] = iq[y];
              kq[y] = tk;
              iq[y] = ti;
            }
          };
          cswap(0, 1);
          cswap(2, 3);
          cswap(0, 2);
          cswap(1, 3);
          cswap(1, 2);
#pragma unroll
          for (int q = 0; q < 4; ++q) top.push(kq[q], iq[q], iq[q] != INT32_MAX, k, l);
          if (top.filtering(k)) {
            filter = true;
            thr_s = slack_thr(top.thr_k);
          }
          A = B;
          continue;
        }
        uint32_t mk = 0;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const bool valid = 128 * g + 32 * s4 + l < deg;
          mk |= (uint32_t)(valid & ares_may_pass_s(u[s4], p[s4], thr_s)) << s4;
        }
        // candidates in rounds of one per lane (the resulting list does not depend on order)
        while (half_ballot(mk != 0)) {
          const bool has = mk != 0;
          const int t = has ? __builtin_ctz(mk) : 0;
          mk &= mk - 1;
          float ut = u[0], pt = p[0];
#pragma unroll
          for (int e = 1; e < 4; ++e) {
            ut = t == e ? u[e] : ut;
            pt = t == e ? p[e] : pt;
          }
          top.push(has ? ares_key(ut, pt) : -__builtin_inff(), (int32_t)(128 * g + 32 * t + l),
                   has, k, l);
          if (!filter && top.filtering(k)) {
            filter = true;
            thr_s = slack_thr(top.thr_k);
            uint32_t keep = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) keep |= (uint32_t)ares_may_pass_s(u[e], p[e], thr_s) << e;
            mk &= keep;
          }
        }
        if (top.filtering(k)) {
          filter = true;
          thr_s = slack_thr(top.thr_k);
        }
        A = B;
      }
      if (l < k) {
        const int64_t v = nb[top.bi];
        rowpos[out + l] = r;
        col[out + l] = v;
        table_record(table, v, S + out + l);
      }
    } else {
      if (deg == 0) return;
      // CDF, 32 edges at a time: lane 0 adds the running aggregate, clamp at 0, then a
      // Kogge-Stone inclusive scan (cub::WarpScan::InclusiveSum), :185-202.
      float *crow = cdf + tboff[r / kTileRows] + tpre2[r];
      float agg = 0.0f, sum = 0.0f;
      for (int64_t base = 0; base < deg; base += 32) {
        const int64_t i = base + l;
        float v = i < deg ? pr[i] : 0.0f;
        if (l == 0) v = __fadd_rn(v, agg);
        v = float_max(v, 0.0f);
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
          const float y = __shfl_up(v, o, 32);
          if (l >= o) v = __fadd_rn(y, v);
        }
        agg = __shfl(v, 31, 32);
        // the reference reads sum = cdf[deg - 1] (:207); lane 31's aggregate can differ from it
        // in the last partial chunk (different association), so take lane (deg - 1) % 32.
        if (base + 32 >= deg) sum = __shfl(v, (int)(deg - 1 - base), 32);
        if (i < deg) __hip_atomic_store(crow + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      for (int64_t p = l; p < k; p += 32) {
        const int64_t q = j >> 2;
        const uint4 o4 =
            philox4x32_10(make_uint4((uint32_t)q, (uint32_t)((uint64_t)q >> 32), sub, 0u), kk);
        const float u = curand_uniform_from(u4_get(o4, (int)(j & 3)));
        ++j;
        const float rnd = __fmul_rn(u, sum);
        // cub::UpperBound probe sequence
        int64_t ret = 0, n = deg;
        while (n > 0) {
          const int64_t half = n >> 1;
          const float cv =
              __hip_atomic_load(crow + ret + half, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (rnd < cv) {
            n = half;
          } else {
            ret = ret + half + 1;
            n = n - (half + 1);
          }
        }
        const int64_t item = ret < deg - 1 ? ret : deg - 1;
        const int64_t v = nb[item];
        rowpos[out + p] = r;
        col[out + p] = v;
        table_record(table, v, S + out + p);
      }
    }
  }
}

template <bool kReplace>
__global__ __launch_bounds__(kTileRows) void k_sample_bias(
    RowSrc src, Count Sc, int64_t k, uint64_t seed, const RowInfo *__restrict__ rowinfo,
    const int32_t *__restrict__ tpre, const int64_t *__restrict__ boff,
    const int32_t *__restrict__ tpre2, const int64_t *__restrict__ tboff, float *cdf,
    int64_t *__restrict__ rowpos, int64_t *__restrict__ col, Table table,
    const int64_t *__restrict__ hubid) {
  latency_prio();
  sample_bias_block<kReplace>(src, Sc, k, seed, rowinfo, tpre, boff, tpre2, tboff, cdf, rowpos,
                              col, table, hubid, blockIdx.x);
}

// ------------------------------------------------------------------------------------
// Biased hub rows (A-Res without replacement, degree > kBiasHubT).  Edge i of a row draws
// curand number j = c_l + i / 32 of subsequence 32w + l (l = i % 32; c_l = draws lane l made on
// the chain's earlier rows), so any half-wave can evaluate any edge's key (see k_bias_boot /
// k_bias_stream below).
struct BiasHubArgs {
  RowSrc src;
  Count Sc;
  int64_t k;
  uint64_t seed;
  const RowInfo *rowinfo;
  const int32_t *tpre;
  const int64_t *boff;
  HubView hub;
  int64_t nworkers;  // half-wave workers of k_bias_stream
  int64_t *rowpos;
  int64_t *col;
  Table table;
  BiasCand cand;
};

// draws lane l made on the earlier rows of row r's (block, warp) chain (no replacement)
__device__ __forceinline__ int64_t chain_draws(const RowInfo *rowinfo, int64_t r, int64_t k,
                                               int l) {
  const int64_t b = r / 16;
  const int w = (int)((r % 16) & 3), m = (int)((r % 16) >> 2);
  int64_t j = 0;
  for (int mm = 0; mm < m; ++mm) {
    const int64_t d = ri_deg(rowinfo[b * 16 + w + 4 * mm]);
    if (d > k) j += lane_draws(d, l);
  }
  return j;
}

__device__ __forceinline__ int64_t bias_worker_c0(int64_t total, int64_t w, int64_t nw) {
  return total * w / nw;
}

// Workers actually used: at least 2 chunks each (parallelism wins over longer row segments).
__device__ __forceinline__ int64_t bias_workers(int64_t total, int64_t max_workers) {
  const int64_t w = total / 2;
  return w < 1 ? 1 : (w > max_workers ? max_workers : w);
}

// Writes row h's k picks (lane l < k: the l-th best, index idx_l).
__device__ __forceinline__ void merge_emit(const BiasHubArgs &a, int64_t S, int64_t h, int32_t idx_l,
                                           int64_t k, int l) {
  const int64_t r = a.hub.row[h];
  const RowInfo ri = a.rowinfo[r];
  const int64_t out = a.boff[r / kTileRows] + a.tpre[r];
  if (l < k) {
    // (a pick outside the row -- only if the filter's proven bound failed -- emits id -1,
    // which the relabel tail reports, instead of reading outside the row)
    const int64_t v = (uint32_t)idx_l < (uint64_t)ri_deg(ri) ? as_global(ri.ptr)[idx_l] : -1;
    a.rowpos[out + l] = r;
    a.col[out + l] = v;
    table_record(a.table, v, S + out + l);
  }
}

// ------------------------------------------------------------------------------------
// Biased hub rows, streaming scheme (round 3).  Round 2's chunked scheme kept a running top-k per
// half-wave worker: 112 VGPRs, 4 waves per SIMD, and its per-edge loop waited on probability and
// threshold loads it could not hide (0.41 T edges/s against ~1 T for the same Philox + filter
// work VALU-bound).  Here the work is split so the per-edge pass holds no top-k state:
//   k_bias_boot    one workgroup per hub row: over a spread sample (8 runs of kBiasSampleSteps
//                  steps, 4096 edges) each lane keeps the largest key_lower() (a provable
//                  lower bound of the exact key, from the hardware log2); the k-th largest of
//                  the 256 lane maxima is a lower bound T of the row's final k-th key.
//   k_bias_stream  every edge of the row: Philox and a cheap linear bound against T; the few
//                  that pass go to the row's candidate list as (u, edge).  The bound is
//                  conservative, so every final pick is kept (they all have key >= final k-th
//                  >= T).  Half-wave workers over contiguous chunk ranges (each lane's chunks
//                  aligned to its Philox blocks), candidates staged in LDS, no exact key.
//   merge          (in k_bias_rows_merge) exact keys of each row's candidates and their top-k;
//                  a row whose list overflowed (or whose sample had no finite k-th key) is
//                  recomputed exactly.
// Every edge's key comes from its reference coordinates, so the picks are the oracle's, bit for
// bit, however the work is split.

struct HubRowCtx {
  int64_t r, deg;
  global_ptr<float> pr;
  uint2 kk;
  uint32_t sub;
  int64_t jb;
};
__device__ __forceinline__ HubRowCtx hub_row_ctx(const BiasHubArgs &a, int64_t h, int64_t G,
                                                 int l) {
  HubRowCtx c;
  c.r = a.hub.row[h];
  c.deg = ri_deg(a.rowinfo[c.r]);
  c.pr = as_global(reinterpret_cast<const float *>(a.hub.aux[h]));
  const uint64_t key = a.seed * (uint64_t)G + (uint64_t)(c.r / 16);
  c.kk = make_uint2((uint32_t)key, (uint32_t)(key >> 32));
  c.sub = (uint32_t)(32 * ((c.r % 16) & 3) + l);
  c.jb = chain_draws(a.rowinfo, c.r, a.k, l);
  return c;
}

// Steps [s0, s1) of a row (step s: edge i = 32 s + l, draw jb + s of the lane's subsequence) into
// `top`: a two-block Philox window refilled once per 4 steps (the loop of sample_bias_block),
// exact keys for the edges the cheap bound lets through.
__device__ __forceinline__ void bias_run(const HubRowCtx &c, int64_t s0, int64_t s1, int64_t k,
                                         int l, HalfTopK &top) {
  const int64_t n = s1 - s0;
  if (n <= 0) return;
  const int64_t j = c.jb + s0;
  const int64_t bl = j >> 2;
  const int off = (int)(j & 3);
  const uint32_t m2 = (off & 2) ? ~0u : 0u, m1 = (off & 1) ? ~0u : 0u;
  uint4 A = philox4x32_10(make_uint4((uint32_t)bl, (uint32_t)((uint64_t)bl >> 32), c.sub, 0u),
                          c.kk);
  bool filter = top.filtering(k);
  float thr_s = filter ? slack_thr(top.thr_k) : -__builtin_inff();
  const int64_t e0 = 32 * s0 + l;
  const int64_t e1 = 32 * s1 < c.deg ? 32 * s1 : c.deg;
  float pn[4];
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) {
    const int64_t i = e0 + 32 * s4;
    pn[s4] = i < e1 ? c.pr[i] : 0.0f;
  }
  for (int64_t g = 0; 4 * g < n; ++g) {
    float p[4];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      p[s4] = pn[s4];
      const int64_t i = e0 + 128 * (g + 1) + 32 * s4;
      pn[s4] = i < e1 ? c.pr[i] : 0.0f;
    }
    const uint64_t qb = (uint64_t)(bl + g + 1);
    const uint4 B = philox4x32_10(make_uint4((uint32_t)qb, (uint32_t)(qb >> 32), c.sub, 0u), c.kk);
    const uint32_t wv[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
    uint32_t w2[5];
#pragma unroll
    for (int e = 0; e < 5; ++e) w2[e] = bitsel(m2, wv[e + 2], wv[e]);
    float u[4];
    uint32_t mk = 0;
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      u[s4] = curand_uniform_from(bitsel(m1, w2[s4 + 1], w2[s4]));
      const bool valid = e0 + 128 * g + 32 * s4 < e1;
      mk |= (uint32_t)(valid & (!filter | ares_may_pass_s(u[s4], p[s4], thr_s))) << s4;
    }
    while (half_ballot(mk != 0)) {
      const bool has = mk != 0;
      const int t = has ? __builtin_ctz(mk) : 0;
      mk &= mk - 1;
      float ut = u[0], pt = p[0];
#pragma unroll
      for (int e = 1; e < 4; ++e) {
        ut = t == e ? u[e] : ut;
        pt = t == e ? p[e] : pt;
      }
      top.push(has ? ares_key(ut, pt) : -__builtin_inff(), (int32_t)(e0 + 128 * g + 32 * t), has,
               k, l);
      if (!filter && top.filtering(k)) {
        filter = true;
        thr_s = slack_thr(top.thr_k);
        uint32_t keep = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) keep |= (uint32_t)ares_may_pass_s(u[e], p[e], thr_s) << e;
        mk &= keep;
      }
    }
    if (top.filtering(k)) {
      filter = true;
      thr_s = slack_thr(top.thr_k);
    }
    A = B;
  }
}

// The 8 half-waves' sorted lists (only the first k of each count) merged pairwise in LDS; the
// k best, sorted, end in s_key[0][0..k) / s_idx[0][0..k).  Every thread of the workgroup calls.
__device__ __forceinline__ void tree_merge8(const HalfTopK &top, int64_t k, int g, int l,
                                            float (*s_key)[32], int32_t (*s_idx)[32]) {
  const bool mine = l < k && top.bi != INT32_MAX;
  s_key[g][l] = mine ? top.bk : -__builtin_inff();
  s_idx[g][l] = mine ? top.bi : INT32_MAX;
  __syncthreads();
#pragma unroll
  for (int step = 1; step < 8; step <<= 1) {
    if ((g & (2 * step - 1)) == 0) {
      float mk = s_key[g][l];
      int32_t mi = s_idx[g][l];
      const float ok = s_key[g + step][31 - l];
      const int32_t oi = s_idx[g + step][31 - l];
      if (ares_better(ok, oi, mk, mi)) {
        mk = ok;
        mi = oi;
      }
#pragma unroll
      for (int stride = 16; stride > 0; stride >>= 1) HalfTopK::cas(mk, mi, stride, (l & stride) == 0);
      s_key[g][l] = mk;
      s_idx[g][l] = mi;
    }
    __syncthreads();
  }
}

// The stream kernel's reject test, in the draw's own domain.  ln u <= u - 1 gives log2 u < p T
// whenever u < 1 + p T ln2, and u = RN(x 2^-32 + 2^-33) < 1 + p T ln2 (1 + 2^-16) - 2^-20
// follows from (float)x < p cx + bx with cx = lin_cx(T) and bx = 2^32 (1 - 2^-20) - 512: the
// margins cover u's rounding, the fma's and the fixed-operation log2's error.  So a rejected
// edge has key < T.  p <= 0 or NaN only lets an edge through (its key is exact later).
__device__ __forceinline__ float lin_cx(float T) {
  return T * (0.6931471805599453f * 1.0000152587890625f) * 4294967296.0f;
}
// The test as the kernel uses it: the lanes of the wave where it does NOT reject, i.e.
// !((float)x < p cx + bx) -- >= or unordered -- as the compare's own 64-bit result (active
// lanes only; a ballot of the predicate would first materialise it in a VGPR).
__device__ __forceinline__ uint64_t lin_pass_mask(uint32_t x, float p, float cx) {
  return __builtin_amdgcn_fcmpf((float)x, __builtin_fmaf(p, cx, 4294962688.0f), 11 /*UGE*/);
}
// (mask & a) | (~mask & b) in one v_bfi_b32 (a ternary on an all-ones / zero mask became a
// compare and a select)
__device__ __forceinline__ uint32_t bfi(uint32_t mask, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(mask), "v"(a), "v"(b));
  return r;
}

// A value <= ares_key(u, p) for every u in (0, 1] and p: the hardware log2 (v_log_f32, within a
// few ulp of dgs_log2f) lowered by 2^-16 relative + 2^-16 absolute, divided through the hardware
// reciprocal and lowered by another 2^-16 relative -- margins far above every rounding on the way
// (< 2^-21 relative), so the result lies below RN(dgs_log2f(u) / p).  p outside [2^-100, 2^100]
// (or not > 0) gives -inf, which keeps every intermediate a normal float.
__device__ __forceinline__ float key_lower(float u, float p) {
  const float L = __builtin_amdgcn_logf(u);
  const float Ll = L - __builtin_fabsf(L) * 1.52587890625e-05f - 1.52587890625e-05f;
  const float q = Ll * __builtin_amdgcn_rcpf(p) * 1.0000152587890625f;
  return ((p >= 7.888609052210118e-31f) & (p <= 1.2676506002282294e+30f)) ? q : -__builtin_inff();
}

// Largest key_lower() of this lane's edges among its draws [A, E), A = the first block boundary
// at or after draw jb + s0 and E = min(A + len, the first block boundary at or after jb + s1):
// whole Philox blocks only (no draw window to select from), and consecutive runs of a row stay
// disjoint, so the lane maxima of different runs are different edges.  Draw jb + s is step s,
// edge 32 s + l (valid below deg).  No cross-lane work.
__device__ __forceinline__ float lane_max_run(const HubRowCtx &c, int64_t s0, int64_t s1,
                                              int64_t len, int l) {
  float best = -__builtin_inff();
  const int64_t A = (c.jb + s0 + 3) & ~int64_t(3);
  const int64_t E1 = (c.jb + s1 + 3) & ~int64_t(3);
  const int64_t E = A + len < E1 ? A + len : E1;
  if (E <= A) return best;
  const PhiloxKeys K = philox_keys(c.kk);
  const int32_t nbk = (int32_t)((E - A) >> 2);
  const uint32_t deg = (uint32_t)c.deg;
  const uint32_t ib = (uint32_t)(32 * (A - c.jb) + l);  // edge of the run's first draw
  // block q's probabilities, 0 past the row's end (key_lower(u, 0) = -inf: no select needed);
  // a block inside the row loads from one address with immediate offsets
  auto load4 = [&](int32_t q, float *p) {
    const uint32_t i0 = ib + 128u * (uint32_t)q;
    if (i0 + 96u < deg) {
      const global_ptr<float> pc = c.pr + i0;
#pragma unroll
      for (int w = 0; w < 4; ++w) p[w] = pc[32 * w];
    } else {
#pragma unroll
      for (int w = 0; w < 4; ++w) p[w] = i0 + 32u * w < deg ? c.pr[i0 + 32u * w] : 0.0f;
    }
  };
  // the next block's probabilities load under this block's Philox and keys
  float pn[4];
  load4(0, pn);
  for (int32_t q = 0; q < nbk; ++q) {
    float p[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) p[w] = pn[w];
    load4(q + 1, pn);
    const uint64_t qb = (uint64_t)((A >> 2) + q);
    const uint4 B = philox4x32_10(make_uint4((uint32_t)qb, (uint32_t)(qb >> 32), c.sub, 0u), K);
    const uint32_t wv[4] = {B.x, B.y, B.z, B.w};
#pragma unroll
    for (int w = 0; w < 4; ++w)  // (max of two non-NaN values in one v_med3_f32)
      best = __builtin_amdgcn_fmed3f(key_lower(curand_uniform_from(wv[w]), p[w]), best,
                                     __builtin_inff());
  }
  return best;
}

// 32 floats across a half-wave sorted descending (bitonic network).
__device__ __forceinline__ float sort32_desc(float v, int l) {
#pragma unroll
  for (int size = 2; size <= 32; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const float o = lane_xor32v(v, stride);
      const bool desc = (l & size) == 0 || size == 32;
      const bool lower = (l & stride) == 0;
      v = (desc == lower) ? fmaxf(v, o) : fminf(v, o);
    }
  }
  return v;
}

// One workgroup per hub row (grid-stride over the hub list): the row's threshold T.  Half-wave g
// samples up to kBiasSampleSteps draws from step ns * g / 8 on, cut at block boundaries (its
// part of the row when the row has fewer than 8 kBiasSampleSteps steps); the 8 sorted lists of
// lane maxima are merged pairwise in LDS and the k-th largest of the 256 is T (a lower bound of
// k distinct edges' keys: the runs are disjoint).
__global__ __launch_bounds__(kTileRows) void k_bias_boot(BiasHubArgs a) {
  latency_prio();
  __shared__ float s_max[8][32];
  const int64_t S = a.Sc.get();
  const int64_t G = (S + 15) / 16;
  const int64_t H = (int64_t)((uint64_t)*a.hub.count >> kHubShift);
  const int l = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int64_t k = a.k;
  for (int64_t h = blockIdx.x; h < H; h += gridDim.x) {
    const HubRowCtx c = hub_row_ctx(a, h, G, l);
    const int64_t ns = (c.deg + 31) / 32;
    // 8 runs spread over the row, each up to kBiasSampleSteps draws (the whole row when it is
    // shorter), cut at block boundaries
    const int64_t s0 = ns * g / 8, s1 = ns * (g + 1) / 8;
    const int64_t len = ns >= 8 * kBiasSampleSteps ? kBiasSampleSteps : s1 - s0 + 4;
    s_max[g][l] = sort32_desc(lane_max_run(c, s0, s1, len, l), l);
    __syncthreads();
#pragma unroll
    for (int step = 1; step < 8; step <<= 1) {
      if ((g & (2 * step - 1)) == 0) {
        // the top 32 of two descending lists: a bitonic sequence, then one bitonic merge
        float v = fmaxf(s_max[g][l], s_max[g + step][31 - l]);
#pragma unroll
        for (int stride = 16; stride > 0; stride >>= 1) {
          const float o = lane_xor32v(v, stride);
          v = (l & stride) == 0 ? fmaxf(v, o) : fminf(v, o);
        }
        s_max[g][l] = v;
      }
      __syncthreads();
    }
    if (threadIdx.x == k - 1) a.hub.thr[h] = key_order(s_max[0][k - 1]);
    __syncthreads();
  }
}

// Every edge of the streamed hub rows against the row's boot threshold T.  Its workgroup 0 first
// does the hop's tile-offset scan (the rows / merge launch after it reads boff).  Row state is
// kept in 32 bits (a row has < 2^31 edges, a lane's draw offset < 2^28, the hop's chunk count
// and candidate room < 2^31): register pressure, not arithmetic, sets this kernel's occupancy.
// DGS_STREAM_COUNTERS (diagnostic builds only): per half-wave candidate flushes, candidates
// and row switches, summed per workgroup into the profiling stamps (DGS_PROF_HUB=1).
#ifndef DGS_STREAM_COUNTERS
#define DGS_STREAM_COUNTERS 0
#endif
struct StreamCounters {
  uint32_t flushes = 0, cands = 0, switches = 0;
};
__device__ __forceinline__ void bias_stream_body(const BiasHubArgs &a, const int64_t *bsum,
                                                 int64_t *boff, int64_t *d_nnz,
                                                 StreamCounters &sc) {
  if (blockIdx.x == 0) {
    __shared__ int64_t lds[kTileRows / 64];
    const int64_t nb = (a.Sc.get() + kTileRows - 1) / kTileRows;
    const int64_t tot = block_scan_range<kTileRows, 8>(bsum, nb, boff, lds);
    if (threadIdx.x == 0) {
      boff[nb] = tot;
      *d_nnz = tot;
    }
  }
  const int64_t S = a.Sc.get();
  const int64_t G = (S + 15) / 16;
  const uint64_t packed = (uint64_t)*a.hub.count;
  const int64_t H = (int64_t)(packed >> kHubShift);
  const int64_t total = (int64_t)(packed & kHubChunkMask);
  if (H == 0 || total == 0) return;
  const int l = threadIdx.x & 31;
  const int64_t wk = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 5;
  const int64_t nw = bias_workers(total, a.nworkers);
  if (wk >= nw) return;
  const uint32_t c0 = (uint32_t)bias_worker_c0(total, wk, nw);
  const uint32_t c1 = (uint32_t)bias_worker_c0(total, wk + 1, nw);
  if (c0 >= c1) return;
  int64_t h = group_search<32>(a.hub.cptr, H, c0);
  uint32_t hstart = 0, hnext = 0, deg = 0, jb = 0, off = 0, sub = 0;
  global_ptr<float> pr = nullptr;
  PhiloxKeys kk;
  float cx = 0.0f;
  bool skip = false;
  auto load_row = [&](int64_t hh) {
    hstart = (uint32_t)a.hub.cptr[hh];
    hnext = hh + 1 < H ? (uint32_t)a.hub.cptr[hh + 1] : (uint32_t)total;
    const HubRowCtx c = hub_row_ctx(a, hh, G, l);
    deg = (uint32_t)c.deg;
    jb = (uint32_t)c.jb;
    off = jb & 3u;
    sub = c.sub;
    kk = philox_keys(c.kk);
    pr = c.pr;
    const float T = key_from_order((int32_t)a.hub.thr[hh]);
    cx = lin_cx(T);
    // no finite sample threshold (weights <= 0): every edge would be a candidate; the merge
    // recomputes the row instead (every worker of the row stores the same marker)
    skip = !(T > -__builtin_inff());
    if (skip && l == 0) a.cand.cnt[hh] = INT32_MAX;
  };
  // Chunks are aligned to the lane's Philox blocks: lane l's chunk q holds its steps
  // s = kStreamT q - off + t (t < kStreamT, off = jb mod 4), i.e. draws jb - off + kStreamT q + t,
  // exactly the words of blocks (jb >> 2) + q kStreamT / 4 + {0, 1}: no draw window to select
  // from and no block carried between chunks (a row has up to one chunk more for it).  Step s
  // is edge 32 s + l, valid when 0 <= s and 32 s + l < deg.
  // The first edge of chunk q in this lane (negative before the row's start) and whether all of
  // the chunk's edges are valid.
  auto chunk_i0 = [&](uint32_t q) { return (int32_t)(32u * (q * kStreamT - off) + (uint32_t)l); };
  auto chunk_whole = [&](int32_t i0) {
    return i0 >= 0 && (uint32_t)i0 + 32u * (kStreamT - 1) < deg;
  };
  // Chunk q's probabilities (clamped into the row outside it; whole chunks: one address and
  // immediate offsets -- the kernel is VALU-issue-bound).
  auto load_probs = [&](uint32_t q, float *p) {
    const int32_t i0 = chunk_i0(q);
    if (chunk_whole(i0)) {
      const global_ptr<float> pc = pr + i0;
#pragma unroll
      for (int t = 0; t < kStreamT; ++t) p[t] = pc[32 * t];
    } else {
#pragma unroll
      for (int t = 0; t < kStreamT; ++t) {
        const int32_t i = i0 + 32 * t;
        p[t] = pr[i < 0 ? 0 : ((uint32_t)i < deg - 1u ? (uint32_t)i : deg - 1u)];
      }
    }
  };
  // Candidates wait in this half-wave's LDS list as (draw, edge, hub row) and reach their rows'
  // global lists in batches (one returning atomic per row and batch).  An atomic per chunk made
  // every chunk wait out a memory round trip, and that wait also drained the next chunk's
  // probability loads.
  __shared__ uint32_t s_x[kTileRows / 32][kStreamBuf], s_i[kTileRows / 32][kStreamBuf];
  __shared__ int32_t s_h[kTileRows / 32][kStreamBuf];
  const int g = threadIdx.x >> 5;
  int nb = 0;  // entries in the list (half-wave uniform)
  // The flush reads entries other lanes of the half-wave wrote: wavefront-scope fences around
  // the scheduling barriers order those LDS accesses (a wave barrier alone only keeps the
  // compiler from moving code across it).
  auto flush = [&]() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int e0 = 0; e0 < nb; e0 += 32) {
      const int e = e0 + l;
      const bool v = e < nb;
      const uint32_t x = v ? s_x[g][e] : 0u;
      const uint32_t ix = v ? s_i[g][e] : 0u;
      const int32_t hh = v ? s_h[g][e] : -1;
      uint32_t todo = half_ballot(v);
      while (todo) {
        const int lead = __builtin_ctz(todo);
        const int32_t hl = __shfl(hh, lead, 32);
        const uint32_t same = half_ballot(v & (hh == hl));
        int32_t old = 0;
        if (l == lead) old = atomicAdd(a.cand.cnt + hl, (int32_t)__builtin_popcount(same));
        old = __shfl(old, lead, 32);
        if ((same >> l) & 1u) {
          const int32_t pos = old + (int32_t)__builtin_popcount(same & ((1u << l) - 1u));
          if (pos < a.cand.cap[hl]) {
            const size_t o = (size_t)a.cand.base[hl] + (size_t)pos;
            a.cand.key[o] = curand_uniform_from(x);
            a.cand.idx[o] = (int32_t)ix;
          }
        }
        todo &= ~same;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (DGS_STREAM_COUNTERS) {
      sc.flushes += 1;
      sc.cands += (uint32_t)nb;
    }
    nb = 0;
  };
  load_row(h);
  // the next chunk's probabilities, loaded under this chunk's Philox (same row only)
  float pn[kStreamT];
  bool have_next = false;
  for (uint32_t ch = c0; ch < c1; ++ch) {
    while (ch >= hnext) {
      ++h;
      load_row(h);
      if (DGS_STREAM_COUNTERS) sc.switches += 1;
    }
    if (skip) continue;
    const uint32_t q = ch - hstart;
    const int32_t i0 = chunk_i0(q);
    const bool whole = chunk_whole(i0);
    if (!have_next) load_probs(q, pn);
    float p[kStreamT];
#pragma unroll
    for (int t = 0; t < kStreamT; ++t) p[t] = pn[t];
    have_next = ch + 1 < c1 && ch + 1 < hnext;
    if (have_next) load_probs(q + 1, pn);
    const uint32_t bc = (jb >> 2) + q * (kStreamT / 4);
    uint32_t xs[kStreamT];
#pragma unroll
    for (int bq = 0; bq < kStreamT / 4; ++bq) {
      const uint4 o = philox4x32_10(make_uint4(bc + bq, 0u, sub, 0u), kk);
      xs[4 * bq + 0] = o.x;
      xs[4 * bq + 1] = o.y;
      xs[4 * bq + 2] = o.z;
      xs[4 * bq + 3] = o.w;
    }
    // Per step t, the wave's lanes whose edge passes the cheap bound, straight from the compares
    // (lin_pass_mask: one convert, one fma and one compare per edge; round 3 A/B against the
    // hardware-log2 bound: +1.7 %); the valid-edge compare only matters in a row's first and
    // last chunks.
    uint64_t pass[kStreamT];
#pragma unroll
    for (int t = 0; t < kStreamT; ++t) pass[t] = lin_pass_mask(xs[t], p[t], cx);
    const uint64_t whole_mask = __ballot(whole);
    if (whole_mask != __builtin_amdgcn_read_exec()) {  // (wave-uniform: a row's first / last chunk)
#pragma unroll
      for (int t = 0; t < kStreamT; ++t)  // (a negative edge compares as a huge unsigned one)
        pass[t] &= whole_mask | __builtin_amdgcn_uicmp((uint32_t)(i0 + 32 * t), deg, 36 /*ULT*/);
    }
    // the few that pass go to the list as (draw, edge); the merge computes their exact keys
    // (keeping the fixed-operation key out of this loop saves registers)
    if (nb > kStreamBuf - kStreamChunk) flush();
    const int hs = threadIdx.x & 32;
#pragma unroll
    for (int t = 0; t < kStreamT; ++t) {
      if (pass[t] == 0) continue;
      const uint32_t b = (uint32_t)(pass[t] >> hs);
      if ((b >> l) & 1u) {
        const int pos = nb + __builtin_popcount(b & ((1u << l) - 1u));
        s_x[g][pos] = xs[t];
        s_i[g][pos] = (uint32_t)(i0 + 32 * t);
        s_h[g][pos] = (int32_t)h;
      }
      nb += __builtin_popcount(b);
    }
  }
  if (nb > 0) flush();
}

__global__ __launch_bounds__(kTileRows) void k_bias_stream(BiasHubArgs a, const int64_t *bsum,
                                                           int64_t *boff, int64_t *d_nnz,
                                                           uint64_t *stamp) {
  // profiling only (DGS_PROF_HUB: stamp != nullptr, a kernel argument: uniform branch)
  if (stamp && threadIdx.x == 0) stamp[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  __shared__ uint32_t s_ctr[3];
  if (DGS_STREAM_COUNTERS && stamp) {
    if (threadIdx.x < 3) s_ctr[threadIdx.x] = 0;
    __syncthreads();
  }
  StreamCounters sc;
  bias_stream_body(a, bsum, boff, d_nnz, sc);
  if (stamp) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (DGS_STREAM_COUNTERS && (threadIdx.x & 31) == 0) {
      atomicAdd(&s_ctr[0], sc.flushes);
      atomicAdd(&s_ctr[1], sc.cands);
      atomicAdd(&s_ctr[2], sc.switches);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      stamp[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
      if (DGS_STREAM_COUNTERS) {
        uint64_t *ctr = stamp + 2 * gridDim.x + 2 * blockIdx.x;
        // the workgroup's CU: HW_ID bits 8-15 (CU, SH, SE) and the XCC id
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);
        ctr[0] = (uint64_t)s_ctr[0] | ((uint64_t)(((hw >> 8) & 0xff) | ((xcc & 0xff) << 8)) << 32);
        ctr[1] = (uint64_t)s_ctr[1] | ((uint64_t)s_ctr[2] << 32);
      }
    }
  }
}

// Candidate e of a streamed row: its exact key from (u, edge) and the row's probabilities.
__device__ __forceinline__ void stream_cand(const BiasHubArgs &a, global_ptr<float> pr, int64_t cb,
                                            int32_t n, int32_t e, float &key, int32_t &idx) {
  const bool v = e < n;
  idx = v ? a.cand.idx[cb + e] : INT32_MAX;
  key = v ? ares_key(a.cand.key[cb + e], pr[idx]) : -__builtin_inff();
}

// Writes row r's k picks (lane l < k: index idx_l) given its node-table entry and output offset.
__device__ __forceinline__ void merge_emit_at(const BiasHubArgs &a, int64_t S, int64_t r,
                                              const RowInfo &ri, int64_t out, int32_t idx_l,
                                              int64_t k, int l) {
  if (l < k) {
    const int64_t v = (uint32_t)idx_l < (uint64_t)ri_deg(ri) ? as_global(ri.ptr)[idx_l] : -1;
    a.rowpos[out + l] = r;
    a.col[out + l] = v;
    table_record(a.table, v, S + out + l);
  }
}

// Emits each hub row's k picks from its candidate list (or recomputes the row when the list
// overflowed).  Lists of at most 64: one half-wave per row.  Longer lists and recomputed rows:
// one workgroup per row, 8 half-waves over interleaved 32-entry batches (or contiguous step
// ranges), merged in LDS.  The loads are grouped by dependence level (the list's header and the
// row's output slot together, both candidate batches together, the next batch's entries under
// the current batch's probabilities): this pass is latency-bound.
#ifndef DGS_MERGE_ILP
#define DGS_MERGE_ILP 4
#endif
constexpr int kMergeIlp = DGS_MERGE_ILP;
__device__ __forceinline__ void stream_merge_block(const BiasHubArgs &a, int64_t blk,
                                                   int64_t nblk) {
  __shared__ float s_key[8][32];
  __shared__ int32_t s_idx[8][32];
  const int64_t S = a.Sc.get();
  const int64_t G = (S + 15) / 16;
  const int64_t H = (int64_t)((uint64_t)*a.hub.count >> kHubShift);
  const int64_t k = a.k;
  const int l = threadIdx.x & 31, g = threadIdx.x >> 5;
  for (int64_t h = blk * 8 + g; h < H; h += nblk * 8) {
    const int32_t n = a.cand.cnt[h], cap = a.cand.cap[h];
    const int64_t cb = a.cand.base[h];
    const global_ptr<float> pr = as_global(reinterpret_cast<const float *>(a.hub.aux[h]));
    const int64_t r = a.hub.row[h];
    if (n > cap || n > 64) continue;
    const RowInfo ri = a.rowinfo[r];
    const int64_t out = a.boff[r / kTileRows] + a.tpre[r];
    const bool v0 = l < n, v1 = 32 + l < n;
    const int32_t i0 = v0 ? a.cand.idx[cb + l] : INT32_MAX;
    const int32_t i1 = v1 ? a.cand.idx[cb + 32 + l] : INT32_MAX;
    const float u0 = v0 ? a.cand.key[cb + l] : 1.0f;
    const float u1 = v1 ? a.cand.key[cb + 32 + l] : 1.0f;
    const float p0 = v0 ? pr[i0] : 1.0f;
    const float p1 = v1 ? pr[i1] : 1.0f;
    HalfTopK top;
    top.push(v0 ? ares_key(u0, p0) : -__builtin_inff(), i0, v0, k, l);
    if (n > 32) top.push(v1 ? ares_key(u1, p1) : -__builtin_inff(), i1, v1, k, l);
    merge_emit_at(a, S, r, ri, out, top.bi, k, l);
  }
  for (int64_t h = blk; h < H; h += nblk) {
    const int32_t n = a.cand.cnt[h], cap = a.cand.cap[h];
    const bool recompute = n > cap;
    if (!recompute && n <= 64) continue;
    HalfTopK top;
    if (recompute) {
      const HubRowCtx c = hub_row_ctx(a, h, G, l);
      const int64_t ns = (c.deg + 31) / 32;
      bias_run(c, ns * g / 8, ns * (g + 1) / 8, k, l, top);
    } else {
      const int64_t cb = a.cand.base[h];
      const global_ptr<float> pr = as_global(reinterpret_cast<const float *>(a.hub.aux[h]));
      // kMergeIlp batches per round: their entries load together, then their probabilities
      // together, and the next round's entries load under this round's probabilities and keys
      // (a long list's chain is its rounds' memory round trips)
      int32_t idx[kMergeIlp];
      float u[kMergeIlp];
      auto load_round = [&](int32_t b0) {
#pragma unroll
        for (int j = 0; j < kMergeIlp; ++j) {
          const int32_t e = b0 + 256 * j + l;
          const bool v = e < n;
          idx[j] = v ? a.cand.idx[cb + e] : INT32_MAX;
          u[j] = v ? a.cand.key[cb + e] : 1.0f;
        }
      };
      load_round(32 * g);
      for (int32_t b0 = 32 * g; b0 < n; b0 += 256 * kMergeIlp) {
        float p[kMergeIlp], uc[kMergeIlp];
        int32_t ic[kMergeIlp];
#pragma unroll
        for (int j = 0; j < kMergeIlp; ++j) {
          p[j] = idx[j] != INT32_MAX ? pr[idx[j]] : 1.0f;
          ic[j] = idx[j];
          uc[j] = u[j];
        }
        if (b0 + 256 * kMergeIlp < n) load_round(b0 + 256 * kMergeIlp);
#pragma unroll
        for (int j = 0; j < kMergeIlp; ++j) {
          const bool v = ic[j] != INT32_MAX;
          if (b0 + 256 * j >= n) break;  // (half-wave uniform)
          top.push(v ? ares_key(uc[j], p[j]) : -__builtin_inff(), ic[j], v, k, l);
        }
      }
    }
    tree_merge8(top, k, g, l, s_key, s_idx);
    if (g == 0) merge_emit(a, S, h, s_idx[0][l], k, l);
    __syncthreads();
  }
}

// The biased hop's non-hub rows (workgroups [0, row_blocks)) and its hub-row merge (the rest) in
// one launch: both only need the hub kernel before them (one launch fewer per hop).
__global__ __launch_bounds__(kTileRows) void k_bias_rows_merge(
    BiasHubArgs a, const int32_t *__restrict__ tpre2, const int64_t *__restrict__ tboff,
    int64_t row_blocks, int64_t merge_blocks) {
  latency_prio();
  if ((int64_t)blockIdx.x < row_blocks)
    sample_bias_block<false>(a.src, a.Sc, a.k, a.seed, a.rowinfo, a.tpre, a.boff, tpre2, tboff,
                             nullptr, a.rowpos, a.col, a.table, a.hub.hubid, blockIdx.x);
  else
    stream_merge_block(a, (int64_t)blockIdx.x - row_blocks, merge_blocks);
}

// The hub-row merge alone (DGS_BIAS_SPLIT_MERGE=1: rows and merge as two launches, profiling).
__global__ __launch_bounds__(kTileRows) void k_bias_hub_merge(BiasHubArgs a) {
  latency_prio();
  stream_merge_block(a, blockIdx.x, gridDim.x);
}

// Test-only (dgs_test_bias_bounds): the exact A-Res key, key_lower() and the two reject tests
// the biased kernels use (bit 0: the stream kernel's linear reject against T, read from the wave
// mask it uses; bit 1: the row / hub-run filter !ares_may_pass_s against thr = T), per (draw x,
// probability p, threshold T).
__global__ void k_test_bias_bounds(const uint32_t *x, const float *p, const float *thr, int64_t n,
                                   float *key, float *klow, uint8_t *flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float u = curand_uniform_from(x[i]);
  const float pi = p[i], T = thr[i];
  key[i] = ares_key(u, pi);
  klow[i] = key_lower(u, pi);
  // the stream kernel's form: the lane's bit of the wave's pass mask
  const bool pass = (lin_pass_mask(x[i], pi, lin_cx(T)) >> (threadIdx.x & 63)) & 1u;
  flags[i] = (uint8_t)((int)!pass | ((int)!ares_may_pass_s(u, pi, slack_thr(T)) << 1));
}

}  // namespace

void test_bias_bounds(const uint32_t *x, const float *p, const float *thr, int64_t n, float *key,
                      float *key_low, uint8_t *flags, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_test_bias_bounds, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, x, p,
                     thr, n, key, key_low, flags);
  DGS_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------
void sample_hop(const RowSrc &src, const int64_t *seeds, Count Sc, int64_t k, bool replace,
                bool bias, uint64_t launch_seed, int64_t *rowpos, int64_t *col, int64_t *d_nnz,
                const Table &table, HopScratch &ws, hipStream_t st, const RelabelTail *tail,
                bool solo) {
  DGS_CHECK(k >= 0, "num_picks must be non-negative");
  const int64_t S = Sc.v;  // exact when Sc.p == nullptr, else an upper bound
  DGS_CHECK(S < (int64_t(1) << 31), "too many seeds in one hop");
  const int64_t nb = ceil_div(S > 0 ? S : 1, kTileRows);
  ws.rowinfo.ensure(sizeof(RowInfo) * (size_t)(S > 0 ? S : 1));
  ws.bsum.ensure(sizeof(int64_t) * (size_t)(2 * nb + 2));
  ws.boff.ensure(sizeof(int64_t) * (size_t)(2 * nb + 4));
  int64_t *bsum = ws.bsum.as<int64_t>();
  int64_t *tsum = bsum + nb;
  int64_t *boff = ws.boff.as<int64_t>();
  int64_t *tboff = boff + nb + 1;
  RowInfo *rowinfo = ws.rowinfo.as<RowInfo>();
  if (S == 0) {
    if (tail) launch_relabel_tail(*tail, st);
    DGS_HIP(hipMemsetAsync(d_nnz, 0, sizeof(int64_t), st));
    return;
  }
  const bool use_hubs = !bias && !replace && k > 0 && S < kHubMaxRows;
  const bool bias_hubs = bias && !replace && k > 0 && S < kHubMaxRows;
  // Two hub counters used by alternate hops (a global hop serial, so calls chain correctly):
  // each prep zeroes the other one; zeroed once at allocation.
  if (ws.hubcount.ensure(128)) DGS_HIP(hipMemsetAsync(ws.hubcount.p, 0, 128, st));
  const uint64_t par = ws.hop_serial++ & 1;
  ws.hub.ensure(HubView::bytes(S));
  HubView hub = HubView::make(ws.hub.as<int64_t>(), S);
  hub.count = ws.hubcount.as<int64_t>() + 8 * par;
  int64_t *next_count = ws.hubcount.as<int64_t>() + 8 * (par ^ 1);
  const bool bias_replace = bias && replace;
  ws.tpre.ensure(sizeof(int32_t) * (size_t)(2 * S));
  int32_t *tpre = ws.tpre.as<int32_t>();
  int32_t *tpre2 = tpre + S;
  if (use_hubs) ws.hubslot.ensure(sizeof(int32_t) * (size_t)(S * k));
  // Biased hubs: per-row candidate lists.  Every row's list fits the room below when the graph's
  // edge count is known (a hop's rows are distinct: their chunks number at most E / chunk + S);
  // otherwise rows past it are recomputed exactly.
  const int sblocks = bias_stream_blocks(solo);
  const int64_t nworkers = (int64_t)sblocks * (kTileRows / 32);
  BiasCand cand{};
  if (bias_hubs) {
    // Hub rows have degree > kBiasHubT.  After the first hop the seeds are a frontier (unique
    // ids, and the sampler passes the previous hop's relabel tail): at most min(S, E / kBiasHubT)
    // hub rows, with at most E / kStreamChunk + 2 per hub chunks.  The first hop's seeds (and the
    // standalone op's) may repeat, so a hub row may count several times: the row bound is S
    // there, and repeated rows' chunks may run past the chunk bound.  Rows whose room lies past
    // the limit get none and are recomputed exactly by the merge (correct either way; only
    // slower).  The room is also capped by a budget (DGS_BIAS_CAND_BUDGET entries, default
    // 2^26 = 512 MB per context).
    const bool seeds_unique = tail != nullptr;
    const int64_t hubs_ub = src.num_edges > 0 && seeds_unique
                                ? std::min<int64_t>(S, src.num_edges / kBiasHubT + 1)
                                : S;
    const int64_t chunks =
        src.num_edges > 0 ? src.num_edges / kStreamChunk + 2 * hubs_ub : (int64_t(1) << 22);
    static const int64_t budget = [] {
      const char *e = getenv("DGS_BIAS_CAND_BUDGET");
      const long long v = e ? atoll(e) : 0;
      return v > 0 ? (int64_t)v : (int64_t(1) << 26);
    }();
    int64_t limit = bias_room_start(hubs_ub, chunks, k);
    if (limit > budget) limit = budget;
    if (limit > INT32_MAX) limit = INT32_MAX;  // 32-bit list offsets (rows past it: recomputed)
    ws.cand.ensure(sizeof(int64_t) * (size_t)S + 2 * sizeof(int32_t) * (size_t)S +
                   (sizeof(float) + sizeof(int32_t)) * (size_t)limit);
    cand.base = ws.cand.as<int64_t>();
    cand.cnt = reinterpret_cast<int32_t *>(cand.base + S);
    cand.cap = cand.cnt + S;
    cand.key = reinterpret_cast<float *>(cand.cap + S);
    cand.idx = reinterpret_cast<int32_t *>(cand.key + limit);
    cand.limit = limit;
    // test hook, read per hop: DGS_BIAS_TEST_CAP=n limits a row's list to n entries (n < k
    // forces the exact recomputation of every hub row)
    const char *e = getenv("DGS_BIAS_TEST_CAP");
    cand.cap_max = e ? atoll(e) : INT64_MAX;
  }
  const PrepArgs pa{src, seeds, Sc, k, (int)replace,
                    use_hubs ? 1 : (bias_hubs ? 2 : 0),
                    (int)bias_replace, rowinfo, tpre, tpre2, bsum, tsum, hub,
                    ws.hubslot.as<int32_t>(), table, next_count, cand};
  if (tail)
    hipLaunchKernelGGL(k_prep_tail, dim3((unsigned)(tail->nblk + nb)), dim3(kTileRows), 0, st, pa,
                       *tail);
  else
    hipLaunchKernelGGL(k_prep, dim3((unsigned)nb), dim3(kTileRows), 0, st, pa);
  DGS_LAUNCH_CHECK();
  if (k == 0) {  // seeds still enter the relabel table (frontier = unique(seeds))
    DGS_HIP(hipMemsetAsync(d_nnz, 0, sizeof(int64_t), st));
    return;
  }
  // (the hub kernels' workgroup 0 does this scan when they run: one launch fewer per hop)
  if (!use_hubs && !bias_hubs) {
    hipLaunchKernelGGL(k_scan_hop, dim3(1), dim3(kScanThreads), 0, st, bsum,
                       bias_replace ? (const int64_t *)tsum : nullptr, Sc, boff, tboff, d_nnz,
                       bsum + 2 * nb + 1);
    DGS_LAUNCH_CHECK();
  }

  if (!bias) {
    DGS_CHECK(replace || k <= kMaxPicksLds, "num_picks > 512 is not supported without replacement");
    const UniformArgs ua{src,    Sc,  k,     launch_seed, rowinfo,
                         tpre,   boff, hub, ws.hubslot.as<int32_t>(),
                         rowpos, col, table, (int)solo};
    const int G = solo ? kGroupSolo : kGroup;
    const int64_t rows_per_block = kTileRows / G;
    const size_t lds = replace ? 16 : sizeof(int32_t) * (size_t)rows_per_block * k;
    const int64_t row_blocks = ceil_div(S, rows_per_block);
    if (use_hubs) {
      hipLaunchKernelGGL(k_hub_reservoir, dim3(hub_blocks()), dim3(256), 0, st, ua,
                         (const int64_t *)bsum, boff, d_nnz, profile_stamps(3, hub_blocks()));
      DGS_LAUNCH_CHECK();
    }
    const dim3 rgrid((unsigned)row_blocks), rblock(kTileRows);
    if (replace && solo)
      hipLaunchKernelGGL((k_sample_uniform<true, kGroupSolo>), rgrid, rblock, lds, st, ua, 0);
    else if (replace)
      hipLaunchKernelGGL((k_sample_uniform<true, kGroup>), rgrid, rblock, lds, st, ua, 0);
    else if (solo)
      hipLaunchKernelGGL((k_sample_uniform<false, kGroupSolo>), rgrid, rblock, lds, st, ua,
                         (int)use_hubs);
    else
      hipLaunchKernelGGL((k_sample_uniform<false, kGroup>), rgrid, rblock, lds, st, ua,
                         (int)use_hubs);
    DGS_LAUNCH_CHECK();
  } else {
    DGS_CHECK(k <= 32, "biased sampling supports num_picks <= 32 (rowwise_sampling_bias.cu:73)");
    float *cdf = nullptr;
    const dim3 grid((unsigned)ceil_div(S, kBiasRowsPerBlock));
    BiasHubArgs ba{};
    if (bias_hubs) {
      ba = BiasHubArgs{src,  Sc,     k,   launch_seed, rowinfo, tpre, boff,
                       hub,  nworkers, rowpos, col, table,   cand};
      hipLaunchKernelGGL(k_bias_boot, dim3((unsigned)std::min<int64_t>(S, bias_boot_blocks())),
                         dim3(kTileRows), 0, st, ba);
      DGS_LAUNCH_CHECK();
      // DGS_BIAS_STATS=1 (diagnostics, synchronises): the hop's hub rows and their edges
      static const bool stats = getenv("DGS_BIAS_STATS") != nullptr;
      if (stats) {
        DGS_HIP(hipStreamSynchronize(st));
        int64_t packed = 0, Sd = S;
        DGS_HIP(hipMemcpy(&packed, hub.count, 8, hipMemcpyDeviceToHost));
        if (Sc.p) DGS_HIP(hipMemcpy(&Sd, Sc.p, 8, hipMemcpyDeviceToHost));
        const int64_t H = (int64_t)((uint64_t)packed >> kHubShift);
        std::vector<int64_t> rows((size_t)H);
        std::vector<RowInfo> ri((size_t)Sd);
        if (H) DGS_HIP(hipMemcpy(rows.data(), hub.row, 8 * H, hipMemcpyDeviceToHost));
        if (Sd) DGS_HIP(hipMemcpy(ri.data(), rowinfo, sizeof(RowInfo) * Sd, hipMemcpyDeviceToHost));
        int64_t edges = 0;
        for (int64_t h = 0; h < H; ++h) {
          const int64_t d = ri[(size_t)rows[(size_t)h]].dl & kOffMask;
          edges += d;
        }
        fprintf(stderr, "[bias stats] S %lld hubs %lld hub edges %lld stream chunks %lld\n",
                (long long)Sd, (long long)H, (long long)edges,
                (long long)((uint64_t)packed & kHubChunkMask));
      }
      // (its workgroup 0 also does the hop's tile-offset scan)
      hipLaunchKernelGGL(k_bias_stream, dim3(sblocks), dim3(kTileRows), 0, st, ba,
                         (const int64_t *)bsum, boff, d_nnz,
                         profile_stamps(4, sblocks, DGS_STREAM_COUNTERS ? 2 : 0));
      DGS_LAUNCH_CHECK();
      if (stats) {  // candidates per hub row after the stream
        DGS_HIP(hipStreamSynchronize(st));
        int64_t packed = 0;
        DGS_HIP(hipMemcpy(&packed, hub.count, 8, hipMemcpyDeviceToHost));
        const int64_t H = (int64_t)((uint64_t)packed >> kHubShift);
        std::vector<int32_t> cnt((size_t)H), cap((size_t)H);
        if (H) {
          DGS_HIP(hipMemcpy(cnt.data(), cand.cnt, 4 * H, hipMemcpyDeviceToHost));
          DGS_HIP(hipMemcpy(cap.data(), cand.cap, 4 * H, hipMemcpyDeviceToHost));
        }
        int64_t tot = 0, over = 0, mx = 0, big64 = 0, big256 = 0, in256 = 0;
        for (int64_t h = 0; h < H; ++h) {
          if (cnt[(size_t)h] > cap[(size_t)h]) { ++over; continue; }
          tot += cnt[(size_t)h];
          mx = std::max<int64_t>(mx, cnt[(size_t)h]);
          big64 += cnt[(size_t)h] > 64;
          big256 += cnt[(size_t)h] > 256;
          in256 += cnt[(size_t)h] > 256 ? cnt[(size_t)h] : 0;
        }
        fprintf(stderr,
                "[bias stats] candidates %lld (max %lld, rows > 64: %lld, rows > 256: %lld holding "
                "%lld) overflowed rows %lld\n",
                (long long)tot, (long long)mx, (long long)big64, (long long)big256,
                (long long)in256, (long long)over);
      }
    }
    if (replace) {
      // CDF scratch = sum of degrees (the reference's temp tensor, :257-259): one D2H.
      int64_t *h = (ws.host.ensure(64), ws.host.as<int64_t>() + 4);
      DGS_HIP(hipMemcpyAsync(h, bsum + 2 * nb + 1, sizeof(int64_t), hipMemcpyDeviceToHost, st));
      DGS_HIP(hipStreamSynchronize(st));
      ws.cdf.ensure(sizeof(float) * (size_t)(h[0] > 0 ? h[0] : 1));
      cdf = ws.cdf.as<float>();
      hipLaunchKernelGGL(k_sample_bias<true>, grid, dim3(kTileRows), 0, st, src, Sc, k,
                         launch_seed, rowinfo, tpre, boff, tpre2, tboff, cdf, rowpos, col, table,
                         (const int64_t *)nullptr);
    } else {
      // DGS_BIAS_SPLIT_MERGE=1: rows and hub merge as two launches (profiling)
      static const bool split = getenv("DGS_BIAS_SPLIT_MERGE") != nullptr;
      if (bias_hubs && split) {
        hipLaunchKernelGGL(k_sample_bias<false>, grid, dim3(kTileRows), 0, st, src, Sc, k,
                           launch_seed, rowinfo, tpre, boff, tpre2, tboff, cdf, rowpos, col,
                           table, (const int64_t *)hub.hubid);
        DGS_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_bias_hub_merge,
                           dim3((unsigned)std::min<int64_t>(S, bias_merge_blocks())),
                           dim3(kTileRows), 0, st, ba);
        DGS_LAUNCH_CHECK();
        return;
      }
      if (bias_hubs) {
        const int64_t mb = std::min<int64_t>(S, bias_merge_blocks());
        hipLaunchKernelGGL(k_bias_rows_merge, dim3((unsigned)(grid.x + mb)), dim3(kTileRows), 0,
                           st, ba, (const int32_t *)tpre2, (const int64_t *)tboff,
                           (int64_t)grid.x, mb);
        DGS_LAUNCH_CHECK();
        return;
      }
      hipLaunchKernelGGL(k_sample_bias<false>, grid, dim3(kTileRows), 0, st, src, Sc, k,
                         launch_seed, rowinfo, tpre, boff, tpre2, tboff, cdf, rowpos, col, table,
                         (const int64_t *)nullptr);
    }
    DGS_LAUNCH_CHECK();
  }
}

}  // namespace dgs
