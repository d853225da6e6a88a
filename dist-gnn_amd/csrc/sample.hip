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
#include "dgs_ops.h"

namespace dgs {
namespace {

constexpr int kTileRows = 256;   // rows per prep / sample workgroup
constexpr int kGroup = 16;       // lanes per row in the uniform kernel
constexpr int kHubT = 1024;      // reservoir tail length above which a row is split
constexpr int kHubBlocks = 512;  // workgroups of the hub kernel
constexpr int kMaxPicksLds = 512;
constexpr int kScanThreads = 1024;

struct RowInfo {
  int64_t off;
  int64_t dl;  // degree | location << 56
};

__device__ __forceinline__ int64_t ri_deg(const RowInfo &r) { return r.dl & kOffMask; }
__device__ __forceinline__ int ri_loc(const RowInfo &r) {
  return (int)((uint64_t)r.dl >> kLocShift);
}

__device__ __forceinline__ RowInfo lookup_row(const RowSrc &src, int64_t v) {
  RowInfo ri;
  if (src.ntab) {
    const NodeEntry e = src.ntab[v];
    ri.off = e.off;
    ri.dl = e.dl;
  } else {
    const int64_t b = src.indptr[v], e = src.indptr[v + 1];
    ri.off = b;
    ri.dl = e - b;  // location 0
  }
  return ri;
}

__device__ __forceinline__ int64_t row_count(int64_t deg, int64_t k, bool replace) {
  return replace ? (deg == 0 ? 0 : k) : (deg < k ? deg : k);
}

// Hub bookkeeping layout inside ws.hub (int64 words):
//   [0] hub count, [1..] pad to 8, then hub_row[S], hub_nch[S + 1], hub_cptr[S + 1], hubid[S]
struct HubView {
  int64_t *count, *row, *nch, *cptr, *hubid;
  __host__ __device__ static HubView make(int64_t *base, int64_t S) {
    HubView h;
    h.count = base;
    h.row = base + 8;
    h.nch = h.row + S;
    h.cptr = h.nch + S + 1;
    h.hubid = h.cptr + S + 1;
    return h;
  }
  static size_t bytes(int64_t S) { return sizeof(int64_t) * (size_t)(8 + 4 * S + 2); }
};

// ------------------------------------------------------------------------------------
// Prep: per-row lookup (one 16-byte node-table load), counts, hub detection, tile sums.
__global__ __launch_bounds__(kTileRows) void k_prep(RowSrc src, const int64_t *__restrict__ seeds,
                                                    int64_t S, int64_t k, int replace,
                                                    int use_hubs, int bias_replace,
                                                    RowInfo *__restrict__ rowinfo,
                                                    int64_t *__restrict__ bsum,
                                                    int64_t *__restrict__ tsum, HubView hub) {
  __shared__ int64_t lds[kTileRows / 64];
  const int64_t i = (int64_t)blockIdx.x * kTileRows + threadIdx.x;
  int64_t cnt = 0, tdeg = 0;
  if (i < S) {
    const RowInfo ri = lookup_row(src, seeds[i]);
    rowinfo[i] = ri;
    const int64_t deg = ri_deg(ri);
    cnt = row_count(deg, k, replace);
    tdeg = deg;
    if (use_hubs) {
      int64_t h = -1;
      if (!replace && deg - k > kHubT) {
        h = atomicAdd((unsigned long long *)hub.count, 1ull);
        hub.row[h] = i;
        hub.nch[h] = (deg - k + 511) / 512;
      }
      hub.hubid[i] = h;
    }
  }
  const int64_t s = block_sum<kTileRows>(cnt, lds);
  if (threadIdx.x == 0) bsum[blockIdx.x] = s;
  if (bias_replace) {
    const int64_t t = block_sum<kTileRows>(tdeg, lds);
    if (threadIdx.x == 0) tsum[blockIdx.x] = t;
  }
}

// Single workgroup: exclusive scan of tile sums (-> boff[0..nb], boff[nb] = nnz), the hub
// chunk prefix and hub slot initialisation (slot s = s, rowwise_sampling.cu:80-82).
__global__ __launch_bounds__(kScanThreads) void k_scan_hop(const int64_t *bsum, int64_t nb,
                                                          int64_t *boff, int use_hubs,
                                                          HubView hub, int64_t k,
                                                          int32_t *hubslot) {
  __shared__ int64_t lds[kScanThreads / 64];
  int64_t carry = 0;
  for (int64_t base = 0; base < nb; base += kScanThreads) {
    const int64_t i = base + threadIdx.x;
    const int64_t v = i < nb ? bsum[i] : 0;
    int64_t tot;
    const int64_t ex = block_exclusive_scan<kScanThreads>(v, &tot, lds);
    if (i < nb) boff[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) boff[nb] = carry;
  if (!use_hubs) return;
  const int64_t H = *hub.count;
  carry = 0;
  for (int64_t base = 0; base < H; base += kScanThreads) {
    const int64_t i = base + threadIdx.x;
    const int64_t v = i < H ? hub.nch[i] : 0;
    int64_t tot;
    const int64_t ex = block_exclusive_scan<kScanThreads>(v, &tot, lds);
    if (i < H) hub.cptr[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) hub.cptr[H] = carry;
  for (int64_t j = threadIdx.x; j < H * k; j += kScanThreads) hubslot[j] = (int32_t)(j % k);
}

// ------------------------------------------------------------------------------------
// Hub reservoir: every wave takes 512-edge chunks (idx = k + 512q + t + 128w, t < 128,
// w < 4 <-> one Philox block per logical thread t) of any hub row and folds its picks into
// the row's k slots with atomicMax (rowwise_sampling.cu:85-92).
__global__ __launch_bounds__(256) void k_hub_reservoir(const RowInfo *__restrict__ rowinfo,
                                                       int64_t S, int64_t k, uint64_t seed,
                                                       HubView hub, int32_t *hubslot) {
  const int64_t H = *hub.count;
  if (H == 0) return;
  const int64_t total = hub.cptr[H];
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t c = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; c < total;
       c += nwaves) {
    int64_t lo = 0, hi = H;  // largest h with cptr[h] <= c
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) >> 1;
      if (hub.cptr[mid] <= c) lo = mid; else hi = mid;
    }
    const int64_t h = lo;
    const int64_t q = c - hub.cptr[h];
    const int64_t r = hub.row[h];
    const int64_t deg = ri_deg(rowinfo[r]);
    const uint64_t key = seed * (uint64_t)S + (uint64_t)r;
    const uint2 kk = make_uint2((uint32_t)key, (uint32_t)(key >> 32));
    int32_t *sl = hubslot + h * k;
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int t = lane + 64 * tt;
      const int64_t base = k + t + 512 * q;
      if (base < deg) {
        const uint4 o4 = philox4x32_10(make_uint4((uint32_t)q, (uint32_t)((uint64_t)q >> 32),
                                                  (uint32_t)t, 0u), kk);
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

// ------------------------------------------------------------------------------------
// Uniform sampling of one 256-row tile.  16-lane groups own rows.
template <bool kReplace>
__global__ __launch_bounds__(kTileRows) void k_sample_uniform(
    RowSrc src, int64_t S, int64_t k, uint64_t seed, const RowInfo *__restrict__ rowinfo,
    const int64_t *__restrict__ boff, HubView hub, const int32_t *__restrict__ hubslot,
    int use_hubs, int64_t *__restrict__ rowpos, int64_t *__restrict__ col) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int64_t *s_off = reinterpret_cast<int64_t *>(smem);                       // [256]
  int64_t *s_scan = s_off + kTileRows;                                       // [4]
  int32_t *s_slot = reinterpret_cast<int32_t *>(s_scan + kTileRows / 64);   // [16][k]

  const int64_t tile0 = (int64_t)blockIdx.x * kTileRows;
  {
    const int64_t i = tile0 + threadIdx.x;
    const int64_t cnt = i < S ? row_count(ri_deg(rowinfo[i]), k, kReplace) : 0;
    int64_t tot;
    const int64_t ex = block_exclusive_scan<kTileRows>(cnt, &tot, s_scan);
    s_off[threadIdx.x] = boff[blockIdx.x] + ex;
  }
  __syncthreads();

  const int g = threadIdx.x / kGroup, L = threadIdx.x % kGroup;
  int32_t *sl = s_slot + g * k;
  for (int rr = g; rr < kTileRows; rr += kTileRows / kGroup) {
    const int64_t r = tile0 + rr;
    if (r >= S) break;
    const RowInfo ri = rowinfo[r];
    const int64_t deg = ri_deg(ri);
    const int64_t begin = ri.off;
    const int64_t *idx_base = reinterpret_cast<const int64_t *>(src.indices.p[ri_loc(ri)]);
    const int64_t out = s_off[rr];
    const uint64_t key = seed * (uint64_t)S + (uint64_t)r;
    const uint2 kk = make_uint2((uint32_t)key, (uint32_t)(key >> 32));
    if (kReplace) {
      if (deg > 0) {
        for (int64_t p = L; p < k; p += kGroup) {
          const int64_t t = p & 127, j = p >> 7;
          const uint4 o4 = philox4x32_10(
              make_uint4((uint32_t)(j >> 2), 0u, (uint32_t)t, 0u), kk);
          const uint32_t x = u4_get(o4, (int)(j & 3));
          const int64_t e = (int64_t)x % deg;
          rowpos[out + p] = r;
          col[out + p] = idx_base[begin + e];
        }
      }
    } else if (deg <= k) {
      for (int64_t p = L; p < deg; p += kGroup) {
        rowpos[out + p] = r;
        col[out + p] = idx_base[begin + p];
      }
    } else {
      const int64_t h = use_hubs ? hub.hubid[r] : -1;
      const int32_t *slots = sl;
      if (h >= 0) {
        slots = hubslot + h * k;
      } else {
        for (int64_t s = L; s < k; s += kGroup) sl[s] = (int32_t)s;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        for (int64_t q = 0; k + 512 * q < deg; ++q) {
          for (int tt = 0; tt < 128 / kGroup; ++tt) {
            const int t = L + kGroup * tt;
            const int64_t base = k + t + 512 * q;
            if (base >= deg) break;
            const uint4 o4 = philox4x32_10(
                make_uint4((uint32_t)q, (uint32_t)((uint64_t)q >> 32), (uint32_t)t, 0u), kk);
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
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
      for (int64_t s = L; s < k; s += kGroup) {
        rowpos[out + s] = r;
        col[out + s] = idx_base[begin + slots[s]];
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  }
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

template <bool kReplace>
__global__ __launch_bounds__(kTileRows) void k_sample_bias(
    RowSrc src, int64_t S, int64_t k, uint64_t seed, const RowInfo *__restrict__ rowinfo,
    const int64_t *__restrict__ boff, const int64_t *__restrict__ tboff, float *cdf,
    int64_t *__restrict__ rowpos, int64_t *__restrict__ col) {
  __shared__ int64_t s_off[kTileRows];
  __shared__ int64_t s_toff[kTileRows];
  __shared__ int64_t s_scan[kTileRows / 64];
  const int64_t tile0 = (int64_t)blockIdx.x * kTileRows;
  {
    const int64_t i = tile0 + threadIdx.x;
    const int64_t deg = i < S ? ri_deg(rowinfo[i]) : 0;
    int64_t tot;
    const int64_t ex = block_exclusive_scan<kTileRows>(row_count(deg, k, kReplace), &tot, s_scan);
    s_off[threadIdx.x] = boff[blockIdx.x] + ex;
    if (kReplace) {
      const int64_t ex2 = block_exclusive_scan<kTileRows>(deg, &tot, s_scan);
      s_toff[threadIdx.x] = tboff[blockIdx.x] + ex2;
    }
  }
  __syncthreads();

  const int64_t G = (S + 15) / 16;  // reference grid: ceil(S / TILE_SIZE=16)
  const int hw = threadIdx.x >> 5, l = threadIdx.x & 31;
  for (int rr = hw; rr < kTileRows; rr += kTileRows / 32) {
    const int64_t r = tile0 + rr;
    if (r >= S) break;
    const RowInfo ri = rowinfo[r];
    const int64_t deg = ri_deg(ri);
    const int64_t begin = ri.off;
    const int loc = ri_loc(ri);
    const int64_t *idx_base = reinterpret_cast<const int64_t *>(src.indices.p[loc]);
    const float *p_base = reinterpret_cast<const float *>(src.probs.p[loc]);
    const int64_t out = s_off[rr];
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
          rowpos[out + p] = r;
          col[out + p] = idx_base[begin + p];
        }
        continue;
      }
      // half-wave top-k: lane q holds the q-th best (key, idx) so far
      float bk = -__builtin_inff();
      int64_t bi = INT64_MAX;
      int cnt = 0;
      float thr_k = 0.0f;
      int64_t thr_i = 0;
      uint4 o4 = make_uint4(0, 0, 0, 0);
      int64_t cached_q = -1;
      for (int64_t base = 0; base < deg; base += 32) {
        const int64_t i = base + l;
        float key_i = -__builtin_inff();
        if (i < deg) {
          const int64_t q = j >> 2;
          if (q != cached_q) {
            o4 = philox4x32_10(make_uint4((uint32_t)q, (uint32_t)((uint64_t)q >> 32), sub, 0u),
                               kk);
            cached_q = q;
          }
          const float u = curand_uniform_from(u4_get(o4, (int)(j & 3)));
          key_i = ares_key(u, p_base[begin + i]);
          ++j;
        }
        bool cand = i < deg && (cnt < k || ares_better(key_i, i, thr_k, thr_i));
        uint32_t mask = half_ballot(cand);
        while (mask) {
          const int c = __builtin_ctz(mask);
          const float ck = __shfl(key_i, c, 32);
          const int64_t ci = __shfl(i, c, 32);
          const uint32_t better = half_ballot(l < cnt && ares_better(bk, bi, ck, ci));
          const int pos = __builtin_popcount(better);
          const float nk = __shfl_up(bk, 1, 32);
          const int64_t ni = __shfl_up(bi, 1, 32);
          if (pos < k) {
            if (l > pos) {
              bk = nk;
              bi = ni;
            } else if (l == pos) {
              bk = ck;
              bi = ci;
            }
            if (cnt < k) ++cnt;
          }
          thr_k = __shfl(bk, (int)(k - 1), 32);
          thr_i = __shfl(bi, (int)(k - 1), 32);
          mask &= ~(1u << c);
          cand = cand && (l != c) && (cnt < k || ares_better(key_i, i, thr_k, thr_i));
          mask &= half_ballot(cand);
        }
      }
      if (l < k) {
        rowpos[out + l] = r;
        col[out + l] = idx_base[begin + bi];
      }
    } else {
      if (deg == 0) continue;
      // CDF, 32 edges at a time: lane 0 adds the running aggregate, clamp at 0, then a
      // Kogge-Stone inclusive scan (cub::WarpScan::InclusiveSum), :185-202.
      float *crow = cdf + s_toff[rr];
      float agg = 0.0f, sum = 0.0f;
      for (int64_t base = 0; base < deg; base += 32) {
        const int64_t i = base + l;
        float v = i < deg ? p_base[begin + i] : 0.0f;
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
        rowpos[out + p] = r;
        col[out + p] = idx_base[begin + item];
      }
    }
  }
}

}  // namespace

// ------------------------------------------------------------------------------------
void sample_hop(const RowSrc &src, const int64_t *seeds, int64_t S, int64_t k, bool replace,
                bool bias, uint64_t launch_seed, int64_t *rowpos, int64_t *col, int64_t *d_nnz,
                HopScratch &ws, hipStream_t st) {
  DGS_CHECK(k >= 0, "num_picks must be non-negative");
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
  if (S == 0 || k == 0) {
    DGS_HIP(hipMemsetAsync(d_nnz, 0, sizeof(int64_t), st));
    return;
  }
  const bool use_hubs = !bias && !replace;
  ws.hub.ensure(HubView::bytes(S));
  HubView hub = HubView::make(ws.hub.as<int64_t>(), S);
  if (use_hubs) {
    DGS_HIP(hipMemsetAsync(hub.count, 0, sizeof(int64_t), st));
    ws.hubslot.ensure(sizeof(int32_t) * (size_t)(S * k));
  }
  const bool bias_replace = bias && replace;
  profile_begin(st, 1);
  hipLaunchKernelGGL(k_prep, dim3((unsigned)nb), dim3(kTileRows), 0, st, src, seeds, S, k,
                     (int)replace, (int)use_hubs, (int)bias_replace, rowinfo, bsum, tsum, hub);
  DGS_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_scan_hop, dim3(1), dim3(kScanThreads), 0, st, bsum, nb, boff,
                     (int)use_hubs, hub, k, ws.hubslot.as<int32_t>());
  DGS_LAUNCH_CHECK();
  DGS_HIP(hipMemcpyAsync(d_nnz, boff + nb, sizeof(int64_t), hipMemcpyDeviceToDevice, st));

  if (!bias) {
    if (use_hubs) {
      hipLaunchKernelGGL(k_hub_reservoir, dim3(kHubBlocks), dim3(256), 0, st, rowinfo, S, k,
                         launch_seed, hub, ws.hubslot.as<int32_t>());
      DGS_LAUNCH_CHECK();
    }
    DGS_CHECK(replace || k <= kMaxPicksLds, "num_picks > 512 is not supported without replacement");
    const size_t lds = sizeof(int64_t) * (kTileRows + kTileRows / 64) +
                       (replace ? 0 : sizeof(int32_t) * (size_t)(kTileRows / kGroup) * k);
    if (replace)
      hipLaunchKernelGGL(k_sample_uniform<true>, dim3((unsigned)nb), dim3(kTileRows), lds, st,
                         src, S, k, launch_seed, rowinfo, boff, hub, ws.hubslot.as<int32_t>(),
                         0, rowpos, col);
    else
      hipLaunchKernelGGL(k_sample_uniform<false>, dim3((unsigned)nb), dim3(kTileRows), lds, st,
                         src, S, k, launch_seed, rowinfo, boff, hub, ws.hubslot.as<int32_t>(),
                         1, rowpos, col);
    DGS_LAUNCH_CHECK();
  } else {
    DGS_CHECK(k <= 32, "biased sampling supports num_picks <= 32 (rowwise_sampling_bias.cu:73)");
    float *cdf = nullptr;
    if (replace) {
      // CDF scratch = sum of degrees (the reference's temp tensor, :257-259): one D2H.
      scan_small(tsum, nb, tboff, st);
      int64_t *h = (ws.host.ensure(16), ws.host.as<int64_t>());
      DGS_HIP(hipMemcpyAsync(h, tboff + nb, sizeof(int64_t), hipMemcpyDeviceToHost, st));
      DGS_HIP(hipStreamSynchronize(st));
      ws.cdf.ensure(sizeof(float) * (size_t)(h[0] > 0 ? h[0] : 1));
      cdf = ws.cdf.as<float>();
      hipLaunchKernelGGL(k_sample_bias<true>, dim3((unsigned)nb), dim3(kTileRows), 0, st, src, S,
                         k, launch_seed, rowinfo, boff, tboff, cdf, rowpos, col);
    } else {
      hipLaunchKernelGGL(k_sample_bias<false>, dim3((unsigned)nb), dim3(kTileRows), 0, st, src,
                         S, k, launch_seed, rowinfo, boff, tboff, cdf, rowpos, col);
    }
    DGS_LAUNCH_CHECK();
  }
  profile_end(st, 1);
}

}  // namespace dgs
