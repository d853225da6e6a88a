// csr.hip -- CSR / cache-construction kernels and the heat propagation ops.
//
// Reference: sampling/cuda/utils.cu:12-101 (ExtractIndptr / ExtractEdgeData),
// hashmap/cuda/hashmap.cu:15-77 (cache map construction) and
// cache/cuda/preprocess_heat.cu:14-121 (frontier heat).
//
// The graph shard context replaces the reference's open-addressing hashmap + per-device
// pointer table with a dense node table NodeEntry ntab[N] (16 B per node: edge offset inside
// the owning location, degree | location << 56).  One 16-byte load per seed gives
// everything the sampler needs; for papers100M (N = 111 M) the table is 1.8 GB of 288 GB HBM.
#include "dgs_block.cuh"
#include "dgs_ops.h"

namespace dgs {
namespace {

__global__ void k_degrees(const int64_t *nids, int64_t n, const int64_t *indptr, int64_t *deg) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int64_t v = nids[i];
    deg[i] = indptr[v + 1] - indptr[v];
  }
}

// One wave per row: copies edge_data[indptr[v] .. indptr[v+1]) into sub at sub_indptr[i].
template <typename T>
__global__ __launch_bounds__(256) void k_extract_rows(const int64_t *nids, int64_t n,
                                                      const int64_t *indptr,
                                                      const int64_t *sub_indptr,
                                                      const T *__restrict__ src,
                                                      T *__restrict__ dst) {
  const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = w; i < n; i += nw) {
    const int64_t v = nids[i];
    const int64_t b = indptr[v], d = indptr[v + 1] - b, o = sub_indptr[i];
    for (int64_t j = lane; j < d; j += 64) dst[o + j] = src[b + j];
  }
}

__global__ void k_ntab_init_host(NodeEntry *ntab, const int64_t *indptr, int64_t n,
                                 const int64_t *indices) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n) {
    const int64_t b = indptr[v], e = indptr[v + 1];
    NodeEntry ne;
    ne.ptr = indices + b;
    ne.dl = (e - b) | ((int64_t)kLocHost << kLocShift);
    ntab[v] = ne;
  }
}

// (the sampler range-checks its cache lists before this runs; the guard keeps a list that
// slipped through from writing outside the table)
__global__ void k_ntab_assign(NodeEntry *ntab, int64_t num_nodes, const int64_t *nids,
                              const int64_t *sub_indptr, int64_t n, int64_t loc,
                              const int64_t *sub_indices) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && (uint64_t)nids[i] < (uint64_t)num_nodes) {
    const int64_t b = sub_indptr[i], e = sub_indptr[i + 1];
    NodeEntry ne;
    ne.ptr = sub_indices + b;
    ne.dl = (e - b) | (loc << kLocShift);
    ntab[nids[i]] = ne;
  }
}

// Heat accumulation: float atomics as the reference (order-dependent rounding), or fixed point
// (deterministic): messages are rounded to multiples of 2^-36 and summed as int64, which is
// associative, so the result does not depend on the order the atomics land in.  Resolution
// 1.5e-11; no overflow below 2^27 unit messages into one node.
constexpr double kHeatFixedScale = 68719476736.0;  // 2^36
struct FloatHeat {
  float *fh;
  __device__ __forceinline__ void add(int64_t v, float m) const { atomicAdd(fh + v, m); }
};
struct FixedHeat {
  unsigned long long *acc;
  __device__ __forceinline__ void add(int64_t v, float m) const {
    atomicAdd(acc + v, (unsigned long long)__double2ll_rn((double)m * kHeatFixedScale));
  }
};

// preprocess_heat.cu:14-33 -- one thread per seed; message min(1, heat * k / deg) per edge.
template <typename Acc>
__global__ void k_heat(const int64_t *seeds, int64_t n, const int64_t *indptr,
                       const int64_t *indices, const float *seeds_heat, int64_t num_picks,
                       int64_t indptr_diff, Acc acc) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const int64_t row = seeds[s];
  const int64_t b = indptr[row] - indptr_diff, e = indptr[row + 1] - indptr_diff;
  const int64_t deg = e - b;
  if (deg <= 0) return;
  const float m = __fdiv_rn(__fmul_rn(seeds_heat[row], (float)num_picks), (float)deg);
  const float msg = (1.0f < m) ? 1.0f : m;
  for (int64_t i = b; i < e; ++i) acc.add(indices[i], msg);
}

// preprocess_heat.cu:58-98 -- the biased variant; row probabilities summed in edge order.
template <typename Acc>
__global__ void k_heat_bias(const int64_t *seeds, int64_t n, const int64_t *indptr,
                            const int64_t *indices, const float *probs, const float *seeds_heat,
                            int64_t num_picks, int64_t indptr_diff, Acc acc) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const int64_t row = seeds[s];
  const int64_t b = indptr[row] - indptr_diff, e = indptr[row + 1] - indptr_diff;
  float psum = 0.0f;
  for (int64_t i = b; i < e; ++i) psum = __fadd_rn(psum, probs[i]);
  const float hk = __fmul_rn(seeds_heat[row], (float)num_picks);
  for (int64_t i = b; i < e; ++i) {
    const float m = __fmul_rn(hk, __fdiv_rn(probs[i], psum));
    const float msg = (1.0f < m) ? 1.0f : m;
    acc.add(indices[i], msg);
  }
}

__global__ void k_heat_fixed_to_float(const unsigned long long *acc, int64_t n, float *fh) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n) fh[v] = (float)((double)(long long)acc[v] / kHeatFixedScale);
}

__global__ void k_cached_flag(const int64_t *tab, int64_t n, int64_t *flag) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n) flag[v] = ((int)((uint64_t)tab[v] >> kLocShift) != kLocHost) ? 1 : 0;
}

__global__ void k_cached_scatter(const int64_t *tab, int64_t n, const int64_t *pos,
                                 int64_t *key, int64_t *idx, int64_t *devid, int64_t *d_count) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v == 0) *d_count = pos[n];
  if (v >= n || !key) return;
  const int64_t e = tab[v];
  const int loc = (int)((uint64_t)e >> kLocShift);
  if (loc == kLocHost) return;
  const int64_t p = pos[v];
  key[p] = v;
  idx[p] = e & kOffMask;
  devid[p] = loc;
}

__global__ void k_loctab_init(int64_t *tab, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) tab[i] = ((int64_t)kLocHost << kLocShift) | i;
}

__global__ void k_loctab_assign(int64_t *tab, int64_t num_nodes, const int64_t *nids, int64_t n,
                                int64_t loc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && (uint64_t)nids[i] < (uint64_t)num_nodes) tab[nids[i]] = (loc << kLocShift) | i;
}

__global__ void k_take_i64(const int64_t *src, const int64_t *idx, int64_t n, int64_t *out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = src[idx[i]];
}

}  // namespace

void extract_indptr(const int64_t *nids, int64_t n, const int64_t *indptr, int64_t *sub_indptr,
                    hipStream_t st) {
  if (n > 0) {
    hipLaunchKernelGGL(k_degrees, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, nids, n,
                       indptr, sub_indptr);
    DGS_LAUNCH_CHECK();
  }
  TmpBuf scratch(scan_scratch_bytes(n), st);
  scan_exclusive(sub_indptr, n, sub_indptr, scratch.p, st);
}

void extract_edge_data(const int64_t *nids, int64_t n, const int64_t *indptr,
                       const int64_t *sub_indptr, const void *edge_data, int64_t elem_bytes,
                       void *sub, hipStream_t st) {
  if (n <= 0) return;
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n, 4), 65536);
  switch (elem_bytes) {
    case 8:
      hipLaunchKernelGGL(k_extract_rows<int64_t>, dim3(grid), dim3(256), 0, st, nids, n, indptr,
                         sub_indptr, (const int64_t *)edge_data, (int64_t *)sub);
      break;
    case 4:
      hipLaunchKernelGGL(k_extract_rows<int32_t>, dim3(grid), dim3(256), 0, st, nids, n, indptr,
                         sub_indptr, (const int32_t *)edge_data, (int32_t *)sub);
      break;
    case 2:
      hipLaunchKernelGGL(k_extract_rows<int16_t>, dim3(grid), dim3(256), 0, st, nids, n, indptr,
                         sub_indptr, (const int16_t *)edge_data, (int16_t *)sub);
      break;
    case 1:
      hipLaunchKernelGGL(k_extract_rows<int8_t>, dim3(grid), dim3(256), 0, st, nids, n, indptr,
                         sub_indptr, (const int8_t *)edge_data, (int8_t *)sub);
      break;
    default:
      DGS_CHECK(false, "edge data element size must be 1, 2, 4 or 8 bytes");
  }
  DGS_LAUNCH_CHECK();
}

void ntab_init_host(NodeEntry *ntab, const int64_t *indptr, int64_t n, const int64_t *indices,
                    hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_ntab_init_host, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, ntab,
                     indptr, n, indices);
  DGS_LAUNCH_CHECK();
}

void ntab_assign(NodeEntry *ntab, int64_t num_nodes, const int64_t *nids,
                 const int64_t *sub_indptr, int64_t n, int loc, const int64_t *sub_indices,
                 hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_ntab_assign, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, ntab,
                     num_nodes, nids, sub_indptr, n, (int64_t)loc, sub_indices);
  DGS_LAUNCH_CHECK();
}

void heat(const int64_t *seeds, int64_t n_seeds, const int64_t *indptr, const int64_t *indices,
          const float *probs, const float *seeds_heat, int64_t num_picks, int64_t indptr_diff,
          float *frontier_heat, int64_t num_nodes, unsigned long long *fixed_acc,
          hipStream_t st) {
  if (probs) n_seeds -= 1;  // preprocess_heat.cu:107 processes seeds.numel() - 1 seeds
  if (fixed_acc) DGS_HIP(hipMemsetAsync(fixed_acc, 0, sizeof(uint64_t) * (size_t)num_nodes, st));
  if (n_seeds > 0) {
    const dim3 grid((unsigned)ceil_div(n_seeds, 128)), block(128);
    if (fixed_acc) {
      const FixedHeat acc{fixed_acc};
      if (probs)
        hipLaunchKernelGGL(k_heat_bias<FixedHeat>, grid, block, 0, st, seeds, n_seeds, indptr,
                           indices, probs, seeds_heat, num_picks, indptr_diff, acc);
      else
        hipLaunchKernelGGL(k_heat<FixedHeat>, grid, block, 0, st, seeds, n_seeds, indptr,
                           indices, seeds_heat, num_picks, indptr_diff, acc);
    } else {
      const FloatHeat acc{frontier_heat};
      if (probs)
        hipLaunchKernelGGL(k_heat_bias<FloatHeat>, grid, block, 0, st, seeds, n_seeds, indptr,
                           indices, probs, seeds_heat, num_picks, indptr_diff, acc);
      else
        hipLaunchKernelGGL(k_heat<FloatHeat>, grid, block, 0, st, seeds, n_seeds, indptr,
                           indices, seeds_heat, num_picks, indptr_diff, acc);
    }
    DGS_LAUNCH_CHECK();
  }
  if (fixed_acc && num_nodes > 0) {
    hipLaunchKernelGGL(k_heat_fixed_to_float, dim3((unsigned)ceil_div(num_nodes, 256)),
                       dim3(256), 0, st, fixed_acc, num_nodes, frontier_heat);
    DGS_LAUNCH_CHECK();
  }
}

void cache_map_compact(const int64_t *tab, int64_t n, int64_t *key, int64_t *idx,
                       int64_t *devid, int64_t *d_count, hipStream_t st) {
  TmpBuf posb(sizeof(int64_t) * (size_t)(n + 1), st), scratch(scan_scratch_bytes(n), st);
  int64_t *pos = posb.as<int64_t>();
  if (n > 0) {
    hipLaunchKernelGGL(k_cached_flag, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, tab,
                       n, pos);
    DGS_LAUNCH_CHECK();
  }
  scan_exclusive(pos, n, pos, scratch.p, st);
  hipLaunchKernelGGL(k_cached_scatter, dim3((unsigned)ceil_div(n > 0 ? n : 1, 256)), dim3(256),
                     0, st, tab, n, pos, key, idx, devid, d_count);
  DGS_LAUNCH_CHECK();
}

void loctab_init_host(int64_t *tab, int64_t n, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_loctab_init, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, tab, n);
  DGS_LAUNCH_CHECK();
}

void loctab_assign(int64_t *tab, int64_t num_nodes, const int64_t *nids, int64_t n, int loc,
                   hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_loctab_assign, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, tab,
                     num_nodes, nids, n, (int64_t)loc);
  DGS_LAUNCH_CHECK();
}

void take_i64(const int64_t *src, const int64_t *idx, int64_t n, int64_t *out, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_take_i64, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, src, idx,
                     n, out);
  DGS_LAUNCH_CHECK();
}

}  // namespace dgs
