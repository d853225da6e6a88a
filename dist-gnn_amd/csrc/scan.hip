// scan.hip -- exclusive prefix sums (cub::DeviceScan::ExclusiveSum replacement used by the
// reference at cub_function.h:11-23).  Reduce-then-scan over 4096-element tiles with a
// single-workgroup scan of the tile sums; wave64 shuffles inside each workgroup.
#include "dgs_block.cuh"
#include "dgs_ops.h"

namespace dgs {
namespace {

constexpr int kScanThreads = 1024;
constexpr int kTileThreads = 256;
constexpr int kTileItems = 16;
constexpr int kTile = kTileThreads * kTileItems;

// out[0..n] = exclusive scan of in[0..n), out[n] = total.  One workgroup.
__global__ __launch_bounds__(kScanThreads) void k_scan_small(const int64_t *in, int64_t n,
                                                             int64_t *out) {
  __shared__ int64_t lds[kScanThreads / 64];
  const int64_t tot = block_scan_range<kScanThreads, 8>(in, n, out, lds);
  if (threadIdx.x == 0) out[n] = tot;
}

__global__ __launch_bounds__(kTileThreads) void k_tile_reduce(const int64_t *in, int64_t n,
                                                              int64_t *tsum) {
  __shared__ int64_t lds[kTileThreads / 64];
  const int64_t base = (int64_t)blockIdx.x * kTile;
  int64_t s = 0;
#pragma unroll
  for (int j = 0; j < kTileItems; ++j) {
    const int64_t i = base + j * kTileThreads + threadIdx.x;
    if (i < n) s += in[i];
  }
  s = block_sum<kTileThreads>(s, lds);
  if (threadIdx.x == 0) tsum[blockIdx.x] = s;
}

__global__ __launch_bounds__(kTileThreads) void k_tile_scan(const int64_t *in, int64_t n,
                                                            const int64_t *toff, int64_t *out) {
  __shared__ int64_t lds[kTileThreads / 64];
  const int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)threadIdx.x * kTileItems;
  int64_t v[kTileItems];
  int64_t s = 0;
#pragma unroll
  for (int j = 0; j < kTileItems; ++j) {
    const int64_t i = base + j;
    v[j] = i < n ? in[i] : 0;
    s += v[j];
  }
  int64_t tot;
  int64_t ex = block_exclusive_scan<kTileThreads>(s, &tot, lds) + toff[blockIdx.x];
#pragma unroll
  for (int j = 0; j < kTileItems; ++j) {
    const int64_t i = base + j;
    if (i < n) out[i] = ex;
    ex += v[j];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = toff[gridDim.x];
}

}  // namespace

void scan_small(const int64_t *in, int64_t n, int64_t *out, hipStream_t st) {
  hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(kScanThreads), 0, st, in, n, out);
  DGS_LAUNCH_CHECK();
}

size_t scan_scratch_bytes(int64_t n) {
  const int64_t nt = ceil_div(n > 0 ? n : 1, kTile);
  return sizeof(int64_t) * (size_t)(2 * nt + 2);
}

void scan_exclusive(const int64_t *in, int64_t n, int64_t *out, void *scratch, hipStream_t st) {
  if (n <= kScanThreads * 4) {
    scan_small(in, n, out, st);
    return;
  }
  const int64_t nt = ceil_div(n, kTile);
  int64_t *tsum = reinterpret_cast<int64_t *>(scratch);
  int64_t *toff = tsum + nt;
  hipLaunchKernelGGL(k_tile_reduce, dim3((unsigned)nt), dim3(kTileThreads), 0, st, in, n, tsum);
  DGS_LAUNCH_CHECK();
  scan_small(tsum, nt, toff, st);
  hipLaunchKernelGGL(k_tile_scan, dim3((unsigned)nt), dim3(kTileThreads), 0, st, in, n, toff,
                     out);
  DGS_LAUNCH_CHECK();
}

}  // namespace dgs
