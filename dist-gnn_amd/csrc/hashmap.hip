// hashmap.hip -- the reference's open-addressing cache map, built for its getter only.
//
// Reference: hashmap/cuda/hashmap.h:12-95 (Hashmap: Murmur3 finaliser, CAS insertion with the
// probe sequence pos <- hash(pos + delta), delta = 1, 2, ...; empty key -1) and
// hashmap/cuda/hashmap.cu:15-77 (CreateNidsP2PCacheHashMapCUDA: dir_size = 2 * _UpPower(total),
// every remote rank's cache list in rotation order, then the local list last, so a node cached
// locally keeps its local (idx, devid)).  The sampler itself never probes this table -- its
// lookups go through the dense node table (csr.hip) -- so it is only built when
// _CAPI_get_local_cache_hashmap_tensors asks for it: the same arrays, capacity and hash as the
// reference (its slot layout depends on the CAS race order in the reference as here).
#include "dgs_ops.h"

namespace dgs {
namespace {

__device__ __forceinline__ uint32_t murmur32(uint32_t k) {
  k ^= k >> 16;
  k *= 0x85ebca6bu;
  k ^= k >> 13;
  k *= 0xc2b2ae35u;
  k ^= k >> 16;
  return k;
}

__device__ __forceinline__ uint64_t murmur64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

// the key's home slot: the 64-bit finaliser for int64 keys, the 32-bit one for int32 keys
__device__ __forceinline__ uint32_t home_slot(int64_t key, uint32_t mask) {
  return (uint32_t)murmur64((uint64_t)key) & mask;
}
__device__ __forceinline__ uint32_t home_slot(int32_t key, uint32_t mask) {
  return murmur32((uint32_t)key) & mask;
}

__device__ __forceinline__ int64_t cas(int64_t *p, int64_t cmp, int64_t val) {
  return (int64_t)atomicCAS(reinterpret_cast<unsigned long long *>(p), (unsigned long long)cmp,
                            (unsigned long long)val);
}
__device__ __forceinline__ int32_t cas(int32_t *p, int32_t cmp, int32_t val) {
  return atomicCAS(reinterpret_cast<int *>(p), cmp, val);
}

template <typename IdT>
__global__ void k_refmap_insert(const int64_t *list, int64_t n, IdT devid, IdT *key, IdT *idx,
                                IdT *dev, uint32_t mask, int *overflow) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const IdT k = (IdT)list[i];
  uint32_t pos = home_slot(k, mask);
  IdT prev = cas(&key[pos], (IdT)-1, k);
  uint32_t delta = 1;
  // (bounded: the reference's probe sequence is not a permutation of the slots)
  while (prev != k && prev != (IdT)-1) {
    if (delta > 4 * (mask + 1)) {
      atomicExch(overflow, 1);
      return;
    }
    pos = murmur32(pos + delta) & mask;
    delta += 1;
    prev = cas(&key[pos], (IdT)-1, k);
  }
  idx[pos] = (IdT)i;
  dev[pos] = devid;
}

template <typename IdT>
__global__ void k_refmap_fill(IdT *a, IdT *b, IdT *c, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = b[i] = c[i] = (IdT)-1;
}

template <typename IdT>
void build(const int64_t *const *lists, const int64_t *counts, const int *order, int nlists,
           int64_t dir, IdT *key, IdT *idx, IdT *dev, hipStream_t st) {
  hipLaunchKernelGGL(k_refmap_fill<IdT>, dim3((unsigned)ceil_div(dir, 256)), dim3(256), 0, st,
                     key, idx, dev, dir);
  DGS_LAUNCH_CHECK();
  TmpBuf ovf(sizeof(int), st);
  DGS_HIP(hipMemsetAsync(ovf.p, 0, sizeof(int), st));
  // one launch per list, in the reference's order: a later list's entry for a key overwrites
  // an earlier one (stream order), so the local list, inserted last, wins
  for (int j = 0; j < nlists; ++j) {
    const int d = order[j];
    if (counts[d] <= 0) continue;
    hipLaunchKernelGGL(k_refmap_insert<IdT>, dim3((unsigned)ceil_div(counts[d], 128)), dim3(128),
                       0, st, lists[d], counts[d], (IdT)d, key, idx, dev, (uint32_t)(dir - 1),
                       ovf.as<int>());
    DGS_LAUNCH_CHECK();
  }
  int h = 0;
  DGS_HIP(hipMemcpyAsync(&h, ovf.p, sizeof(int), hipMemcpyDeviceToHost, st));
  DGS_HIP(hipStreamSynchronize(st));
  DGS_CHECK(h == 0, "cache hashmap: a probe sequence found no free slot");
}
}  // namespace

// _UpPower (hashmap.h:91-94): 1 << (uint32)(log2(key) + 1), a power of two above key
int64_t refmap_dir_size(int64_t total) {
  DGS_CHECK(total >= 1, "cache hashmap: no cached node (the reference requires a cache)");
  int64_t up = 1;
  while (up <= total) up <<= 1;
  DGS_CHECK(2 * up <= (int64_t(1) << 32), "cache hashmap: too many cached nodes");
  return 2 * up;
}

void refmap_build(const int64_t *const *lists, const int64_t *counts, const int *order,
                  int nlists, int id_bytes, int64_t dir, void *key, void *idx, void *dev,
                  hipStream_t st) {
  if (id_bytes == 8)
    build<int64_t>(lists, counts, order, nlists, dir, (int64_t *)key, (int64_t *)idx,
                   (int64_t *)dev, st);
  else if (id_bytes == 4)
    build<int32_t>(lists, counts, order, nlists, dir, (int32_t *)key, (int32_t *)idx,
                   (int32_t *)dev, st);
  else
    DGS_CHECK(false, "cache hashmap: ids are int32 or int64");
}

}  // namespace dgs
