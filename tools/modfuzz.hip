// Exactness check of the sampler's fast modulo forms (csrc/dgs_mod.cuh) against x % d on the
// GPU, with the definitions the sampler compiles:
//   mod_mid<false>  every (x, d), x < 2^32, 1 <= d <= kModMidMax
//   mod_mid<true>   every (x, d), x < 2^32, 257 <= d <= kModMidMax
//   mod_big<false>  every x for ~1K divisors in [2^12, 2^30) (range ends, powers of two +-1, a
//                   dense run above the threshold) + 2^34 random (x, d) pairs biased to x near
//                   multiples of d
//   mod_big<true>   the same with d < 2^24
//   hipcc --offload-arch=gfx950 -O3 -I dist-gnn_amd/csrc -o /tmp/modfuzz tools/modfuzz.hip
//   /tmp/modfuzz [mid|big|all]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "dgs_mod.cuh"

using dgs::kModBigMin;
using dgs::kModMidMax;

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e) {                                                               \
      printf("hip error %s at %d\n", hipGetErrorString(e), __LINE__);      \
      exit(2);                                                             \
    }                                                                      \
  } while (0)

enum Form { kMidGeneric = 0, kMidU24 = 1, kBigGeneric = 2, kBigU24 = 3 };

template <int F>
__device__ __forceinline__ uint32_t fmod_of(uint32_t x, uint32_t d) {
  if (F == kMidGeneric) return dgs::mod_mid<false>(x, d);
  if (F == kMidU24) return dgs::mod_mid<true>(x, d);
  if (F == kBigGeneric) return dgs::mod_big<false>(x, d);
  return dgs::mod_big<true>(x, d);
}

__device__ __forceinline__ uint4 mix(uint64_t i, uint32_t s) {
  uint4 c = make_uint4((uint32_t)i, (uint32_t)(i >> 32), s, 0x9e3779b9u);
  uint2 k = make_uint2(s * 0x85ebca6bu, 0xc2b2ae35u);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    c = make_uint4((uint32_t)(p1 >> 32) ^ c.y ^ k.x, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k.y,
                   (uint32_t)p0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

// every x for the divisors ds[blockIdx.y]
template <int F>
__global__ void k_exhaustive(const uint32_t *ds, unsigned long long *bad) {
  const uint32_t d = ds[blockIdx.y];
  unsigned long long b = 0;
  for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < (1ull << 32);
       x += (uint64_t)gridDim.x * blockDim.x)
    b += fmod_of<F>((uint32_t)x, d) != (uint32_t)x % d;
  if (b) atomicAdd(bad, b);
}

template <int F>
__global__ void k_random(uint64_t n, uint32_t seed, uint32_t dmax, unsigned long long *bad) {
  unsigned long long b = 0;
  const uint32_t span = dmax - kModBigMin;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 r = mix(i, seed);
    uint32_t d, x = r.x;
    switch (i & 7) {
      case 0: d = kModBigMin + r.y % 100000u; break;
      case 1: d = kModBigMin + r.y % span; break;
      case 2: d = kModBigMin + (r.y & 0xfffu); break;
      case 3:  // x = m*d - 1, m*d, m*d + 1 for large m
        d = kModBigMin + r.y % 65536u;
        x = (uint32_t)((uint64_t)(r.z % (0xffffffffu / d)) * d + (r.w % 3) - 1);
        break;
      case 4: d = kModBigMin + r.y % span; x = 0xffffffffu - (r.z & 1023u); break;
      case 5: d = kModBigMin + (r.y & 0x3ffu); x = 0xffffffffu - r.z % (4 * d); break;
      case 6: d = kModBigMin + r.y % 1000000u; x = (x / d) * d + d - 1; break;
      default: d = kModBigMin + r.y % 400000u; x = (x / d) * d; break;
    }
    b += fmod_of<F>(x, d) != x % d;
  }
  if (b) atomicAdd(bad, b);
}

template <int F>
static unsigned long long run_exhaustive(const std::vector<uint32_t> &ds, const char *name) {
  uint32_t *dd = nullptr;
  unsigned long long *bad = nullptr, hb = 0;
  CK(hipMalloc(&dd, sizeof(uint32_t) * ds.size()));
  CK(hipMalloc(&bad, sizeof(unsigned long long)));
  CK(hipMemset(bad, 0, sizeof(unsigned long long)));
  CK(hipMemcpy(dd, ds.data(), sizeof(uint32_t) * ds.size(), hipMemcpyHostToDevice));
  // 16 divisors (2^36 pairs) per launch, so no single launch runs long
  for (size_t i = 0; i < ds.size(); i += 16) {
    const int nd = (int)(ds.size() - i < 16 ? ds.size() - i : 16);
    hipLaunchKernelGGL(k_exhaustive<F>, dim3(4096, nd), dim3(256), 0, 0, dd + i, bad);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    if ((i / 16) % 128 == 127) {
      printf("  %s: %zu / %zu divisors\n", name, i + nd, ds.size());
      fflush(stdout);
    }
  }
  CK(hipMemcpy(&hb, bad, sizeof(hb), hipMemcpyDeviceToHost));
  CK(hipFree(dd));
  CK(hipFree(bad));
  printf("%s exhaustive: %zu divisors x 2^32, mismatches %llu\n", name, ds.size(), hb);
  fflush(stdout);
  return hb;
}

template <int F>
static unsigned long long run_random(uint32_t dmax, const char *name) {
  unsigned long long *bad = nullptr, hb = 0;
  CK(hipMalloc(&bad, sizeof(unsigned long long)));
  CK(hipMemset(bad, 0, sizeof(unsigned long long)));
  const uint64_t n = 1ull << 34;
  for (uint32_t s = 0; s < 16; ++s) {
    hipLaunchKernelGGL(k_random<F>, dim3(8192), dim3(256), 0, 0, n / 16, s + 1, dmax, bad);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
  }
  CK(hipMemcpy(&hb, bad, sizeof(hb), hipMemcpyDeviceToHost));
  CK(hipFree(bad));
  printf("%s random: 2^34 pairs, mismatches %llu\n", name, hb);
  fflush(stdout);
  return hb;
}

static std::vector<uint32_t> big_divisors(uint32_t dmax) {
  std::vector<uint32_t> ds;
  for (uint32_t d = kModBigMin; d < kModBigMin + 512; ++d) ds.push_back(d);
  for (int e = 12; e <= 30; ++e)
    for (int o = -3; o <= 3; ++o) {
      const int64_t d = (int64_t(1) << e) + o;
      if (d >= kModBigMin && d < (int64_t)dmax) ds.push_back((uint32_t)d);
    }
  for (uint32_t d = dmax - 64; d < dmax; ++d) ds.push_back(d);
  for (uint32_t i = 0; i < 256; ++i)
    ds.push_back(kModBigMin + (uint32_t)((i * 2654435761u) % (dmax - kModBigMin)));
  return ds;
}

int main(int argc, char **argv) {
  const char *what = argc > 1 ? argv[1] : "all";
  const bool mid = !strcmp(what, "mid") || !strcmp(what, "all");
  const bool big = !strcmp(what, "big") || !strcmp(what, "all");
  unsigned long long bad = 0;
  if (mid) {
    std::vector<uint32_t> all, u24;
    for (uint32_t d = 1; d <= kModMidMax; ++d) {
      all.push_back(d);
      if (d >= 257) u24.push_back(d);
    }
    bad += run_exhaustive<kMidU24>(u24, "mod_mid<u24>");
    bad += run_exhaustive<kMidGeneric>(all, "mod_mid");
  }
  if (big) {
    bad += run_exhaustive<kBigU24>(big_divisors(1u << 24), "mod_big<u24>");
    bad += run_random<kBigU24>(1u << 24, "mod_big<u24>");
    bad += run_exhaustive<kBigGeneric>(big_divisors(1u << 30), "mod_big");
    bad += run_random<kBigGeneric>(1u << 30, "mod_big");
  }
  printf("total mismatches %llu\n", bad);
  return bad ? 1 : 0;
}
