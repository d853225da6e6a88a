// Exactness check of the sampler's fast modulo (csrc/sample.hip mod_big) against x % d on the
// GPU: every x for ~1K divisors (range ends, powers of two +-1, a dense run above the
// threshold) and 2^34 random (x, d) pairs biased to x near multiples of d.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/modfuzz tools/modfuzz.hip && /tmp/modfuzz
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e) {                                                               \
      printf("hip error %s at %d\n", hipGetErrorString(e), __LINE__);      \
      exit(2);                                                             \
    }                                                                      \
  } while (0)

constexpr uint32_t kMin = 4096;

// the sampler's definition (keep in sync with csrc/sample.hip)
__device__ __forceinline__ uint32_t mod_big(uint32_t x, uint32_t d) {
  const float rcp = __builtin_amdgcn_rcpf((float)d);
  const uint32_t q = (uint32_t)(int32_t)__builtin_fmaf((float)x, rcp, -0.5f);
  const uint32_t r = x - q * d;
  return r >= d ? r - d : r;
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

__global__ void k_exhaustive(const uint32_t *ds, int nd, unsigned long long *bad) {
  const uint32_t d = ds[blockIdx.y];
  unsigned long long b = 0;
  for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < (1ull << 32);
       x += (uint64_t)gridDim.x * blockDim.x)
    b += mod_big((uint32_t)x, d) != (uint32_t)x % d;
  if (b) atomicAdd(bad, b);
}

__global__ void k_random(uint64_t n, uint32_t seed, unsigned long long *bad) {
  unsigned long long b = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 r = mix(i, seed);
    uint32_t d, x = r.x;
    switch (i & 7) {
      case 0: d = kMin + r.y % 100000u; break;
      case 1: d = kMin + r.y % ((1u << 30) - kMin); break;
      case 2: d = kMin + (r.y & 0xfffu); break;
      case 3:  // x = m*d - 1, m*d, m*d + 1 for large m
        d = kMin + r.y % 65536u;
        x = (uint32_t)((uint64_t)(r.z % (0xffffffffu / d)) * d + (r.w % 3) - 1);
        break;
      case 4: d = kMin + r.y % ((1u << 30) - kMin); x = 0xffffffffu - (r.z & 1023u); break;
      case 5: d = kMin + (r.y & 0x3ffu); x = 0xffffffffu - r.z % (4 * d); break;
      case 6: d = kMin + r.y % 1000000u; x = (x / d) * d + d - 1; break;
      default: d = kMin + r.y % 400000u; x = (x / d) * d; break;
    }
    b += mod_big(x, d) != x % d;
  }
  if (b) atomicAdd(bad, b);
}

int main() {
  std::vector<uint32_t> ds;
  for (uint32_t d = kMin; d < kMin + 512; ++d) ds.push_back(d);
  for (int e = 12; e <= 30; ++e)
    for (int o = -3; o <= 3; ++o) {
      const int64_t d = (int64_t(1) << e) + o;
      if (d >= kMin && d < (int64_t(1) << 30)) ds.push_back((uint32_t)d);
    }
  for (uint32_t d = (1u << 30) - 64; d < (1u << 30); ++d) ds.push_back(d);
  for (uint32_t i = 0; i < 256; ++i) ds.push_back(kMin + (uint32_t)((i * 2654435761u) % ((1u << 30) - kMin)));
  uint32_t *dd = nullptr;
  unsigned long long *bad = nullptr, hb[2] = {0, 0};
  CK(hipMalloc(&dd, sizeof(uint32_t) * ds.size()));
  CK(hipMalloc(&bad, 2 * sizeof(unsigned long long)));
  CK(hipMemset(bad, 0, 2 * sizeof(unsigned long long)));
  CK(hipMemcpy(dd, ds.data(), sizeof(uint32_t) * ds.size(), hipMemcpyHostToDevice));
  // one y-slice per divisor, every x; chunked so no single launch runs long
  for (size_t i = 0; i < ds.size(); i += 64) {
    const int nd = (int)(ds.size() - i < 64 ? ds.size() - i : 64);
    hipLaunchKernelGGL(k_exhaustive, dim3(2048, nd), dim3(256), 0, 0, dd + i, nd, bad);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
  }
  const uint64_t n = 1ull << 34;
  for (uint32_t s = 0; s < 16; ++s) {
    hipLaunchKernelGGL(k_random, dim3(8192), dim3(256), 0, 0, n / 16, s + 1, bad + 1);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
  }
  CK(hipMemcpy(hb, bad, sizeof(hb), hipMemcpyDeviceToHost));
  printf("divisors exhaustive: %zu x 2^32 pairs, mismatches %llu; random: 2^34 pairs, mismatches %llu\n",
         ds.size(), hb[0], hb[1]);
  return hb[0] || hb[1] ? 1 : 0;
}
