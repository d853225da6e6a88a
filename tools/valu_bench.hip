// valu_bench.hip -- issue-cost microbenchmark for the hub kernels' inner loops (gfx950).
// Measures, on every CU with W waves per SIMD, the throughput of:
//   philox   : one Philox4x32-10 block per iteration (as in dgs_common.h: 20 v_mad_u64_u32)
//   mad64    : 20 v_mad_u64_u32 per iteration (the multiply alone)
//   modbig   : 8 mod_big<true> modulos per iteration (the uniform reservoir's draw test)
//   fma      : 20 v_fma_f32 per iteration (reference: full-rate VALU)
// so the hub kernels' VALU floor can be priced.
//   hipcc -O3 --offload-arch=gfx950 -I../dist-gnn_amd/csrc valu_bench.hip -o valu_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "dgs_common.h"
#include "dgs_mod.cuh"

using namespace dgs;

constexpr int kIters = 4096;

__global__ __launch_bounds__(256) void k_philox(uint32_t seed, uint32_t *out) {
  const uint2 kk = make_uint2(seed, seed ^ 0x1234567u);
  uint32_t acc = 0;
  uint32_t t = threadIdx.x + blockIdx.x * 256;
  for (int i = 0; i < kIters; ++i) {
    const uint4 o = philox4x32_10(make_uint4((uint32_t)i, 0u, t, 0u), kk);
    acc ^= o.x ^ o.y ^ o.z ^ o.w;
  }
  if (acc == 0x9e3779b9u) out[t] = acc;
}

__global__ __launch_bounds__(256) void k_mad64(uint32_t seed, uint32_t *out) {
  uint32_t a = seed + threadIdx.x, b = seed ^ threadIdx.x;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      const uint64_t p0 = (uint64_t)0xD2511F53u * a;
      const uint64_t p1 = (uint64_t)0xCD9E8D57u * b;
      a = (uint32_t)(p0 >> 32) ^ (uint32_t)p1 ^ (uint32_t)i;
      b = (uint32_t)(p1 >> 32) ^ (uint32_t)p0;
    }
  }
  if ((a ^ b) == 0x9e3779b9u) out[threadIdx.x] = a;
}

__global__ __launch_bounds__(256) void k_modbig(uint32_t seed, uint32_t *out) {
  uint32_t x = seed * (threadIdx.x + 1), acc = 0;
  const uint32_t d0 = 5000 + threadIdx.x;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      acc += mod_big<true>(x, d0 + 128u * w + (uint32_t)i);
      x = x * 1664525u + 1013904223u;
    }
  }
  if (acc == 0x9e3779b9u) out[threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_fma(float seed, float *out) {
  float a = seed + threadIdx.x, b = seed - threadIdx.x, c = 1.0001f;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      a = __builtin_fmaf(a, c, b);
      b = __builtin_fmaf(b, c, a);
    }
  }
  if (a == 123.0f) out[threadIdx.x] = b;
}

template <typename F>
float time_it(F launch) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  launch();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int r = 0; r < 5; ++r) launch();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t *out = nullptr;
  (void)hipMalloc(&out, sizeof(uint32_t) << 24);
  for (int wps : {1, 2, 4, 8}) {
    const int blocks = cus * wps;  // 256-thread blocks: 4 waves = one per SIMD
    const double waves = (double)blocks * 4;
    const double lanes = waves * 64;
    const double slots = cus * 4 * 2.4e9 / 2;  // wave64 VALU issue slots/s at 2 cycles each
    float ms = time_it([&] { hipLaunchKernelGGL(k_philox, dim3(blocks), dim3(256), 0, 0, 7u, out); });
    const double blk_s = lanes * kIters / (ms * 1e-3);
    printf("waves/SIMD=%d philox: %.3f ms, %.1f G blocks/s = %.1f G draws/s\n", wps, ms,
           blk_s / 1e9, 4 * blk_s / 1e9);
    ms = time_it([&] { hipLaunchKernelGGL(k_mad64, dim3(blocks), dim3(256), 0, 0, 7u, out); });
    printf("waves/SIMD=%d mad64: %.3f ms, %.2f T lane-mad/s, %.2f full-rate slots each\n", wps,
           ms, lanes * kIters * 20 / (ms * 1e-3) / 1e12,
           slots / (waves * kIters * 20 / (ms * 1e-3)));
    ms = time_it([&] { hipLaunchKernelGGL(k_modbig, dim3(blocks), dim3(256), 0, 0, 7u, out); });
    printf("waves/SIMD=%d modbig: %.3f ms, %.1f G lane-mods/s, %.2f slots each\n", wps, ms,
           lanes * kIters * 8 / (ms * 1e-3) / 1e9, slots / (waves * kIters * 8 / (ms * 1e-3)));
    ms = time_it([&] {
      hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, 1.5f, (float *)out);
    });
    printf("waves/SIMD=%d fma: %.3f ms, %.2f T lane-fma/s, %.2f slots each\n", wps, ms,
           lanes * kIters * 20 / (ms * 1e-3) / 1e12, slots / (waves * kIters * 20 / (ms * 1e-3)));
  }
  (void)hipFree(out);
  return 0;
}
