// Checks the half-wave lane moves of dist-gnn_amd/csrc/dgs_lane.cuh against HIP's __shfl forms
// on the GPU: every helper, with the whole wave active and with only one half active.
//   hipcc --offload-arch=gfx950 -O3 -I dist-gnn_amd/csrc tools/lane_ops_test.hip -o tools/lane_ops_test
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "dgs_lane.cuh"

using namespace dgs;

#define CHECK(x)                                          \
  do {                                                    \
    if ((x) != hipSuccess) {                              \
      printf("%s failed\n", #x);                          \
      exit(2);                                            \
    }                                                     \
  } while (0)

// out[t * 64 + lane]: mismatch flags of test t (0 = equal)
__global__ void k_lane_test(const int32_t *in, int32_t *bad, int mode, int q) {
  const int lane = threadIdx.x;
  const int32_t x = in[blockIdx.x * 64 + lane];
  const bool active = mode == 0 || (mode == 1 && lane < 32) || (mode == 2 && lane >= 32);
  if (!active) return;
  int32_t *b = bad + (size_t)blockIdx.x * 9 * 64;
  const int l = lane & 31;
  // every helper runs with the whole half active (as in the kernels): a DPP move reading a lane
  // whose exec bit is clear does not see its value
  const int32_t up1 = lane_up1_32(x), up1_ref = __shfl_up(x, 1, 32);
  const int32_t wshr = dpp_keep<0x138>(x, x);
  const int32_t rdl = (threadIdx.x & 32) ? __builtin_amdgcn_readlane(x, 47)
                                         : __builtin_amdgcn_readlane(x, 15);
  const int32_t up1_rl = (threadIdx.x & 31) == 16 ? rdl : dpp_keep<0x111>(x, x);
  b[0 * 64 + lane] = lane_xor32<1>(x) != __shfl_xor(x, 1, 32);
  b[1 * 64 + lane] = lane_xor32<2>(x) != __shfl_xor(x, 2, 32);
  b[2 * 64 + lane] = lane_xor32<4>(x) != __shfl_xor(x, 4, 32);
  b[3 * 64 + lane] = lane_xor32<8>(x) != __shfl_xor(x, 8, 32);
  b[4 * 64 + lane] = lane_xor32<16>(x) != __shfl_xor(x, 16, 32);
  b[5 * 64 + lane] = lane_rev32(x) != __shfl(x, 31 - l, 32);
  b[6 * 64 + lane] = l > 0 && up1 != up1_ref;
  b[7 * 64 + lane] = half_bcast(x, q) != __shfl(x, q, 32);
  // (not used) the wave-wide DPP shift wave_shr:1 and the readlane patch, lanes 1-31 of each half
  b[8 * 64 + lane] = (l > 0 && wshr != up1_ref) | ((l > 0 && up1_rl != up1_ref) << 1);
}

int main() {
  const int nb = 64;
  int32_t *h = (int32_t *)malloc(sizeof(int32_t) * nb * 64);
  srand(7);
  for (int i = 0; i < nb * 64; ++i) h[i] = rand() ^ (rand() << 16);
  int32_t *din, *dbad;
  CHECK(hipMalloc(&din, sizeof(int32_t) * nb * 64));
  CHECK(hipMalloc(&dbad, sizeof(int32_t) * nb * 9 * 64));
  CHECK(hipMemcpy(din, h, sizeof(int32_t) * nb * 64, hipMemcpyHostToDevice));
  int32_t *hb = (int32_t *)malloc(sizeof(int32_t) * nb * 9 * 64);
  const char *names[9] = {"xor1", "xor2", "xor4", "xor8", "xor16", "rev32", "up1", "bcast",
                          "(wave_shr1)"};
  int total = 0;
  for (int mode = 0; mode < 3; ++mode) {
    for (int q = 0; q < 32; q += 13) {
      CHECK(hipMemset(dbad, 0, sizeof(int32_t) * nb * 9 * 64));
      hipLaunchKernelGGL(k_lane_test, dim3(nb), dim3(64), 0, 0, din, dbad, mode, q);
      if (hipDeviceSynchronize() != hipSuccess) {
        printf("kernel failed\n");
        return 2;
      }
      CHECK(hipMemcpy(hb, dbad, sizeof(int32_t) * nb * 9 * 64, hipMemcpyDeviceToHost));
      for (int t = 0; t < 9; ++t) {
        int n = 0, first = -1;
        for (int blk = 0; blk < nb; ++blk)
          for (int lane = 0; lane < 64; ++lane)
            if (hb[(blk * 9 + t) * 64 + lane]) {
              ++n;
              if (first < 0) first = lane;
            }
        if (n) printf("mode %d q %d %s: %d mismatches (first lane %d)\n", mode, q, names[t], n, first);
        if (t < 8) total += n;
      }
    }
  }
  printf("lane ops: %s (%d mismatches)\n", total ? "FAIL" : "ok", total);
  return total ? 1 : 0;
}
