// launch_cost.hip -- host cost of one kernel launch through each HIP launch entry point (round 6
// probe for the synchronous sample call, whose 16 launches take ~48 us of host time).
//
// A chain of N launches of a short kernel with a realistic argument block (256 B, the size of
// the sampler's PrepArgs / UniformArgs) on one stream, through:
//   (a) hipLaunchKernelGGL (the library's path: hipLaunchKernel with an argument array)
//   (b) hipModuleLaunchKernel on the hipFunction_t from hipGetFuncBySymbol, argument array
//   (c) hipModuleLaunchKernel with the argument block passed whole (HIP_LAUNCH_PARAM_BUFFER_*)
//   (d) hipExtLaunchKernel
// Reports host microseconds per launch (mean over reps, after warm-up) and the wall time of the
// chain to completion.  Build: hipcc --offload-arch=gfx950 -O3 tools/launch_cost.hip -o ...
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

struct Args {
  unsigned long long *out;
  int idx;
  int pad[61];  // 256 B in all
};
static_assert(sizeof(Args) == 256, "256-B argument block");

__global__ void k_short(Args a) {
  if (threadIdx.x == 0 && blockIdx.x == 0) a.out[a.idx & 15] += (unsigned long long)a.pad[3];
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int main(int argc, char **argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 16;
  const int reps = argc > 2 ? atoi(argv[2]) : 300;
  const unsigned blocks = 64;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  unsigned long long *out;
  CK(hipMalloc(&out, 16 * sizeof(unsigned long long)));
  CK(hipMemset(out, 0, 16 * sizeof(unsigned long long)));
  hipFunction_t fn;
  CK(hipGetFuncBySymbol(&fn, reinterpret_cast<const void *>(&k_short)));

  auto run = [&](int mode, Args &a) {
    switch (mode) {
      case 0:
        hipLaunchKernelGGL(k_short, dim3(blocks), dim3(256), 0, st, a);
        break;
      case 1: {
        void *params[] = {&a};
        CK(hipModuleLaunchKernel(fn, blocks, 1, 1, 256, 1, 1, 0, st, params, nullptr));
        break;
      }
      case 2: {
        size_t sz = sizeof(a);
        void *extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                         HIP_LAUNCH_PARAM_END};
        CK(hipModuleLaunchKernel(fn, blocks, 1, 1, 256, 1, 1, 0, st, nullptr, extra));
        break;
      }
      case 3: {
        void *params[] = {&a};
        CK(hipExtLaunchKernel(reinterpret_cast<const void *>(&k_short), dim3(blocks), dim3(256),
                              params, 0, st, nullptr, nullptr, 0));
        break;
      }
    }
  };
  const char *names[] = {"hipLaunchKernelGGL", "hipModuleLaunchKernel (args)",
                         "hipModuleLaunchKernel (buffer)", "hipExtLaunchKernel"};
  printf("chain of %d launches, 256-B arguments, %u workgroups, %d reps\n", N, blocks, reps);
  for (int round = 0; round < 2; ++round) {
    for (int mode = 0; mode < 4; ++mode) {
      Args a{};
      a.out = out;
      a.pad[3] = 1;
      for (int r = 0; r < 20; ++r)
        for (int i = 0; i < N; ++i) {
          a.idx = i;
          run(mode, a);
        }
      CK(hipStreamSynchronize(st));
      std::vector<double> host, wall;
      for (int r = 0; r < reps; ++r) {
        const double t0 = now_us();
        for (int i = 0; i < N; ++i) {
          a.idx = i;
          run(mode, a);
        }
        const double t1 = now_us();
        CK(hipStreamSynchronize(st));
        const double t2 = now_us();
        host.push_back((t1 - t0) / N);
        wall.push_back(t2 - t0);
      }
      CK(hipGetLastError());
      std::sort(host.begin(), host.end());
      std::sort(wall.begin(), wall.end());
      printf("round %d  %-32s host %.2f us/launch (p10 %.2f, p90 %.2f), chain wall median %.1f us\n",
             round, names[mode], host[reps / 2], host[reps / 10], host[reps * 9 / 10],
             wall[reps / 2]);
    }
  }
  unsigned long long h[16];
  CK(hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost));
  printf("check %llu\n", h[0]);
  return 0;
}
