// Host cost of the HIP calls a loader step makes (diagnostics): median ns per call of
// hipGetDevice, hipEventRecord, hipStreamWaitEvent and an empty-kernel launch, alone and while a
// second thread launches on another stream (the sampler's launcher thread does that).
//   hipcc --offload-arch=gfx950 -O2 -o tools/hip_api_cost tools/hip_api_cost.hip -lpthread
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

__global__ void k_empty(int *p) {
  if (p && threadIdx.x == 1024) p[0] = 1;
}

#define CK(x)                                                       \
  do {                                                              \
    hipError_t e_ = (x);                                            \
    if (e_ != hipSuccess) {                                         \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));           \
      return 1;                                                     \
    }                                                               \
  } while (0)

using clk = std::chrono::steady_clock;

template <class F>
double med_ns(F f, int n) {
  std::vector<double> t(n);
  for (int i = 0; i < n; ++i) {
    auto a = clk::now();
    f();
    t[i] = std::chrono::duration<double, std::nano>(clk::now() - a).count();
  }
  std::sort(t.begin(), t.end());
  return t[n / 2];
}

int run(const char *tag, hipStream_t a, hipStream_t b, hipEvent_t ev) {
  const int n = 4000;
  int dev = 0;
  double g = med_ns([&] { (void)hipGetDevice(&dev); }, n);
  double r = med_ns([&] { (void)hipEventRecord(ev, a); }, n);
  double w = med_ns([&] { (void)hipStreamWaitEvent(b, ev, 0); }, n);
  double k = med_ns([&] { hipLaunchKernelGGL(k_empty, dim3(64), dim3(256), 0, b, nullptr); }, n);
  double k8 = med_ns([&] {
    hipLaunchKernelGGL(k_empty, dim3(64), dim3(256), 0, b, nullptr);
    hipLaunchKernelGGL(k_empty, dim3(64), dim3(256), 0, b, nullptr);
  }, n);
  CK(hipDeviceSynchronize());
  std::printf("%-28s getDevice %6.0f ns  eventRecord %6.0f ns  streamWaitEvent %6.0f ns  "
              "launch %6.0f ns  2 launches %6.0f ns\n", tag, g, r, w, k, k8);
  return 0;
}

int main() {
  hipStream_t a, b, c;
  hipEvent_t ev;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, a, nullptr);
  CK(hipDeviceSynchronize());
  if (run("alone", a, b, ev)) return 1;
  std::atomic<bool> stop{false};
  std::thread other([&] {
    while (!stop.load(std::memory_order_relaxed)) {
      for (int i = 0; i < 16; ++i) hipLaunchKernelGGL(k_empty, dim3(64), dim3(256), 0, c, nullptr);
      (void)hipStreamSynchronize(c);
    }
  });
  int rc = run("with a launching thread", a, b, ev);
  stop = true;
  other.join();
  CK(hipDeviceSynchronize());
  return rc;
}
