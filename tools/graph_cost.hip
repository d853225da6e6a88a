// graph_cost.hip -- what a HIP graph would buy the synchronous sample call (round 5 probe).
//
// A sample call is a chain of 16 dependent kernel launches.  This measures, for a chain of N
// short kernels (each spins ~T us, stamping s_memrealtime at entry and exit):
//   (a) plain hipLaunchKernelGGL launches: host time to enqueue, wall to completion, and the
//       device-side gaps between consecutive kernels;
//   (b) the same chain captured once into a graph and replayed with hipGraphLaunch;
//   (c) (b) plus hipGraphExecKernelNodeSetParams on every node before each replay (the cost of
//       changing per-call arguments such as output pointers and launch seeds).
// Build: hipcc --offload-arch=gfx950 -O3 tools/graph_cost.hip -o tools/graph_cost
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

struct Args {
  unsigned long long *stamps;
  int idx;
  unsigned spin;  // device clock ticks (100 MHz) to spin
  int pad[8];     // a kernel argument block of realistic size
};

__global__ void k_step(Args a) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) a.stamps[2 * a.idx] = t0;
  unsigned long long t = t0;
  while (t - t0 < a.spin) t = __builtin_amdgcn_s_memrealtime();
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0)
    a.stamps[2 * a.idx + 1] = __builtin_amdgcn_s_memrealtime();
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int main(int argc, char **argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 16;
  const unsigned spin = argc > 2 ? (unsigned)atoi(argv[2]) : 400;  // 4 us
  const int reps = 200;
  const int blocks = 256;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  unsigned long long *stamps;
  CK(hipMalloc(&stamps, sizeof(unsigned long long) * 2 * N));
  std::vector<unsigned long long> h(2 * N);
  auto launch_chain = [&](hipStream_t s) {
    for (int i = 0; i < N; ++i) {
      Args a{stamps, i, spin, {}};
      hipLaunchKernelGGL(k_step, dim3(blocks), dim3(256), 0, s, a);
    }
  };
  auto gaps = [&](double *gap_sum, double *span) {
    CK(hipMemcpy(h.data(), stamps, sizeof(unsigned long long) * 2 * N, hipMemcpyDeviceToHost));
    double g = 0;
    for (int i = 1; i < N; ++i) g += (double)(h[2 * i] - h[2 * i - 1]) / 100.0;
    *gap_sum += g;
    *span += (double)(h[2 * N - 1] - h[0]) / 100.0;
  };
  // warm up
  for (int r = 0; r < 20; ++r) launch_chain(st);
  CK(hipStreamSynchronize(st));

  // (a) plain launches
  double host_a = 0, wall_a = 0, gap_a = 0, span_a = 0;
  std::vector<double> wa;
  for (int r = 0; r < reps; ++r) {
    const double t0 = now_us();
    launch_chain(st);
    const double t1 = now_us();
    CK(hipStreamSynchronize(st));
    const double t2 = now_us();
    host_a += t1 - t0;
    wall_a += t2 - t0;
    wa.push_back(t2 - t0);
    gaps(&gap_a, &span_a);
  }

  // (b) captured graph
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  launch_chain(st);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int r = 0; r < 20; ++r) CK(hipGraphLaunch(ge, st));
  CK(hipStreamSynchronize(st));
  double host_b = 0, wall_b = 0, gap_b = 0, span_b = 0;
  std::vector<double> wb;
  for (int r = 0; r < reps; ++r) {
    const double t0 = now_us();
    CK(hipGraphLaunch(ge, st));
    const double t1 = now_us();
    CK(hipStreamSynchronize(st));
    const double t2 = now_us();
    host_b += t1 - t0;
    wall_b += t2 - t0;
    wb.push_back(t2 - t0);
    gaps(&gap_b, &span_b);
  }

  // (c) per-node parameter updates before each replay
  size_t nn = 0;
  CK(hipGraphGetNodes(g, nullptr, &nn));
  std::vector<hipGraphNode_t> nodes(nn);
  CK(hipGraphGetNodes(g, nodes.data(), &nn));
  std::vector<hipKernelNodeParams> kp(nn);
  for (size_t i = 0; i < nn; ++i) CK(hipGraphKernelNodeGetParams(nodes[i], &kp[i]));
  std::vector<Args> args(nn);
  std::vector<void *> argp(nn);
  double host_c = 0, upd_c = 0, wall_c = 0, gap_c = 0, span_c = 0;
  std::vector<double> wc;
  for (int r = 0; r < reps; ++r) {
    const double t0 = now_us();
    for (size_t i = 0; i < nn; ++i) {
      // node order from hipGraphGetNodes is not guaranteed to be launch order: keep each
      // node's own index (read back from its captured argument)
      const Args *old = reinterpret_cast<const Args *>(kp[i].kernelParams[0]);
      args[i] = *old;
      args[i].pad[0] = r;
      argp[i] = &args[i];
      hipKernelNodeParams p = kp[i];
      p.kernelParams = &argp[i];
      CK(hipGraphExecKernelNodeSetParams(ge, nodes[i], &p));
    }
    const double tu = now_us();
    CK(hipGraphLaunch(ge, st));
    const double t1 = now_us();
    CK(hipStreamSynchronize(st));
    const double t2 = now_us();
    upd_c += tu - t0;
    host_c += t1 - t0;
    wall_c += t2 - t0;
    wc.push_back(t2 - t0);
    gaps(&gap_c, &span_c);
  }
  // (d) a fresh capture of the chain every call, folded into the instantiated graph with
  // hipGraphExecUpdate (new arguments without knowing the node layout), then a replay
  double host_d = 0, cap_d = 0, wall_d = 0, gap_d = 0, span_d = 0;
  std::vector<double> wd;
  int upd_fail = 0;
  for (int r = 0; r < reps; ++r) {
    const double t0 = now_us();
    hipGraph_t g2;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    launch_chain(st);
    CK(hipStreamEndCapture(st, &g2));
    const double tc = now_us();
    hipGraphExecUpdateResult ur;
    hipGraphNode_t en = nullptr;
    if (hipGraphExecUpdate(ge, g2, &en, &ur) != hipSuccess) ++upd_fail;
    CK(hipGraphLaunch(ge, st));
    const double t1 = now_us();
    CK(hipStreamSynchronize(st));
    const double t2 = now_us();
    CK(hipGraphDestroy(g2));
    cap_d += tc - t0;
    host_d += t1 - t0;
    wall_d += t2 - t0;
    wd.push_back(t2 - t0);
    gaps(&gap_d, &span_d);
  }
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  printf("chain of %d kernels, %u ticks spin each, %d reps (means; wall also median)\n", N, spin,
         reps);
  printf("(a) launches     : host %.1f us, wall %.1f us (median %.1f), device span %.1f us, "
         "sum of gaps %.1f us\n",
         host_a / reps, wall_a / reps, med(wa), span_a / reps, gap_a / reps);
  printf("(b) graph        : host %.1f us, wall %.1f us (median %.1f), device span %.1f us, "
         "sum of gaps %.1f us\n",
         host_b / reps, wall_b / reps, med(wb), span_b / reps, gap_b / reps);
  printf("(c) graph+update : host %.1f us (updates %.1f), wall %.1f us (median %.1f), device span "
         "%.1f us, sum of gaps %.1f us\n",
         host_c / reps, upd_c / reps, wall_c / reps, med(wc), span_c / reps, gap_c / reps);
  printf("(d) capture+update: host %.1f us (capture %.1f), wall %.1f us (median %.1f), device "
         "span %.1f us, sum of gaps %.1f us, update failures %d\n",
         host_d / reps, cap_d / reps, wall_d / reps, med(wd), span_d / reps, gap_d / reps,
         upd_fail);
  return 0;
}
