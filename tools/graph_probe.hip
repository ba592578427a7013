// Launch-path probe for small windows: what four dependent launches cost from the host's call to
// the stream's completion, launched one by one or as one HIP graph (captured once; replayed as
// is, or with its kernel nodes' arguments updated before each replay, as per-window arguments
// would need).  The kernels are as small as a 16-topic window's: one block each, a few stores.
//
//   hipcc --offload-arch=gfx950 -O3 tools/graph_probe.hip -o graph_probe && ./graph_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

// each kernel reads the previous one's word and writes its own (a dependent chain)
__global__ void k_step(uint32_t* w, uint32_t i, uint32_t n) {
  if (threadIdx.x < n) w[i * 64 + 64 + threadIdx.x] = w[i * 64 + threadIdx.x] + i + 1;
}

using clk = std::chrono::steady_clock;

static double pct(std::vector<double> v, double p) {
  std::sort(v.begin(), v.end());
  return v[(size_t)(p * (v.size() - 1))];
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 2000;
  const int K = 4;
  uint32_t* w;
  CHK(hipMalloc(&w, 64 * 4 * (K + 1)));
  CHK(hipMemset(w, 0, 64 * 4 * (K + 1)));
  hipStream_t s;
  CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev;
  CHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));

  auto launches = [&](uint32_t n) {
    for (int i = 0; i < K; ++i) hipLaunchKernelGGL(k_step, dim3(1), dim3(64), 0, s, w, (uint32_t)i, n);
  };
  // one graph of the same four launches
  hipGraph_t g;
  hipGraphExec_t ge;
  CHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  launches(64);
  CHK(hipStreamEndCapture(s, &g));
  CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  size_t nn = 0;
  CHK(hipGraphGetNodes(g, nullptr, &nn));
  std::vector<hipGraphNode_t> nodes(nn);
  CHK(hipGraphGetNodes(g, nodes.data(), &nn));

  // a wait as the engine's: poll the event, then block
  auto wait = [&]() {
    while (hipEventQuery(ev) == hipErrorNotReady) {
    }
  };
  struct Row {
    const char* name;
    std::vector<double> call, done;
  };
  std::vector<Row> rows = {{"4 launches", {}, {}}, {"graph replay", {}, {}}, {"graph + set params", {}, {}}};
  for (int mode = 0; mode < 3; ++mode) {
    for (int r = 0; r < reps + 100; ++r) {
      const uint32_t n = 32 + (r & 31);
      auto t0 = clk::now();
      if (mode == 0) {
        launches(n);
      } else {
        if (mode == 2) {
          for (size_t j = 0; j < nn; ++j) {
            hipKernelNodeParams p;
            CHK(hipGraphKernelNodeGetParams(nodes[j], &p));
            uint32_t i = (uint32_t)j;
            void* args[] = {&w, &i, (void*)&n};
            p.kernelParams = args;
            CHK(hipGraphExecKernelNodeSetParams(ge, nodes[j], &p));
          }
        }
        CHK(hipGraphLaunch(ge, s));
      }
      CHK(hipEventRecord(ev, s));
      auto t1 = clk::now();
      wait();
      auto t2 = clk::now();
      if (r >= 100) {
        rows[mode].call.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        rows[mode].done.push_back(std::chrono::duration<double, std::micro>(t2 - t0).count());
      }
    }
  }
  printf("{\"reps\": %d, \"kernels\": %d, \"us\": {", reps, K);
  for (int m = 0; m < 3; ++m)
    printf("%s\"%s\": {\"call_p50\": %.1f, \"done_p10\": %.1f, \"done_p50\": %.1f, \"done_p90\": %.1f}",
           m ? ", " : "", rows[m].name, pct(rows[m].call, 0.5), pct(rows[m].done, 0.1),
           pct(rows[m].done, 0.5), pct(rows[m].done, 0.9));
  printf("}}\n");
  CHK(hipGraphExecDestroy(ge));
  CHK(hipGraphDestroy(g));
  CHK(hipFree(w));
  return 0;
}
