// latency_probe.hip -- the per-iteration floor of a latency-bound walk on this MI355X (diagnostic
// for the k_walk small-batch latency).  Every lane chases `steps` dependent
// random 64-B lines (four 16-B loads, the k_walk probe) in a table of `mb` MiB; optional extras
// per step: a 12-B store per lane (a staged pair), a returning atomic on one hot counter per
// wave every 4 steps (a chunk reservation).  Timed with HIP events, reported as
// (t(64 steps) - t(8 steps)) / 56 = the cost of one dependent step, and t(0) = launch + drain.
// Build: hipcc --offload-arch=gfx950 -O3 tools/latency_probe.hip -o build/latency_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33;
  return k;
}

__global__ __launch_bounds__(256) void k_chase(const uint4* __restrict__ tab, uint64_t nlines, int steps,
                                               int mode, uint3* out, uint32_t* ctr, uint32_t* sink) {
  const uint64_t gid = blockIdx.x * 256ull + threadIdx.x;
  uint64_t s = mix(gid + 1);
  uint32_t acc = 0, base = 0;
  for (int r = 0; r < steps; ++r) {
    const uint4* q = tab + (s % nlines) * 4;
    const uint4 a = q[0], b = q[1], c = q[2], d = q[3];
    const uint32_t x = a.x ^ b.y ^ c.z ^ d.w;
    acc += x;
    s = mix(s + x + 1);
    if (mode & 1) out[(uint64_t)r * gridDim.x * 256 + gid] = make_uint3((uint32_t)gid, x, r);
    if ((mode & 2) && (r & 3) == 0) {
      uint32_t v = 0;
      if ((threadIdx.x & 63) == 0) v = atomicAdd(ctr, 256u);
      base += __builtin_amdgcn_readfirstlane(v);
    }
  }
  if (acc == 0x12345678u) sink[0] = acc + base;
}

int main(int argc, char** argv) {
  const int waves_list[] = {1, 16, 1564, 4096};
  const uint64_t mbs[] = {8, 4096};
  uint4* tab;
  const uint64_t maxb = 4096ull << 20;
  CHK(hipMalloc(&tab, maxb));
  CHK(hipMemset(tab, 3, maxb));
  uint3* out;
  const size_t out_bytes = (size_t)4096 * 64 * 64 * sizeof(uint3);
  CHK(hipMalloc(&out, out_bytes));
  uint32_t *ctr, *sink;
  CHK(hipMalloc(&ctr, 256));
  CHK(hipMalloc(&sink, 256));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  auto run = [&](uint64_t mb, int waves, int steps, int mode) {
    const int blocks = (waves * 64 + 255) / 256;
    float best = 1e9f;
    for (int rep = 0; rep < 5; ++rep) {
      CHK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_chase, dim3(blocks), dim3(waves < 4 ? waves * 64 : 256), 0, 0, tab,
                         (mb << 20) / 64, steps, mode, out, ctr, sink);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    return best * 1000.0f;
  };
  printf("launch+drain (0 steps, 1 wave): %.2f us\n", run(8, 1, 0, 0));
  for (uint64_t mb : mbs)
    for (int waves : waves_list)
      for (int mode = 0; mode < 4; ++mode) {
        const float t8 = run(mb, waves, 8, mode), t64 = run(mb, waves, 64, mode);
        printf("table %5llu MiB waves %5d mode %d (store %d atomic %d): 8 steps %7.2f us, 64 steps %7.2f us, per step %.3f us\n",
               (unsigned long long)mb, waves, mode, mode & 1, (mode >> 1) & 1, t8, t64, (t64 - t8) / 56.0f);
      }
  return 0;
}
