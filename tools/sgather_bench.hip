// sgather_bench.hip -- does the scalar memory path add random-line throughput beside the vector
// path?  The trie walk and the exact probe are bound by ~55-67 outstanding vector L1 misses per
// CU (profiles/r02/pmc_walk_cfg3_4m_issue_and_vmem.txt).  Scalar loads of a
// wave-uniform address go through the scalar cache to the L2 on a path of their own.  Each
// wave runs `rounds` dependent rounds; per round every lane issues `vdepth` random 64-B vector
// loads and the wave issues `sdepth` random 64-B scalar loads (16 dwords each), the next
// addresses depending on the loaded data.  Prints random lines/s for each mix.
// Build: hipcc --offload-arch=gfx950 -O3 tools/sgather_bench.hip -o tools/sgather_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33;
  return k;
}

typedef uint32_t Line __attribute__((ext_vector_type(16)));
typedef const __attribute__((address_space(4))) Line* CLine;

template <int VD, int SD>
__global__ __launch_bounds__(256) void k_mix(const uint4* __restrict__ tab, uint64_t nlines, int rounds,
                                             uint64_t* out) {
  const uint64_t gid = blockIdx.x * 256ull + threadIdx.x;
  uint64_t vs[VD > 0 ? VD : 1];
  for (int d = 0; d < VD; ++d) vs[d] = mix(gid * 8 + d + 1);
  // wave-uniform scalar states
  const uint32_t wave = __builtin_amdgcn_readfirstlane((uint32_t)(gid >> 6));
  uint64_t ss[SD > 0 ? SD : 1];
  for (int d = 0; d < SD; ++d) ss[d] = mix(((uint64_t)wave << 8) + d + 0x9999);
  uint32_t acc = 0, sacc = 0;
  for (int r = 0; r < rounds; ++r) {
    uint4 v[VD > 0 ? VD : 1][4];
#pragma unroll
    for (int d = 0; d < VD; ++d) {
      const uint64_t s = vs[d] % nlines;
#pragma unroll
      for (int w = 0; w < 4; ++w) v[d][w] = tab[s * 4 + w];
    }
    Line sl[SD > 0 ? SD : 1];
#pragma unroll
    for (int d = 0; d < SD; ++d) {
      const uint64_t s = ss[d] % nlines;
      const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)s);
      const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(s >> 32));
      CLine p = (CLine)(const void*)tab;
      sl[d] = p[((uint64_t)hi << 32) | lo];
    }
#pragma unroll
    for (int d = 0; d < VD; ++d) {
      uint32_t x = 0;
#pragma unroll
      for (int w = 0; w < 4; ++w) x ^= v[d][w].x ^ v[d][w].y ^ v[d][w].z ^ v[d][w].w;
      acc += x;
      vs[d] = mix(vs[d] + x + 1);
    }
#pragma unroll
    for (int d = 0; d < SD; ++d) {
      uint32_t x = 0;
#pragma unroll
      for (int w = 0; w < 16; ++w) x ^= sl[d][w];
      sacc += x;
      ss[d] = mix(ss[d] + x + 1);
    }
  }
  if (acc + sacc == 0x12345678u) out[0] = acc;
}

template <int VD, int SD>
static void run(const uint4* tab, uint64_t nlines, int blocks, int rounds, uint64_t* out) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  float ms = 0;
  for (int rep = 0; rep < 2; ++rep) {
    CHK(hipEventRecord(a));
    hipLaunchKernelGGL((k_mix<VD, SD>), dim3(blocks), dim3(256), 0, 0, tab, nlines, rounds, out);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    CHK(hipEventElapsedTime(&ms, a, b));
  }
  const double vacc = (double)blocks * 256 * rounds * VD;
  const double sacc = (double)blocks * 4 * rounds * SD;
  printf("vdepth %d sdepth %d: %.3f ms  vector %.2f G lines/s  scalar %.2f G lines/s  total %.2f G lines/s\n",
         VD, SD, ms, vacc / ms / 1e6, sacc / ms / 1e6, (vacc + sacc) / ms / 1e6);
}

int main(int argc, char** argv) {
  // usage: sgather_bench [table_MiB=2048] [wg_per_cu=8] [rounds=64]
  const uint64_t mb = argc > 1 ? atoll(argv[1]) : 2048;
  const int wgpc = argc > 2 ? atoi(argv[2]) : 8;
  const int rounds = argc > 3 ? atoi(argv[3]) : 64;
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const uint64_t bytes = mb << 20;
  uint4* tab;
  uint64_t* out;
  CHK(hipMalloc(&tab, bytes));
  CHK(hipMalloc(&out, 64));
  CHK(hipMemset(tab, 1, bytes));
  const uint64_t nlines = bytes / 64;
  const int blocks = p.multiProcessorCount * wgpc;
  printf("table %llu MiB, %d CUs x %d WG, %d rounds\n", (unsigned long long)mb, p.multiProcessorCount, wgpc, rounds);
  run<1, 0>(tab, nlines, blocks, rounds, out);
  run<2, 0>(tab, nlines, blocks, rounds, out);
  run<0, 1>(tab, nlines, blocks, rounds, out);
  run<0, 2>(tab, nlines, blocks, rounds, out);
  run<0, 4>(tab, nlines, blocks, rounds, out);
  run<1, 1>(tab, nlines, blocks, rounds, out);
  run<1, 2>(tab, nlines, blocks, rounds, out);
  run<1, 4>(tab, nlines, blocks, rounds, out);
  run<2, 2>(tab, nlines, blocks, rounds, out);
  run<2, 4>(tab, nlines, blocks, rounds, out);
  return 0;
}
