// gather_bench.hip -- what random small-line gathers cost on this MI355X (calibration for the
// k_walk roofline).  Every lane issues `depth` independent random loads per round of `width`
// bytes (16/32/64) from a table of `table_mb` MiB, for `rounds` dependent rounds (the next
// address depends on the loaded data, like a trie walk).  Prints lines/s and GB/s.  With `part`
// each workgroup draws from one range of the table (r05: profiles/r05/gather_part.txt).
// Build: hipcc --offload-arch=gfx950 -O3 tools/gather_bench.hip -o tools/gather_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <algorithm>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33;
  return k;
}

template <int W>  // W = 16-B loads per access
__global__ __launch_bounds__(256) void k_gather(const uint4* __restrict__ tab, uint64_t nslots,
                                                int rounds, int depth, uint64_t* out, int part) {
  const uint64_t gid = blockIdx.x * 256ull + threadIdx.x;
  // part > 0: block b draws from range b % part of the table (blocks are dealt to the 8 XCDs
  // round-robin, so part = 8 gives each XCD one eighth); part < 0: range b * |part| / grid (each
  // range spread over every XCD)
  const uint64_t np = part ? (uint64_t)(part > 0 ? part : -part) : 1ull;
  const uint64_t rs = nslots / np;
  const uint64_t base = rs * (part > 0 ? blockIdx.x % np : part < 0 ? (uint64_t)blockIdx.x * np / gridDim.x : 0ull);
  uint64_t st[4];
  for (int d = 0; d < 4; ++d) st[d] = mix(gid * 4 + d + 1);
  uint32_t acc = 0;
  for (int r = 0; r < rounds; ++r) {
    uint4 v[4][W];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      if (d < depth) {
        const uint64_t s = base + st[d] % rs;
#pragma unroll
        for (int w = 0; w < W; ++w) v[d][w] = tab[s * W + w];
      }
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      if (d < depth) {
        uint32_t x = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) x ^= v[d][w].x ^ v[d][w].w;
        acc += x;
        st[d] = mix(st[d] + x + 1);  // next address depends on the data
      }
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
  // usage: gather_bench [table_MiB=2048] [wg_per_cu=8] [width_16B_units=0 (all)] [depth=0 (all)]
  //                     [alloc=0: hipMalloc, 1: hipExtMallocWithFlags(hipDeviceMallocContiguous),
  //                      2: hipMemCreate/hipMemMap at 1 GiB granularity] [part=0, see k_gather]
  const uint64_t mb = argc > 1 ? atoll(argv[1]) : 2048;
  const int wgpc = argc > 2 ? atoi(argv[2]) : 8;
  const int only_w = argc > 3 ? atoi(argv[3]) : 0;
  const int only_d = argc > 4 ? atoi(argv[4]) : 0;
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const uint64_t bytes = mb << 20;
  uint4* tab;
  uint64_t* out;
  const int alloc = argc > 5 ? atoi(argv[5]) : 0;
  const int part = argc > 6 ? atoi(argv[6]) : 0;  // see k_gather
  if (alloc == 1) {
    CHK(hipExtMallocWithFlags((void**)&tab, bytes, hipDeviceMallocContiguous));
  } else if (alloc == 2) {
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gran = 0;
    CHK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
    const size_t chunk = std::max<size_t>(gran, 1ull << 30);
    const size_t total = (bytes + chunk - 1) / chunk * chunk;
    void* va = nullptr;
    CHK(hipMemAddressReserve(&va, total, chunk, nullptr, 0));
    for (size_t o = 0; o < total; o += chunk) {
      hipMemGenericAllocationHandle_t hnd;
      CHK(hipMemCreate(&hnd, chunk, &prop, 0));
      CHK(hipMemMap((char*)va + o, chunk, 0, hnd, 0));
    }
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    CHK(hipMemSetAccess(va, total, &acc, 1));
    tab = (uint4*)va;
    printf("vmm granularity %zu, chunk %zu\n", gran, chunk);
  } else {
    CHK(hipMalloc(&tab, bytes));
  }
  CHK(hipMalloc(&out, 64));
  CHK(hipMemset(tab, 1, bytes));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const int blocks = p.multiProcessorCount * wgpc;
  const int rounds = 64;
  printf("table %llu MiB, %d CUs x %d WG, %d rounds, alloc %d, part %d\n", (unsigned long long)mb, p.multiProcessorCount, wgpc, rounds, alloc, part);
  for (int W : {1, 2, 4}) {
    if (only_w && W != only_w) continue;
    for (int depth : {1, 2, 4}) {
      if (only_d && depth != only_d) continue;
      const uint64_t nslots = bytes / (16ull * W);
      for (int rep = 0; rep < 2; ++rep) {
        CHK(hipEventRecord(a));
        if (W == 1) hipLaunchKernelGGL(k_gather<1>, dim3(blocks), dim3(256), 0, 0, tab, nslots, rounds, depth, out, part);
        if (W == 2) hipLaunchKernelGGL(k_gather<2>, dim3(blocks), dim3(256), 0, 0, tab, nslots, rounds, depth, out, part);
        if (W == 4) hipLaunchKernelGGL(k_gather<4>, dim3(blocks), dim3(256), 0, 0, tab, nslots, rounds, depth, out, part);
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        const double acc = (double)blocks * 256 * rounds * depth;
        if (rep == 1)
          printf("width %2d B depth %d: %.3f ms  %.2f G accesses/s  %.1f GB/s\n", 16 * W, depth, ms,
                 acc / ms / 1e6, acc * 16 * W / ms / 1e6);
      }
    }
  }
  return 0;
}
