// fake_hip.cpp -- TEST INFRASTRUCTURE for tests/host_harness: the HIP runtime calls and kernel
// launchers the engine's host code (emqx_amd/csrc/gm_engine.cpp) makes, restated on the CPU so
// that its registry / trie model / delta-commit / epoch bookkeeping runs under ASan + UBSan.
// "Device" memory is malloc'ed host memory; every asynchronous call completes at once.
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime.h>

#include "../../emqx_amd/csrc/gm_kernels.h"

struct ihipStream_t {
  int dummy;
};
struct ihipEvent_t {
  int dummy;
};

hipError_t hipGetDeviceCount(int* n) {
  *n = 1;
  return hipSuccess;
}
hipError_t hipSetDevice(int d) { return d == 0 ? hipSuccess : hipErrorInvalidDevice; }
hipError_t hipGetDeviceProperties(hipDeviceProp_t* p, int) {
  p->multiProcessorCount = 4;
  return hipSuccess;
}
const char* hipGetErrorString(hipError_t) { return "fake hip error"; }
// device / pinned allocations and frees so far (tests/test_hook_alloc.py: a subscribe's commit
// must not allocate)
static unsigned long long g_allocs = 0, g_frees = 0;
extern "C" unsigned long long fakehip_allocs(void) { return __atomic_load_n(&g_allocs, __ATOMIC_RELAXED); }
extern "C" unsigned long long fakehip_frees(void) { return __atomic_load_n(&g_frees, __ATOMIC_RELAXED); }

hipError_t hipMalloc(void** p, size_t bytes) {
  __atomic_fetch_add(&g_allocs, 1, __ATOMIC_RELAXED);
  *p = malloc(bytes ? bytes : 1);
  if (*p) memset(*p, 0xA5, bytes);  // device memory starts undefined: poison it
  return *p ? hipSuccess : hipErrorUnknown;
}
hipError_t hipFree(void* p) {
  if (p) __atomic_fetch_add(&g_frees, 1, __ATOMIC_RELAXED);
  free(p);
  return hipSuccess;
}
hipError_t hipHostMalloc(void** p, size_t bytes, unsigned) { return hipMalloc(p, bytes); }
hipError_t hipHostFree(void* p) { return hipFree(p); }
hipError_t hipGetLastError() { return hipSuccess; }
hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned) {
  *d = h;
  return hipSuccess;
}
hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind) {
  if (n) memmove(d, s, n);
  return hipSuccess;
}
hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind k, hipStream_t) {
  return hipMemcpy(d, s, n, k);
}
hipError_t hipMemsetAsync(void* d, int v, size_t n, hipStream_t) {
  if (n) memset(d, v, n);
  return hipSuccess;
}
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned) {
  *s = new ihipStream_t();
  return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) {
  delete s;
  return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned) { return hipSuccess; }
hipError_t hipEventCreate(hipEvent_t* e) {
  *e = new ihipEvent_t();
  return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) { return hipEventCreate(e); }
hipError_t hipEventDestroy(hipEvent_t e) {
  delete e;
  return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
hipError_t hipEventQuery(hipEvent_t) { return hipSuccess; }
hipError_t hipEventElapsedTime(float* ms, hipEvent_t, hipEvent_t) {
  *ms = 0.f;
  return hipSuccess;
}

namespace gm {

WalkGeom walk_geometry(int, uint32_t wg) {
  WalkGeom g;
  g.cus = 4;
  g.blocks = 4 * (wg ? wg : 4);
  g.lanes = g.blocks * 256;
  return g;
}
uint32_t scan_tmp_words(uint32_t n) { return n / 4096 + 2; }

// k_patch: the one launcher whose effect the harness checks (delta commits patch the tables)
hipError_t launch_patch(const PatchEnt* ents, uint32_t n, const uint32_t* src, hipStream_t) {
  for (uint32_t e = 0; e < n; ++e)
    memcpy((void*)(uintptr_t)ents[e].dst, src + ents[e].s, 4u * ents[e].w);
  return hipSuccess;
}

// the match pipeline does not run in the harness (it walks the tables on the CPU itself)
#define NOT_HERE return hipErrorUnknown
hipError_t launch_scan(const uint32_t*, uint32_t*, uint32_t, uint32_t*, uint32_t*, hipStream_t) { NOT_HERE; }
hipError_t launch_tok(const uint8_t*, const uint32_t*, uint32_t, const DevIndex&, Scratch&, hipStream_t, uint32_t, bool, const uint32_t*, const uint8_t*, const uint32_t*) { NOT_HERE; }
void walk_claim_init(const WalkGeom&, uint32_t, uint32_t, uint32_t*) {}
hipError_t launch_exact(const uint8_t*, const uint32_t*, uint32_t, const DevIndex&, Scratch&, const WalkGeom&, hipStream_t) { NOT_HERE; }
hipError_t launch_exact_owned(const uint8_t*, const uint32_t*, uint32_t, const DevIndex&, uint32_t, uint32_t, uint32_t*, hipStream_t) { NOT_HERE; }
hipError_t launch_walk(const DevIndex&, Scratch&, uint32_t, const WalkGeom&, hipStream_t, unsigned long long*, uint32_t, uint32_t) { NOT_HERE; }
uint32_t walk_blocks(const WalkGeom&, uint32_t, uint32_t) { return 0; }
bool walk_pair(const WalkGeom&, uint32_t, uint32_t) { return false; }
uint32_t walk_static_chunks(const WalkGeom&, uint32_t, uint32_t, uint32_t) { return 0; }
hipError_t launch_verify(const uint8_t*, const uint32_t*, const DevIndex&, Scratch&, uint32_t, const WalkGeom&, hipStream_t) { NOT_HERE; }
hipError_t launch_scatter(Scratch&, uint32_t, const WalkGeom&, hipStream_t, bool, bool) { NOT_HERE; }
hipError_t launch_scan_ctl(const uint32_t*, uint32_t*, uint32_t, uint32_t*, uint32_t*, const uint32_t*, uint32_t*, hipStream_t) { NOT_HERE; }
hipError_t launch_verify_scatter(const uint8_t*, const uint32_t*, const DevIndex&, Scratch&, uint32_t, hipStream_t) { NOT_HERE; }
hipError_t launch_fixup(Scratch&, uint32_t, hipStream_t) { NOT_HERE; }
hipError_t launch_row64(const uint32_t*, uint64_t, uint64_t*, uint32_t, hipStream_t) { NOT_HERE; }
hipError_t launch_fanout(const DevIndex&, const Scratch&, FanScratch&, uint32_t, bool, hipStream_t) { NOT_HERE; }
hipError_t launch_rules(const uint8_t*, const uint32_t*, uint32_t, const uint8_t*, const uint32_t*, const uint32_t*, uint32_t, uint64_t, uint32_t*, hipStream_t) { NOT_HERE; }
hipError_t launch_copy_out(const CopyOut&, const CopyOut&, const CopyOut&, hipStream_t) { NOT_HERE; }
hipError_t launch_ctl_out(const uint32_t*, uint32_t*, hipStream_t) { NOT_HERE; }
hipError_t launch_export(const uint32_t*, const uint32_t*, const uint32_t*, uint32_t, uint32_t, const uint32_t*, uint32_t*, uint32_t*, uint32_t*, hipStream_t) { NOT_HERE; }
hipError_t launch_merge(const uint32_t* const*, uint32_t, uint32_t, uint32_t*, uint32_t*, uint32_t*, uint32_t*, uint32_t*, uint32_t*, hipStream_t) { NOT_HERE; }

hipError_t launch_wire_export(const uint32_t*, const uint32_t*, const uint32_t*, uint32_t, uint32_t, const uint32_t*, uint32_t, uint8_t*, uint8_t*, uint2*, uint2*, uint32_t*, hipStream_t) { NOT_HERE; }
hipError_t launch_wire_rows(const uint8_t*, uint32_t, const uint2*, uint32_t, uint32_t, uint32_t*, uint32_t*, uint32_t*, hipStream_t) { NOT_HERE; }
hipError_t launch_wire_ids(const uint8_t*, uint32_t, uint32_t*, hipStream_t) { NOT_HERE; }
hipError_t launch_wire_exact(const uint2* const*, const uint32_t*, uint32_t, uint32_t, uint32_t*, hipStream_t) { NOT_HERE; }
hipError_t launch_filter_len(const uint32_t*, uint32_t, const uint64_t*, uint32_t*, uint32_t*, uint32_t*, uint32_t*, hipStream_t) { NOT_HERE; }
hipError_t launch_filter_gather(const uint32_t*, uint32_t, const uint64_t*, const uint8_t*, const uint32_t*, uint8_t*, hipStream_t) { NOT_HERE; }
hipError_t launch_filter_len_dev(const uint32_t*, const uint32_t*, uint32_t, const uint64_t*, uint32_t*, uint32_t*, uint32_t*, uint32_t*, hipStream_t) { NOT_HERE; }
hipError_t launch_fb_small(const uint32_t*, const uint32_t*, const uint64_t*, const uint8_t*, const uint32_t*, const uint32_t*, uint32_t, uint32_t, uint64_t, uint8_t*, hipStream_t) { NOT_HERE; }
hipError_t launch_fb_pack(const uint32_t*, const uint32_t*, const uint64_t*, const uint8_t*, const uint32_t*, const uint32_t*, const uint32_t*, const uint32_t*, uint32_t, uint32_t, uint64_t, uint8_t*, hipStream_t) { NOT_HERE; }

}  // namespace gm
