// gm_kernels.h -- launch interface of the gfx950 match pipeline (gm_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gm {

// Committed device index (all pointers are device memory).
struct DevIndex {
  const uint4* edges = nullptr;   // SLOT_U4 x uint4 per slot (gm_common.h "edge slots")
  uint64_t emask = 0;             // slot capacity - 1
  const uint32_t* multi = nullptr;  // [count, fid...] lists
  uint32_t root_cf = 0, root_hf = 0xFFFFFFFFu;
  uint32_t root_q[6] = {0u, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0xFFFFFFFFu, 0xFFFFFFFFu};  // p, pp
  const uint4* exact = nullptr;   // exact slots {hash.lo, hash.hi, fid, len}
  uint64_t xmask = 0;
  const uint8_t* fbytes = nullptr;  // filter string pool
  const uint64_t* foff = nullptr;   // [n_filters+1]
  const uint4* fver = nullptr;      // 64-B verification record per filter id
  const uint32_t* fvbits = nullptr; // bit per filter id: its trie pairs need byte verification
  uint64_t test_mask = 0;           // != 0: collision-test tokens (every word hashed, masked)
  uint64_t full_mask = ~0ull;
  uint32_t max_depth = 0;           // deepest trie filter in levels
  bool trie_empty = true;
  bool exact_empty = true;
  bool needs_verify = false;        // some trie filter has a hashed (long or test) token
};

// Per-batch scratch (device memory, owned by the engine, grown on demand).
struct Scratch {
  uint32_t n_cap = 0;  // topic capacity
  uint64_t w_cap = 0;  // word capacity
  uint32_t* nw = nullptr;     // [n]   words per topic
  uint64_t* wh = nullptr;     // [w]   level tokens
  uint4* rec = nullptr;       // [n]   {wbase, n_words | flags << 24, tok0.lo, tok0.hi}
  uint32_t* cnt = nullptr;    // [n]   trie matches per topic
  uint32_t* row = nullptr;    // [n+1]
  uint32_t* row2 = nullptr;   // [n+1] (legacy fix-up)
  uint32_t* rej = nullptr;    // [n]   rejected pairs per topic
  uint32_t* exact_id = nullptr;  // [n]
  uint32_t p_cap = 0;   // pair staging capacity
  uint32_t* pt = nullptr;     // staged pair: topic
  uint32_t* pf = nullptr;     // staged pair: filter
  uint32_t* pr = nullptr;     // staged pair: rank within topic (bit 31 = rejected)
  uint32_t o_cap = 0;
  uint32_t* out = nullptr;    // [pairs] CSR filter ids
  uint32_t* out2 = nullptr;   // legacy fix-up target
  uint32_t* scan_tmp = nullptr;  // scan partials
  uint32_t scan_tmp_cap = 0;
  uint32_t* ctl = nullptr;    // control words (see CTL_*)
  uint4* spill = nullptr;     // walk stack spill (depth beyond LDS)
  uint64_t spill_cap = 0;     // entries
  uint2* rlist = nullptr;     // rejected (topic, rank) list
  uint32_t r_cap = 0;
  uint32_t* ctl_host = nullptr;  // pinned host mirror of ctl
  unsigned long long* census = nullptr;  // [4] diagnostic walk counters
};

enum : int {
  CTL_TOPIC_CTR = 0,  // walk topic-block claim counter
  CTL_PAIR_TOP = 1,   // staged pair slots reserved
  CTL_ANY_REJ = 2,    // a verification rejected some pair
  CTL_TOTAL = 3,      // total pairs (row[n]) copied here
  CTL_WORDS = 4,      // total words
  CTL_NREJ = 5,       // rejected pairs appended to rlist
  CTL_LEGACY = 6,     // deferred scatter could not place rejects: re-run with the fix-up path
  CTL_N = 8
};

constexpr uint32_t REJ_BIT = 0x80000000u;
constexpr uint32_t REJ_SCAN_MAX = 4096;  // rejects the deferred scatter handles in-line
constexpr uint32_t WALK_LDS_STACK = 4;   // walk stack entries per lane kept in LDS (rest spill)
constexpr uint32_t SPILL_U4 = 3;         // uint4 per spilled walk stack entry

struct WalkGeom {
  uint32_t blocks = 0;      // persistent workgroups
  uint32_t lanes = 0;       // blocks * 256
  uint32_t cus = 0;
};

WalkGeom walk_geometry(int device, uint32_t wg_per_cu);

// Pipeline stages (all asynchronous on `s`).
hipError_t launch_scan(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* tmp,
                       uint32_t* total_dst, hipStream_t s);
uint32_t scan_tmp_words(uint32_t n);
// tokenise: levels (nw), level tokens (wh), topic records (rec), exact route-key ids; adds the
// batch's level count to ctl[CTL_WORDS]
hipError_t launch_tok(const uint8_t* bytes, const uint32_t* off, uint32_t n, const DevIndex& ix,
                      Scratch& sc, hipStream_t s);
// census != nullptr selects the diagnostic walk that adds {states, slot loads} to census[0..1]
hipError_t launch_walk(const DevIndex& ix, Scratch& sc, uint32_t n, const WalkGeom& g,
                       hipStream_t s, unsigned long long* census = nullptr);
// production: verify (flags + counts) -> [scan] -> deferred scatter
hipError_t launch_verify(const uint8_t* bytes, const uint32_t* off, const DevIndex& ix,
                         Scratch& sc, uint32_t n, const WalkGeom& g, hipStream_t s);
hipError_t launch_scatter(Scratch& sc, uint32_t n, const WalkGeom& g, hipStream_t s);
// legacy path (reject list overflow): scan -> verify+scatter -> compaction
hipError_t launch_verify_scatter(const uint8_t* bytes, const uint32_t* off, const DevIndex& ix,
                                 Scratch& sc, uint32_t n, hipStream_t s);
hipError_t launch_fixup(Scratch& sc, uint32_t n, hipStream_t s);

}  // namespace gm
