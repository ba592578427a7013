// gm_kernels.h -- launch interface of the gfx950 match pipeline (gm_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gm {

// Committed device index (all pointers are device memory).
struct DevIndex {
  const uint4* edges = nullptr;   // SLOT_U4 x uint4 per slot (gm_common.h "edge slots")
  uint64_t emask = 0;             // bucket count - 1
  const uint32_t* multi = nullptr;  // [count, fid...] lists
  uint32_t root_cf = 0, root_hf = 0xFFFFFFFFu;
  uint32_t root_pcf = 0, root_phf = 0xFFFFFFFFu;  // root's '+' child (cf 0: none)
  uint32_t root_sig = 0x3Fu;                       // root's child signature (gm_common.h)
  // the root's fat half (gm_common.h FAT_ID): its only literal child's slot, as a bucket's
  // second half would hold it (rh0.z = NONE: the root's literal children are probed by hash)
  uint4 rh0 = {0u, 0u, 0xFFFFFFFFu, 0u}, rh1 = {0u, 0u, 0u, 0u};
  const uint32_t* tn_of = nullptr;  // per node: non-wildcard trie keys ending there
  // publish fan-out tables (gm_fanout.inc), per filter id < fan_nf
  const uint4* fan = nullptr;        // [fan_nf] {rt off, rt count, dl off, dl count}
  const uint32_t* rt_dst = nullptr;  // aggre entries (dest handles)
  const uint32_t* dl_sub = nullptr;  // local deliveries (subscriber ids)
  uint32_t fan_nf = 0;
  // exact route-key buckets (gm_common.h "Exact route-key table"): plain (non-wildcard) keys
  // in buckets [0, xmask], wildcard keys in [xwbase, xwbase + xwmask]
  const uint4* exact = nullptr;
  const uint32_t* xovf = nullptr;  // per bucket: keys were placed past it (gm_common.h)
  uint64_t xmask = 0;             // plain region bucket count - 1
  uint64_t xwbase = 0;            // first bucket of the wildcard-key region
  uint64_t xwmask = 0;            // wildcard region bucket count - 1
  const uint8_t* fbytes = nullptr;  // filter string pool
  const uint64_t* foff = nullptr;   // [n_filters+1]
  const uint4* fver = nullptr;      // 64-B verification record per filter id
  const uint32_t* fvbits = nullptr; // bit per filter id: its trie pairs need byte verification
  uint64_t test_mask = 0;           // != 0: collision-test tokens (every word hashed, masked)
  uint64_t full_mask = ~0ull;
  uint32_t max_depth = 0;           // deepest trie filter in levels
  uint64_t fid_bound = 0;           // every filter id the walk can emit is below it (0: unknown)
  bool trie_empty = true;
  bool plain_empty = true;         // no committed non-wildcard route key
  bool wild_empty = true;          // no committed wildcard route key
  bool needs_verify = false;        // some trie filter has a hashed (long or test) token
  uint32_t leafp_mask = (1u << 26) | (1u << 29);  // CF_HMASK: depth-code pruning (0: off)
};

// Layout of the staged pairs of one pass.  Wide: {topic, filter, rank | REJ_BIT}, 12 B.  Packed
// (pk, when the batch's topic ids, the index's filter ids and a rank field of at least
// STG_MIN_RANK_BITS fit 64 bits): one 8-B word, topic << tsh | filter << fsh | rank << 1 | rejected
// -- a third less for the walk to write and the scatter to read.  A topic with more pairs than
// the rank field holds flags CTL_PKOVF and the pass is redone wide.
struct StgFmt {
  uint32_t pk = 0;
  uint32_t tsh = 0, fsh = 0;  // shifts of the topic and filter fields
  uint32_t fmask = 0;         // filter field mask
  uint32_t rmask = 0;         // rank field mask (ranks <= rmask)
};
constexpr uint32_t STG_MIN_RANK_BITS = 10;

// Per-batch scratch (device memory, owned by the engine, grown on demand).
struct Scratch {
  uint32_t n_cap = 0;  // topic capacity
  uint64_t w_cap = 0;  // word capacity
  uint32_t* nw = nullptr;     // [n]   words per topic
  uint64_t* wh = nullptr;     // [w]   level tokens
  uint4* rec = nullptr;       // [n * REC_U4] 64-B topic records (gm_common.h)
  uint32_t* cnt = nullptr;    // [n]   trie matches per topic
  uint32_t* row = nullptr;    // [n+1]
  uint32_t* row2 = nullptr;   // [n+1] (legacy fix-up)
  uint32_t* rej = nullptr;    // [n]   rejected pairs per topic
  uint32_t* exact_id = nullptr;  // [n]
  uint2* xh = nullptr;        // [n]   exact probe over a huge table: {home bucket, h32} per name
  uint32_t p_cap = 0;   // pair staging capacity
  uint3* stg = nullptr;       // staged pairs {topic, filter, rank | REJ_BIT} (12 B), CH-slot chunks
                              // (or 8-B packed words, fmt)
  StgFmt fmt;                 // this pass's staging layout (set by the engine per pass)
  uint32_t* chk = nullptr;    // per staged chunk: pairs in it (written by the walk)
  uint32_t xseq = 1;          // this pass's sequence number (CTL_XHIT), set by the engine
  uint32_t o_cap = 0;
  uint32_t* out = nullptr;    // [pairs] CSR filter ids
  uint32_t* out2 = nullptr;   // legacy fix-up target
  uint32_t* scan_tmp = nullptr;  // scan partials
  uint32_t scan_tmp_cap = 0;
  uint32_t* ctl = nullptr;    // control words (see CTL_*)
  uint2* spill = nullptr;     // walk probe items beyond the LDS stack
  uint32_t spill_items = 0;   // spill entries per walk lane
  uint32_t spill_lanes = 0;   // walk lanes the spill was sized for
  uint2* rlist = nullptr;     // rejected (topic, rank) list
  uint32_t r_cap = 0;
  uint32_t* ctl_host = nullptr;  // pinned host mirror of ctl (mapped: k_ctl_out writes it)
  uint32_t* ctl_host_dev = nullptr;  // its device-side address
  unsigned long long* census = nullptr;  // [CENSUS_N] diagnostic walk counters
};

enum : int {
  CTL_TOPIC_CTR = 0,  // walk topic-block claim counter
  CTL_PAIR_TOP = 1,   // staged pair slots reserved
  CTL_ANY_REJ = 2,    // a verification rejected some pair
  CTL_TOTAL = 3,      // total pairs (row[n]) copied here
  CTL_XHIT = 4,       // == Scratch::xseq: some name of the batch has an exact route key (else
                      // exact_id is all NONE); the word is never cleared, k_tok zeroes the rest
  CTL_NREJ = 5,       // rejected pairs appended to rlist
  CTL_LEGACY = 6,     // deferred scatter could not place rejects: re-run with the fix-up path
  CTL_ERR = 7,        // walk item stack outgrew its spill: re-run with a larger spill
  CTL_PKOVF = 8,      // a topic's rank outgrew the packed staging's field: re-run wide
  CTL_FAN_R = 9,      // publish fan-out: aggre entries of the batch
  CTL_FAN_D = 10,     //   local deliveries of the batch
  CTL_CLAIM0 = 16,    // walk topic-claim counters, one per shard, CTL_CLAIM_STRIDE apart
  CTL_SHARDS_OUT = 16 + 8 * 32,  // walk: bit c = claim shard c ran out (a line of its own)
  CTL_N = 16 + 9 * 32
};

// diagnostic walk counters: states, slot loads, lane iterations, wave iterations
constexpr uint32_t CENSUS_N = 4;
// then edge-bucket loads per probed level (levels >= CENSUS_DEPTHS - 1 lumped), literal probes
// at [CENSUS_N + d], '+' probes at [CENSUS_N + CENSUS_DEPTHS + d]; the per-wave timeline after
constexpr uint32_t CENSUS_DEPTHS = 16;
constexpr uint32_t CENSUS_HDR = CENSUS_N + 2 * CENSUS_DEPTHS;

// The walk claims topics from WALK_SHARDS counters on separate 128-B lines (one hot counter
// serialises at ~88 claims/us chip-wide); a wave starts on shard blockIdx % 8 (its XCD under
// round-robin dispatch) and moves on when that shard's topics are exhausted.
constexpr uint32_t WALK_SHARDS = 8;
constexpr uint32_t CTL_CLAIM_STRIDE = 32;

constexpr uint32_t STAGE_CHUNK = 1024;  // staged-pair slots a walk wave reserves per atomic
constexpr uint32_t REJ_BIT = 0x80000000u;
constexpr uint32_t REJ_SCAN_MAX = 4096;  // rejects the deferred scatter handles in-line
// Walk probe items per lane kept in LDS.  Passes start with the shallow stack (34 KB of LDS per
// walk block: four blocks per CU leave room for the other pipe's tokenizer tile beside them);
// an index whose walks outgrow it moves to the deep one (47 KB: three blocks per CU), then to the
// deep stack continued in global memory (spill).  Measured on cfg2, whose walks outgrow 6 items
// (profiles/r02/session2/ab_walk_stack.txt, ab_walk_stack_deep.txt): pipelined step 1.59 ms
// spilling past 6, 1.38 ms past 8, 1.21 ms with 12 or 14 (3 blocks per CU), 1.45 ms with 16
// (2 blocks per CU); cfg3 never leaves the shallow stack (an 8-deep one cost it ~1.5%).
// Walk item stacks per variant level: SHALLOW and DEEP keep compact 32-bit items in LDS (12 at
// four blocks per CU, 24 at three: gm_walk.inc CPT), SPILL keeps 12 {node, level} pairs in LDS
// and continues in global memory (r03: compact items made cfg2's walk 1.274 -> 1.229 ms;
// an 18-item deep stack made its pipelined step slower, profiles/r03/results/ab_*).
constexpr bool WALK_CPT = true;
constexpr uint32_t WALK_STK_SHALLOW = 12;
constexpr uint32_t WALK_STK_DEEP = 24;
constexpr uint32_t WALK_STK_SPILL = 12;
// The walk variant a committed index needs, raised when a pass's lanes outgrow their stack:
// shallow LDS stack (pairs for small batches only), shallow stack with pairs for every batch (two
// lanes share a topic's items), deep stack with pairs, deep + global spill (one lane per topic).
enum WalkLevel : uint32_t { WALK_SHALLOW = 0, WALK_PAIRED = 1, WALK_DEEP = 2, WALK_SPILL = 3 };
constexpr uint32_t WALK_SPILL_MIN = 32;  // initial spill items per lane (grown on overflow)
// spill items per lane that no walk can exceed: a resolved probe pushes <= 4 items spanning
// 3 levels, and the LIFO holds <= 3 unexplored siblings per level of the current path
inline uint32_t walk_spill_bound(uint32_t max_depth) { return 4u * (max_depth + 2u) + 8u; }

struct WalkGeom {
  uint32_t blocks = 0;      // persistent workgroups
  uint32_t lanes = 0;       // blocks * 256
  uint32_t cus = 0;
  // exact route-key probe in passes over bucket ranges of this many bytes (0: one pass; see
  // launch_exact); set by the engine, emqxgm_tune("exact_range_kb")
  uint64_t xrange_bytes = 0;
  // two lanes per topic (k_walk PAIR) for batches of at most half the grid's lanes;
  // emqxgm_tune("walk_pair", 0) turns it off (A/B)
  uint32_t pair = 1;
};

WalkGeom walk_geometry(int device, uint32_t wg_per_cu);

// Pipeline stages (all asynchronous on `s`).
hipError_t launch_scan(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* tmp,
                       uint32_t* total_dst, hipStream_t s);
uint32_t scan_tmp_words(uint32_t n);
// tokenise: levels (nw), 64-B topic records (rec: first REC_TOKS tokens inline), tokens of
// deeper levels (wh, at off[t] + t + level); exact route-key ids (exact_id, NONE if absent)
// of wildcard names when there are no plain keys, else X_WILDPEND marks for launch_exact.
// src_bytes / src_off (copy-through, TokArgs): the input is read there (pinned host memory) and
// stored into bytes / off, the pass's device buffers.
hipError_t launch_tok(const uint8_t* bytes, const uint32_t* off, uint32_t n, const DevIndex& ix,
                      Scratch& sc, hipStream_t s, uint32_t pair_top0, bool zero_rej,
                      const uint32_t* claim0 = nullptr, const uint8_t* src_bytes = nullptr,
                      const uint32_t* src_off = nullptr);
// exact route-key ids of every name (after launch_tok; a no-op when there are no plain keys)
// the route-key probe of the names key shard `part` of `parts` owns (others: NONE) into out
hipError_t launch_exact_owned(const uint8_t* bytes, const uint32_t* off, uint32_t n,
                              const DevIndex& ix, uint32_t parts, uint32_t part, uint32_t* out,
                              hipStream_t s);
hipError_t launch_exact(const uint8_t* bytes, const uint32_t* off, uint32_t n, const DevIndex& ix,
                        Scratch& sc, const WalkGeom& g, hipStream_t s);

// Per-batch scratch of the publish fan-out (gm_fanout.inc).
struct FanScratch {
  uint32_t n_cap = 0, r_cap = 0, d_cap = 0;
  uint32_t *cr = nullptr, *cd = nullptr, *rp = nullptr, *dp = nullptr;
  uint32_t *o_rf = nullptr, *o_rd = nullptr, *o_df = nullptr, *o_ds = nullptr;
};
// first rule (emqx_topic:match/2, or equality for RULE_EQ) matching each name, NONE if none
hipError_t launch_rules(const uint8_t* nb, const uint32_t* no, uint32_t n, const uint8_t* rb,
                        const uint32_t* ro, const uint32_t* rf, uint32_t nr, uint64_t rbytes,
                        uint32_t* out, hipStream_t s);
// Committed retained-topic store (gm_retain.inc / gm_retain.cpp), device pointers.
struct RetainDev {
  const uint4* rn = nullptr;      // per node {tb | RTERM, te, c0, c1}
  const uint4* redge = nullptr;   // edge slots {tok.lo, tok.hi, parent, child}
  uint64_t rmask = 0;
  const uint32_t* rch = nullptr;  // children lists
  const uint2* rw = nullptr;      // per node {pool offset, length} of its word
  const uint8_t* pool = nullptr;  // topic bytes
  const uint32_t* sid = nullptr;  // topic id per sorted position
  const uint64_t* sexp = nullptr; // expiry per sorted position (~0: deleted)
};
// count (fill = false: cnt = runs + cnt_in) or fill (at rbase + rshift) the runs of each
// filter in one store; delta tags its runs
hipError_t launch_retain_walk(const RetainDev& st, const uint8_t* fb, const uint32_t* fo, uint32_t n,
                              const uint8_t* tail, uint4* frames, uint32_t max_plus, uint32_t* cnt,
                              const uint32_t* cnt_in, const uint32_t* rbase,
                              const uint32_t* rshift, bool delta, uint2* runs, bool fill,
                              hipStream_t s);
// count (adds to *total) or write the live topic ids of each run (base or delta store)
hipError_t launch_retain_runs(const RetainDev& base, const RetainDev& delta, const uint2* runs,
                              uint32_t nr, uint64_t now, uint32_t* acnt, const uint32_t* abase,
                              uint32_t* out, unsigned long long* total, bool fill, hipStream_t s);
hipError_t launch_retain_ptr(const uint32_t* rbase, const uint32_t* abase, uint32_t n,
                             uint32_t* ptr, hipStream_t s);
// One patch of a delta commit: w (1..64) dwords from src[s..] to the device address dst.
struct PatchEnt {
  uint64_t dst;
  uint32_t s, w;
};
hipError_t launch_patch(const PatchEnt* ents, uint32_t n, const uint32_t* src, hipStream_t s);
// count pass (fill = false) or fill pass over the match result in sc (row, out, exact_id)
hipError_t launch_fanout(const DevIndex& ix, const Scratch& sc, FanScratch& fs, uint32_t n,
                         bool fill, hipStream_t s);

// census != nullptr selects the diagnostic walk (adds to census[0..CENSUS_N)); level (WalkLevel)
// the probe-item stack: shallow or deep in LDS, or deep continued in global memory (spill)
// the walk's workgroup count and its static staged-pair chunks (one per wave, or 0); k_tok
// starts CTL_PAIR_TOP at static_chunks * STAGE_CHUNK
uint32_t walk_blocks(const WalkGeom& g, uint32_t n, uint32_t level);
// whether the walk of n topics runs two lanes per topic (k_walk PAIR)
bool walk_pair(const WalkGeom& g, uint32_t n, uint32_t level);
uint32_t walk_static_chunks(const WalkGeom& g, uint32_t n, uint32_t level, uint32_t pcap);
// the claim counters' start values past the walk's static first claims (k_tok sets them)
void walk_claim_init(const WalkGeom& g, uint32_t n, uint32_t level, uint32_t claim0[WALK_SHARDS]);
hipError_t launch_walk(const DevIndex& ix, Scratch& sc, uint32_t n, const WalkGeom& g,
                       hipStream_t s, unsigned long long* census = nullptr,
                       uint32_t level = WALK_SHALLOW, uint32_t stat_chunks = 0);
// production: verify (flags + counts) -> [scan] -> deferred scatter
hipError_t launch_verify(const uint8_t* bytes, const uint32_t* off, const DevIndex& ix,
                         Scratch& sc, uint32_t n, const WalkGeom& g, hipStream_t s);
// fuse_scan: the row scan inside k_scatter (n <= SCATTER_SCAN_MAX; no launch_scan_ctl before)
constexpr uint32_t SCATTER_SCAN_MAX = 4096;  // = SCAN_TILE (gm_kernels.hip)
hipError_t launch_scatter(Scratch& sc, uint32_t n, const WalkGeom& g, hipStream_t s,
                          bool mirror_ctl = false, bool fuse_scan = false);
// a pass's row scan whose last block also copies the control words to the host mirror
hipError_t launch_scan_ctl(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* tmp,
                           uint32_t* total_dst, const uint32_t* ctl, uint32_t* ctl_host_dev,
                           hipStream_t s);
// legacy path (reject list overflow): scan -> verify+scatter -> compaction
hipError_t launch_verify_scatter(const uint8_t* bytes, const uint32_t* off, const DevIndex& ix,
                                 Scratch& sc, uint32_t n, hipStream_t s);
hipError_t launch_fixup(Scratch& sc, uint32_t n, hipStream_t s);
// A result array copied into pinned host memory by a kernel (PCIe writes from the GPU): its
// count is n, or min(*n_dev, cap) when n_dev is set (a pass's pair total, read on the device, so
// nothing on the host sizes the copy).  dst is the device-side address of the host buffer.
struct CopyOut {
  const uint32_t* src;
  uint32_t* dst;
  uint32_t n;
  const uint32_t* n_dev;
  uint32_t cap;
};
// The pass's control words into the mapped host mirror (one block; replaces a D2H copy, which
// the runtime runs as a blit with more overhead between two pipes' passes).
hipError_t launch_ctl_out(const uint32_t* ctl, uint32_t* ctl_host_dev, hipStream_t s);
hipError_t launch_copy_out(const CopyOut& a, const CopyOut& b, const CopyOut& c, hipStream_t s);
// Filter-sharded layout: a shard's result copied with its ids mapped to global ids (map NULL:
// identity), and np shards' results merged (parts: np x {row, fid, exact} device pointers, in
// device memory); cnt/tmp: scratch of n / scan_tmp_words(n) words; *total = merged pairs.
hipError_t launch_export(const uint32_t* row, const uint32_t* fid, const uint32_t* exact, uint32_t n,
                         uint32_t pairs, const uint32_t* map, uint32_t* orow, uint32_t* ofid,
                         uint32_t* oexact, hipStream_t s);
hipError_t launch_merge(const uint32_t* const* parts, uint32_t np, uint32_t n, uint32_t* cnt,
                        uint32_t* tmp, uint32_t* orow, uint32_t* ofid, uint32_t* oexact,
                        uint32_t* total, hipStream_t s);
// The compact wire form of a shard's result: counts (u8, or two bit planes with
// flags & 1), mapped ids (u32, or u16 + u8 planes with flags & 2), sparse (topic, exact id) xs
// and (topic, count) ovf lists; ctr[0] / ctr[1] = their lengths.
hipError_t launch_wire_export(const uint32_t* row, const uint32_t* fid, const uint32_t* exact,
                              uint32_t n, uint32_t pairs, const uint32_t* map, uint32_t flags,
                              uint8_t* cnt, uint8_t* ofid, uint2* xs, uint2* ovf, uint32_t* ctr,
                              hipStream_t s);
// a received part's row pointers [n+1] from its counts and overflow list (counts/tmp scratch)
hipError_t launch_wire_rows(const uint8_t* cnt, uint32_t flags, const uint2* ovf, uint32_t novf,
                            uint32_t n, uint32_t* counts, uint32_t* tmp, uint32_t* row,
                            hipStream_t s);
// a received part's 24-bit ids widened to u32
hipError_t launch_wire_ids(const uint8_t* fid, uint32_t pairs, uint32_t* out, hipStream_t s);
// the merged exact ids [n]: NONE, then every part's (topic, id) entries (host arrays of device
// pointers / lengths)
hipError_t launch_wire_exact(const uint2* const* xs, const uint32_t* nx, uint32_t parts, uint32_t n,
                             uint32_t* exact, hipStream_t s);
// The bytes of the filters fid[0..pairs) from the device string pool (foff: pool offsets per
// filter id): ooff = exclusive scan of their lengths (pairs + 1 entries; *total = bytes; len /
// tmp scratch), then out[ooff[j] ..] = filter fid[j]'s bytes.
hipError_t launch_filter_len(const uint32_t* fid, uint32_t pairs, const uint64_t* foff,
                             uint32_t* len, uint32_t* ooff, uint32_t* tmp, uint32_t* total,
                             hipStream_t s);
hipError_t launch_filter_gather(const uint32_t* fid, uint32_t pairs, const uint64_t* foff,
                                const uint8_t* pool, const uint32_t* ooff, uint8_t* out,
                                hipStream_t s);
// The length scan behind a pass, its pair count read on the device (pairs_dev, at most cap): no
// host round trip.
hipError_t launch_filter_len_dev(const uint32_t* fid, const uint32_t* pairs_dev, uint32_t cap,
                                 const uint64_t* foff, uint32_t* len, uint32_t* ooff, uint32_t* tmp,
                                 uint32_t* total, hipStream_t s);
// A host window's whole result packed into one block (one D2H copy): byte offsets of the
// block's parts for n topics and up to cap_p pairs; the filter bytes follow at `bytes`.
struct FbLayout {
  uint64_t total = 0, ooff, fid, exact, row, bytes;
  FbLayout(uint32_t n, uint32_t cap_p) {
    ooff = 16;
    fid = (ooff + 4ull * (cap_p + 1) + 15) & ~15ull;
    exact = (fid + 4ull * cap_p + 15) & ~15ull;
    row = (exact + 4ull * n + 15) & ~15ull;
    bytes = (row + 4ull * (n + 1) + 15) & ~15ull;
  }
};
// {byte total, byte offsets, filter ids, exact ids, row pointers, bytes} of a pass into `block`
// (FbLayout), its pair count read on the device; beyond cap_p pairs or cap_b bytes only the total
// is written.
hipError_t launch_fb_pack(const uint32_t* fid, const uint32_t* pairs_dev, const uint64_t* foff,
                          const uint8_t* pool, const uint32_t* ooff, const uint32_t* total,
                          const uint32_t* exact, const uint32_t* row, uint32_t n, uint32_t cap_p,
                          uint64_t cap_b, uint8_t* block, hipStream_t s);
// launch_filter_len_dev + launch_fb_pack in one single-block launch, for cap_p <= SCAN_TILE pairs
// (the scan of the lengths in LDS); -> hipErrorInvalidValue beyond
hipError_t launch_fb_small(const uint32_t* fid, const uint32_t* pairs_dev, const uint64_t* foff,
                           const uint8_t* pool, const uint32_t* exact, const uint32_t* row,
                           uint32_t n, uint32_t cap_p, uint64_t cap_b, uint8_t* block, hipStream_t s);
constexpr uint32_t FB_SMALL_PAIRS = 4096;  // = SCAN_TILE (gm_kernels.hip)
// out[i] = base + row[i], i < m (u64 CSR row pointers of the host API, built on the device)
hipError_t launch_row64(const uint32_t* row, uint64_t base, uint64_t* out, uint32_t m,
                        hipStream_t s);

}  // namespace gm
