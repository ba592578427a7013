// gm_engine.cpp -- host side of the MI355X topic-match engine: filter registry, device index
// builder (snapshot/commit), batch driver and the C-ABI declared in include/emqx_gpumatch.h.
//
// Reference semantics mirrored here:
//   * trie membership is a SET of filters (emqx_trie:insert is idempotent, delete of an absent
//     filter is a no-op: emqx_trie.erl:121-127, 139-144);
//   * route keys are refcounted by dests (the emqx_route bag, emqx_router_utils.erl:31-71);
//   * readers only ever see committed state (mria transactions), so every mutation lands in
//     the pending registry and becomes visible atomically at emqxgm_commit.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <new>
#include <shared_mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/emqx_gpumatch.h"
#include "gm_common.h"
#include "gm_internal.h"
#include "gm_kernels.h"
#include "gm_roctx.h"

using namespace gm;

namespace {

uint64_t pow2_at_least(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

// Open-addressing map (parent node, level token) -> child node (host-side trie; kept between
// commits for delta commits, so it also erases: a freed entry becomes a TOMB that lookups pass).
struct EdgeMap {
  struct Ent {
    uint64_t tok;
    uint32_t parent;  // NONE = empty, TOMB = erased
    uint32_t child;
  };
  std::vector<Ent> ents;
  uint64_t mask = 0, used = 0;  // used counts erased entries too
  void init(uint64_t expect) {
    const uint64_t cap = pow2_at_least(std::max<uint64_t>(16, expect * 2));
    ents.assign(cap, Ent{0, NONE, 0});
    mask = cap - 1;
    used = 0;
  }
  void grow() {
    std::vector<Ent> old;
    old.swap(ents);
    ents.assign(old.size() * 2, Ent{0, NONE, 0});
    mask = ents.size() - 1;
    used = 0;
    bool ins;
    for (const Ent& e : old)
      if (e.parent != NONE && e.parent != TOMB) *get_or_insert(e.parent, e.tok, ins) = e.child;
  }
  // returns pointer to the child slot; inserted=true if new
  uint32_t* get_or_insert(uint32_t parent, uint64_t tok, bool& inserted) {
    if ((used + 1) * 2 > mask + 1) grow();
    uint64_t i = edge_slot(parent, tok, mask), free_at = ~0ull;
    for (;;) {
      Ent& e = ents[i];
      if (e.parent == parent && e.tok == tok) {
        inserted = false;
        return &e.child;
      }
      if (e.parent == TOMB && free_at == ~0ull) free_at = i;
      if (e.parent == NONE) {
        if (free_at == ~0ull) {
          free_at = i;
          ++used;
        }
        Ent& f = ents[free_at];
        f.parent = parent;
        f.tok = tok;
        inserted = true;
        return &f.child;
      }
      i = (i + 1) & mask;
    }
  }
  uint32_t* find(uint32_t parent, uint64_t tok) {
    if (ents.empty()) return nullptr;
    for (uint64_t i = edge_slot(parent, tok, mask);; i = (i + 1) & mask) {
      Ent& e = ents[i];
      if (e.parent == parent && e.tok == tok) return &e.child;
      if (e.parent == NONE) return nullptr;
    }
  }
  bool erase(uint32_t parent, uint64_t tok) {
    uint32_t* c = find(parent, tok);
    if (!c) return false;
    Ent* e = (Ent*)((uint8_t*)c - offsetof(Ent, child));
    e->parent = TOMB;
    return true;
  }
};

// Level tokens of a filter/topic string, exactly as the device tokenizer computes them.
// is_plus/is_hash flag words that are exactly '+' / '#'; `hashed` = some literal word got a
// hashed token (its trie pairs need byte verification).
void tokenize(const uint8_t* p, uint32_t len, uint64_t test_mask, std::vector<uint64_t>& toks,
              std::vector<uint8_t>& is_plus, std::vector<uint8_t>& is_hash, bool& hashed) {
  toks.clear();
  is_plus.clear();
  is_hash.clear();
  hashed = false;
  uint32_t s = 0;
  for (uint32_t i = 0; i <= len; ++i) {
    if (i == len || p[i] == '/') {
      const uint32_t wl = i - s;
      uint64_t packed = 0, fnv = FNV_OFF;
      for (uint32_t q = 0; q < wl; ++q) {
        if (q < 8) packed |= (uint64_t)p[s + q] << (8 * q);
        fnv = fnv_step(fnv, p[s + q]);
      }
      const bool pl = (wl == 1 && p[s] == '+');
      const bool hs = (wl == 1 && p[s] == '#');
      const uint64_t tok = word_token(packed, fnv, wl, test_mask);
      toks.push_back(tok);
      is_plus.push_back(pl);
      is_hash.push_back(hs);
      if (!pl && !hs && (tok & TOK_HASHED)) hashed = true;
      s = i + 1;
    }
  }
}

struct Filter {
  uint64_t off;
  uint32_t len;
  uint8_t in_trie;
  uint8_t wild;
  uint8_t trie_committed;
  uint8_t route_committed;
  uint32_t route_refs;
  uint32_t sync_gen;  // emqxgm_route_set: the resync generation that last set it present
};

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

// Device buffers freed together.  Epochs share them: consecutive delta commits patch one table
// set in place, and an append-only mirror that outgrows its buffer moves to a new one while the
// epochs still reading the old buffer keep it alive.
struct DevOwner {
  std::vector<DevBuf> bufs;
  DevOwner() = default;
  explicit DevOwner(std::vector<DevBuf>&& b) : bufs(std::move(b)) {}
  DevOwner(const DevOwner&) = delete;
  DevOwner& operator=(const DevOwner&) = delete;
  ~DevOwner() {
    for (auto& b : bufs)
      if (b.p) (void)hipFree(b.p);
  }
};
using OwnerP = std::shared_ptr<DevOwner>;

// One committed index as match passes read it (the reference's committed mria state: readers
// never see a transaction half applied, emqx_router_utils.erl:74-135).  A pass takes the current
// epoch under emqxgm::emu and enqueues every launch that reads the tables before letting go, so a
// later delta commit -- which patches the shared tables in place -- is ordered behind it on the
// GPU (hipStreamWaitEvent on the pass's `done` event); a full build writes new tables and never
// waits for readers at all.
struct Epoch {
  uint64_t id = 0;
  DevIndex ix;
  std::vector<OwnerP> owners;   // tables, fan-out tables, pool mirrors
  hipEvent_t ready = nullptr;   // this epoch's uploads / patches are complete (writer stream)
  // the walk variant its passes need (WalkLevel: shallow LDS stack, deep, deep + spill), learnt
  // by passes whose lanes outgrew a stack; only ever raised
  std::atomic<uint32_t> walk_level{WALK_SHALLOW};
  std::atomic<uint32_t> census_level{WALK_SHALLOW};  // the same for diagnostic census passes
                                                      // (their unpruned walks stack deeper)
  // a topic outgrew the packed staging's rank field (StgFmt): this epoch's passes stage wide
  std::atomic<bool> wide_stage{false};
  mutable std::atomic<bool> ready_seen{false};  // `ready` has completed (passes skip the query)
  // retired by a background build's install: the last epoch on the replaced tables frees
  // gigabytes (hipFree synchronises), so the builder thread frees it, not a subscribe's commit
  bool heavy = false;
  ~Epoch() {
    if (ready) (void)hipEventDestroy(ready);
  }
};
using EpochP = std::shared_ptr<Epoch>;

// A reader's pass resources: scratch, stream, timing events.  One for synchronous calls, one per
// pipelined pass slot (device-resident and host-in/host-out pipes).
struct PassCtx {
  Scratch sc;
  std::vector<DevBuf> bufs;
  hipStream_t stream = nullptr;
  hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};  // start, probe, walk, end, tok
  hipEvent_t done = nullptr;  // recorded after each pass enqueued here (guarded by emqxgm::emu)
  bool done_rec = false;
  EpochP epoch;               // epoch of the pass last enqueued here (kept until it completes)
  bool own_stream = false;    // false: the stream is one of the handle's shared pipe streams
  uint32_t walk_level = 0;    // walk variant of that pass (WalkLevel)
  bool census = false;        // that pass was a census pass
  bool packed = false;        // that pass staged its pairs packed (StgFmt)
  bool pipelined = false;     // a device / host pipe (walks with emqxgm::geom_pipe)
  // copy-through input of the next pass enqueued here (pinned host memory, k_tok's TokArgs);
  // cleared by the enqueue
  const uint8_t* src_bytes = nullptr;
  const uint32_t* src_off = nullptr;
};

constexpr uint64_t DEAD = ~0ull;  // TrieModel::slot of the root and of removed nodes
constexpr uint64_t ROOTH = ~1ull; // TrieModel::slot of the root's fat half (kernel arguments)

// Device writes staged by one commit (k_patch): dword runs to device addresses, uploaded in
// one copy and applied by one launch on the engine stream.
struct PatchList {
  std::vector<PatchEnt> ents;
  std::vector<uint32_t> src;
  void add(void* dst, const void* vals, uint64_t words) {
    const uint32_t* v = (const uint32_t*)vals;
    uint8_t* d = (uint8_t*)dst;
    while (words) {
      const uint32_t w = (uint32_t)std::min<uint64_t>(words, 64);
      ents.push_back(PatchEnt{(uint64_t)(uintptr_t)d, (uint32_t)src.size(), w});
      src.insert(src.end(), v, v + w);
      v += w;
      d += 4ull * w;
      words -= w;
    }
  }
  void clear() {
    ents.clear();
    src.clear();
  }
};

// Host model of the committed trie and exact table, kept so that a commit with a small delta
// patches the device tables in place (commit_delta) instead of rebuilding them.  A slot's 32 B
// are a function of its node's state (node_slot), so only positions and occupancy are mirrored.
struct TrieModel {
  bool valid = false;  // false: the next commit is a full build
  EdgeMap emap;
  // per node (root = 0): hf/tw/tn are NONE, a filter id, or LIST_MULTI | multi[] position
  std::vector<uint32_t> parent, ref, nlit, pchild, hf, tw, tn;
  std::vector<uint8_t> sig;    // gm_common.h sig_bit classes of the node's literal children
  std::vector<uint8_t> hcode;  // depth code (gm_common.h CF_H0/CF_H1): exact at a full build,
                               // only reset to 0 (unbounded) by delta commits
  std::vector<uint64_t> tok;
  std::vector<uint64_t> slot;       // edge slot of the node's incoming edge (DEAD: root/removed,
                                    // ROOTH: the root's fat half, carried in the arguments)
  // fat buckets (gm_common.h FAT_ID): fchild = the node's only literal child when that child's
  // slot is the second half of the node's bucket (the root's: the arguments), else 0; half = the
  // node is such a child
  std::vector<uint32_t> fchild;
  std::vector<uint8_t> half;
  std::vector<uint8_t> keyed;  // the node's children are placed by token (gm_common.h edge_home)
  std::vector<uint64_t> occ, tomb;  // bitmaps over edge slots: used (live or TOMB), TOMB
  uint64_t nbk = 0, ecap = 0, n_occ = 0, n_edges = 0, tn_cap = 0, fv_cap = 0;
  std::vector<uint32_t> fvbits;
  std::vector<uint32_t> multi;  // [count, fid...] lists of nodes shared by several filters
  bool needs_verify = false;
  uint32_t max_depth = 0;
  uint64_t n_trie = 0, n_route = 0;
  uint64_t n_nodes0 = 0, fv_words0 = 0;  // nodes / verify words at the build (headroom used since)
  // exact route keys: entry per committed key, bitmaps over entries.  Two regions of one
  // table: plain (non-wildcard) keys in buckets [0, xcap_p), wildcard keys in [xcap_p,
  // xcap_p + xcap_w); a name can only equal a key of its own kind (same bytes, same words).
  std::vector<uint32_t> xpos;
  std::vector<uint64_t> xocc, xtomb, xovf;  // xovf: a bit per bucket (gm_common.h)
  uint64_t xcap_p = 0, xcap_w = 0, x_occ_p = 0, x_occ_w = 0, n_route_p = 0, n_route_w = 0;
  uint64_t xbase(bool w) const { return w ? xcap_p : 0; }
  uint64_t xcapr(bool w) const { return w ? xcap_w : xcap_p; }
  uint64_t& xoccr(bool w) { return w ? x_occ_w : x_occ_p; }
  uint64_t& nroute(bool w) { return w ? n_route_w : n_route_p; }
  // home bucket of a key hash in its region, and the next bucket of its probe sequence
  uint64_t xhome(bool w, uint64_t fh) const { return xbase(w) + exact_slot(fh, xcapr(w) - 1); }
  uint64_t xnext(bool w, uint64_t b) const {
    return xbase(w) + ((b - xbase(w) + 1) & (xcapr(w) - 1));
  }
  // device tables patched in place (owned by emqxgm::o_tab)
  uint32_t *d_edges = nullptr, *d_exact = nullptr, *d_tn = nullptr, *d_fv = nullptr,
           *d_xovf = nullptr;

  uint32_t cf(uint32_t i) const {  // gm_common.h cf: id | flags
    uint32_t f = i;
    if (nlit[i]) f |= CF_LIT;
    if (pchild[i]) f |= CF_PLUS;
    if (tw[i] != NONE) f |= CF_TW;
    if (tn[i] != NONE) f |= CF_TN;
    return cf_with_depth_code(f, hcode[i]);
  }
  uint32_t hfd(uint32_t i) const { return hf[i]; }  // id, LIST_MULTI | multi index, or NONE
  void node_slot(uint32_t c, uint4* sl) const {  // the 2 x uint4 of c's incoming edge
    const uint32_t p = pchild[c];
    sl[0] = make_uint4((uint32_t)tok[c], (uint32_t)(tok[c] >> 32),
                       (half[c] ? FAT_ID : parent[c]) | ((keyed[c] ? 0u : (uint32_t)sig[c]) << SIG_SHIFT),
                       cf(c));
    sl[1] = make_uint4(hfd(c), tw[c], p ? pcf(p) : 0u, p ? phf(p) : NONE);
  }
  // the carried copy of '+' child p (gm_common.h CF_PTW): its '#' filter, or -- when it has
  // none -- its terminal filters, flagged
  bool ptw(uint32_t p) const { return hf[p] == NONE && tw[p] != NONE; }
  uint32_t pcf(uint32_t p) const { return cf(p) | (ptw(p) ? CF_PTW : 0u); }
  uint32_t phf(uint32_t p) const { return ptw(p) ? tw[p] : hfd(p); }
  uint32_t new_node(uint32_t par, uint64_t t) {
    const uint32_t c = (uint32_t)parent.size();
    parent.push_back(par);
    tok.push_back(t);
    ref.push_back(0);
    nlit.push_back(0);
    pchild.push_back(0);
    hf.push_back(NONE);
    tw.push_back(NONE);
    tn.push_back(NONE);
    hcode.push_back(0);
    sig.push_back(0);
    slot.push_back(DEAD);
    fchild.push_back(0);
    half.push_back(0);
    keyed.push_back(0);
    return c;
  }
  // home bucket of the edge (par, t): a keyed parent's literal children by token, its '+' child
  // (probed by IT_PLUS items, never keyed) like every other edge
  uint64_t home(uint32_t par, uint64_t t) const {
    return edge_home(par, t, nbk - 1, keyed[par] != 0 && t != PLUS_TOK);
  }
  // the root's fat half as the walk's arguments carry it (rh0.z = NONE: none)
  void root_half(DevIndex& x) const {
    uint4 sl[2] = {make_uint4(0u, 0u, NONE, 0u), make_uint4(0u, 0u, 0u, 0u)};
    if (fchild[0]) node_slot(fchild[0], sl);
    x.rh0 = sl[0];
    x.rh1 = sl[1];
  }
  // a filter was added along path[0] = root .. path[m] (its end node; hash_last: a '#' filter
  // hanging off path[m]): a code its ancestors can no longer guarantee is reset to unbounded
  void widen_codes(const std::vector<uint32_t>& path, bool hash_last,
                   std::vector<uint32_t>& dirty) {
    const size_t m = path.size() - 1;
    for (size_t i = 0; i < m; ++i) {
      const uint32_t x = path[i];
      if (hcode[x] && (hash_last || m - i > hcode[x])) {
        hcode[x] = 0;
        dirty.push_back(x);
      }
    }
  }
};

// Host side of the publish fan-out tables (gm_fanout.inc): entries per filter id and the used
// and reserved sizes of the two append-only pools.
struct FanModel {
  bool valid = false;
  uint64_t cap = 0;  // filter ids with an entry (0: no tables)
  uint64_t rt_used = 0, rt_cap = 0, dl_used = 0, dl_cap = 0, garbage = 0;
  std::vector<uint4> ent;
  uint32_t *d_ent = nullptr, *d_rt = nullptr, *d_dl = nullptr;  // owned by emqxgm::o_fan
};

// What a full build reads and how (build_model / upload_tables).  A background build (bg) runs
// on a thread of its own while writers keep changing the registry: it reads the registry in
// slices (for_slices) and records per filter the membership it read (seen: bit 0 trie member,
// bit 1 route key), from which its install replays every change made since (install_build).
struct BuildIn {
  bool bg = false;
  uint64_t nf = 0;           // filters [0, nf) are read
  uint64_t n_trie_hint = 0;  // expected trie members (edge map sizing)
  uint64_t test_mask = 0, fmask = ~0ull;
  uint32_t fat_mode = 1, keyed_mode = 1;
  std::vector<uint8_t>* seen = nullptr;
};

// A full build running beside the writers (r05).  Until its install the readers keep the index
// they have, and commits patch it (delta commits); the install swaps the build's tables in with
// the changes since its start replayed onto them as one more delta.
struct BuildJob {
  BuildIn in;
  std::vector<uint8_t> seen;
  std::vector<uint32_t> covered;  // changes pending at the start: the build includes them
  TrieModel m;
  DevIndex nx;  // its table fields (upload_tables)
  OwnerP o;     // and their buffers
  int rc = 0;
  std::chrono::steady_clock::time_point t0;
  double build_ms = 0;
};

inline bool bit(const std::vector<uint64_t>& b, uint64_t i) { return (b[i >> 6] >> (i & 63)) & 1; }
inline void bset(std::vector<uint64_t>& b, uint64_t i) { b[i >> 6] |= 1ull << (i & 63); }
inline void bclr(std::vector<uint64_t>& b, uint64_t i) { b[i >> 6] &= ~(1ull << (i & 63)); }

}  // namespace

// Device mirror of an append-only host array (filter pool, offsets, verification records).
struct Mirror {
  DevBuf b;
  OwnerP o;              // owns b; epochs that read b hold it too
  uint64_t uploaded = 0; // bytes already on the device
};

// Locking (include/emqx_gpumatch.h "Threading"):
//   wmu  writers: registry mutations and commit (a full build runs under it for seconds);
//   pmu  the registry's storage (pool, filters, slots): writers hold it exclusively only while
//        they grow it, filter_bytes / lookup_id / trie_member read under it shared;
//   emu  the current epoch and the reader streams' done events: a reader holds it while it
//        enqueues a pass, a writer while it orders its patches behind those passes and swaps;
//   mmu  the readers' pass resources (sync context, pipes, geometry): match calls serialise
//        on it among themselves, never against a writer;
//   stmu / errmu  statistics and the last-error string.
struct emqxgm {
  std::mutex wmu, emu, mmu, stmu, errmu;
  std::shared_mutex pmu;
  emqxgm_cfg cfg{};
  // writer stream (patch uploads, k_patch): the sync context's stream.  HIP maps streams onto
  // GPU_MAX_HW_QUEUES (4) hardware queues; a stream of its own pushed a pipe onto a shared queue
  // and serialised the two pipelined passes (profiles/r02: pipelined step 0.374 vs 0.312 ms)
  hipStream_t wstream = nullptr;
  std::string err;

  // ---- registry (pending state) ----
  std::vector<uint8_t> pool;
  std::vector<Filter> filters;
  std::vector<uint32_t> slots;  // id+1, open addressing on string hash
  uint64_t slot_mask = 0;
  uint64_t n_trie_pending = 0, n_route_pending = 0;
  bool dirty = false;
  // emqxgm_route_sync_begin/_end: generation of the resync in progress (0: none)
  uint32_t sync_gen = 0, sync_next = 1;
  // filters whose local subscriber list a set call gave during the resync in progress (bitmap):
  // _end clears every other list (a topic whose subscribers all went is absent from the table
  // the resync scans; its old list must not survive it -- r06, with handle reuse)
  std::vector<uint64_t> sub_seen;

  // ---- the writer's working copy of the committed index (published as epochs) ----
  uint64_t epoch = 0;
  DevIndex ix;
  OwnerP o_tab;  // edge slots, multi lists, tn side array, verify bits, exact table
  Mirror m_pool, m_foff, m_fver;
  std::vector<uint64_t> foff_host;  // [n_filters+1]
  std::vector<uint8_t> fver_host;   // 64 B per filter
  emqxgm_stats st{};

  // ---- what readers see ----
  EpochP cur;                      // current epoch (emu)
  std::atomic<int> cur_trie_empty{1};  // cur->ix.trie_empty, readable without emu (which a
                                       // commit holds across its patch wait)
  std::vector<EpochP> graveyard;   // retired epochs a reader may still hold (swept by writers)

  // ---- reader side (mmu) ----
  PassCtx sync;                    // synchronous calls
  WalkGeom geom;
  // the walk geometry of pipelined passes (device and host pipes: two passes in flight), never
  // wider than geom.  Three workgroups per CU instead of four leave room beside a walk for the
  // other pass's tokenizer and scatter (a walk of four holds ~450 of a SIMD's 512 VGPRs): r04
  // cfg3 pipelined step 0.412 -> 0.403 ms, 9.71 -> 9.93 G topics/s, though the walk alone is
  // slower at three (0.319 -> 0.377 ms; one pass at a time keeps four).  tune "walk_wg_per_cu_pipe"
  WalkGeom geom_pipe;
  uint32_t pipe_wg_per_cu = 3;
  uint32_t leafp_mask = CF_HMASK;  // depth-code pruning (tune "leaf_prune")
  uint64_t census_depth[2 * CENSUS_DEPTHS] = {};  // the last census pass's loads per level
  uint8_t* d_in_bytes = nullptr;
  uint32_t* d_in_off = nullptr;
  uint64_t in_bytes_cap = 0, in_off_cap = 0;

  // ---- host outputs (match_batch: pinned, filled by D2H copies straight from the device) ----
  struct Pinned {
    void* p = nullptr;
    size_t cap = 0;
  };
  Pinned hp_row, hp_fid, hp_exact;
  uint64_t* d_row64 = nullptr;  // device u64 row pointers of one chunk
  uint64_t row64_cap = 0;

  // ---- publish fan-out state (host registry; device tables built at commit) ----
  std::unordered_map<uint32_t, std::vector<std::pair<uint32_t, uint32_t>>> rdest;  // (node, group)
  std::unordered_map<uint32_t, std::vector<uint32_t>> lsubs;  // local subscribers per filter
  uint32_t local_node = NONE;
  FanScratch fs;
  std::vector<DevBuf> fan_bufs, fan_out_bufs;
  std::vector<uint64_t> h_rp, h_dp;
  std::vector<uint32_t> h_rf, h_rd, h_df, h_ds, h_tmp32;

  bool profiling = false;
  uint32_t spill_want = 0;         // walk spill items per lane (grown on overflow)
  uint32_t reject_cap = 1u << 20;  // cfg.reject_cap overrides (tests force the legacy path)
  uint64_t test_mask = 0;          // != 0: collision-test tokens (cfg.word_hash_bits)

  // ---- pipelined device passes (emqxgm_match_device_submit / _wait): each pipe has its own
  // scratch, stream and events, so a batch can be enqueued while the previous one still runs
  // (its walk's tail then overlaps the next batch's tokenizer and walk) ----
  struct Pipe {
    PassCtx c;
    uint64_t ticket = 0;  // last ticket submitted here (0: never)
    int state = 0;        // 0 idle / result taken, 1 in flight, 2 result ready
    const uint8_t* d_bytes = nullptr;
    const uint32_t* d_off = nullptr;
    uint32_t n = 0, pairs = 0;
    uint64_t bytes_len = 0;
  } pipes[EMQXGM_PIPES];
  uint64_t next_ticket = 1;

  // ---- pipelined host passes (emqxgm_match_batch_submit / _wait): the pipe's stream carries the
  // H2D copy of its batch, the pass and the copy of its result into pinned host memory, so one
  // batch's upload, another's pass and a third's download overlap ----
  struct HostPipe {
    PassCtx c;
    uint64_t ticket = 0;
    int state = 0;  // as Pipe
    uint8_t* d_bytes = nullptr;
    uint32_t* d_off = nullptr;
    uint64_t bytes_cap = 0, off_cap = 0;
    uint32_t* h_row = nullptr;  // pinned results: row pointers [n+1], exact ids [n], filter ids
    uint32_t* h_exact = nullptr;
    uint32_t* h_none = nullptr;  // [row_cap] all NONE: the exact ids of a batch without any hit
    bool exact_none = false;
    uint32_t* h_fid = nullptr;
    uint64_t row_cap = 0, fid_cap = 0;  // entries
    uint32_t n = 0, pairs = 0;
    uint64_t bytes_len = 0;
    // emqxgm_match_batch_wait_filters: the pairs' filter bytes gathered on the device
    // ([len | off | scan | total] words, then bytes) and copied into pinned memory
    DevBuf d_fb;
    Pinned h_fboff, h_fb;
    uint64_t fb_bytes = 0;
    // emqxgm_match_batch_submit_filters: the gather and every copy were enqueued behind the
    // pass, sized by the estimates below; the wait then takes one stream synchronisation
    bool fb_async = false;
    bool rows_enq = false;  // the submit enqueued the row pointers' copy into h_row
    bool zc = false;        // this submit's input / result block went without DMA copies
    uint64_t fb_pairs_copy = 0, fb_bytes_copy = 0;  // pairs / bytes the packed block holds
    Pinned h_blk;                                   // the packed block (FbLayout)
    bool fb_fast = false;                           // the last completion came from the block
    double fb_ppt = 0, fb_bpp = 0;                  // pairs per topic, bytes per pair (decaying max)
    // recorded behind everything a submit enqueued: a waiter blocks on it without holding mmu,
    // so other threads keep submitting (and waiting for other tickets) meanwhile
    hipEvent_t fin = nullptr;
  } hpipes[EMQXGM_HOST_PIPES];
  uint64_t next_hticket = 1;
  hipStream_t pipe_streams[EMQXGM_HOST_PIPES] = {};  // pipe_stream(): shared by both pipe kinds
  // results to the host: 0 = hipMemcpyAsync (SDMA; default), 1 = copy kernel writing host
  // memory over PCIe.  Measured on cfg3 (profiles/r02/pcie_e2e.json): 1.24 vs 1.02 G topics/s
  // host-in/host-out -- the kernel's PCIe writes contend with the uploads
  uint32_t host_out_mode = 0;
  // host windows with the filter-byte gather (emqxgm_match_batch_submit_filters: the concurrent
  // entry's, the batcher's) of up to this many topics (and 8 MiB of topic bytes) in pinned memory
  // go without DMA copies: k_tok reads the window itself (copy-through) and k_fb_pack writes the
  // result block into pinned memory (emqxgm_tune "zc_topics"; 0: always DMA)
  uint32_t zc_topics = 65536;
  // a host pipe's wait polls its completion event for up to this long before it blocks in
  // hipEventSynchronize (emqxgm_tune "spin_us"; 0: block at once).  r04: one 16-topic window
  // 67.6 -> 63.0 us, the concurrent entry's 16k windows p50 373 -> 294 us (the waiter -- a
  // completer thread -- burns its core while a window is in flight, up to this long)
  std::atomic<uint32_t> spin_us{200};
  uint64_t xrange_bytes = 0;  // emqxgm_tune("exact_range_kb")
  uint32_t walk_pair_on = 1;  // emqxgm_tune("walk_pair")

  // ---- delta commits (writer side) ----
  TrieModel tm;
  std::vector<uint32_t> changed;  // filter ids whose trie / route-key membership may differ
  FanModel fm;
  std::vector<uint32_t> fan_changed;  // filter ids whose fan-out lists may differ
  bool fan_rebuild = false;           // every filter's lists may differ (local node changed)
  OwnerP o_fan;                       // the fan-out tables
  OwnerP o_fv;                        // a regrown verify-bit array (grow_fv; until a full build)
  PatchList patches;
  DevBuf d_patch;                   // device copy of the staged patch list
  DevBuf d_rules;                   // emqxgm_match_rules inputs and output
  DevBuf d_merge;                   // emqxgm_merge pointer table and scratch
  uint8_t* h_stage = nullptr;       // pinned host staging of the patch list
  uint64_t h_stage_bytes = 0;
  hipEvent_t patch_ev = nullptr;    // the last patch upload + launch
  uint32_t delta_mode = 1;        // 0: always rebuild, 1: delta when small, 2: delta if possible
  uint64_t delta_max = 0;         // "small": changes per delta (tune "delta_max"; 0: max(4096, n/8))
  uint32_t fat_mode = 1;          // 1: fat buckets at full builds (gm_common.h FAT_ID), 0: none
  uint32_t keyed_mode = 1;        // token-keyed parents at full builds (select_keyed): 0 / 1 / 2
  bool roctx = false;             // roctx ranges / launch markers (gm_roctx.h)

  // ---- background full builds (r05; wmu) ----
  std::unique_ptr<BuildJob> job;   // in flight (installed by its own thread when done)
  std::thread builder;             // its thread (joined before the next one starts)
  std::condition_variable bcv;     // a job was installed
  uint64_t builds_started = 0, builds_done = 0;
  int build_rc = 0;                // the last install's result
  std::vector<uint32_t> build_log; // filters whose membership changed since the job started
  // full builds of registries of at least this many filters run in the background (tune
  // "bg_build"; 0: never): a commit the current tables cannot take waits for the build, every
  // other commit meanwhile is a delta on the index the readers have
  uint64_t bg_min = 16384;
  std::atomic<uint32_t> bg_delay_ms{0};
  // synchronous sets (EMQXGM_SET_COMMIT) waiting for the writer lock: a bulk set lets them in
  // between two of its slices (sync_lock / let_prio_in)
  std::atomic<uint32_t> prio_waiting{0};  // tune "bg_delay_ms": a build holds its install back (tests)

  // ---- health (r06, SURVEY 5 "Failure detection"; hmu): a failed commit, a set that failed
  // half-way, or the host's report of a timeout marks the index STALE -- it may lack a change the
  // caller's tables already hold -- and every match entry refuses with -ESTALE (the caller takes
  // the reference's path) until a repair: a successful emqxgm_commit (after a full resync begun
  // after the last mark, when a mark asked for one) and a probe of the device's streams ----
  std::mutex hmu;
  std::atomic<uint32_t> stale{0};  // EMQXGM_STALE_* bits
  uint64_t stale_seq = 0;          // marks so far
  uint64_t resync_from = 0;        // stale_seq at the last emqxgm_route_sync_begin
  uint64_t resynced = ~0ull;       // stale_seq the last completed resync covers (~0: none)
  int32_t stale_err = 0;           // the last mark's errno (negative)
  std::atomic<uint64_t> refused{0};
  uint64_t repairs = 0;
  uint32_t probe_ms = 2000;        // the repair's bounded wait on the streams (tune "probe_ms")
  // fault injection (tune "fail_commits" / "fail_errno" / "hang_ms"): the next n commits fail
  // before they touch anything; host-pipe waits and publish passes stall this long first
  std::atomic<int64_t> inject_commits{0};
  std::atomic<int32_t> inject_errno{EIO};
  std::atomic<uint32_t> hang_ms{0};
  // packed staging's rank field capped at this many bits (tune "stage_rank_bits", tests of the
  // wide redo; 0: as many as fit)
  std::atomic<uint32_t> stage_rank_bits{0};
};

namespace {

void set_err(emqxgm* h, std::string msg) {
  std::lock_guard<std::mutex> g(h->errmu);
  h->err = std::move(msg);
}

int fail(emqxgm* h, hipError_t e, const char* what) {
  set_err(h, std::string(what) + ": " + hipGetErrorString(e));
  return -EIO;
}

#define HIPCHK(h, expr)                          \
  do {                                           \
    hipError_t _e = (expr);                      \
    if (_e != hipSuccess) return fail(h, _e, #expr); \
  } while (0)

// ---- health (emqxgm::stale) ----
void mark_stale(emqxgm* h, uint32_t bits, int err) {
  std::lock_guard<std::mutex> g(h->hmu);
  h->stale.fetch_or(bits, std::memory_order_seq_cst);
  h->stale_seq += 1;
  h->stale_err = err;
}

// -ESTALE for a match entry while the index is stale (counted), else 0
int refuse_stale(emqxgm* h) {
  if (h->stale.load(std::memory_order_acquire) == 0) return 0;
  h->refused.fetch_add(1, std::memory_order_relaxed);
  set_err(h, "the device index is stale (a failed commit or a timeout): repair it with a resync "
             "and emqxgm_commit; callers take the reference path meanwhile");
  return -ESTALE;
}

// The injected failure of a commit (tune "fail_commits"), before it touches anything
int injected(emqxgm* h) {
  if (h->inject_commits.load(std::memory_order_relaxed) <= 0) return 0;
  if (h->inject_commits.fetch_sub(1) <= 0) return 0;
  set_err(h, "injected commit failure (tune fail_commits)");
  return -h->inject_errno.load(std::memory_order_relaxed);
}

// tune "hang_ms": a host-pipe wait or a publish pass stalls first (tests: a window that does
// not complete within the caller's timeout)
void injected_hang(emqxgm* h) {
  if (const uint32_t ms = h->hang_ms.load(std::memory_order_relaxed))
    std::this_thread::sleep_for(std::chrono::milliseconds(ms));
}

uint64_t str_hash(const uint8_t* p, uint32_t len) {
  uint64_t x = FNV_OFF;
  for (uint32_t i = 0; i < len; ++i) x = fnv_step(x, p[i]);
  return fmix64(x);
}

// The 32-B exact-table entry of a route key (gm_common.h "Exact route-key table").
void xent(uint64_t fh, uint32_t id, const uint8_t* p, uint32_t len, uint4 e[XENT_U4]) {
  uint32_t w[5] = {0, 0, 0, 0, 0};
  memcpy(w, p, std::min<uint32_t>(len, XINL));
  e[0] = make_uint4((uint32_t)(fh >> 32), id, len, w[0]);
  e[1] = make_uint4(w[1], w[2], w[3], w[4]);
}

bool is_wild(const uint8_t* p, uint32_t len) {  // emqx_topic:wildcard/1
  uint32_t s = 0;
  for (uint32_t i = 0; i <= len; ++i) {
    if (i == len || p[i] == '/') {
      if (i - s == 1 && (p[s] == '+' || p[s] == '#')) return true;
      s = i + 1;
    }
  }
  return false;
}

void slots_grow(emqxgm* h) {
  // at least twice the registered filters (a snapshot load re-indexes them all at once)
  const uint64_t cap = std::max<uint64_t>(
      std::max<uint64_t>(1024, (h->slot_mask + 1) * 2), pow2_at_least(4 * h->filters.size()));
  std::vector<uint32_t> ns(cap, 0);
  for (uint32_t id = 0; id < h->filters.size(); ++id) {
    const Filter& f = h->filters[id];
    uint64_t i = str_hash(h->pool.data() + f.off, f.len) & (cap - 1);
    while (ns[i]) i = (i + 1) & (cap - 1);
    ns[i] = id + 1;
  }
  h->slots.swap(ns);
  h->slot_mask = cap - 1;
}

// Find or (if create) register a filter string; returns id or NONE.
uint32_t find_id(emqxgm* h, const uint8_t* p, uint32_t len, bool create) {
  if (h->slots.empty()) {
    if (!create) return NONE;
    slots_grow(h);
  }
  if (create && (h->filters.size() + 1) * 2 > h->slot_mask + 1) slots_grow(h);
  uint64_t i = str_hash(p, len) & h->slot_mask;
  for (;;) {
    const uint32_t v = h->slots[i];
    if (v == 0) break;
    const Filter& f = h->filters[v - 1];
    if (f.len == len && memcmp(h->pool.data() + f.off, p, len) == 0) return v - 1;
    i = (i + 1) & h->slot_mask;
  }
  if (!create) return NONE;
  const uint32_t id = (uint32_t)h->filters.size();
  Filter f;
  f.off = h->pool.size();
  f.len = len;
  f.in_trie = 0;
  f.trie_committed = 0;
  f.route_committed = 0;
  f.wild = is_wild(p, len) ? 1 : 0;
  f.route_refs = 0;
  f.sync_gen = 0;
  h->pool.insert(h->pool.end(), p, p + len);
  h->filters.push_back(f);
  h->slots[i] = id + 1;
  return id;
}

template <class T>
int dev_upload(emqxgm* h, std::vector<DevBuf>& keep, const std::vector<T>& v, const T** out) {
  DevBuf b;
  b.bytes = std::max<size_t>(sizeof(T), v.size() * sizeof(T));
  HIPCHK(h, hipMalloc(&b.p, b.bytes));
  keep.push_back(b);
  // in 64-MiB pieces: a background build uploads gigabytes, and the small copies of the commits
  // and passes running meanwhile queue on the same copy engines -- between pieces, not behind
  // a whole table
  constexpr size_t PIECE = 64ull << 20;
  const size_t total = v.size() * sizeof(T);
  for (size_t o = 0; o < total; o += PIECE)
    HIPCHK(h, hipMemcpy((uint8_t*)b.p + o, (const uint8_t*)v.data() + o, std::min(PIECE, total - o),
                        hipMemcpyHostToDevice));
  *out = (const T*)b.p;
  return 0;
}

void free_bufs(std::vector<DevBuf>& v) {
  for (auto& b : v)
    if (b.p) (void)hipFree(b.p);
  v.clear();
}

// Node-level filter list during the build: NONE, a single fid, or LIST_MULTI|index.
struct ListBuild {
  std::vector<std::vector<uint32_t>> lists;
  void add(uint32_t& slot, uint32_t fid) {
    if (slot == NONE) {
      slot = fid;
    } else if (slot & LIST_MULTI) {
      lists[slot & ~LIST_MULTI].push_back(fid);
    } else {
      lists.push_back({slot, fid});
      slot = LIST_MULTI | (uint32_t)(lists.size() - 1);
    }
  }
};

int patch_wait(emqxgm* h);

// Grow-and-append a device mirror of an append-only host array (bytes [uploaded, total)).
// Without growth and with a patch list, the new tail (whole dwords) goes into the list.  Readers
// of committed epochs only read the prefix those epochs knew, so the tail is written while they
// run; a grown mirror moves to a new buffer and the epochs holding the old one keep it.
// A mirror regrown to hold `need` bytes with headroom (half again, at least 1 MiB, or double):
// a new buffer holding [0, uploaded).  A synchronous allocation and device copy (a ~1 GB mirror at
// cfg3: milliseconds), so it runs at full builds and on the commit paths off the hook
// (grow_ahead), never -- while the headroom lasts -- inside a subscribe.
int mirror_grow(emqxgm* h, Mirror& m, uint64_t need) {
  if (int rc = patch_wait(h)) return rc;  // earlier patches into the old buffer have landed
  DevBuf nb;
  nb.bytes = std::max<uint64_t>(need + std::max<uint64_t>(need / 2, 1u << 20), m.b.bytes * 2);
  nb.bytes = (nb.bytes + 15) & ~15ull;
  HIPCHK(h, hipMalloc(&nb.p, nb.bytes));
  auto o = std::make_shared<DevOwner>();
  o->bufs.push_back(nb);
  if (m.uploaded) HIPCHK(h, hipMemcpy(nb.p, m.b.p, m.uploaded, hipMemcpyDeviceToDevice));
  m.b = nb;
  m.o = std::move(o);  // the old buffer lives on with the epochs that read it
  std::lock_guard<std::mutex> g(h->stmu);
  h->st.buffer_grows += 1;
  return 0;
}

int append_upload(emqxgm* h, Mirror& m, const void* src, uint64_t total, PatchList* pl) {
  DevBuf& buf = m.b;
  uint64_t& uploaded = m.uploaded;
  const uint64_t need = std::max<uint64_t>(16, (total + 3) & ~3ull);
  if (need > buf.bytes) {
    if (int rc = mirror_grow(h, m, need)) return rc;
    pl = nullptr;
  }
  if (total > uploaded) {
    if (pl) {
      const uint64_t a = uploaded & ~3ull;
      std::vector<uint32_t> tmp((total - a + 3) / 4, 0u);
      memcpy(tmp.data(), (const uint8_t*)src + a, total - a);
      pl->add((uint8_t*)buf.p + a, tmp.data(), tmp.size());
    } else {
      HIPCHK(h, hipMemcpy((uint8_t*)buf.p + uploaded, (const uint8_t*)src + uploaded,
                          total - uploaded, hipMemcpyHostToDevice));
    }
  }
  uploaded = total;
  return 0;
}

// Upload the staged patch list: one copy through pinned memory and one k_patch launch on the
// writer stream (publish_epoch orders it behind the passes already enqueued and every later pass
// behind it).  patch_wait() before the staging is reused or a patched buffer is freed.
int patch_wait(emqxgm* h) {
  if (h->patch_ev) HIPCHK(h, hipEventSynchronize(h->patch_ev));
  return 0;
}

constexpr uint64_t PATCH_STAGE0 = 4ull << 20;  // patch staging at create (pinned and device)

int patch_flush(emqxgm* h) {
  PatchList& pl = h->patches;
  if (pl.ents.empty()) return 0;
  int rc = patch_wait(h);
  if (rc) return rc;
  const uint64_t eb = pl.ents.size() * sizeof(PatchEnt), total = eb + pl.src.size() * 4;
  if (total > h->h_stage_bytes) {
    if (h->h_stage) (void)hipHostFree(h->h_stage);
    h->h_stage = nullptr;
    h->h_stage_bytes = 0;
    const uint64_t bytes = std::max<uint64_t>(total * 2, 1u << 16);
    HIPCHK(h, hipHostMalloc((void**)&h->h_stage, bytes, hipHostMallocDefault));
    h->h_stage_bytes = bytes;
  }
  if (total > h->d_patch.bytes) {
    if (h->d_patch.p) (void)hipFree(h->d_patch.p);
    h->d_patch = DevBuf();
    const uint64_t bytes = std::max<uint64_t>(total * 2, 1u << 16);
    HIPCHK(h, hipMalloc(&h->d_patch.p, bytes));
    h->d_patch.bytes = bytes;
  }
  memcpy(h->h_stage, pl.ents.data(), eb);
  memcpy(h->h_stage + eb, pl.src.data(), pl.src.size() * 4);
  HIPCHK(h, hipMemcpyAsync(h->d_patch.p, h->h_stage, total, hipMemcpyHostToDevice, h->wstream));
  HIPCHK(h, launch_patch((const PatchEnt*)h->d_patch.p, (uint32_t)pl.ents.size(),
                         (const uint32_t*)((uint8_t*)h->d_patch.p + eb), h->wstream));
  if (!h->patch_ev) HIPCHK(h, hipEventCreateWithFlags(&h->patch_ev, hipEventDisableTiming));
  HIPCHK(h, hipEventRecord(h->patch_ev, h->wstream));
  pl.clear();
  return 0;
}

// Filter string pool, offsets and 64-B verification records: append-only device mirrors
// (pl: stage the appended tails in a delta commit's patch list).
int upload_pool(emqxgm* h, PatchList* pl) {
  const uint64_t nf = h->filters.size();
  if (h->foff_host.empty()) h->foff_host.push_back(0);
  for (uint64_t i = h->foff_host.size() - 1; i < nf; ++i)  // pool is append-only
    h->foff_host.push_back(h->filters[i].off + h->filters[i].len);
  for (uint64_t i = h->fver_host.size() / VREC; i < nf; ++i) {
    const Filter& f = h->filters[i];
    uint8_t r[VREC] = {0};
    memcpy(r, &f.len, 4);
    memcpy(r + 4, h->pool.data() + f.off, std::min<uint32_t>(f.len, VINL));
    h->fver_host.insert(h->fver_host.end(), r, r + VREC);
  }
  int rc = 0;
  if ((rc = append_upload(h, h->m_pool, h->pool.data(), h->pool.size(), pl)) ||
      (rc = append_upload(h, h->m_foff, h->foff_host.data(),
                          h->foff_host.size() * sizeof(uint64_t), pl)) ||
      (rc = append_upload(h, h->m_fver, h->fver_host.data(), h->fver_host.size(), pl)))
    return rc;
  h->ix.fbytes = (const uint8_t*)h->m_pool.b.p;
  h->ix.foff = (const uint64_t*)h->m_foff.b.p;
  h->ix.fver = (const uint4*)h->m_fver.b.p;
  return 0;
}

// Publish fan-out lists of one filter id (gm_fanout.inc): its aggre/1 entries (plain node
// dests, then each group once: emqx_broker.erl:284-300) and, when it routes to the local node,
// its local subscribers (dispatch/2, :326-355).
void fan_lists(emqxgm* h, uint32_t id, std::vector<uint32_t>& rt, std::vector<uint32_t>& dl,
               std::vector<uint32_t>& groups) {
  auto it = h->rdest.find(id);
  if (it == h->rdest.end()) return;
  bool local = false;
  groups.clear();
  for (const auto& d : it->second) {
    if (d.second == NONE) {
      rt.push_back(d.first);
      local = local || d.first == h->local_node;
    } else {
      groups.push_back(EMQXGM_DEST_GROUP | d.second);
    }
  }
  std::sort(groups.begin(), groups.end());
  groups.erase(std::unique(groups.begin(), groups.end()), groups.end());
  rt.insert(rt.end(), groups.begin(), groups.end());
  if (local) {
    auto sit = h->lsubs.find(id);
    if (sit != h->lsubs.end()) dl.insert(dl.end(), sit->second.begin(), sit->second.end());
  }
}

// Full build of the fan-out tables: entries for every filter id (with headroom for new ids)
// and both pools packed (with headroom for delta appends).
int fan_full(emqxgm* h) {
  const uint64_t nf = h->filters.size();
  FanModel& m = h->fm;
  m = FanModel();
  DevIndex& ix = h->ix;
  std::vector<DevBuf> nb;
  if (!h->rdest.empty() || !h->lsubs.empty()) {
    m.cap = nf + std::max<uint64_t>(4096, nf / 4);
    m.ent.assign(m.cap, make_uint4(0u, 0u, 0u, 0u));
    std::vector<uint32_t> rt, dl, groups;
    for (uint32_t id = 0; id < nf; ++id) {
      const uint32_t r0 = (uint32_t)rt.size(), d0 = (uint32_t)dl.size();
      fan_lists(h, id, rt, dl, groups);
      m.ent[id] = make_uint4(r0, (uint32_t)rt.size() - r0, d0, (uint32_t)dl.size() - d0);
    }
    m.rt_used = rt.size();
    m.dl_used = dl.size();
    m.rt_cap = m.rt_used + std::max<uint64_t>(16384, m.rt_used / 4);
    m.dl_cap = m.dl_used + std::max<uint64_t>(16384, m.dl_used / 4);
    if (m.rt_cap >= 0xFFFFFFFFull || m.dl_cap >= 0xFFFFFFFFull) {
      set_err(h, "fan-out pools exceed 2^32 entries");
      return -E2BIG;
    }
    rt.resize(m.rt_cap, 0u);
    dl.resize(m.dl_cap, 0u);
    DevIndex t;
    int rc = 0;
    if ((rc = dev_upload(h, nb, m.ent, &t.fan)) || (rc = dev_upload(h, nb, rt, &t.rt_dst)) ||
        (rc = dev_upload(h, nb, dl, &t.dl_sub))) {
      free_bufs(nb);
      return rc;
    }
    ix.fan = t.fan;
    ix.rt_dst = t.rt_dst;
    ix.dl_sub = t.dl_sub;
    m.d_ent = (uint32_t*)t.fan;
    m.d_rt = (uint32_t*)t.rt_dst;
    m.d_dl = (uint32_t*)t.dl_sub;
  } else {
    ix.fan = nullptr;
    ix.rt_dst = ix.dl_sub = nullptr;
  }
  ix.fan_nf = (uint32_t)m.cap;
  h->o_fan = std::make_shared<DevOwner>(std::move(nb));  // the old tables live on with their epochs
  h->fan_changed.clear();
  h->fan_rebuild = false;
  m.valid = true;
  return 0;
}

// Fan-out tables after a registry change: a changed filter's lists are appended to the pools
// and its entry re-pointed (k_patch); a full build when the tables are absent, an id or a pool
// passes its headroom, stale entries pass half the pools, or the local node changed.
int fan_commit(emqxgm* h) {
  FanModel& m = h->fm;
  auto& ch = h->fan_changed;
  if (!m.valid || h->fan_rebuild || (m.cap == 0 && !ch.empty())) return fan_full(h);
  if (ch.empty()) return 0;
  std::sort(ch.begin(), ch.end());
  ch.erase(std::unique(ch.begin(), ch.end()), ch.end());
  std::vector<uint32_t> rt, dl, groups, changed;
  uint64_t garbage = m.garbage;
  for (uint32_t id : ch) {
    if (id >= m.cap) return fan_full(h);
    const uint32_t r0 = (uint32_t)rt.size(), d0 = (uint32_t)dl.size();
    fan_lists(h, id, rt, dl, groups);
    const uint4 old = m.ent[id];
    garbage += old.y + old.w;
    const uint4 e = make_uint4((uint32_t)(m.rt_used + r0), (uint32_t)rt.size() - r0,
                               (uint32_t)(m.dl_used + d0), (uint32_t)dl.size() - d0);
    m.ent[id] = e;
    changed.push_back(id);
  }
  if (m.rt_used + rt.size() > m.rt_cap || m.dl_used + dl.size() > m.dl_cap ||
      garbage * 2 > m.rt_used + m.dl_used + 65536)
    return fan_full(h);
  PatchList& pl = h->patches;
  pl.add(m.d_rt + m.rt_used, rt.data(), rt.size());
  pl.add(m.d_dl + m.dl_used, dl.data(), dl.size());
  for (uint32_t id : changed) pl.add(m.d_ent + 4ull * id, &m.ent[id], 4);
  m.rt_used += rt.size();
  m.dl_used += dl.size();
  m.garbage = garbage;
  ch.clear();
  return 0;
}

void commit_stats(emqxgm* h, double ms, bool delta) {
  const TrieModel& m = h->tm;
  std::lock_guard<std::mutex> g(h->stmu);
  h->st.epoch = h->epoch;
  h->st.n_filters = h->filters.size();
  h->st.n_trie_filters = m.n_trie;
  h->st.n_route_keys = m.n_route;
  h->st.n_nodes = m.n_edges + 1;
  h->st.n_edges = m.n_edges;
  h->st.edge_slots = m.ecap;
  // keyed flags are chosen by full builds only (a delta's new nodes are never keyed); counting
  // them is O(nodes), 2 ms at cfg3, so a delta commit keeps the count
  if (!delta) h->st.keyed_nodes = (uint64_t)std::count(m.keyed.begin(), m.keyed.end(), (uint8_t)1);
  h->st.exact_slots = (m.xcap_p + m.xcap_w) * XBUCKET;
  h->st.max_depth = m.max_depth;
  h->st.device_bytes = m.ecap * SLOT_U4 * 16 + (m.xcap_p + m.xcap_w) * XBUCKET * XENT_U4 * 16 + m.tn_cap * 4 +
                       m.fv_cap * 4 + h->pool.size() + (h->filters.size() + 1) * 8 +
                       h->filters.size() * VREC;
  h->st.last_commit_ms = ms;
  (delta ? h->st.delta_commits : h->st.full_commits) += 1;
}

// f(i0, i1, filters, pool) over the registered filters [0, n) in slices.  A background build
// (bg) reads the registry while writers change it: it holds the registry lock shared for one
// slice at a time and, before each slice, takes and drops the writer lock, so that a writer
// waiting for either gets in first -- a subscribe waits for at most one slice, never for the
// build.  (A filter's bytes, offset and length never change once registered; its membership
// flags only change under the registry lock held exclusively.)
//
// The slice is copied out under the locks -- its records and their bytes, offsets rebased -- and
// f works on the copy after they are released: f's own work (tokenising, growing the model's
// node arrays and hash map: a reallocation of a 10M-entry array takes ~100 ms) never holds a
// writer (r05: synchronous sets waited up to 91 ms for the registry lock).  f(i0, i1, F, pool):
// filter id is F[id - i0], its bytes pool + F[id - i0].off.
constexpr uint64_t REG_SLICE = 1024;
template <class F>
void for_slices(emqxgm* h, bool bg, uint64_t n, F f) {
  std::vector<Filter> lf;
  std::vector<uint8_t> lp;
  for (uint64_t i0 = 0; i0 < n; i0 += REG_SLICE) {
    const uint64_t i1 = std::min<uint64_t>(n, i0 + REG_SLICE);
    if (!bg) {
      f(i0, i1, h->filters.data() + i0, h->pool.data());
      continue;
    }
    {
      { std::lock_guard<std::mutex> w(h->wmu); }
      std::shared_lock<std::shared_mutex> g(h->pmu);
      lf.assign(h->filters.begin() + i0, h->filters.begin() + i1);
      lp.clear();
      for (Filter& x : lf) {
        const uint64_t o = lp.size();
        lp.insert(lp.end(), h->pool.data() + x.off, h->pool.data() + x.off + x.len);
        x.off = o;
      }
    }
    f(i0, i1, lf.data(), lp.data());
  }
}

// f(F, pool) with the registry readable (a background build takes and drops the writer lock
// first, then holds the registry lock shared): for short reads of arbitrary ids.
template <class F>
void with_registry(emqxgm* h, bool bg, F f) {
  std::shared_lock<std::shared_mutex> g(h->pmu, std::defer_lock);
  if (bg) {
    { std::lock_guard<std::mutex> w(h->wmu); }
    g.lock();
  }
  f(h->filters.data(), h->pool.data());
}

// The device tables of a host model (its node slots, side array, verify bits, exact entries,
// overflow bits, multi lists): generated from the model -- a full build and a snapshot load
// share this -- and uploaded into a new table set: nx's table fields, o its buffers (the caller
// swaps them in; nx's pool and fan-out fields are left as they are).
int upload_tables(emqxgm* h, const BuildIn& in, TrieModel& m, DevIndex& nx, OwnerP& o) {
  const uint64_t n_nodes = m.parent.size();
  std::vector<uint4> eslots(SLOT_U4 * m.ecap, make_uint4(0u, 0u, 0u, 0u));
  for (uint64_t i = 0; i < m.ecap; ++i)
    eslots[SLOT_U4 * i] = make_uint4(0u, 0u, bit(m.tomb, i) ? TOMB : NONE, 0u);
  for (uint32_t c = 1; c < n_nodes; ++c)
    if (m.slot[c] != DEAD && m.slot[c] != ROOTH) m.node_slot(c, &eslots[SLOT_U4 * m.slot[c]]);
  std::vector<uint32_t> tn_of(m.tn_cap, NONE);
  for (size_t i = 0; i < n_nodes; ++i) tn_of[i] = m.tn[i];
  const uint64_t fmask = in.fmask;
  const uint64_t xcap = m.xcap_p + m.xcap_w;
  std::vector<uint4> xslots(xcap * XBUCKET * XENT_U4, make_uint4(0u, 0u, 0u, 0u));
  for (uint64_t e = 0; e < xcap * XBUCKET; ++e) xslots[XENT_U4 * e].y = bit(m.xtomb, e) ? TOMB : NONE;
  for_slices(h, in.bg, m.xpos.size(), [&](uint64_t i0, uint64_t i1, const Filter* F, const uint8_t* pool) {
    for (uint64_t id = i0; id < i1; ++id) {
      if (m.xpos[id] == NONE) continue;
      const Filter& f = F[id - i0];
      const uint8_t* p = pool + f.off;
      xent(key_hash(p, f.len, fmask), (uint32_t)id, p, f.len, &xslots[XENT_U4 * (uint64_t)m.xpos[id]]);
    }
  });
  std::vector<DevBuf> nbufs;
  int rc = 0;
  if ((rc = dev_upload(h, nbufs, eslots, &nx.edges)) ||
      (rc = dev_upload(h, nbufs, m.multi, &nx.multi)) ||
      (rc = dev_upload(h, nbufs, tn_of, &nx.tn_of)) ||
      (rc = dev_upload(h, nbufs, m.fvbits, &nx.fvbits)) ||
      (rc = dev_upload(h, nbufs, xslots, &nx.exact)) ||
      (rc = dev_upload(h, nbufs, m.xovf, (const uint64_t**)&nx.xovf))) {
    free_bufs(nbufs);
    return rc;
  }
  m.d_edges = (uint32_t*)nx.edges;
  m.d_exact = (uint32_t*)nx.exact;
  m.d_tn = (uint32_t*)nx.tn_of;
  m.d_fv = (uint32_t*)nx.fvbits;
  m.d_xovf = (uint32_t*)nx.xovf;
  nx.emask = m.nbk - 1;
  nx.xmask = m.xcap_p - 1;
  nx.xwbase = m.xcap_p;
  nx.xwmask = m.xcap_w - 1;
  const uint32_t root_p = m.pchild[0];
  nx.root_cf = m.cf(0);
  nx.root_sig = m.sig[0];
  nx.root_hf = m.hfd(0);
  nx.root_pcf = root_p ? m.pcf(root_p) : 0u;
  nx.root_phf = root_p ? m.phf(root_p) : NONE;
  m.root_half(nx);
  nx.test_mask = in.test_mask;
  nx.needs_verify = m.needs_verify;
  nx.full_mask = fmask;
  nx.max_depth = m.max_depth;
  nx.fid_bound = (uint64_t)m.fv_cap * 32;
  nx.trie_empty = (m.n_trie == 0);
  nx.plain_empty = (m.n_route_p == 0);
  nx.wild_empty = (m.n_route_w == 0);
  o = std::make_shared<DevOwner>(std::move(nbufs));
  return 0;
}

// The table fields of `from` into `to` (its pool and fan-out fields stay).
void set_tables(DevIndex& to, const DevIndex& from) {
  DevIndex x = from;
  x.fan = to.fan;
  x.rt_dst = to.rt_dst;
  x.dl_sub = to.dl_sub;
  x.fan_nf = to.fan_nf;
  x.fbytes = to.fbytes;
  x.foff = to.foff;
  x.fver = to.fver;
  x.leafp_mask = to.leafp_mask;
  to = x;
}

BuildIn build_in(emqxgm* h, bool bg) {
  BuildIn in;
  in.bg = bg;
  in.nf = h->filters.size();
  in.n_trie_hint = h->n_trie_pending;
  in.test_mask = h->test_mask;
  in.fmask = h->cfg.full_hash_bits >= 64 ? ~0ull : ((1ull << h->cfg.full_hash_bits) - 1ull);
  in.fat_mode = h->fat_mode;
  in.keyed_mode = h->keyed_mode;
  return in;
}

// The tables of model m uploaded and swapped into the writer's index (the old ones live on with
// the epochs that read them): a blocking full build and a snapshot load.
int upload_model(emqxgm* h, TrieModel& m) {
  DevIndex nx = h->ix;
  OwnerP o;
  if (int rc = upload_tables(h, build_in(h, false), m, nx, o)) return rc;
  h->o_tab = std::move(o);
  h->o_fv.reset();  // (the new tables have their own verify bits)
  h->ix = nx;
  return 0;
}

// Token-keyed parents (gm_common.h edge_home) of a full build.  mode 1: parents with at least
// KEYED_MIN_FANOUT literal children, none of whose child tokens is the child of more than
// KEYED_MAX_SHARE candidates and at most 1/16 of them of more than EBUCKET (their edges then
// share one bucket per token; the few crowded tokens only lengthen their own chains -- on cfg3 the
// device ids 0..9999 are also site numbers, children of `site`); mode 2 (tests): every eligible
// parent; 0: none.  Never the root or a node reached by a '+' edge.
constexpr uint32_t KEYED_MIN_FANOUT = 16;
constexpr uint32_t KEYED_MAX_SHARE = 8;
void select_keyed(TrieModel& m, uint32_t mode) {
  const size_t nn = m.parent.size();
  m.keyed.assign(nn, 0u);
  if (mode == 0) return;
  auto eligible = [&](uint32_t x) {
    return x != 0 && m.tok[x] != PLUS_TOK && m.nlit[x] > 0 &&
           (mode == 2 || m.nlit[x] >= KEYED_MIN_FANOUT);
  };
  if (mode == 2) {
    for (uint32_t x = 1; x < nn; ++x) m.keyed[x] = eligible(x) ? 1 : 0;
    return;
  }
  // child tokens of the candidates, counted by sorting
  std::vector<uint64_t> toks;
  for (uint32_t c = 1; c < nn; ++c)
    if (m.tok[c] != PLUS_TOK && eligible(m.parent[c])) toks.push_back(m.tok[c]);
  if (toks.empty()) return;
  std::sort(toks.begin(), toks.end());
  std::vector<std::pair<uint64_t, uint32_t>> crowded;  // tokens under more than EBUCKET candidates
  for (size_t i = 0; i < toks.size();) {
    size_t j = i;
    while (j < toks.size() && toks[j] == toks[i]) ++j;
    if (j - i > EBUCKET) crowded.emplace_back(toks[i], (uint32_t)std::min<size_t>(j - i, ~0u));
    i = j;
  }
  std::vector<uint32_t> n_crowded(nn, 0);
  std::vector<uint8_t> ok(nn, 0);
  for (uint32_t x = 1; x < nn; ++x) ok[x] = eligible(x) ? 1 : 0;
  for (uint32_t c = 1; c < nn; ++c) {
    const uint32_t p = m.parent[c];
    if (!ok[p] || m.tok[c] == PLUS_TOK) continue;
    auto it = std::lower_bound(crowded.begin(), crowded.end(), std::make_pair(m.tok[c], 0u));
    if (it == crowded.end() || it->first != m.tok[c]) continue;
    if (it->second > KEYED_MAX_SHARE) ok[p] = 0;
    else n_crowded[p] += 1;
  }
  for (uint32_t x = 1; x < nn; ++x) m.keyed[x] = ok[x] && n_crowded[x] * 16 <= m.nlit[x];
}

// The host model (TrieModel) of a full build of the registry's filters [0, in.nf): trie nodes,
// edge-slot placement, exact-key placement.  No device work; a background build runs it beside
// the writers (in.bg, for_slices).
int build_model(emqxgm* h, const BuildIn& in, TrieModel& m) {
  const uint64_t test_mask = in.test_mask;
  const uint64_t fmask = in.fmask;
  const uint64_t nf = in.nf;

  // ---- trie: nodes keyed by (parent, level token); root = node 0 ----
  m.new_node(NONE, 0);
  m.emap.init(std::max<uint64_t>(1024, in.n_trie_hint * 2));
  ListBuild lb;
  m.fvbits.assign((nf + 31) / 32 + 1, 0u);
  std::vector<uint64_t> toks;
  std::vector<uint8_t> is_plus, is_hash;
  int rc = 0;
  for_slices(h, in.bg, nf, [&](uint64_t i0, uint64_t i1, const Filter* F, const uint8_t* pool) {
    for (uint64_t i = i0; i < i1 && !rc; ++i) {
      const uint32_t id = (uint32_t)i;
      const Filter& f = F[i - i0];
      if (in.seen) (*in.seen)[id] = f.in_trie ? 1 : 0;
      if (!f.in_trie) continue;
      ++m.n_trie;
      bool hashed;
      tokenize(pool + f.off, f.len, test_mask, toks, is_plus, is_hash, hashed);
      if (hashed) {
        m.fvbits[id >> 5] |= 1u << (id & 31);
        m.needs_verify = true;
      }
      const size_t nw = toks.size();
      const bool hash_last = is_hash[nw - 1];
      const size_t path_len = hash_last ? nw - 1 : nw;  // '#' last: attach to the parent node
      uint32_t cur = 0;
      for (size_t w = 0; w < path_len; ++w) {
        const uint64_t tok = is_plus[w] ? PLUS_TOK : toks[w];
        bool ins;
        uint32_t* v = m.emap.get_or_insert(cur, tok, ins);
        if (ins) {
          if (m.parent.size() >= MAX_NODES) {
            set_err(h, "trie exceeds 2^26-1 nodes");
            rc = -E2BIG;
            return;
          }
          const uint32_t child = m.new_node(cur, tok);
          *v = child;
          if (is_plus[w])
            m.pchild[cur] = child;
          else
            m.nlit[cur] += 1;
        }
        cur = *v;
        m.ref[cur] += 1;
      }
      m.max_depth = std::max<uint32_t>(m.max_depth, (uint32_t)path_len);
      lb.add(hash_last ? m.hf[cur] : f.wild ? m.tw[cur] : m.tn[cur], id);
    }
  });
  if (rc) return rc;
  // child signatures
  for (size_t y = 1; y < m.parent.size(); ++y)
    if (m.tok[y] != PLUS_TOK) m.sig[m.parent[y]] |= (uint8_t)sig_bit(m.tok[y]);
  // depth codes: H(x) = how many levels below x the filters under x reach (a '#' filter below
  // x: unbounded), bottom-up over node ids (a parent's id is smaller than its children's)
  {
    const size_t nn = m.parent.size();
    constexpr uint32_t INF = 0xFFu;
    std::vector<uint8_t> H(nn, 0);
    for (size_t y = nn; y-- > 1;) {
      const uint32_t up = (m.hf[y] != NONE || H[y] == INF) ? INF : std::min<uint32_t>(H[y] + 1u, INF - 1);
      uint8_t& hp = H[m.parent[y]];
      hp = (uint8_t)std::max<uint32_t>(hp, up);
    }
    m.hcode.assign(nn, 0);
    for (size_t x = 0; x < nn; ++x) m.hcode[x] = (H[x] >= 1 && H[x] <= 3) ? H[x] : 0;
  }
  // flatten multi lists
  std::vector<uint32_t> multi(1, 0);
  std::vector<uint32_t> list_pos(lb.lists.size());
  for (size_t i = 0; i < lb.lists.size(); ++i) {
    list_pos[i] = (uint32_t)multi.size();
    multi.push_back((uint32_t)lb.lists[i].size());
    multi.insert(multi.end(), lb.lists[i].begin(), lb.lists[i].end());
  }
  auto resolve = [&](uint32_t& v) {
    if (v != NONE && (v & LIST_MULTI)) v = LIST_MULTI | list_pos[v & ~LIST_MULTI];
  };
  const size_t n_nodes = m.parent.size();
  for (size_t i = 0; i < n_nodes; ++i) {
    resolve(m.hf[i]);
    resolve(m.tw[i]);
    resolve(m.tn[i]);
  }
  m.n_edges = n_nodes - 1;
  m.multi = std::move(multi);
  // 32-B slots in 64-B buckets (gm_common.h "edge slots"); load factor <= 1/EDGE_SLACK.  Each
  // slot carries its child's '+' child {cf, hf}, so the walk expands most '+' children
  // without a probe.
  m.ecap = pow2_at_least(std::max<uint64_t>(64, m.n_edges * EDGE_SLACK));
  m.nbk = m.ecap / EBUCKET;
  m.occ.assign(m.ecap / 64 + 1, 0ull);
  m.tomb.assign(m.ecap / 64 + 1, 0ull);
  // fat buckets (gm_common.h FAT_ID): a node at depth 2, 4 or 6 reached by a literal edge whose
  // only literal child is G takes a bucket of its own with G in the second half (halves are at
  // odd depths, so a half is never fat itself); the root's only literal child rides in the
  // kernel arguments.  Fat nodes are placed first, each only into its home bucket when both
  // of its slots are free (else the node stays thin): no lookup chain grows past a bucket
  // that still has a free slot (r03 A/B: TOMBing passed buckets lengthened cfg2's miss chains).
  m.fchild.assign(n_nodes, 0u);
  m.half.assign(n_nodes, 0u);
  select_keyed(m, in.keyed_mode);
  if (in.fat_mode) {
    std::vector<uint8_t> depth(n_nodes, 0);
    std::vector<uint32_t> lit(n_nodes, 0);
    for (uint32_t c = 1; c < n_nodes; ++c) {
      depth[c] = (uint8_t)std::min<uint32_t>(depth[m.parent[c]] + 1u, 255u);
      if (m.tok[c] != PLUS_TOK) lit[m.parent[c]] = c;
    }
    for (uint32_t x = 0; x < n_nodes; ++x)
      if (m.nlit[x] == 1 && (x == 0 || (depth[x] % 2 == 0 && depth[x] <= FAT_MAX_DEPTH &&
                                        m.tok[x] != PLUS_TOK))) {
        m.fchild[x] = lit[x];
        m.half[lit[x]] = 1;
      }
  }
  for (uint32_t c = 1; c < n_nodes; ++c) {
    if (!m.fchild[c]) continue;
    const uint64_t q = m.home(m.parent[c], m.tok[c]) * EBUCKET;
    if (bit(m.occ, q) || bit(m.occ, q + 1)) {  // home bucket taken: thin
      m.half[m.fchild[c]] = 0;
      m.fchild[c] = 0;
      continue;
    }
    bset(m.occ, q);
    bset(m.occ, q + 1);
    m.slot[c] = q;
    m.slot[m.fchild[c]] = q + 1;
  }
  if (m.fchild[0]) m.slot[m.fchild[0]] = ROOTH;
  // the children of keyed parents before the other thin edges, so that the edges sharing a token
  // find their home bucket free and share its line
  for (int pass = 0; pass < 2; ++pass)
    for (uint32_t c = 1; c < n_nodes; ++c) {
      if (m.fchild[c] || m.half[c] || (m.keyed[m.parent[c]] != 0) != (pass == 0)) continue;
      uint64_t b = m.home(m.parent[c], m.tok[c]), i;
      for (;;) {
        uint32_t j = 0;
        while (j < EBUCKET && bit(m.occ, b * EBUCKET + j) && !bit(m.tomb, b * EBUCKET + j)) ++j;
        if (j < EBUCKET) {
          i = b * EBUCKET + j;
          break;
        }
        b = (b + 1) & (m.nbk - 1);
      }
      bset(m.occ, i);
      bclr(m.tomb, i);
      m.slot[c] = i;
    }
  m.n_occ = 0;
  for (uint64_t w : m.occ) m.n_occ += (uint64_t)__builtin_popcountll(w);
  // node side array with headroom for delta-commit growth
  m.tn_cap = n_nodes + std::max<uint64_t>(4096, n_nodes / 4);
  m.n_nodes0 = n_nodes;
  m.fv_words0 = m.fvbits.size();
  m.fv_cap = m.fvbits.size() + std::max<uint64_t>(1024, m.fvbits.size() / 4);
  m.fvbits.resize(m.fv_cap, 0u);

  // ---- exact route keys: buckets of XBUCKET entries, load factor <= 1/2 per region, filled
  // in order; plain keys and wildcard keys in separate regions ----
  std::vector<uint32_t> rids;  // the route keys, in id order (read once: a background build's
                               // registry may change between two reads)
  for_slices(h, in.bg, nf, [&](uint64_t i0, uint64_t i1, const Filter* F, const uint8_t*) {
    for (uint64_t id = i0; id < i1; ++id) {
      if (!F[id - i0].route_refs) continue;
      if (in.seen) (*in.seen)[id] |= 2;
      rids.push_back((uint32_t)id);
      m.nroute(F[id - i0].wild) += 1;
    }
  });
  m.n_route = m.n_route_p + m.n_route_w;
  m.xcap_p = pow2_at_least(std::max<uint64_t>(16, (m.n_route_p * 2 + XBUCKET - 1) / XBUCKET));
  m.xcap_w = pow2_at_least(std::max<uint64_t>(16, (m.n_route_w * 2 + XBUCKET - 1) / XBUCKET));
  const uint64_t xcap = m.xcap_p + m.xcap_w;
  m.xocc.assign(xcap * XBUCKET / 64 + 1, 0ull);
  m.xtomb.assign(xcap * XBUCKET / 64 + 1, 0ull);
  m.xovf.assign(xcap / 64 + 1, 0ull);
  m.xpos.assign(nf, NONE);
  for (uint64_t k0 = 0; k0 < rids.size(); k0 += REG_SLICE) {
    const uint64_t k1 = std::min<uint64_t>(rids.size(), k0 + REG_SLICE);
    // (bytes of registered filters never change: only the storage may move, under the lock)
    with_registry(h, in.bg, [&](const Filter* F, const uint8_t* pool) {
      for (uint64_t k = k0; k < k1; ++k) {
        const uint32_t id = rids[k];
        const Filter& f = F[id];
        const uint64_t fh = key_hash(pool + f.off, f.len, fmask);
        const bool w = f.wild;
        uint64_t b = m.xhome(w, fh);
        for (;;) {
          uint32_t j = 0;
          while (j < XBUCKET && bit(m.xocc, b * XBUCKET + j)) ++j;
          if (j < XBUCKET) {
            const uint64_t e = b * XBUCKET + j;
            bset(m.xocc, e);
            m.xpos[id] = (uint32_t)e;
            break;
          }
          bset(m.xovf, b);  // the key goes on past this full bucket
          b = m.xnext(w, b);
        }
      }
    });
  }
  m.x_occ_p = m.n_route_p;
  m.x_occ_w = m.n_route_w;
  return 0;
}

// Full build of the device index from the pending registry, in the caller's thread (wmu held:
// no writer runs meanwhile); swaps it in and rebuilds the host model (TrieModel) that later delta
// commits patch.
void model_room(TrieModel& m);

int commit_full(emqxgm* h) {
  const BuildIn in = build_in(h, false);
  h->tm = TrieModel();  // frees the old model before the new one is built
  TrieModel m;
  int rc = build_model(h, in, m);
  if (rc) return rc;
  if (hipSetDevice(h->cfg.device) != hipSuccess) return fail(h, hipErrorInvalidDevice, "hipSetDevice");
  if ((rc = upload_pool(h, nullptr)) || (rc = fan_full(h)) || (rc = upload_model(h, m))) return rc;
  m.valid = true;
  model_room(m);
  h->tm = std::move(m);
  h->changed.clear();  // every filter's committed flags follow at publish (commit_locked)
  return 0;
}

// Delta commit: apply the membership changes since the last commit to the host model and patch
// the device tables in place (k_patch).  Returns 0 when applied, 1 when the delta does not fit
// (too large, a table would pass its load bound, a node list would need a multi[] list, ...):
// the caller then runs the full build, which also rebuilds the model.  The patches are only
// staged here; publish_epoch applies them on the GPU after every pass already enqueued and before
// every later one, so no match sees a half-applied delta.
//
// The model's state per filter is its committed flags -- or, for the catch-up of a background
// build (install_build), `base`: the membership the build read (bit 0 trie, bit 1 route key;
// ids past its end: none).  The declines for size and for table capacity come before anything
// changes, so they leave the model valid (a background build then runs while later deltas still
// patch it); only a delta that would need a multi[] list (level-token collisions) gives the model
// up half-way.
// The verify-bit array of the writer's index regrown to `need` words plus headroom: a new
// buffer (owner o_fv until the next full build brings its own) filled from the host model; the
// epochs reading the old array keep it.
int grow_fv(emqxgm* h, TrieModel& m, uint64_t need) {
  const uint64_t cap = need + std::max<uint64_t>(1024, need / 4);
  if (int rc = patch_wait(h)) return rc;  // (patches to the old array have landed)
  auto o = std::make_shared<DevOwner>();
  DevBuf nb;
  nb.bytes = cap * 4;
  HIPCHK(h, hipMalloc(&nb.p, nb.bytes));
  o->bufs.push_back(nb);
  m.fvbits.resize(cap, 0u);
  HIPCHK(h, hipMemcpy(nb.p, m.fvbits.data(), cap * 4, hipMemcpyHostToDevice));
  m.fv_cap = cap;
  m.d_fv = (uint32_t*)nb.p;
  h->ix.fvbits = (const uint32_t*)nb.p;
  h->o_fv = std::move(o);
  return 0;
}

int commit_delta(emqxgm* h, const std::vector<uint8_t>* base = nullptr) {
  TrieModel& m = h->tm;
  if (!m.valid || h->delta_mode == 0) return 1;
  const uint64_t nf = h->filters.size();
  auto& ch = h->changed;
  std::sort(ch.begin(), ch.end());
  ch.erase(std::unique(ch.begin(), ch.end()), ch.end());
  std::vector<uint32_t> tadd, tdel, radd, rdel;
  for (uint32_t id : ch) {
    const Filter& f = h->filters[id];
    const uint8_t b = base ? (id < base->size() ? (*base)[id] : 0u)
                           : (uint8_t)((f.trie_committed ? 1u : 0u) | (f.route_committed ? 2u : 0u));
    if ((bool)f.in_trie != (bool)(b & 1)) (f.in_trie ? tadd : tdel).push_back(id);
    const bool r = f.route_refs > 0;
    if (r != (bool)(b & 2)) (r ? radd : rdel).push_back(id);
  }
  const uint64_t nchg = tadd.size() + tdel.size() + radd.size() + rdel.size();
  if (h->delta_mode == 1 &&
      nchg > (h->delta_max ? h->delta_max : std::max<uint64_t>(4096, (m.n_trie + m.n_route) / 8)))
    return 1;
  if ((nf + 31) / 32 + 1 > m.fv_cap) {
    // filter ids registered past the verify bits' headroom (a bulk registration, whose build
    // runs in the background): a larger array, from the host model
    if (int rc = grow_fv(h, m, (nf + 31) / 32 + 1)) return rc;
  }

  const uint64_t test_mask = h->test_mask;
  std::vector<uint64_t> toks;
  std::vector<uint8_t> is_plus, is_hash;
  {
    // the nodes and slots the delta can take at most: each added filter's path levels that are
    // not in the trie yet, plus every node a delete may free and an add re-create
    // (and a fat half moved out of its parent's bucket where the first new node is a second
    // literal child: one more slot)
    uint64_t new_nodes = 0, moved = 0, xa[2] = {0, 0};
    std::unordered_map<uint32_t, uint32_t> dpass;  // node -> deleted filters passing it
    auto walk = [&](uint32_t id, auto&& on_node) {
      const Filter& f = h->filters[id];
      bool hashed;
      tokenize(h->pool.data() + f.off, f.len, test_mask, toks, is_plus, is_hash, hashed);
      const size_t path_len = is_hash.back() ? toks.size() - 1 : toks.size();
      uint32_t cur = 0;
      size_t w = 0;
      for (; w < path_len; ++w) {
        const uint32_t* v = m.emap.find(cur, is_plus[w] ? PLUS_TOK : toks[w]);
        if (!v) break;
        cur = *v;
        on_node(cur);
      }
      new_nodes += path_len - w;
      if (w < path_len && !is_plus[w] && m.fchild[cur]) moved += 1;
    };
    if (!tadd.empty())
      for (uint32_t id : tdel) walk(id, [&](uint32_t n) { dpass[n] += 1; });
    new_nodes = moved = 0;
    for (uint32_t id : tadd)
      walk(id, [&](uint32_t n) {  // a node the deletes free is created again
        auto it = dpass.find(n);
        if (it != dpass.end() && it->second >= m.ref[n]) new_nodes += 1;
      });
    if (m.parent.size() + new_nodes > std::min<uint64_t>(MAX_NODES, m.tn_cap) ||
        (m.n_occ + new_nodes + moved) * 2 > m.ecap)
      return 1;
    for (uint32_t id : radd) xa[h->filters[id].wild ? 1 : 0] += 1;
    for (int w = 0; w < 2; ++w)
      if (xa[w] && (m.xoccr(w != 0) + xa[w]) * 4 > m.xcapr(w != 0) * XBUCKET * 3) return 1;
  }
  m.valid = false;  // from here a declined delta leaves the model to the full build

  const uint64_t fmask =
      h->cfg.full_hash_bits >= 64 ? ~0ull : ((1ull << h->cfg.full_hash_bits) - 1ull);
  std::unordered_map<uint64_t, uint32_t> epatch;  // edge slot -> node (NONE: TOMB)
  struct XE {
    uint4 e[XENT_U4];
  };
  std::unordered_map<uint64_t, XE> xpatch;        // exact entry -> content
  std::vector<uint32_t> dirty;                    // nodes whose slot / side entry changed
  std::vector<uint32_t> fv_words;  // changed words of the verify bitmap
  std::vector<uint32_t> ovf_words; // changed words of the exact table's overflow bitmap
  std::vector<uint32_t> path;

  // ---- trie deletes: drop the key from its end node, free nodes no filter passes any more ----
  for (uint32_t id : tdel) {
    const Filter& f = h->filters[id];
    bool hashed;
    tokenize(h->pool.data() + f.off, f.len, test_mask, toks, is_plus, is_hash, hashed);
    const size_t nw = toks.size();
    const bool hash_last = is_hash[nw - 1];
    const size_t path_len = hash_last ? nw - 1 : nw;
    path.clear();
    uint32_t cur = 0;
    for (size_t w = 0; w < path_len; ++w) {
      const uint32_t* v = m.emap.find(cur, is_plus[w] ? PLUS_TOK : toks[w]);
      if (!v) return 1;
      cur = *v;
      path.push_back(cur);
    }
    uint32_t& fld = hash_last ? m.hf[cur] : f.wild ? m.tw[cur] : m.tn[cur];
    if (fld != id) return 1;  // part of a multi[] list
    fld = NONE;
    dirty.push_back(cur);
    for (size_t k = path.size(); k-- > 0;) {
      const uint32_t n = path[k];
      if (--m.ref[n] != 0) continue;
      const uint32_t par = m.parent[n];
      m.emap.erase(par, m.tok[n]);
      if (m.tok[n] == PLUS_TOK)
        m.pchild[par] = 0;
      else
        m.nlit[par] -= 1;
      if (m.half[n]) {  // its slot is the parent's second half (or the root's arguments)
        m.fchild[par] = 0;
        m.half[n] = 0;
      }
      if (m.slot[n] != ROOTH) {
        bset(m.tomb, m.slot[n]);
        epatch[m.slot[n]] = NONE;
      }
      m.slot[n] = DEAD;
      m.n_edges -= 1;
      dirty.push_back(par);
    }
    m.n_trie -= 1;
  }

  // ---- trie inserts: new nodes take the first free or TOMB slot of their bucket chain ----
  auto alloc_slot = [&](uint32_t par, uint64_t tok) {
    uint64_t b = m.home(par, tok), i = DEAD;
    while (i == DEAD) {
      for (uint32_t j = 0; j < EBUCKET && i == DEAD; ++j) {
        const uint64_t q = b * EBUCKET + j;
        if (!bit(m.occ, q)) {
          bset(m.occ, q);
          m.n_occ += 1;
          i = q;
        } else if (bit(m.tomb, q)) {
          bclr(m.tomb, q);
          i = q;
        }
      }
      b = (b + 1) & (m.nbk - 1);
    }
    return i;
  };
  for (uint32_t id : tadd) {
    const Filter& f = h->filters[id];
    bool hashed;
    tokenize(h->pool.data() + f.off, f.len, test_mask, toks, is_plus, is_hash, hashed);
    if (hashed) {
      m.fvbits[id >> 5] |= 1u << (id & 31);
      m.needs_verify = true;
      fv_words.push_back(id >> 5);
    }
    const size_t nw = toks.size();
    const bool hash_last = is_hash[nw - 1];
    const size_t path_len = hash_last ? nw - 1 : nw;
    uint32_t cur = 0;
    path.assign(1, 0u);  // root .. end node
    for (size_t w = 0; w < path_len; ++w) {
      const uint64_t tok = is_plus[w] ? PLUS_TOK : toks[w];
      bool ins;
      uint32_t* v = m.emap.get_or_insert(cur, tok, ins);
      if (ins) {
        if (m.parent.size() >= std::min<uint64_t>(MAX_NODES, m.tn_cap)) return 1;
        if ((m.n_occ + 1) * 2 > m.ecap) return 1;  // load bound of a delta-patched table
        const uint32_t fc = m.fchild[cur];
        if (fc && !is_plus[w]) {
          // a second literal child: the fat half moves to its own hash position (its old slot
          // becomes TOMB), so cur's literal children are probed by hash from now on
          if ((m.n_occ + 2) * 2 > m.ecap) return 1;
          if (m.slot[fc] != ROOTH) {
            bset(m.tomb, m.slot[fc]);
            epatch[m.slot[fc]] = NONE;
          }
          m.half[fc] = 0;
          m.fchild[cur] = 0;
          m.slot[fc] = alloc_slot(cur, m.tok[fc]);
          epatch[m.slot[fc]] = fc;
          dirty.push_back(fc);
        }
        const uint32_t c = m.new_node(cur, tok);
        *v = c;
        const uint64_t i = alloc_slot(cur, tok);
        m.slot[c] = i;
        epatch[i] = c;
        m.n_edges += 1;
        if (is_plus[w]) {
          m.pchild[cur] = c;
        } else {
          m.nlit[cur] += 1;
          m.sig[cur] |= (uint8_t)sig_bit(tok);
        }
        dirty.push_back(cur);
        dirty.push_back(c);
      }
      cur = *v;
      m.ref[cur] += 1;
      path.push_back(cur);
    }
    m.max_depth = std::max<uint32_t>(m.max_depth, (uint32_t)path_len);
    uint32_t& fld = hash_last ? m.hf[cur] : f.wild ? m.tw[cur] : m.tn[cur];
    if (fld != NONE) return 1;  // a second key at one node needs a multi[] list
    fld = id;
    m.widen_codes(path, hash_last, dirty);
    dirty.push_back(cur);
    m.n_trie += 1;
  }

  // ---- exact route keys ----
  m.xpos.resize(nf, NONE);
  for (uint32_t id : rdel) {
    const uint32_t e = m.xpos[id];
    if (e == NONE) return 1;
    bset(m.xtomb, e);
    xpatch[e] = XE{{make_uint4(0u, TOMB, 0u, 0u), make_uint4(0u, 0u, 0u, 0u)}};
    m.xpos[id] = NONE;
    m.n_route -= 1;
    m.nroute(h->filters[id].wild) -= 1;
  }
  for (uint32_t id : radd) {
    const Filter& f = h->filters[id];
    const bool w = f.wild;
    if ((m.xoccr(w) + 1) * 4 > m.xcapr(w) * XBUCKET * 3) return 1;
    const uint64_t fh = key_hash(h->pool.data() + f.off, f.len, fmask);
    uint64_t b = m.xhome(w, fh), e = DEAD;
    while (e == DEAD) {
      for (uint32_t j = 0; j < XBUCKET && e == DEAD; ++j) {
        const uint64_t q = b * XBUCKET + j;
        if (!bit(m.xocc, q)) {
          bset(m.xocc, q);
          m.xoccr(w) += 1;
          e = q;
        } else if (bit(m.xtomb, q)) {
          bclr(m.xtomb, q);
          e = q;
        }
      }
      if (e == DEAD && !bit(m.xovf, b)) {  // the key goes on past this full bucket
        bset(m.xovf, b);
        ovf_words.push_back((uint32_t)(b >> 5));
      }
      b = m.xnext(w, b);
    }
    xent(fh, id, h->pool.data() + f.off, f.len, xpatch[e].e);
    m.xpos[id] = (uint32_t)e;
    m.n_route += 1;
    m.nroute(w) += 1;
  }

  // ---- patch lists: a dirty node rewrites its own slot, and its parent's slot when it is the
  // parent's '+' child (the parent's slot carries its {cf, hf}) ----
  std::sort(dirty.begin(), dirty.end());
  dirty.erase(std::unique(dirty.begin(), dirty.end()), dirty.end());
  std::vector<uint32_t> tn_nodes;
  for (uint32_t n : dirty) {
    if (n != 0 && m.slot[n] == DEAD) continue;  // removed
    if (n != 0 && m.slot[n] != ROOTH) epatch[m.slot[n]] = n;  // ROOTH: the arguments, below
    tn_nodes.push_back(n);
    const uint32_t par = n ? m.parent[n] : NONE;
    if (par != NONE && par != 0 && m.pchild[par] == n && m.slot[par] != ROOTH)
      epatch[m.slot[par]] = par;
  }
  // ---- stage the patches, upload them in one copy, apply them in one launch ----
  if (hipSetDevice(h->cfg.device) != hipSuccess) return fail(h, hipErrorInvalidDevice, "hipSetDevice");
  PatchList& pl = h->patches;
  for (const auto& p : epatch) {
    uint4 sl[2] = {make_uint4(0u, 0u, TOMB, 0u), make_uint4(0u, 0u, 0u, 0u)};
    if (p.second != NONE) m.node_slot(p.second, sl);
    pl.add(m.d_edges + 8 * p.first, sl, 8);
  }
  for (const auto& p : xpatch) pl.add(m.d_exact + 4 * XENT_U4 * p.first, p.second.e, 4 * XENT_U4);
  for (uint32_t n : tn_nodes) pl.add(m.d_tn + n, &m.tn[n], 1);
  std::sort(fv_words.begin(), fv_words.end());
  fv_words.erase(std::unique(fv_words.begin(), fv_words.end()), fv_words.end());
  for (uint32_t w : fv_words) pl.add(m.d_fv + w, &m.fvbits[w], 1);
  std::sort(ovf_words.begin(), ovf_words.end());
  ovf_words.erase(std::unique(ovf_words.begin(), ovf_words.end()), ovf_words.end());
  for (uint32_t w : ovf_words) {
    const uint32_t v = (uint32_t)(m.xovf[w >> 1] >> (32 * (w & 1)));
    pl.add(m.d_xovf + w, &v, 1);
  }
  int rc = 0;
  if ((rc = upload_pool(h, &pl)) || (rc = fan_commit(h))) return rc;

  DevIndex& ix = h->ix;
  const uint32_t root_p = m.pchild[0];
  ix.root_cf = m.cf(0);
  ix.root_sig = m.sig[0];
  ix.root_hf = m.hfd(0);
  ix.root_pcf = root_p ? m.pcf(root_p) : 0u;
  ix.root_phf = root_p ? m.phf(root_p) : NONE;
  m.root_half(ix);
  ix.needs_verify = m.needs_verify;
  ix.max_depth = m.max_depth;
  ix.fid_bound = (uint64_t)m.fv_cap * 32;
  ix.trie_empty = (m.n_trie == 0);
  ix.plain_empty = (m.n_route_p == 0);
  ix.wild_empty = (m.n_route_w == 0);
  m.valid = true;  // h->changed: their committed flags follow at publish (commit_locked)
  return 0;
}

// The reader contexts whose passes a writer orders its patches behind.
template <class F>
void for_each_reader(emqxgm* h, F f) {
  f(h->sync);
  for (auto& p : h->pipes) f(p.c);
  for (auto& p : h->hpipes) f(p.c);
}

// Publishes the writer's working index as the next epoch (under emu).  A delta commit's patches
// rewrite tables that passes enqueued on the current epoch may still read: the writer stream
// first waits for each reader stream's last pass (GPU-side, the host does not block), then runs
// the patch upload and k_patch, and the new epoch's `ready` event follows them -- every later
// pass waits on it.  A full build's tables are new, so it waits for nobody.
int publish_epoch(emqxgm* h, bool delta) {
  auto E = std::make_shared<Epoch>();
  E->id = h->epoch + 1;
  E->ix = h->ix;
  E->owners = {h->o_tab, h->o_fan, h->m_pool.o, h->m_foff.o, h->m_fver.o, h->o_fv};
  HIPCHK(h, hipEventCreateWithFlags(&E->ready, hipEventDisableTiming));
  std::lock_guard<std::mutex> g(h->emu);
  if (delta && h->cur) {
    E->walk_level.store(h->cur->walk_level.load());
    E->census_level.store(h->cur->census_level.load());
  }
  if (!h->patches.ents.empty()) {
    int rc = 0;
    // every pass was enqueued under emu, which this commit holds: an event recorded now on a
    // reader's stream follows its last pass (no event per pass: r03)
    for_each_reader(h, [&](PassCtx& c) {
      if (!rc && c.stream && c.done &&
          (hipEventRecord(c.done, c.stream) != hipSuccess ||
           hipStreamWaitEvent(h->wstream, c.done, 0) != hipSuccess))
        rc = fail(h, hipErrorUnknown, "hipStreamWaitEvent(writer, reader pass)");
    });
    if (rc || (rc = patch_flush(h))) return rc;
  }
  HIPCHK(h, hipEventRecord(E->ready, h->wstream));
  // an epoch that holds a buffer the new one does not (replaced tables, a regrown mirror, rebuilt
  // fan-out tables) is heavy: its last reference frees device memory (a hipFree synchronises the
  // device), so a subscribe's commit never sweeps it -- emqxgm_commit and the builder thread do
  auto heavy = [&](Epoch& x) {
    for (const OwnerP& o : x.owners)
      if (o && std::find(E->owners.begin(), E->owners.end(), o) == E->owners.end()) {
        x.heavy = true;
        return;
      }
  };
  if (h->cur) heavy(*h->cur);
  for (auto& e : h->graveyard) heavy(*e);
  if (h->cur) h->graveyard.push_back(std::move(h->cur));
  h->cur = std::move(E);
  h->cur_trie_empty.store(h->cur->ix.trie_empty ? 1 : 0);
  h->epoch += 1;
  return 0;
}

// Frees retired epochs no reader holds any more (writers only: readers never free).
// all = false (writers): heavy epochs are left to the builder thread.  Returns the heavy epochs
// still retired (held by a pass).
size_t sweep_graveyard(emqxgm* h, bool all = false) {
  std::vector<EpochP> dead;
  size_t left = 0;
  {
    std::lock_guard<std::mutex> g(h->emu);
    auto& gy = h->graveyard;
    for (size_t i = 0; i < gy.size();) {
      if (gy[i].use_count() == 1 && (all || !gy[i]->heavy)) {
        dead.push_back(std::move(gy[i]));
        gy[i] = std::move(gy.back());
        gy.pop_back();
      } else {
        ++i;
      }
    }
    for (const auto& e : gy) left += e->heavy ? 1u : 0u;
  }
  // dead epochs (and the device buffers only they owned) are freed here, outside emu
  dead.clear();
  return left;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// EMQXGM_DEBUG_SLOW=<ms>: writer-side steps slower than that are reported on stderr (diagnosis
// of the subscribe path's tail; off by default)
double debug_slow_ms() {
  static const double v = [] {
    const char* e = getenv("EMQXGM_DEBUG_SLOW");
    return e ? atof(e) : 0.0;
  }();
  return v;
}
void debug_slow(const char* what, double ms) {
  const double lim = debug_slow_ms();
  if (lim > 0 && ms >= lim) fprintf(stderr, "[emqxgm slow] %s %.1f ms\n", what, ms);
}

// The registry's committed flags (trie_member, route_member, the next delta's base) follow the
// published epoch: for the listed filters, or for all.
void flip_committed(emqxgm* h, const std::vector<uint32_t>* ids) {
  std::unique_lock<std::shared_mutex> g(h->pmu);
  auto flip = [](Filter& f) {
    f.trie_committed = f.in_trie;
    f.route_committed = f.route_refs > 0;
  };
  if (ids) {
    for (uint32_t id : *ids) flip(h->filters[id]);
  } else {
    for (Filter& f : h->filters) flip(f);
  }
}

// A delta commit of the pending changes published, or 1 when it does not fit (nothing changed
// then, unless the model gave way: tm.valid false).  During a background build its changes are
// logged for the build's install.
int try_delta(emqxgm* h, std::chrono::steady_clock::time_point t0) {
  sweep_graveyard(h);
  h->patches.clear();
  int rc = patch_wait(h);  // the previous commit's patches are applied before buffers change
  if (rc) return rc;
  rc = commit_delta(h);
  if (rc) {
    h->patches.clear();  // a declined delta stages nothing
    return rc;
  }
  if ((rc = publish_epoch(h, true))) return rc;
  flip_committed(h, &h->changed);
  if (h->job) h->build_log.insert(h->build_log.end(), h->changed.begin(), h->changed.end());
  h->changed.clear();
  h->dirty = false;
  commit_stats(h, ms_since(t0), true);
  return 0;
}

// A blocking full build of the whole registry, published.
int full_now(emqxgm* h, std::chrono::steady_clock::time_point t0) {
  sweep_graveyard(h);
  h->patches.clear();
  int rc = patch_wait(h);
  if (rc || (rc = commit_full(h)) || (rc = publish_epoch(h, false))) return rc;
  flip_committed(h, nullptr);
  h->changed.clear();
  h->build_log.clear();
  h->dirty = false;
  const double ms = ms_since(t0);
  commit_stats(h, ms, false);
  std::lock_guard<std::mutex> g(h->stmu);
  h->st.last_build_ms = ms;
  return 0;
}

// Host-side room for the deltas ahead: a vector past 7/8 of its capacity gets a quarter more
// (a full build sizes the model's per-node arrays exactly: the first subscribe's new node then
// reallocated a dozen 11M-entry arrays, ~6 ms at cfg3 -- VERDICT r05 item 2), and the edge map
// is rehashed before a delta's insert would do it.  Returns whether anything moved.
template <class V>
bool room_ahead(V& v) {
  if (v.size() * 8 <= v.capacity() * 7 && v.capacity() - v.size() >= 1024) return false;
  v.reserve(v.size() + std::max<size_t>(v.size() / 4, 4096));
  return true;
}
void model_room(TrieModel& m) {
  if (!m.valid) return;
  for (auto* v : {&m.parent, &m.ref, &m.nlit, &m.pchild, &m.hf, &m.tw, &m.tn, &m.fchild,
                  &m.fvbits, &m.multi, &m.xpos})
    room_ahead(*v);
  for (auto* v : {&m.sig, &m.hcode, &m.half, &m.keyed}) room_ahead(*v);
  for (auto* v : {&m.tok, &m.slot}) room_ahead(*v);
  if ((m.emap.used + 4096) * 2 > m.emap.mask + 1) m.emap.grow();
}
void registry_room(emqxgm* h) {
  std::unique_lock<std::shared_mutex> g(h->pmu);
  room_ahead(h->filters);
  room_ahead(h->pool);
  room_ahead(h->foff_host);
  room_ahead(h->fver_host);
  if (!h->slots.empty() && (h->filters.size() + 4096) * 2 > h->slot_mask + 1) slots_grow(h);
}

// Off the hook path (emqxgm_commit, a background build's install; wmu held): an append-only
// mirror (filter pool, offsets, verify records) past 7/8 of its buffer, or fan-out tables past 7/8
// of their ids or pools (or with stale entries past a quarter), are regrown now, so that the
// subscribes' delta commits keep finding room and never allocate.  The index
// is left dirty: the caller's commit publishes the new buffers.
int grow_ahead(emqxgm* h) {
  registry_room(h);
  model_room(h->tm);
  bool grew = false;
  for (Mirror* m : {&h->m_pool, &h->m_foff, &h->m_fver})
    if (m->b.bytes && m->uploaded * 8 > m->b.bytes * 7) {
      if (int rc = mirror_grow(h, *m, m->uploaded)) return rc;
      grew = true;
    }
  if (grew) {
    h->ix.fbytes = (const uint8_t*)h->m_pool.b.p;
    h->ix.foff = (const uint64_t*)h->m_foff.b.p;
    h->ix.fver = (const uint4*)h->m_fver.b.p;
  }
  const FanModel& fm = h->fm;
  if (fm.valid && fm.cap &&
      (h->filters.size() * 8 > fm.cap * 7 || fm.rt_used * 8 > fm.rt_cap * 7 ||
       fm.dl_used * 8 > fm.dl_cap * 7 || fm.garbage * 4 > fm.rt_used + fm.dl_used + 65536)) {
    if (int rc = patch_wait(h)) return rc;
    if (int rc = fan_full(h)) return rc;
    grew = true;
  }
  if (grew) h->dirty = true;
  return 0;
}

bool bg_allowed(const emqxgm* h) {
  return h->bg_min != 0 && h->filters.size() >= h->bg_min && h->delta_mode != 0;
}

// A table of the current index well on its way to a delta bound (edge slots past 3/8 of 1/2,
// an exact region past 5/8 of 3/4, half the node or verify-word headroom used): rebuilt in the
// background while deltas still fit, so that a subscribe does not meet a full table.
bool nearly_full(const emqxgm* h) {
  const TrieModel& m = h->tm;
  if (!m.valid) return false;
  if (m.n_occ * 8 > m.ecap * 3) return true;
  for (bool w : {false, true})
    if (m.xcapr(w) > 16 && (w ? m.x_occ_w : m.x_occ_p) * 8 > m.xcapr(w) * XBUCKET * 5) return true;
  if (m.parent.size() * 2 > m.tn_cap + m.n_nodes0) return true;
  const uint64_t fvw = (h->filters.size() + 31) / 32 + 1;
  return m.fv_words0 && fvw * 2 > m.fv_cap + m.fv_words0;
}

int install_build(emqxgm* h, std::unique_ptr<BuildJob>& spent);

// The background build's thread: build the model and upload its tables without the writer lock
// (for_slices lets writers in between slices), then install it under the lock.
void build_thread(emqxgm* h, BuildJob* J) {
  int rc = 0;
  if (hipSetDevice(h->cfg.device) != hipSuccess) rc = -EIO;
  if (!rc) rc = build_model(h, J->in, J->m);
  if (!rc) rc = upload_tables(h, J->in, J->m, J->nx, J->o);
  J->rc = rc;
  if (!rc) {
    J->m.valid = true;
    model_room(J->m);  // (its own model: no lock needed; the install keeps it)
    J->m.valid = false;
  }
  J->build_ms = ms_since(J->t0);
  if (const uint32_t d = h->bg_delay_ms.load()) std::this_thread::sleep_for(std::chrono::milliseconds(d));
  std::unique_ptr<BuildJob> spent;
  {
    const auto tw = std::chrono::steady_clock::now();
    std::lock_guard<std::mutex> g(h->wmu);
    debug_slow("install: waited for the writer lock", ms_since(tw));
    const auto ti = std::chrono::steady_clock::now();
    h->build_rc = install_build(h, spent);
    if (h->build_rc) mark_stale(h, EMQXGM_STALE_COMMIT, h->build_rc);  // (no caller may be waiting)
    debug_slow("install", ms_since(ti));
    h->builds_done += 1;
    h->bcv.notify_all();
  }
  const auto tf = std::chrono::steady_clock::now();
  // The replaced host model (tens of millions of entries at cfg3) is freed here, without the
  // writer lock, and so are the replaced device tables once the passes that read them are done
  // -- not by the next subscribe's commit (sweep_graveyard takes only the epoch lock).
  spent.reset();
  debug_slow("free the replaced model", ms_since(tf));
  const auto ts = std::chrono::steady_clock::now();
  for (int i = 0; i < 10000 && sweep_graveyard(h, true) != 0; ++i)
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  debug_slow("free the replaced tables", ms_since(ts));
  std::lock_guard<std::mutex> g(h->emu);  // (a pass held on for 10 s: writers free them later)
  for (auto& e : h->graveyard) e->heavy = false;
}

// Starts a background full build of the registry as it is now (wmu held): the changes pending now
// are the build's to publish (`covered`); the index readers have stays until the install.
int start_build(emqxgm* h) {
  if (h->builder.joinable()) h->builder.join();  // the previous one is installed and gone
  std::unique_ptr<BuildJob> J(new (std::nothrow) BuildJob());
  if (!J) return -ENOMEM;
  J->in = build_in(h, true);
  J->seen.assign(J->in.nf, 0);
  J->in.seen = &J->seen;
  J->covered.swap(h->changed);
  J->t0 = std::chrono::steady_clock::now();
  h->build_log.clear();
  h->dirty = false;
  BuildJob* jp = J.get();
  h->job = std::move(J);
  h->builds_started += 1;
  try {
    h->builder = std::thread([h, jp] { build_thread(h, jp); });
  } catch (...) {
    h->changed.swap(jp->covered);
    h->job.reset();
    h->builds_started -= 1;
    h->dirty = true;
    return -ENOMEM;
  }
  std::lock_guard<std::mutex> g(h->stmu);
  h->st.bg_builds += 1;
  return 0;
}

// Waits (releasing the writer lock) until the build in flight is installed.
int wait_build(emqxgm* h, std::unique_lock<std::mutex>& lk) {
  const uint64_t target = h->builds_started;
  h->bcv.wait(lk, [&] { return h->builds_done >= target; });
  return h->build_rc;
}

// Swaps the finished background build in (wmu held, by its thread): its tables replace the
// writer's index, the changes made since it read the registry (the log of the deltas committed
// meanwhile and whatever is pending) are replayed onto its model as one delta against the
// membership it read, and the result is published.  A failed build, or a catch-up too large for
// a delta, ends in a blocking full build.
int install_build(emqxgm* h, std::unique_ptr<BuildJob>& spent) {
  spent = std::move(h->job);
  BuildJob* J = spent.get();
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<uint32_t> ch = std::move(h->build_log);
  h->build_log.clear();
  ch.insert(ch.end(), h->changed.begin(), h->changed.end());
  int rc = J->rc;
  if (rc == 0) {
    sweep_graveyard(h);
    h->patches.clear();
    rc = patch_wait(h);
  }
  if (rc == 0) {
    J->m.valid = true;
    std::swap(h->tm, J->m);  // J->m: the replaced model, freed by the caller after the lock
    h->o_tab = std::move(J->o);
    h->o_fv.reset();
    set_tables(h->ix, J->nx);
    h->changed = ch;
    rc = commit_delta(h, &J->seen);
    if (rc > 0) {
      h->patches.clear();
      rc = commit_full(h);  // (the catch-up did not fit: every filter, now)
      ch.clear();
      J->covered.clear();
      if (rc == 0) J->covered.push_back(NONE);  // flip every flag below
    }
    if (rc == 0) {
      {
        std::lock_guard<std::mutex> g(h->emu);  // every epoch on the replaced tables
        if (h->cur) h->cur->heavy = true;
        for (auto& e : h->graveyard) e->heavy = true;
      }
      rc = publish_epoch(h, false);
    }
  } else {
    h->changed = ch;
    set_err(h, "background build failed: a blocking full build follows");
    rc = full_now(h, t0);
    J->covered.clear();
    ch.clear();
    if (rc == 0) return 0;
  }
  if (rc) {
    h->tm.valid = false;  // the next commit rebuilds
    h->dirty = true;
    return rc;
  }
  const uint64_t n_catchup = ch.size();
  if (!J->covered.empty() && J->covered[0] == NONE) {
    flip_committed(h, nullptr);
  } else {
    ch.insert(ch.end(), J->covered.begin(), J->covered.end());
    flip_committed(h, &ch);
  }
  h->changed.clear();
  h->dirty = false;
  commit_stats(h, ms_since(t0), false);
  {
    std::lock_guard<std::mutex> g(h->stmu);
    h->st.last_build_ms = J->build_ms;
    h->st.catchup_changes = n_catchup;
  }
  // room for the subscribes that follow (the install's publish already holds the index; what
  // this regrows goes out with the next commit)
  return grow_ahead(h);
}

// Make the pending registry the committed index (wmu held; lk: the caller's lock on it, which
// waiting for a background build releases -- nullptr: never build in the background).
//   * No build in flight: a delta commit when it fits; else a full build -- in the background
//     when the registry is large enough (bg_allowed), the caller waiting for its install.
//   * A build in flight: the pending changes go into the index readers have now as a delta
//     commit (and are replayed onto the build at its install).  wait_all (emqxgm_commit) then
//     waits for the install too, since changes made before the build started -- possibly this
//     caller's -- become visible only with it; the synchronous subscribe path
//     (EMQXGM_SET_COMMIT, whose changes are made under the same lock hold) returns at once.
//     A delta the current tables cannot take waits for the install, which includes it.
int commit_locked(emqxgm* h, std::unique_lock<std::mutex>* lk, bool wait_all) {
  const auto t0 = std::chrono::steady_clock::now();
  RoctxRange rr(h->roctx, "emqxgm.commit");
  if (h->job) {
    if (!lk) return -EBUSY;
    int rc = h->dirty ? try_delta(h, t0) : 0;
    if (rc < 0) return rc;
    if (rc == 0 && !wait_all) return 0;
    if (rc > 0) {
      std::lock_guard<std::mutex> g(h->stmu);
      h->st.bg_waits += 1;
    }
    return wait_build(h, *lk);
  }
  if (!h->dirty) return 0;
  int rc = try_delta(h, t0);
  if (rc == 0) {
    if (lk && bg_allowed(h) && nearly_full(h)) (void)start_build(h);  // not waited for
    return 0;
  }
  if (rc < 0) return rc;
  if (lk && bg_allowed(h) && start_build(h) == 0) return wait_build(h, *lk);
  return full_now(h, t0);
}

int dev_alloc(emqxgm* h, PassCtx& c, void** p, size_t bytes) {
  HIPCHK(h, hipMalloc(p, std::max<size_t>(bytes, 16)));
  DevBuf b;
  b.p = *p;
  b.bytes = bytes;
  c.bufs.push_back(b);
  return 0;
}

// A reader context's stream and events (created on first use).
// Stream k of the pipelined passes, shared by device pipe k and host pipe k.  HIP maps streams
// onto GPU_MAX_HW_QUEUES (4) hardware queues: the synchronous context's stream plus these three
// keep one queue each, where separate streams for the two device pipes and the three host pipes
// (six in all) doubled pipes up on queues and serialised them (cfg1 host-in/host-out 46 M
// topics/s in a process that had used both kinds, 366 M with host pipes alone).
static_assert(EMQXGM_PIPES <= EMQXGM_HOST_PIPES, "device pipe k borrows host pipe k's stream");
hipStream_t pipe_stream(emqxgm* h, uint32_t k) {
  if (!h->pipe_streams[k] &&
      hipStreamCreateWithFlags(&h->pipe_streams[k], hipStreamNonBlocking) != hipSuccess)
    h->pipe_streams[k] = nullptr;
  return h->pipe_streams[k];
}

// emqxgm::geom_pipe from geom and pipe_wg_per_cu (same CUs, at most geom's workgroups per CU,
// so the scratch sized for geom -- spill lanes, census waves -- fits it)
void set_pipe_geometry(emqxgm* h) {
  const uint32_t wg = std::max<uint32_t>(1, std::min(h->pipe_wg_per_cu, h->geom.blocks / std::max<uint32_t>(1, h->geom.cus)));
  h->geom_pipe = walk_geometry(h->cfg.device, wg);
  h->geom_pipe.xrange_bytes = h->geom.xrange_bytes;
  h->geom_pipe.pair = h->geom.pair;
}

int ctx_init(emqxgm* h, PassCtx& c, hipStream_t shared = nullptr) {
  if (c.stream) return 0;
  if (shared) {
    c.stream = shared;
  } else {
    HIPCHK(h, hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    c.own_stream = true;
  }
  for (auto& e : c.ev) HIPCHK(h, hipEventCreate(&e));
  HIPCHK(h, hipEventCreateWithFlags(&c.done, hipEventDisableTiming));
  return 0;
}

void ctx_free(PassCtx& c) {
  if (c.stream) {
    (void)hipStreamSynchronize(c.stream);
    if (c.own_stream) (void)hipStreamDestroy(c.stream);
  }
  for (auto& e : c.ev)
    if (e) (void)hipEventDestroy(e);
  if (c.done) (void)hipEventDestroy(c.done);
  free_bufs(c.bufs);
  if (c.sc.ctl_host) (void)hipHostFree(c.sc.ctl_host);
  c = PassCtx();
}

// (Re)allocate a context's batch scratch for n topics, `words` words and `pairs` staged pairs.
int ensure_scratch(emqxgm* h, PassCtx& c, uint32_t n, uint64_t words, uint32_t pairs) {
  Scratch& s = c.sc;
  const uint32_t spill_need = std::max<uint32_t>(h->spill_want, WALK_SPILL_MIN);
  if (n <= s.n_cap && words <= s.w_cap && pairs <= s.p_cap && spill_need <= s.spill_items &&
      s.spill_lanes == h->geom.lanes && s.ctl)
    return 0;
  HIPCHK(h, hipStreamSynchronize(c.stream));
  h->st.buffer_grows += 1;
  const uint32_t ncap = std::max(n, s.n_cap);
  const uint64_t wcap = std::max(words, s.w_cap);
  const uint32_t pcap = (std::max(pairs, s.p_cap) + STAGE_CHUNK - 1) / STAGE_CHUNK * STAGE_CHUNK;
  const uint32_t scap = std::max(spill_need, s.spill_items);
  free_bufs(c.bufs);
  if (s.ctl_host) {
    (void)hipHostFree(s.ctl_host);
    s.ctl_host = nullptr;
  }
  s = Scratch();
  int rc = 0;
  const uint32_t stw = scan_tmp_words(ncap);
  if ((rc = dev_alloc(h, c, (void**)&s.nw, (size_t)ncap * 4)) ||
      (rc = dev_alloc(h, c, (void**)&s.wh, (size_t)wcap * 8)) ||
      (rc = dev_alloc(h, c, (void**)&s.rec, (size_t)(ncap + REC_BLOCK - 1) / REC_BLOCK * REC_BLOCK * 16 * REC_U4)) ||
      (rc = dev_alloc(h, c, (void**)&s.cnt, (size_t)ncap * 4)) ||
      (rc = dev_alloc(h, c, (void**)&s.row, (size_t)(ncap + 1) * 4)) ||
      (rc = dev_alloc(h, c, (void**)&s.row2, (size_t)(ncap + 1) * 4)) ||
      (rc = dev_alloc(h, c, (void**)&s.rej, (size_t)ncap * 4)) ||
      (rc = dev_alloc(h, c, (void**)&s.exact_id, (size_t)ncap * 4)) ||
      (rc = dev_alloc(h, c, (void**)&s.xh, (size_t)ncap * 8)) ||
      (rc = dev_alloc(h, c, (void**)&s.stg, (size_t)pcap * 12)) ||
      (rc = dev_alloc(h, c, (void**)&s.chk, (size_t)(pcap / STAGE_CHUNK + 1) * 4)) ||
      (rc = dev_alloc(h, c, (void**)&s.out, (size_t)pcap * 4)) ||
      (rc = dev_alloc(h, c, (void**)&s.out2, (size_t)pcap * 4)) ||
      (rc = dev_alloc(h, c, (void**)&s.scan_tmp, (size_t)stw * 4)) ||
      (rc = dev_alloc(h, c, (void**)&s.ctl, CTL_N * 4)) ||
      (rc = dev_alloc(h, c, (void**)&s.census,
                      (CENSUS_HDR + 3 * (h->geom.lanes / 64)) * sizeof(unsigned long long))) ||
      (rc = dev_alloc(h, c, (void**)&s.spill, (size_t)scap * h->geom.lanes * sizeof(uint2))) ||
      (rc = dev_alloc(h, c, (void**)&s.rlist, (size_t)h->reject_cap * 8)))
    return rc;
  s.r_cap = h->reject_cap;
  HIPCHK(h, hipHostMalloc((void**)&s.ctl_host, CTL_N * 4, hipHostMallocMapped | hipHostMallocPortable));
  HIPCHK(h, hipHostGetDevicePointer((void**)&s.ctl_host_dev, s.ctl_host, 0));
  s.n_cap = ncap;
  s.w_cap = wcap;
  s.p_cap = pcap;
  s.o_cap = pcap;
  s.scan_tmp_cap = stw;
  s.spill_items = scap;
  s.spill_lanes = h->geom.lanes;
  return 0;
}

// One device pass over n topics already in HBM.  Leaves results in the context's scratch (row,
// out, exact_id) and the total pair count in *pairs.
//
// Production order: tokenise -> walk -> verify (flags rejects, fixes counts) -> scan -> scatter.
// If a batch rejected more pairs than k_scatter adjusts in-line (a weak-hash test config or an
// adversarial index), the pass is redone on the legacy path: scan -> verify+scatter -> compaction.
//
// The pass is split so that a pipelined caller (emqxgm_match_device_submit/_wait,
// emqxgm_match_batch_submit/_wait) can enqueue one batch while an earlier one still runs on
// another stream: pass_prepare (scratch), pass_submit (takes the current epoch and enqueues every
// launch, then the control words to the host, no synchronisation), pass_check (after the stream
// has drained: 0 done, 1 redo, < 0 error) and pass_finish.

// Scratch for n topics; returns 0, or 2 when n == 0 (then the empty result is already set).
int pass_prepare(emqxgm* h, PassCtx& c, uint32_t n, uint64_t bytes_len) {
  const uint64_t words = bytes_len + n + 1;  // token array: level k of topic t at off[t] + t + k
  if (words > 0xFFFFFFFFull) {
    set_err(h, "batch too large: topic bytes + topics must stay below 2^32");
    return -E2BIG;
  }
  uint32_t want_pairs = std::max<uint32_t>(c.sc.p_cap, std::max<uint32_t>(1u << 20, n * 4u));
  // room for every walk wave's static first chunk (walk_static_chunks; without it each wave's
  // first flush takes an atomic on one counter, serialised at ~88/us), up to 16M slots
  const uint64_t stat_need = (uint64_t)walk_blocks(h->geom, n, WALK_SHALLOW) * (256 / 64) * STAGE_CHUNK;
  want_pairs = std::max<uint32_t>(want_pairs, (uint32_t)std::min<uint64_t>(stat_need, 1u << 24));
  int rc = ensure_scratch(h, c, std::max<uint32_t>(n, 1), words, want_pairs);
  if (rc) return rc;
  if (n == 0) {
    HIPCHK(h, hipMemsetAsync(c.sc.row, 0, 4, c.stream));
    HIPCHK(h, hipStreamSynchronize(c.stream));
    return 2;
  }
  return 0;
}

// The staging layout of a pass over n topics (StgFmt): packed when topic ids, filter ids below
// fid_bound and a rank field of at least STG_MIN_RANK_BITS fit one 64-bit word with the reject
// bit.  The legacy path (k_verify_scatter) and an epoch that saw a rank outgrow the field stage
// wide.
StgFmt stg_format(uint32_t n, uint64_t fid_bound, bool wide, uint32_t rank_bits_cap) {
  StgFmt F;
  auto bits = [](uint64_t v) {  // bits to hold every value below v
    uint32_t b = 1;
    while (b < 64 && (1ull << b) < v) ++b;
    return b;
  };
  static const bool force_wide = getenv("EMQXGM_STAGE_WIDE") != nullptr;  // (A/B runs)
  if (wide || fid_bound == 0 || force_wide) return F;
  const uint32_t tb = bits(n), fb = bits(fid_bound);
  if (tb + fb + 1 + std::min(STG_MIN_RANK_BITS, rank_bits_cap ? rank_bits_cap : 31u) > 64) return F;
  const uint32_t rb = std::min<uint32_t>({64 - 1 - tb - fb, 31u, rank_bits_cap ? rank_bits_cap : 31u});
  F.pk = 1;
  F.fsh = 1 + rb;
  F.tsh = 64 - tb;
  F.fmask = (uint32_t)((1ull << fb) - 1);
  F.rmask = (uint32_t)((1ull << rb) - 1);
  return F;
}

// Every launch of one pass against epoch E on the context's stream (caller holds emu).
int pass_enqueue(emqxgm* h, PassCtx& c, const Epoch& E, const uint8_t* d_bytes,
                 const uint32_t* d_off, uint32_t n, bool legacy, bool census) {
  Scratch& s = c.sc;
  hipStream_t st = c.stream;
  DevIndex ix = E.ix;
  ix.leafp_mask = h->leafp_mask;
  // the epoch's uploads / patches must have landed (a full build's have: its wait is skipped)
  if (!E.ready_seen.load(std::memory_order_relaxed)) {
    if (hipEventQuery(E.ready) == hipSuccess)
      E.ready_seen.store(true, std::memory_order_relaxed);
    else
      HIPCHK(h, hipStreamWaitEvent(st, E.ready, 0));
  }
  if (h->profiling) HIPCHK(h, hipEventRecord(c.ev[0], st));
  RoctxRange rr(h->roctx, census ? "emqxgm.pass.census" : "emqxgm.pass");
  bool ctl_sent = false;  // the control words already go to the host mirror
  // k_tok starts the control words (no memset launch); CTL_XHIT compares to this pass's number
  s.xseq = s.xseq + 1 ? s.xseq + 1 : 1;
  if (census)
    HIPCHK(h, hipMemsetAsync(s.census, 0,
                             (CENSUS_HDR + 3 * (h->geom.lanes / 64)) * sizeof(unsigned long long),
                             st));
  c.census = census;
  c.walk_level = (census ? E.census_level : E.walk_level).load(std::memory_order_relaxed);
  s.fmt = stg_format(n, ix.fid_bound, legacy || E.wide_stage.load(std::memory_order_relaxed),
                     h->stage_rank_bits.load(std::memory_order_relaxed));
  c.packed = s.fmt.pk != 0;
  // (census passes and the synchronous ones keep the full geometry)
  WalkGeom WG_ = (c.pipelined && !census) ? h->geom_pipe : h->geom;
  if (census) WG_.pair = 0;  // census walks are one lane per topic (their buffers count lanes)
  if (!s.fmt.pk) WG_.pair = 0;  // the pair walk stages packed only (gm_walk.inc put)
  const uint32_t stat = ix.trie_empty ? 0u : walk_static_chunks(WG_, n, c.walk_level, s.p_cap);
  roctx_mark(h->roctx, "k_tok");
  // (per-topic reject counts: only the verification passes write -- and then read -- them;
  // k_tok zeroes them as it goes, like the control words: a memset launch between the passes of
  // two pipes serialised them, r03)
  uint32_t claim0[WALK_SHARDS] = {};
  if (!ix.trie_empty) walk_claim_init(WG_, n, c.walk_level, claim0);
  HIPCHK(h, launch_tok(d_bytes, d_off, n, ix, s, st, stat * STAGE_CHUNK,
                       !ix.trie_empty && (ix.needs_verify || legacy), claim0, c.src_bytes, c.src_off));
  c.src_bytes = nullptr;
  c.src_off = nullptr;
  if (h->profiling) HIPCHK(h, hipEventRecord(c.ev[4], st));
  roctx_mark(h->roctx, "k_exact");
  HIPCHK(h, launch_exact(d_bytes, d_off, n, ix, s, h->geom, st));
  if (h->profiling) HIPCHK(h, hipEventRecord(c.ev[1], st));
  if (ix.trie_empty) {
    HIPCHK(h, hipMemsetAsync(s.row, 0, (size_t)(n + 1) * 4, st));
  } else {
    roctx_mark(h->roctx, "k_walk");
    HIPCHK(h, launch_walk(ix, s, n, WG_, st, census ? s.census : nullptr, c.walk_level, stat));
    if (h->profiling) HIPCHK(h, hipEventRecord(c.ev[2], st));
    if (!legacy) {
      // pairs of filters made of short (exact) tokens need no byte check (gm_verify.inc)
      roctx_mark(h->roctx && ix.needs_verify, "k_verify");
      if (ix.needs_verify) HIPCHK(h, launch_verify(d_bytes, d_off, ix, s, n, h->geom, st));
      // the scan's last block mirrors the control words to the host (no launch of its own); a
      // batch of one scan tile has its scan done inside k_scatter (one launch less)
      const bool fuse = n <= SCATTER_SCAN_MAX;
      if (!fuse) {
        roctx_mark(h->roctx, "k_scan");
        HIPCHK(h, launch_scan_ctl(s.cnt, s.row, n, s.scan_tmp, s.ctl + CTL_TOTAL, s.ctl, s.ctl_host_dev, st));
      }
      ctl_sent = true;
      roctx_mark(h->roctx, "k_scatter");
      HIPCHK(h, launch_scatter(s, n, h->geom, st, ctl_sent, fuse));
    } else {
      HIPCHK(h, launch_scan(s.cnt, s.row, n, s.scan_tmp, s.ctl + CTL_TOTAL, st));
      HIPCHK(h, launch_verify_scatter(d_bytes, d_off, ix, s, n, st));
    }
  }
  if (h->profiling) HIPCHK(h, hipEventRecord(c.ev[3], st));
  if (!ctl_sent) {
    HIPCHK(h, launch_ctl_out(s.ctl, s.ctl_host_dev, st));
  }
  return 0;
}

// Marks the end of the table reads a context enqueued (caller holds emu): a later delta commit
// orders its patches behind this point.
int mark_done(emqxgm* h, PassCtx& c) {
  (void)h, (void)c;  // (until r03 an event per pass; a commit now records them itself)
  return 0;
}

// Takes the current epoch and enqueues one pass on it.  emu is held for the enqueue only (a few
// asynchronous launches); the pass then runs while writers build, patch and swap.
int pass_submit(emqxgm* h, PassCtx& c, const uint8_t* d_bytes, const uint32_t* d_off,
                uint32_t n, bool legacy, bool census) {
  std::lock_guard<std::mutex> g(h->emu);
  c.epoch = h->cur;
  int rc = pass_enqueue(h, c, *c.epoch, d_bytes, d_off, n, legacy, census);
  return rc ? rc : mark_done(h, c);
}

// After the pass's stream drained: 0 = done, 1 = redo (scratch grown / walk variant or path
// switched), < 0 = error.
int pass_check(emqxgm* h, PassCtx& c, uint32_t n, uint64_t bytes_len, int attempt, bool& legacy) {
  Scratch& s = c.sc;
  Epoch& E = *c.epoch;
  const uint64_t words = bytes_len + n + 1;
  if (attempt > 6) {
    set_err(h, "match pass did not converge");
    return -ENOMEM;
  }
  const uint32_t top = s.ctl_host[CTL_PAIR_TOP];
  auto rerun = [&]() {
    std::lock_guard<std::mutex> g(h->stmu);
    h->st.reruns += 1;
  };
  if (top > s.p_cap) {
    // staging overflow: nothing beyond the capacity was written; grow and redo the pass
    rerun();
    const uint64_t np = std::min<uint64_t>(0xF0000000ull, (uint64_t)top * 2 + (1u << 20));
    int rc = ensure_scratch(h, c, n, words, (uint32_t)np);
    return rc ? rc : 1;
  }
  if (s.ctl_host[CTL_ERR] && c.walk_level < WALK_SPILL) {
    // a walk lane's item stack outgrew its LDS stack: redo with the next variant (deep stack,
    // then deep + spill), kept for this committed index
    rerun();
    std::atomic<uint32_t>& lvl = c.census ? E.census_level : E.walk_level;
    // the next variant; WALK_PAIRED is skipped when it would launch the kernel that just
    // overflowed (a batch already walked in pairs) or pairs nothing (census and wide passes,
    // pairs off): ADVICE r05, one wasted re-run per epoch otherwise
    uint32_t next = c.walk_level + 1;
    if (next == WALK_PAIRED) {
      WalkGeom g = c.pipelined && !c.census ? h->geom_pipe : h->geom;
      if (c.census || !c.packed) g.pair = 0;
      if (!walk_pair(g, n, WALK_PAIRED) || walk_pair(g, n, c.walk_level)) next = WALK_DEEP;
    }
    uint32_t cur = lvl.load();
    while (cur < next && !lvl.compare_exchange_weak(cur, next)) {
    }
    return 1;
  }
  if (s.ctl_host[CTL_ERR]) {
    // a walk lane's item stack outgrew the spill: grow it to the proven bound and redo
    const uint32_t bound = walk_spill_bound(E.ix.max_depth);
    if (s.spill_items >= bound) {
      set_err(h, "walk item stack exceeded its bound");
      return -EIO;
    }
    rerun();
    h->spill_want = bound;
    int rc = ensure_scratch(h, c, n, words, s.p_cap);
    return rc ? rc : 1;
  }
  if (c.packed && s.ctl_host[CTL_PKOVF]) {
    // a topic's rank outgrew the packed staging's field: stage this epoch's passes wide
    rerun();
    E.wide_stage.store(true, std::memory_order_relaxed);
    return 1;
  }
  if (!legacy && s.ctl_host[CTL_LEGACY]) {
    rerun();
    legacy = true;
    return 1;
  }
  return 0;
}

int pass_finish(emqxgm* h, PassCtx& c, uint32_t n, bool legacy, uint32_t* pairs, uint64_t* census) {
  Scratch& s = c.sc;
  hipStream_t st = c.stream;
  float tok = 0, exact = 0, walk = 0, all = 0;
  const bool timed = h->profiling;
  const bool walked = !c.epoch->ix.trie_empty;
  if (timed) {
    HIPCHK(h, hipEventElapsedTime(&tok, c.ev[0], c.ev[4]));
    HIPCHK(h, hipEventElapsedTime(&exact, c.ev[4], c.ev[1]));
    if (walked) HIPCHK(h, hipEventElapsedTime(&walk, c.ev[1], c.ev[2]));
    HIPCHK(h, hipEventElapsedTime(&all, c.ev[0], c.ev[3]));
  }
  if (legacy && s.ctl_host[CTL_ANY_REJ]) {
    HIPCHK(h, launch_fixup(s, n, st));
    HIPCHK(h, hipMemcpyAsync(s.ctl_host + CTL_TOTAL, s.ctl + CTL_TOTAL, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    std::swap(s.row, s.row2);
    std::swap(s.out, s.out2);
  }
  *pairs = s.ctl_host[CTL_TOTAL];
  {
    std::lock_guard<std::mutex> g(h->stmu);
    if (timed) {
      h->st.tok_ms += tok;
      h->st.tok_launches += 1;
      h->st.exact_ms += exact;
      if (walked) {
        h->st.walk_ms += walk;
        h->st.walk_launches += 1;
      }
      h->st.total_ms += all;
    }
    if (s.ctl_host[CTL_ANY_REJ]) h->st.rejected_pairs += legacy ? 0 : s.ctl_host[CTL_NREJ];
    if (legacy) h->st.legacy_batches += 1;
    h->st.batches += 1;
    h->st.topics += n;
    h->st.pairs += *pairs;
  }
  if (census) {
    if (const char* wf = getenv("EMQXGM_WAVE_TIMES")) {  // diagnostic: per-wave timeline
      std::vector<unsigned long long> wt(3 * (h->geom.lanes / 64));
      HIPCHK(h, hipMemcpy(wt.data(), s.census + CENSUS_HDR, wt.size() * 8, hipMemcpyDeviceToHost));
      if (FILE* fp = fopen(wf, "wb")) {
        fwrite(wt.data(), 8, wt.size(), fp);
        fclose(fp);
      }
    }
    unsigned long long cv[CENSUS_HDR] = {0};
    HIPCHK(h, hipMemcpy(cv, s.census, sizeof cv, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < 2 * CENSUS_DEPTHS; ++i) h->census_depth[i] = cv[CENSUS_N + i];
    census[0] = cv[0];
    census[1] = cv[1];
    census[2] = *pairs;
    std::vector<uint32_t> nw(n);
    HIPCHK(h, hipMemcpy(nw.data(), s.nw, (size_t)n * 4, hipMemcpyDeviceToHost));
    uint64_t nwords = 0;
    for (uint32_t v : nw) nwords += v;
    census[3] = nwords;
    census[4] = cv[2];
    census[5] = cv[3];
  }
  return 0;
}

// A whole synchronous pass on context c (redone until it converges).  c.epoch is the epoch the
// result belongs to; the caller drops it when done with the result.
int run_device(emqxgm* h, PassCtx& c, const uint8_t* d_bytes, const uint32_t* d_off, uint32_t n,
               uint64_t bytes_len, uint32_t* pairs, uint64_t* census = nullptr) {
  int rc = pass_prepare(h, c, n, bytes_len);
  if (rc == 2) {
    *pairs = 0;
    return 0;
  }
  if (rc) return rc;
  bool legacy = false;
  for (int attempt = 0;; ++attempt) {
    if ((rc = pass_submit(h, c, d_bytes, d_off, n, legacy, census != nullptr))) return rc;
    HIPCHK(h, hipStreamSynchronize(c.stream));
    rc = pass_check(h, c, n, bytes_len, attempt, legacy);
    if (rc < 0) return rc;
    if (rc == 0) break;
  }
  return pass_finish(h, c, n, legacy, pairs, census);
}

int fan_alloc(emqxgm* h, std::vector<DevBuf>& keep, uint32_t** p, size_t words) {
  HIPCHK(h, hipMalloc((void**)p, std::max<size_t>(words * 4, 16)));
  DevBuf b;
  b.p = *p;
  b.bytes = words * 4;
  keep.push_back(b);
  return 0;
}

// Publish fan-out over the match result of the last run_device pass on the sync context (n
// topics): counts, two scans, then (outputs grown to the totals) the fill.  Leaves the results in
// h->fs.  The fan-out tables must be those of the epoch the match ran against: emu is held from
// the count pass to the fill pass (one short host wait in between), and 1 is returned when a
// commit published another epoch since the match (the caller redoes both).
int run_fanout(emqxgm* h, uint32_t n, uint32_t* n_routes, uint32_t* n_deliv) {
  PassCtx& c = h->sync;
  FanScratch& f = h->fs;
  Scratch& s = c.sc;
  hipStream_t st = c.stream;
  int rc = 0;
  if (n > f.n_cap || !f.cr) {
    HIPCHK(h, hipStreamSynchronize(st));
    free_bufs(h->fan_bufs);
    const uint32_t cap = std::max(n, f.n_cap);
    if ((rc = fan_alloc(h, h->fan_bufs, &f.cr, cap)) || (rc = fan_alloc(h, h->fan_bufs, &f.cd, cap)) ||
        (rc = fan_alloc(h, h->fan_bufs, &f.rp, (size_t)cap + 1)) ||
        (rc = fan_alloc(h, h->fan_bufs, &f.dp, (size_t)cap + 1)))
      return rc;
    f.n_cap = cap;
  }
  if (n == 0) {
    *n_routes = *n_deliv = 0;
    return 0;
  }
  std::lock_guard<std::mutex> g(h->emu);
  if (h->cur != c.epoch) return 1;
  const DevIndex& ix = c.epoch->ix;
  HIPCHK(h, launch_fanout(ix, s, f, n, false, st));
  HIPCHK(h, launch_scan(f.cr, f.rp, n, s.scan_tmp, s.ctl + CTL_FAN_R, st));
  HIPCHK(h, launch_scan(f.cd, f.dp, n, s.scan_tmp, s.ctl + CTL_FAN_D, st));
  HIPCHK(h, hipMemcpyAsync(s.ctl_host + CTL_FAN_R, s.ctl + CTL_FAN_R, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(h, hipStreamSynchronize(st));
  const uint32_t nr = s.ctl_host[CTL_FAN_R], nd = s.ctl_host[CTL_FAN_D];
  if (nr > f.r_cap || nd > f.d_cap || !f.o_rf) {
    free_bufs(h->fan_out_bufs);
    const uint32_t rc_ = std::max(nr, f.r_cap), dc = std::max(nd, f.d_cap);
    if ((rc = fan_alloc(h, h->fan_out_bufs, &f.o_rf, rc_)) ||
        (rc = fan_alloc(h, h->fan_out_bufs, &f.o_rd, rc_)) ||
        (rc = fan_alloc(h, h->fan_out_bufs, &f.o_df, dc)) ||
        (rc = fan_alloc(h, h->fan_out_bufs, &f.o_ds, dc)))
      return rc;
    f.r_cap = rc_;
    f.d_cap = dc;
  }
  HIPCHK(h, launch_fanout(ix, s, f, n, true, st));
  if ((rc = mark_done(h, c))) return rc;
  *n_routes = nr;
  *n_deliv = nd;
  return 0;
}

// Grows a pinned host buffer to `bytes` (keep: preserve the old contents).
int pinned_reserve(emqxgm* h, emqxgm::Pinned& b, size_t bytes, bool keep) {
  if (bytes <= b.cap) return 0;
  h->st.buffer_grows += 1;
  const size_t cap = std::max<size_t>(bytes + bytes / 2, 1 << 16);
  void* p = nullptr;
  HIPCHK(h, hipHostMalloc(&p, cap, hipHostMallocDefault));
  if (keep && b.p && b.cap) memcpy(p, b.p, b.cap);
  if (b.p) (void)hipHostFree(b.p);
  b.p = p;
  b.cap = cap;
  return 0;
}

int ensure_input(emqxgm* h, uint64_t bytes, uint64_t offs) {
  if (bytes > h->in_bytes_cap) {
    if (h->d_in_bytes) (void)hipFree(h->d_in_bytes);
    h->d_in_bytes = nullptr;
    const uint64_t cap = std::max<uint64_t>(bytes, 1 << 20);
    HIPCHK(h, hipMalloc((void**)&h->d_in_bytes, cap));
    h->in_bytes_cap = cap;
  }
  if (offs > h->in_off_cap) {
    if (h->d_in_off) (void)hipFree(h->d_in_off);
    h->d_in_off = nullptr;
    const uint64_t cap = std::max<uint64_t>(offs, 1 << 16);
    HIPCHK(h, hipMalloc((void**)&h->d_in_off, cap * 4));
    h->in_off_cap = cap;
  }
  return 0;
}

// Completes an in-flight device pipe (stream drained, checked, redone synchronously if it has
// to be).
int pipe_complete(emqxgm* h, emqxgm::Pipe& p) {
  if (p.state != 1) return 0;
  HIPCHK(h, hipStreamSynchronize(p.c.stream));
  bool legacy = false;
  int rc = pass_check(h, p.c, p.n, p.bytes_len, 0, legacy);
  if (rc < 0) {
    p.state = 0;
    p.c.epoch.reset();
    return rc;
  }
  rc = rc == 0 ? pass_finish(h, p.c, p.n, false, &p.pairs, nullptr)
               : run_device(h, p.c, p.d_bytes, p.d_off, p.n, p.bytes_len, &p.pairs);
  p.state = rc ? 0 : 2;
  p.c.epoch.reset();
  return rc;
}

int drain_pipes(emqxgm* h) {
  for (auto& p : h->pipes)
    if (int rc = pipe_complete(h, p)) return rc;
  return 0;
}

// Pinned host buffer a kernel can write (its device-side address in *dev).
int host_buf(emqxgm* h, uint32_t** p, uint64_t entries) {
  HIPCHK(h, hipHostMalloc((void**)p, std::max<uint64_t>(entries, 16) * 4,
                          hipHostMallocMapped | hipHostMallocPortable));
  return 0;
}

int host_pipe_reserve(emqxgm* h, emqxgm::HostPipe& p, uint64_t n, uint64_t bytes, uint64_t fid) {
  if (bytes > p.bytes_cap) {
    h->st.buffer_grows += 1;
    if (p.d_bytes) (void)hipFree(p.d_bytes);
    p.d_bytes = nullptr;
    p.bytes_cap = 0;
    const uint64_t cap = std::max<uint64_t>(bytes + bytes / 4, 1 << 20);
    HIPCHK(h, hipMalloc((void**)&p.d_bytes, cap));
    p.bytes_cap = cap;
  }
  if (n + 1 > p.off_cap) {
    h->st.buffer_grows += 1;
    if (p.d_off) (void)hipFree(p.d_off);
    p.d_off = nullptr;
    p.off_cap = 0;
    const uint64_t cap = std::max<uint64_t>(n + 1 + n / 4, 1 << 16);
    HIPCHK(h, hipMalloc((void**)&p.d_off, cap * 4));
    p.off_cap = cap;
  }
  if (n + 1 > p.row_cap) {
    h->st.buffer_grows += 1;
    if (p.h_row) (void)hipHostFree(p.h_row);
    if (p.h_exact) (void)hipHostFree(p.h_exact);
    delete[] p.h_none;
    p.h_row = p.h_exact = p.h_none = nullptr;
    p.row_cap = 0;
    const uint64_t cap = std::max<uint64_t>(n + 1 + n / 4, 1 << 16);
    int rc = 0;
    if ((rc = host_buf(h, &p.h_row, cap)) || (rc = host_buf(h, &p.h_exact, cap))) return rc;
    p.h_none = new (std::nothrow) uint32_t[cap];
    if (!p.h_none) return -ENOMEM;
    std::fill(p.h_none, p.h_none + cap, NONE);
    p.row_cap = cap;
  }
  if (fid > p.fid_cap) {
    h->st.buffer_grows += 1;
    if (p.h_fid) (void)hipHostFree(p.h_fid);
    p.h_fid = nullptr;
    p.fid_cap = 0;
    int rc = host_buf(h, &p.h_fid, fid);
    if (rc) return rc;
    p.fid_cap = fid;
  }
  return 0;
}

// The pass's results into the host pipe's pinned buffers, enqueued on its stream: by a copy
// kernel writing host memory over PCIe (the pair count is read on the device, so nothing waits
// for the host), or by hipMemcpyAsync for the row pointers (the filter ids then follow in _wait,
// once their count is known, and so do the exact ids, only when some name has a route key:
// CTL_XHIT; otherwise the batch's exact ids are a prefilled all-NONE buffer and nothing crosses
// PCIe for them -- a 4M-topic batch's 16 MB).
int host_pipe_copy_out(emqxgm* h, emqxgm::HostPipe& p) {
  const Scratch& s = p.c.sc;
  if (h->host_out_mode == 1) {
    void *dr = nullptr, *de = nullptr, *df = nullptr;
    HIPCHK(h, hipHostGetDevicePointer(&dr, p.h_row, 0));
    HIPCHK(h, hipHostGetDevicePointer(&de, p.h_exact, 0));
    HIPCHK(h, hipHostGetDevicePointer(&df, p.h_fid, 0));
    CopyOut a{s.row, (uint32_t*)dr, p.n + 1, nullptr, p.n + 1};
    CopyOut b{s.exact_id, (uint32_t*)de, p.n, nullptr, p.n};
    CopyOut f{s.out, (uint32_t*)df, 0, s.ctl + CTL_TOTAL, (uint32_t)std::min<uint64_t>(p.fid_cap, s.p_cap)};
    HIPCHK(h, launch_copy_out(a, b, f, p.c.stream));
  } else {
    HIPCHK(h, hipMemcpyAsync(p.h_row, s.row, ((size_t)p.n + 1) * 4, hipMemcpyDeviceToHost, p.c.stream));
  }
  return 0;
}

// Completes an in-flight host pipe: checks the pass (redoing it synchronously when it has to be)
// and makes sure every result array is in its pinned buffer.
int grow_dev(emqxgm* h, DevBuf& b, uint64_t bytes, hipStream_t s);

// The pairs' filter bytes of a completed pass (its epoch still held: the device string pool
// the gather reads is the epoch's), into the pipe's pinned buffers.
int host_pipe_gather(emqxgm* h, emqxgm::HostPipe& p) {
  const Scratch& s = p.c.sc;
  const DevIndex& ix = p.c.epoch->ix;
  const uint32_t m = p.pairs;
  const uint64_t tw = scan_tmp_words(std::max<uint32_t>(m, 1));
  const uint64_t words = 2ull * m + 1 + tw + 2;
  int rc = grow_dev(h, p.d_fb, words * 4, p.c.stream);
  if (rc) return rc;
  uint32_t* len = (uint32_t*)p.d_fb.p;
  uint32_t* ooff = len + m;
  uint32_t* total = ooff + m + 1;
  uint32_t* tmp = total + 2;
  HIPCHK(h, launch_filter_len(s.out, m, ix.foff, len, ooff, tmp, total, p.c.stream));
  uint32_t nb = 0;
  HIPCHK(h, hipMemcpyAsync(&nb, total, 4, hipMemcpyDeviceToHost, p.c.stream));
  HIPCHK(h, hipStreamSynchronize(p.c.stream));
  if (m == 0) nb = 0;
  const uint64_t at = ((words * 4 + 255) / 256) * 256;  // the bytes after the words
  if ((rc = grow_dev(h, p.d_fb, at + nb + 1, p.c.stream)) ||
      (rc = pinned_reserve(h, p.h_fboff, ((size_t)m + 1) * 4, false)) ||
      (rc = pinned_reserve(h, p.h_fb, (size_t)nb + 1, false)))
    return rc;
  len = (uint32_t*)p.d_fb.p;  // (grown: re-derive; the scan results were kept by grow_dev)
  ooff = len + m;
  uint8_t* out = (uint8_t*)p.d_fb.p + at;
  HIPCHK(h, launch_filter_gather(s.out, m, ix.foff, ix.fbytes, ooff, out, p.c.stream));
  HIPCHK(h, hipMemcpyAsync(p.h_fboff.p, ooff, ((size_t)m + 1) * 4, hipMemcpyDeviceToHost, p.c.stream));
  if (nb) HIPCHK(h, hipMemcpyAsync(p.h_fb.p, out, nb, hipMemcpyDeviceToHost, p.c.stream));
  HIPCHK(h, hipStreamSynchronize(p.c.stream));
  p.fb_bytes = nb;
  return 0;
}

int host_pipe_complete(emqxgm* h, emqxgm::HostPipe& p, bool gather = false) {
  if (p.state != 1) return 0;
  HIPCHK(h, hipStreamSynchronize(p.c.stream));
  bool legacy = false;
  int rc = pass_check(h, p.c, p.n, p.bytes_len, 0, legacy);
  // copy_out enqueued the row pointers behind the pass (both modes; with the gather behind the
  // pass they travel in its block instead), the copy kernel (mode 1) the exact ids and up to
  // fid_cap filter ids too; a redone pass copies everything here
  bool rows_copied = p.rows_enq, redone = false;
  if (rc == 0) {
    rc = pass_finish(h, p.c, p.n, false, &p.pairs, nullptr);
  } else if (rc == 1) {
    rc = run_device(h, p.c, p.d_bytes, p.d_off, p.n, p.bytes_len, &p.pairs);
    rows_copied = false;
    redone = true;
  }
  // submitted with the gather behind the pass: done when its copies covered the window
  const uint32_t blk_total = p.fb_async ? *(const uint32_t*)p.h_blk.p : 0u;
  const bool async_done = rc == 0 && gather && p.fb_async && !redone &&
                          p.pairs <= p.fb_pairs_copy && blk_total <= p.fb_bytes_copy;
  if (async_done) p.fb_bytes = p.pairs ? blk_total : 0;
  p.fb_fast = async_done;
  if (rc == 0 && gather && !async_done) {
    if (p.fb_async) h->st.sync_gathers += 1;
    rc = host_pipe_gather(h, p);
  }
  p.fb_async = false;
  p.c.epoch.reset();
  if (rc < 0) {
    p.state = 0;
    return rc;
  }
  if (gather && p.n) {  // the next async window's copy sizes follow the recent windows
    const double ppt = (double)p.pairs / p.n, bpp = p.pairs ? (double)p.fb_bytes / p.pairs : 0.0;
    p.fb_ppt = std::max(ppt, 0.9 * p.fb_ppt);
    p.fb_bpp = std::max(bpp, 0.9 * p.fb_bpp);
  }
  if (async_done) {  // filter ids, exact ids, byte offsets and bytes are in the packed block
    p.state = 2;
    return 0;
  }
  const Scratch& s = p.c.sc;
  const bool mode1 = h->host_out_mode == 1;
  const bool fids_copied = rows_copied && mode1 && p.pairs <= p.fid_cap;
  if (p.pairs > p.fid_cap &&
      (rc = host_pipe_reserve(h, p, p.n, 0, (uint64_t)p.pairs + p.pairs / 4))) {
    p.state = 0;
    return rc;
  }
  bool enq = false;
  if (!rows_copied) {
    HIPCHK(h, hipMemcpyAsync(p.h_row, s.row, ((size_t)p.n + 1) * 4, hipMemcpyDeviceToHost, p.c.stream));
    enq = true;
  }
  // a redone pass refreshed ctl_host
  const bool exact_copied = rows_copied && mode1;
  p.exact_none = !exact_copied && s.ctl_host[CTL_XHIT] != s.xseq;
  if (!exact_copied && !p.exact_none) {
    HIPCHK(h, hipMemcpyAsync(p.h_exact, s.exact_id, (size_t)p.n * 4, hipMemcpyDeviceToHost, p.c.stream));
    enq = true;
  }
  if (!fids_copied && p.pairs) {
    HIPCHK(h, hipMemcpyAsync(p.h_fid, s.out, (size_t)p.pairs * 4, hipMemcpyDeviceToHost, p.c.stream));
    enq = true;
  }
  if (enq) HIPCHK(h, hipStreamSynchronize(p.c.stream));
  p.state = 2;
  return 0;
}

// A device buffer of at least `bytes`, its contents kept (stream-ordered on s).
int grow_dev(emqxgm* h, DevBuf& b, uint64_t bytes, hipStream_t s) {
  if (bytes <= b.bytes && b.p) return 0;
  h->st.buffer_grows += 1;
  const uint64_t cap = std::max<uint64_t>(bytes + bytes / 2, 1 << 20);
  void* p = nullptr;
  HIPCHK(h, hipMalloc(&p, cap));
  if (b.p) {
    HIPCHK(h, hipMemcpyAsync(p, b.p, b.bytes, hipMemcpyDeviceToDevice, s));
    HIPCHK(h, hipStreamSynchronize(s));
    (void)hipFree(b.p);
  }
  b.p = p;
  b.bytes = cap;
  return 0;
}

void host_pipe_free(emqxgm::HostPipe& p) {
  ctx_free(p.c);
  if (p.fin) (void)hipEventDestroy(p.fin);
  if (p.d_fb.p) (void)hipFree(p.d_fb.p);
  for (void* q : {p.h_fboff.p, p.h_fb.p})
    if (q) (void)hipHostFree(q);
  if (p.d_bytes) (void)hipFree(p.d_bytes);
  if (p.d_off) (void)hipFree(p.d_off);
  for (uint32_t* q : {p.h_row, p.h_exact, p.h_fid})
    if (q) (void)hipHostFree(q);
  delete[] p.h_none;
  p = emqxgm::HostPipe();
}

// Writers hold wmu then pmu (exclusive) while they may grow the registry.
struct WriterLock {
  std::lock_guard<std::mutex> w;
  std::unique_lock<std::shared_mutex> p;
  explicit WriterLock(emqxgm* h) : w(h->wmu), p(h->pmu) {}
};

// The writer lock of a batch set.  A synchronous one (prio: EMQXGM_SET_COMMIT, the writing
// node's hook) announces itself, so that a bulk set (a resync's 64k-topic chunk) lets it in
// between two of its slices: a subscribe waits for one slice, not for the chunk.
std::unique_lock<std::mutex> set_lock(emqxgm* h, bool prio) {
  if (!prio) return std::unique_lock<std::mutex>(h->wmu);
  h->prio_waiting.fetch_add(1);
  std::unique_lock<std::mutex> lk(h->wmu);
  h->prio_waiting.fetch_sub(1);
  return lk;
}
constexpr uint64_t SET_SLICE = 4096;  // topics of a bulk set per writer-lock hold
void let_prio_in(emqxgm* h, std::unique_lock<std::mutex>& lk) {
  if (h->prio_waiting.load() == 0) return;
  lk.unlock();
  while (h->prio_waiting.load() != 0) std::this_thread::yield();
  lk.lock();
}

}  // namespace

extern "C" {

int emqxgm_abi_version(void) { return EMQXGM_ABI_VERSION; }
int emqxgm_device_pipes(void) { return EMQXGM_PIPES; }

int emqxgm_create(const emqxgm_cfg* cfg, emqxgm_t** out) {
  if (!out) return -EINVAL;
  *out = nullptr;
  emqxgm* h = new (std::nothrow) emqxgm();
  if (!h) return -ENOMEM;
  if (cfg) h->cfg = *cfg;
  // word_hash_bits 0 (or >= 63): production tokens (short words exact, long words hashed);
  // 1..62: collision-test mode, every word hashed and masked to that many bits
  if (h->cfg.word_hash_bits >= 63) h->cfg.word_hash_bits = 0;
  h->test_mask = h->cfg.word_hash_bits ? ((1ull << h->cfg.word_hash_bits) - 1ull) : 0ull;
  if (h->cfg.full_hash_bits == 0 || h->cfg.full_hash_bits > 64) h->cfg.full_hash_bits = 64;
  if (h->cfg.batch_max == 0) h->cfg.batch_max = 4u << 20;
  if (h->cfg.reject_cap) h->reject_cap = h->cfg.reject_cap;
  if (const char* e = getenv("EMQXGM_ROCTX")) h->roctx = e[0] == '1';
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || h->cfg.device < 0 ||
      h->cfg.device >= ndev) {
    delete h;
    return -EIO;
  }
  if (hipSetDevice(h->cfg.device) != hipSuccess ||
      ctx_init(h, h->sync) != 0) {
    emqxgm_destroy(h);
    return -EIO;
  }
  h->wstream = h->sync.stream;
  // the delta commits' patch staging (pinned + device) and its event, sized now: a subscribe's
  // commit never allocates (patch_flush grows them only for larger deltas)
  h->h_stage_bytes = h->d_patch.bytes = PATCH_STAGE0;
  if (hipHostMalloc((void**)&h->h_stage, PATCH_STAGE0, hipHostMallocDefault) != hipSuccess ||
      hipMalloc(&h->d_patch.p, PATCH_STAGE0) != hipSuccess ||
      hipEventCreateWithFlags(&h->patch_ev, hipEventDisableTiming) != hipSuccess ||
      hipEventRecord(h->patch_ev, h->wstream) != hipSuccess) {
    emqxgm_destroy(h);
    return -EIO;
  }
  {
    // a kernel's first launch in the process loads its code object (r05's first subscribe paid
    // 5-8 ms for it): k_patch runs once now -- one entry copying a staging word onto another --
    // so the first subscribe's delta commit does not
    PatchEnt pe{};
    pe.dst = (uint64_t)(uintptr_t)((uint8_t*)h->d_patch.p + 64);
    pe.s = 0;
    pe.w = 1;
    memcpy(h->h_stage, &pe, sizeof pe);
    memset(h->h_stage + sizeof pe, 0, 16);
    const uint32_t* src = (const uint32_t*)((uint8_t*)h->d_patch.p + sizeof pe);
    if (hipMemcpyAsync(h->d_patch.p, h->h_stage, sizeof pe + 16, hipMemcpyHostToDevice, h->wstream) != hipSuccess ||
        launch_patch((const PatchEnt*)h->d_patch.p, 1, src, h->wstream) != hipSuccess ||
        hipStreamSynchronize(h->wstream) != hipSuccess) {
      emqxgm_destroy(h);
      return -EIO;
    }
  }
  h->geom = walk_geometry(h->cfg.device, h->cfg.walk_wg_per_cu);
  h->geom.xrange_bytes = h->xrange_bytes;
  h->geom.pair = h->walk_pair_on;
  set_pipe_geometry(h);
  h->dirty = true;
  int rc = commit_locked(h, nullptr, true);  // empty index: epoch 1
  if (rc) {
    emqxgm_destroy(h);
    return rc;
  }
  *out = h;
  return 0;
}

void emqxgm_destroy(emqxgm_t* h) {
  if (!h) return;
  {
    std::unique_lock<std::mutex> lk(h->wmu);
    if (h->job) (void)wait_build(h, lk);
  }
  if (h->builder.joinable()) h->builder.join();
  (void)hipSetDevice(h->cfg.device);
  for (auto& p : h->pipes) ctx_free(p.c);
  for (auto& p : h->hpipes) host_pipe_free(p);
  for (auto& st : h->pipe_streams)
    if (st) (void)hipStreamDestroy(st);
  ctx_free(h->sync);
  for (auto* b : {&h->hp_row, &h->hp_fid, &h->hp_exact})
    if (b->p) (void)hipHostFree(b->p);
  if (h->d_row64) (void)hipFree(h->d_row64);
  h->cur.reset();
  h->graveyard.clear();
  h->o_tab.reset();
  h->o_fan.reset();
  h->m_pool.o.reset();
  h->m_foff.o.reset();
  h->m_fver.o.reset();
  free_bufs(h->fan_bufs);
  free_bufs(h->fan_out_bufs);
  if (h->d_patch.p) (void)hipFree(h->d_patch.p);
  if (h->h_stage) (void)hipHostFree(h->h_stage);
  if (h->patch_ev) (void)hipEventDestroy(h->patch_ev);
  if (h->d_rules.p) (void)hipFree(h->d_rules.p);
  if (h->d_merge.p) (void)hipFree(h->d_merge.p);
  if (h->d_in_bytes) (void)hipFree(h->d_in_bytes);
  if (h->d_in_off) (void)hipFree(h->d_in_off);
  delete h;
}

static int trie_insert_locked(emqxgm* h, const uint8_t* p, uint32_t len, uint32_t* id) {
  if (len > 65535) return -EINVAL;  // emqx_topic.erl:47 MAX_TOPIC_LEN
  if (h->filters.size() >= 0x7FFFFFFFu) return -E2BIG;
  const uint32_t i = find_id(h, p, len, true);
  if (!h->filters[i].in_trie) {
    h->filters[i].in_trie = 1;
    ++h->n_trie_pending;
    h->changed.push_back(i);
    h->dirty = true;
  }
  if (id) *id = i;
  return 0;
}

static int route_ref_locked(emqxgm* h, const uint8_t* p, uint32_t len, uint32_t* id) {
  if (len > 65535) return -EINVAL;
  if (h->filters.size() >= 0x7FFFFFFFu) return -E2BIG;
  const uint32_t i = find_id(h, p, len, true);
  if (h->filters[i].route_refs++ == 0) {
    ++h->n_route_pending;
    h->changed.push_back(i);
    h->dirty = true;
  }
  if (id) *id = i;
  return 0;
}

int emqxgm_trie_insert(emqxgm_t* h, const uint8_t* filter, uint32_t len, uint32_t* id) {
  if (!h || (!filter && len)) return -EINVAL;
  WriterLock g(h);
  return trie_insert_locked(h, filter, len, id);
}

int emqxgm_trie_delete(emqxgm_t* h, const uint8_t* filter, uint32_t len) {
  if (!h || (!filter && len)) return -EINVAL;
  WriterLock g(h);
  const uint32_t i = find_id(h, filter, len, false);
  if (i != NONE && h->filters[i].in_trie) {  // absent filter: no-op (emqx_trie.erl:139-144)
    h->filters[i].in_trie = 0;
    --h->n_trie_pending;
    h->changed.push_back(i);
    h->dirty = true;
  }
  return 0;
}

int emqxgm_route_ref(emqxgm_t* h, const uint8_t* filter, uint32_t len, uint32_t* id) {
  if (!h || (!filter && len)) return -EINVAL;
  WriterLock g(h);
  return route_ref_locked(h, filter, len, id);
}

int emqxgm_route_unref(emqxgm_t* h, const uint8_t* filter, uint32_t len) {
  if (!h || (!filter && len)) return -EINVAL;
  WriterLock g(h);
  const uint32_t i = find_id(h, filter, len, false);
  if (i == NONE || h->filters[i].route_refs == 0) return -ENOENT;
  if (--h->filters[i].route_refs == 0) {
    --h->n_route_pending;
    h->changed.push_back(i);
    h->dirty = true;
  }
  return 0;
}

// Level-triggered route-key membership (emqx_router_utils.erl:34-39, 57-71 as a state): the
// route key exists, and a wildcard filter is in the trie, exactly when `present`.  Overrides the
// refcount route_ref/route_unref keep (a mirror that calls this never counts).
static void route_set_locked(emqxgm* h, uint32_t i, bool present) {
  Filter& f = h->filters[i];
  const bool was = f.route_refs > 0;
  if (present) f.sync_gen = h->sync_gen;
  if (present == was && (!f.wild || (bool)f.in_trie == present)) return;
  if (present != was) {
    f.route_refs = present ? 1 : 0;
    if (present) ++h->n_route_pending; else --h->n_route_pending;
  }
  if (f.wild && (bool)f.in_trie != present) {
    f.in_trie = present ? 1 : 0;
    if (present) ++h->n_trie_pending; else --h->n_trie_pending;
  }
  h->changed.push_back(i);
  h->dirty = true;
}

int emqxgm_route_set(emqxgm_t* h, const uint8_t* filter, uint32_t len, int present) {
  if (!h || (!filter && len) || len > 65535) return -EINVAL;
  WriterLock g(h);
  if (!present) {
    const uint32_t i = find_id(h, filter, len, false);
    if (i != NONE) route_set_locked(h, i, false);
    return 0;
  }
  if (h->filters.size() >= 0x7FFFFFFFu) return -E2BIG;
  route_set_locked(h, find_id(h, filter, len, true), true);
  return 0;
}

int emqxgm_route_set_many(emqxgm_t* h, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                          int present) {
  if (!h || !offsets || (!bytes && n)) return -EINVAL;
  for (uint64_t i = 0; i < n; ++i)
    if (offsets[i + 1] < offsets[i] || offsets[i + 1] - offsets[i] > 65535) return -EINVAL;
  std::unique_lock<std::mutex> lk = set_lock(h, false);
  for (uint64_t i0 = 0; i0 < n; i0 += SET_SLICE) {
    if (i0) let_prio_in(h, lk);
    std::unique_lock<std::shared_mutex> g(h->pmu);
    for (uint64_t i = i0; i < std::min(n, i0 + SET_SLICE); ++i) {
      const uint8_t* p = bytes + offsets[i];
      const uint32_t len = (uint32_t)(offsets[i + 1] - offsets[i]);
      const uint32_t id = find_id(h, p, len, present != 0);
      if (id == NONE) continue;
      if (h->filters.size() >= 0x7FFFFFFFu) return -E2BIG;
      route_set_locked(h, id, present != 0);
    }
  }
  return 0;
}

int emqxgm_route_sync_begin(emqxgm_t* h, uint32_t* gen) {
  if (!h) return -EINVAL;
  WriterLock g(h);
  h->sync_gen = h->sync_next++;
  if (h->sync_next == 0) h->sync_next = 1;  // 0 means "no resync"
  if (gen) *gen = h->sync_gen;
  std::lock_guard<std::mutex> hg(h->hmu);
  h->resync_from = h->stale_seq;  // a repair needs a resync begun after the last mark
  return 0;
}

int emqxgm_route_sync_end(emqxgm_t* h, uint32_t gen, uint64_t* removed) {
  if (!h) return -EINVAL;
  WriterLock g(h);
  if (gen == 0 || gen != h->sync_gen) return -ESTALE;
  uint64_t k = 0;
  for (uint32_t i = 0; i < (uint32_t)h->filters.size(); ++i) {
    const Filter& f = h->filters[i];
    if (f.route_refs > 0 && f.sync_gen != gen) {
      route_set_locked(h, i, false);
      ++k;
    }
  }
  // local subscriber lists the resync did not give (their topics left the subscriber table)
  for (auto it = h->lsubs.begin(); it != h->lsubs.end();) {
    const uint64_t id = it->first;
    if ((id >> 6) < h->sub_seen.size() && bit(h->sub_seen, id)) {
      ++it;
      continue;
    }
    h->fan_changed.push_back(it->first);
    h->dirty = true;
    it = h->lsubs.erase(it);
  }
  std::vector<uint64_t>().swap(h->sub_seen);
  h->sync_gen = 0;
  if (removed) *removed = k;
  std::lock_guard<std::mutex> hg(h->hmu);
  h->resynced = h->resync_from;
  return 0;
}

int emqxgm_route_member(emqxgm_t* h, const uint8_t* filter, uint32_t len) {
  if (!h || (!filter && len)) return -EINVAL;
  std::shared_lock<std::shared_mutex> g(h->pmu);
  const uint32_t i = find_id(h, filter, len, false);
  return (i != NONE && h->filters[i].route_committed) ? 1 : 0;
}

// ---- publish fan-out registry ----

int emqxgm_route_add(emqxgm_t* h, const uint8_t* filter, uint32_t len, uint32_t node,
                     uint32_t group) {
  if (!h || (!filter && len) || len > 65535 || node == NONE ||
      (group != NONE && (group & EMQXGM_DEST_GROUP)))
    return -EINVAL;
  WriterLock g(h);
  if (h->filters.size() >= 0x7FFFFFFFu) return -E2BIG;
  const uint32_t i = find_id(h, filter, len, true);
  auto& v = h->rdest[i];
  const std::pair<uint32_t, uint32_t> d(node, group);
  if (std::find(v.begin(), v.end(), d) != v.end()) return 0;  // already routed
  v.push_back(d);
  h->fan_changed.push_back(i);
  if (h->filters[i].route_refs++ == 0) {
    ++h->n_route_pending;
    h->changed.push_back(i);
    // insert_trie_route: the first route of a wildcard filter (emqx_router_utils.erl:34-39)
    if (is_wild(filter, len) && !h->filters[i].in_trie) {
      h->filters[i].in_trie = 1;
      ++h->n_trie_pending;
    }
  }
  h->dirty = true;
  return 0;
}

int emqxgm_route_delete(emqxgm_t* h, const uint8_t* filter, uint32_t len, uint32_t node,
                        uint32_t group) {
  if (!h || (!filter && len)) return -EINVAL;
  WriterLock g(h);
  const uint32_t i = find_id(h, filter, len, false);
  if (i == NONE) return 0;
  auto it = h->rdest.find(i);
  if (it == h->rdest.end()) return 0;
  auto& v = it->second;
  auto p = std::find(v.begin(), v.end(), std::make_pair(node, group));
  if (p == v.end()) return 0;  // absent route: no-op
  v.erase(p);
  if (v.empty()) h->rdest.erase(it);
  h->fan_changed.push_back(i);
  if (h->filters[i].route_refs && --h->filters[i].route_refs == 0) {
    --h->n_route_pending;
    h->changed.push_back(i);
    // delete_trie_route: the last route of a wildcard filter (emqx_router_utils.erl:57-71)
    if (is_wild(filter, len) && h->filters[i].in_trie) {
      h->filters[i].in_trie = 0;
      --h->n_trie_pending;
    }
  }
  h->dirty = true;
  return 0;
}

int emqxgm_set_local_node(emqxgm_t* h, uint32_t node) {
  if (!h) return -EINVAL;
  std::lock_guard<std::mutex> g(h->wmu);
  if (h->local_node != node) {
    h->local_node = node;
    h->fan_rebuild = true;
    h->dirty = true;
  }
  return 0;
}

int emqxgm_subscriber_add(emqxgm_t* h, const uint8_t* filter, uint32_t len, uint32_t sub) {
  if (!h || (!filter && len) || len > 65535) return -EINVAL;
  WriterLock g(h);
  if (h->filters.size() >= 0x7FFFFFFFu) return -E2BIG;
  const uint32_t i = find_id(h, filter, len, true);
  auto& v = h->lsubs[i];
  if (std::find(v.begin(), v.end(), sub) == v.end()) {
    v.push_back(sub);
    h->fan_changed.push_back(i);
    h->dirty = true;
  }
  return 0;
}

int emqxgm_subscriber_delete(emqxgm_t* h, const uint8_t* filter, uint32_t len, uint32_t sub) {
  if (!h || (!filter && len)) return -EINVAL;
  WriterLock g(h);
  const uint32_t i = find_id(h, filter, len, false);
  if (i == NONE) return 0;
  auto it = h->lsubs.find(i);
  if (it == h->lsubs.end()) return 0;
  auto p = std::find(it->second.begin(), it->second.end(), sub);
  if (p == it->second.end()) return 0;
  it->second.erase(p);
  if (it->second.empty()) h->lsubs.erase(it);
  h->fan_changed.push_back(i);
  h->dirty = true;
  return 0;
}

int emqxgm_trie_insert_many(emqxgm_t* h, const uint8_t* bytes, const uint64_t* offsets,
                            uint64_t n, uint32_t* ids) {
  if (!h || !offsets || (!bytes && n)) return -EINVAL;
  WriterLock g(h);
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t b = offsets[i], e = offsets[i + 1];
    if (e < b || e - b > 65535) return -EINVAL;
    int rc = trie_insert_locked(h, bytes + b, (uint32_t)(e - b), ids ? ids + i : nullptr);
    if (rc) return rc;
  }
  return 0;
}

int emqxgm_route_ref_many(emqxgm_t* h, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                          uint32_t* ids) {
  if (!h || !offsets || (!bytes && n)) return -EINVAL;
  WriterLock g(h);
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t b = offsets[i], e = offsets[i + 1];
    if (e < b || e - b > 65535) return -EINVAL;
    int rc = route_ref_locked(h, bytes + b, (uint32_t)(e - b), ids ? ids + i : nullptr);
    if (rc) return rc;
  }
  return 0;
}

}  // extern "C"
namespace {

// Every stream the passes and the writer use answers within probe_ms (a repair's proof that the
// device runs again): an event recorded on each, polled.  -ETIMEDOUT: some stream did not.
int probe_streams(emqxgm* h) {
  std::vector<hipEvent_t> evs;
  int rc = 0;
  auto rec = [&](hipStream_t s) {
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return (rc = -EIO), false;
    evs.push_back(e);
    if (hipEventRecord(e, s) != hipSuccess) return (rc = -EIO), false;
    return true;
  };
  if (hipSetDevice(h->cfg.device) != hipSuccess) return -EIO;
  if (rec(h->wstream))
    for (hipStream_t s : h->pipe_streams)
      if (s && !rec(s)) break;
  const auto t0 = std::chrono::steady_clock::now();
  for (size_t i = 0; !rc && i < evs.size();) {
    const hipError_t q = hipEventQuery(evs[i]);
    if (q == hipSuccess) {
      ++i;
    } else if (q != hipErrorNotReady) {
      rc = -EIO;
    } else if (ms_since(t0) > h->probe_ms) {
      (void)hipGetLastError();
      rc = -ETIMEDOUT;
    } else {
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
  }
  for (hipEvent_t e : evs) (void)hipEventDestroy(e);
  if (rc) set_err(h, rc == -ETIMEDOUT ? "repair: a device stream did not answer within probe_ms"
                                      : "repair: the stream probe failed");
  return rc;
}

// After a successful commit of a stale index (wmu held): clear the mark when no mark came since
// seq0, a mark that asked for a resync has one that began after it, and the streams answer.
// 0: healthy again; -ESTALE: still stale (a mark since, or no covering resync); -ETIMEDOUT/-EIO:
// the probe failed.
int try_repair(emqxgm* h, uint64_t seq0) {
  {
    std::lock_guard<std::mutex> g(h->hmu);
    if (h->stale_seq != seq0 ||
        ((h->stale.load() & EMQXGM_STALE_RESYNC) && h->resynced != seq0)) {
      set_err(h, "still stale: a resync begun after the last mark must complete before the commit");
      return -ESTALE;
    }
  }
  if (int rc = probe_streams(h)) return rc;
  std::lock_guard<std::mutex> g(h->hmu);
  if (h->stale_seq != seq0) return -ESTALE;
  h->stale.store(0, std::memory_order_seq_cst);
  h->repairs += 1;
  return 0;
}

}  // namespace
extern "C" {

int emqxgm_commit(emqxgm_t* h, uint64_t* epoch) {
  if (!h) return -EINVAL;
  std::unique_lock<std::mutex> lk(h->wmu);
  uint64_t seq0;
  {
    std::lock_guard<std::mutex> g(h->hmu);
    seq0 = h->stale_seq;
  }
  int rc = injected(h);
  if (rc == 0) rc = commit_locked(h, &lk, true);
  if (epoch) *epoch = h->epoch;
  // room for the subscribes that follow: buffers and host arrays past 7/8 grow now, off their
  // path (a build in flight: its install does it)
  if (rc == 0 && !h->job) rc = grow_ahead(h);
  if (rc < 0) {
    mark_stale(h, EMQXGM_STALE_COMMIT, rc);
    return rc;
  }
  // the replaced buffers of earlier commits are freed here, off the subscribe path (a pass that
  // still reads one is waited for briefly; what is left goes with the next commit)
  for (int i = 0; i < 200 && sweep_graveyard(h, true) != 0; ++i)
    std::this_thread::sleep_for(std::chrono::microseconds(500));
  return h->stale.load() ? try_repair(h, seq0) : 0;
}

int emqxgm_get_health(emqxgm_t* h, emqxgm_health_t* out) {
  if (!h || !out) return -EINVAL;
  std::lock_guard<std::mutex> g(h->hmu);
  out->stale = h->stale.load();
  out->last_error = h->stale_err;
  out->marks = h->stale_seq;
  out->repairs = h->repairs;
  out->refused = h->refused.load();
  return (int)out->stale;
}

int emqxgm_mark_stale(emqxgm_t* h, int err) {
  if (!h) return -EINVAL;
  mark_stale(h, EMQXGM_STALE_RESYNC, err > 0 ? -err : err);
  return 0;
}

// The commit of a synchronous set (EMQXGM_SET_COMMIT): a delta of this call's own changes (those
// appended to h->changed since c0, and the filters `mine` -- every filter the call resolved --
// whose state another caller left pending: a resync chunk that already set the state this call
// asks for leaves this call nothing to append, and its hook must still see the filter committed
// when it returns); other callers' pending changes stay pending -- they are not this
// caller's to publish, and a bulk of them (a resync's chunks) must not make a single subscribe
// wait for its full build.  When this delta does not fit, everything pending takes the usual
// path (commit_locked).
static int commit_mine(emqxgm* h, std::unique_lock<std::mutex>& lk, size_t c0,
                       std::vector<uint32_t>& mine) {
  const auto t0 = std::chrono::steady_clock::now();
  struct Slow {
    std::chrono::steady_clock::time_point t0;
    ~Slow() { debug_slow("synchronous commit", ms_since(t0)); }
  } slow{t0};
  if (int rc = injected(h)) return rc;
  if (c0 == 0) return commit_locked(h, &lk, false);
  std::sort(mine.begin(), mine.end());
  std::vector<uint32_t> rest, own;
  rest.reserve(c0);
  for (size_t i = 0; i < c0; ++i) {
    const uint32_t id = h->changed[i];
    (std::binary_search(mine.begin(), mine.end(), id) ? own : rest).push_back(id);
  }
  own.insert(own.end(), h->changed.begin() + c0, h->changed.end());
  h->changed.swap(own);
  int rc = try_delta(h, std::chrono::steady_clock::now());
  if (rc == 0) {
    h->changed.swap(rest);
    h->dirty = true;
    return 0;
  }
  h->changed.insert(h->changed.end(), rest.begin(), rest.end());
  h->dirty = true;
  return rc < 0 ? rc : commit_locked(h, &lk, false);
}

// A synchronous set's end: its commit, and the health mark when the set or its commit failed (the
// caller's table holds a change the index may now lack: matches refuse until a repair)
static int set_done(emqxgm* h, std::unique_lock<std::mutex>& lk, int rc, uint32_t flags, size_t c0,
                    std::vector<uint32_t>& mine, uint64_t* epoch) {
  if (rc == -E2BIG) mark_stale(h, EMQXGM_STALE_RESYNC, rc);  // half applied
  if (rc == 0 && (flags & EMQXGM_SET_COMMIT)) {
    rc = commit_mine(h, lk, c0, mine);
    if (rc < 0) mark_stale(h, EMQXGM_STALE_COMMIT, rc);
  }
  if (epoch) *epoch = h->epoch;
  return rc;
}

int emqxgm_route_set_batch(emqxgm_t* h, const uint8_t* bytes, const uint64_t* offsets,
                           const uint8_t* present, uint64_t n, uint32_t flags, uint64_t* epoch) {
  if (!h || !offsets || (!bytes && n && offsets[n]) || (flags & ~EMQXGM_SET_COMMIT)) return -EINVAL;
  for (uint64_t i = 0; i < n; ++i)
    if (offsets[i + 1] < offsets[i] || offsets[i + 1] - offsets[i] > 65535) return -EINVAL;
  const bool sync = (flags & EMQXGM_SET_COMMIT) != 0;
  const auto tl = std::chrono::steady_clock::now();
  std::unique_lock<std::mutex> lk = set_lock(h, sync);
  if (sync) debug_slow("synchronous set: waited for the writer lock", ms_since(tl));
  const size_t c0 = h->changed.size();  // changes pending from other callers
  std::vector<uint32_t> mine;
  int rc = 0;
  for (uint64_t i0 = 0; i0 < n && !rc; i0 += sync ? n : SET_SLICE) {
    if (i0) let_prio_in(h, lk);
    const auto tp = std::chrono::steady_clock::now();
    std::unique_lock<std::shared_mutex> g(h->pmu);
    if (sync) debug_slow("synchronous set: waited for the registry lock", ms_since(tp));
    for (uint64_t i = i0; i < (sync ? n : std::min(n, i0 + SET_SLICE)); ++i) {
      const bool pr = !present || present[i];
      const uint8_t* p = bytes + offsets[i];
      const uint32_t len = (uint32_t)(offsets[i + 1] - offsets[i]);
      if (pr && h->filters.size() >= 0x7FFFFFFFu) {
        rc = -E2BIG;
        break;
      }
      const uint32_t id = find_id(h, p, len, pr);
      if (id == NONE) continue;
      route_set_locked(h, id, pr);
      if (sync) mine.push_back(id);
    }
  }
  return set_done(h, lk, rc, flags, c0, mine, epoch);
}

int emqxgm_route_dests_batch(emqxgm_t* h, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                             const uint32_t* dptr, const uint32_t* node, const uint32_t* group,
                             uint32_t flags, uint64_t* epoch) {
  if (!h || !offsets || !dptr || (!bytes && n && offsets[n]) || (flags & ~EMQXGM_SET_COMMIT)) return -EINVAL;
  for (uint64_t i = 0; i < n; ++i) {
    if (offsets[i + 1] < offsets[i] || offsets[i + 1] - offsets[i] > 65535 || dptr[i + 1] < dptr[i])
      return -EINVAL;
    for (uint32_t j = dptr[i]; j < dptr[i + 1]; ++j)
      if (!node || !group || node[j] == NONE || (group[j] != NONE && (group[j] & EMQXGM_DEST_GROUP)))
        return -EINVAL;
  }
  const bool sync = (flags & EMQXGM_SET_COMMIT) != 0;
  std::unique_lock<std::mutex> lk = set_lock(h, sync);
  const size_t c0 = h->changed.size();  // changes pending from other callers
  std::vector<std::pair<uint32_t, uint32_t>> ds;
  std::vector<uint32_t> mine;
  int rc = 0;
  for (uint64_t i0 = 0; i0 < n && !rc; i0 += sync ? n : SET_SLICE) {
    if (i0) let_prio_in(h, lk);
    std::unique_lock<std::shared_mutex> g(h->pmu);
    for (uint64_t i = i0; i < (sync ? n : std::min(n, i0 + SET_SLICE)); ++i) {
      ds.clear();
      for (uint32_t j = dptr[i]; j < dptr[i + 1]; ++j) ds.emplace_back(node[j], group[j]);
      std::sort(ds.begin(), ds.end());
      ds.erase(std::unique(ds.begin(), ds.end()), ds.end());
      const uint8_t* p = bytes + offsets[i];
      const uint32_t len = (uint32_t)(offsets[i + 1] - offsets[i]);
      if (!ds.empty() && h->filters.size() >= 0x7FFFFFFFu) {
        rc = -E2BIG;
        break;
      }
      const uint32_t id = find_id(h, p, len, !ds.empty());
      if (id == NONE) continue;  // absent and unknown: nothing to remove
      auto it = h->rdest.find(id);
      std::vector<std::pair<uint32_t, uint32_t>> old;
      if (it != h->rdest.end()) old = it->second;
      std::sort(old.begin(), old.end());
      if (old != ds) {
        if (ds.empty())
          h->rdest.erase(id);
        else
          h->rdest[id] = ds;
        h->fan_changed.push_back(id);
        h->dirty = true;
      }
      route_set_locked(h, id, !ds.empty());
      if (sync) mine.push_back(id);
    }
  }
  return set_done(h, lk, rc, flags, c0, mine, epoch);
}

int emqxgm_subscribers_batch(emqxgm_t* h, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                             const uint32_t* sptr, const uint32_t* subs, uint32_t flags,
                             uint64_t* epoch) {
  if (!h || !offsets || !sptr || (!bytes && n && offsets[n]) || (flags & ~EMQXGM_SET_COMMIT)) return -EINVAL;
  for (uint64_t i = 0; i < n; ++i)
    if (offsets[i + 1] < offsets[i] || offsets[i + 1] - offsets[i] > 65535 || sptr[i + 1] < sptr[i] ||
        (sptr[i + 1] > sptr[i] && !subs))
      return -EINVAL;
  const bool sync = (flags & EMQXGM_SET_COMMIT) != 0;
  std::unique_lock<std::mutex> lk = set_lock(h, sync);
  const size_t c0 = h->changed.size();  // changes pending from other callers
  std::vector<uint32_t> ss, mine;  // (fan-out changes commit whole: nothing of `mine` needed)
  int rc = 0;
  for (uint64_t i0 = 0; i0 < n && !rc; i0 += sync ? n : SET_SLICE) {
    if (i0) let_prio_in(h, lk);
    std::unique_lock<std::shared_mutex> g(h->pmu);
    for (uint64_t i = i0; i < (sync ? n : std::min(n, i0 + SET_SLICE)); ++i) {
      ss.assign(subs + sptr[i], subs + sptr[i + 1]);
      std::sort(ss.begin(), ss.end());
      ss.erase(std::unique(ss.begin(), ss.end()), ss.end());
      const uint8_t* p = bytes + offsets[i];
      const uint32_t len = (uint32_t)(offsets[i + 1] - offsets[i]);
      if (!ss.empty() && h->filters.size() >= 0x7FFFFFFFu) {
        rc = -E2BIG;
        break;
      }
      const uint32_t id = find_id(h, p, len, !ss.empty());
      if (id == NONE) continue;
      if (h->sync_gen) {
        if (((uint64_t)id >> 6) >= h->sub_seen.size()) h->sub_seen.resize(((uint64_t)id >> 6) + 1, 0);
        bset(h->sub_seen, id);
      }
      auto it = h->lsubs.find(id);
      std::vector<uint32_t> old;
      if (it != h->lsubs.end()) old = it->second;
      std::sort(old.begin(), old.end());
      if (old == ss) continue;
      if (ss.empty())
        h->lsubs.erase(id);
      else
        h->lsubs[id] = ss;
      h->fan_changed.push_back(id);
      h->dirty = true;
    }
  }
  return set_done(h, lk, rc, flags, c0, mine, epoch);
}

// ---- index snapshot (SURVEY 5 "checkpoint / resume"): the committed registry and the host
// model of the device index in one file, so a restart restores the index without rebuilding it
// (the reference rebuilds its ram_copies route tables from peers, emqx_router.erl:78-92) ----
}  // extern "C"
namespace {

constexpr uint64_t SNAP_MAGIC = 0x31534d47584d45ull;  // "EMXGMS1"
constexpr uint32_t SNAP_VERSION = 3;  // 2: fat buckets (TrieModel fchild / half), 3: Filter::sync_gen, keyed

struct SnapOut {
  FILE* f;
  bool ok = true;
  void raw(const void* p, size_t n) { ok = ok && (n == 0 || fwrite(p, 1, n, f) == n); }
  template <class T>
  void pod(const T& v) { raw(&v, sizeof v); }
  template <class T>
  void vec(const std::vector<T>& v) {
    pod<uint64_t>(v.size());
    raw(v.data(), v.size() * sizeof(T));
  }
};

struct SnapIn {
  FILE* f;
  bool ok = true;
  void raw(void* p, size_t n) { ok = ok && (n == 0 || fread(p, 1, n, f) == n); }
  template <class T>
  void pod(T& v) { raw(&v, sizeof v); }
  template <class T>
  void vec(std::vector<T>& v) {
    uint64_t n = 0;
    pod(n);
    if (!ok || n > (1ull << 40) / sizeof(T)) {
      ok = false;
      return;
    }
    v.resize(n);
    raw(v.data(), n * sizeof(T));
  }
};

template <class IO, class M>
void snap_model(IO& io, M& m) {
  io.vec(m.emap.ents);
  io.pod(m.emap.mask);
  io.pod(m.emap.used);
  io.vec(m.parent);
  io.vec(m.ref);
  io.vec(m.nlit);
  io.vec(m.pchild);
  io.vec(m.hf);
  io.vec(m.tw);
  io.vec(m.tn);
  io.vec(m.sig);
  io.vec(m.hcode);
  io.vec(m.tok);
  io.vec(m.slot);
  io.vec(m.fchild);
  io.vec(m.keyed);
  io.vec(m.half);
  io.vec(m.occ);
  io.vec(m.tomb);
  io.pod(m.nbk);
  io.pod(m.ecap);
  io.pod(m.n_occ);
  io.pod(m.n_edges);
  io.pod(m.tn_cap);
  io.pod(m.fv_cap);
  io.vec(m.fvbits);
  io.vec(m.multi);
  io.pod(m.needs_verify);
  io.pod(m.max_depth);
  io.pod(m.n_trie);
  io.pod(m.n_route);
  io.vec(m.xpos);
  io.vec(m.xocc);
  io.vec(m.xtomb);
  io.vec(m.xovf);
  io.pod(m.xcap_p);
  io.pod(m.xcap_w);
  io.pod(m.x_occ_p);
  io.pod(m.x_occ_w);
  io.pod(m.n_route_p);
  io.pod(m.n_route_w);
}

// Internal consistency of a loaded model against the registry it came with: every index
// upload_model and the delta-commit code take from the file stays inside its array.  A
// snapshot that fails this is rejected with -EINVAL instead of writing past host buffers.
bool pow2(uint64_t x) { return x && !(x & (x - 1)); }

bool model_consistent(const TrieModel& m, uint64_t n_filters, std::string& why) {
  const uint64_t n = m.parent.size();
  auto bad = [&](const char* w) {
    why = w;
    return false;
  };
  if (n == 0 || n > MAX_NODES) return bad("node count");
  for (const auto* v : {&m.ref, &m.nlit, &m.pchild, &m.hf, &m.tw, &m.tn})
    if (v->size() != n) return bad("per-node array size");
  if (m.sig.size() != n || m.hcode.size() != n || m.tok.size() != n || m.slot.size() != n ||
      m.fchild.size() != n || m.half.size() != n || m.keyed.size() != n)
    return bad("per-node array size");
  if (!pow2(m.nbk) || m.ecap != m.nbk * EBUCKET || m.ecap > (1ull << 40)) return bad("edge capacity");
  if (m.occ.size() < m.ecap / 64 + 1 || m.tomb.size() < m.ecap / 64 + 1) return bad("edge bitmaps");
  if (m.tn_cap < n || m.tn_cap > (1ull << 32)) return bad("side array capacity");
  if (m.fvbits.size() < (n_filters + 31) / 32 || m.fv_cap != m.fvbits.size()) return bad("verify bits");
  if (!pow2(m.emap.ents.size()) || m.emap.mask + 1 != m.emap.ents.size() ||
      m.emap.used > m.emap.ents.size())
    return bad("edge map");
  for (const auto& e : m.emap.ents)
    if (e.parent != NONE && e.parent != TOMB && (e.parent >= n || e.child >= n)) return bad("edge map entry");
  auto fid_ok = [&](uint32_t v) {
    if (v == NONE) return true;
    if (!(v & LIST_MULTI)) return v < n_filters;
    const uint64_t i = v & ~LIST_MULTI;
    if (i >= m.multi.size() || m.multi[i] + i + 1 > m.multi.size()) return false;
    for (uint64_t k = 0; k < m.multi[i]; ++k)
      if (m.multi[i + 1 + k] >= n_filters) return false;
    return true;
  };
  if (m.slot[0] != DEAD) return bad("root slot");
  for (uint64_t c = 0; c < n; ++c) {
    if (c && m.slot[c] != DEAD && m.slot[c] != ROOTH && m.slot[c] >= m.ecap) return bad("slot position");
    if (m.slot[c] == ROOTH && (!m.half[c] || m.parent[c] != 0)) return bad("root half");
    if (m.keyed[c] && (c == 0 || m.tok[c] == PLUS_TOK)) return bad("keyed node");
    if (const uint32_t g = m.fchild[c]) {  // the half sits right after its fat parent's slot
      if (g >= n || !m.half[g] || m.parent[g] != c) return bad("fat child");
      if (c ? (m.slot[c] == DEAD || m.slot[c] % EBUCKET != 0 || m.slot[g] != m.slot[c] + 1)
            : m.slot[g] != ROOTH)
        return bad("fat bucket");
    }
    if (m.half[c] && (c == 0 || m.parent[c] >= n || m.fchild[m.parent[c]] != c)) return bad("half");
    if (c && m.parent[c] != NONE && m.parent[c] >= c) return bad("parent id");
    if (m.pchild[c] >= n) return bad("'+' child id");
    if (!fid_ok(m.hf[c]) || !fid_ok(m.tw[c]) || !fid_ok(m.tn[c])) return bad("node filter id");
  }
  if (!pow2(m.xcap_p) || !pow2(m.xcap_w) || m.xcap_p + m.xcap_w > (1ull << 36)) return bad("key capacity");
  const uint64_t xent_n = (m.xcap_p + m.xcap_w) * XBUCKET;
  if (m.xocc.size() < xent_n / 64 + 1 || m.xtomb.size() < xent_n / 64 + 1 ||
      m.xovf.size() < (m.xcap_p + m.xcap_w) / 64 + 1)
    return bad("key bitmaps");
  if (m.xpos.size() > n_filters) return bad("key positions");
  for (uint32_t v : m.xpos)
    if (v != NONE && v >= xent_n) return bad("key position");
  if (m.max_depth > 65536) return bad("depth");
  return true;
}

// A handle whose snapshot load failed half-way returns to the fresh state (empty registry,
// no model): the next commit is a full build and another load may be tried.
void reset_loaded(emqxgm* h) {
  {
    std::unique_lock<std::shared_mutex> pg(h->pmu);
    h->pool.clear();
    h->filters.clear();
    h->slots.clear();
    h->slot_mask = 0;
  }
  h->n_trie_pending = 0;
  h->n_route_pending = 0;
  h->local_node = NONE;
  h->rdest.clear();
  h->lsubs.clear();
  h->foff_host.clear();
  h->fver_host.clear();
  h->tm = TrieModel();
  h->changed.clear();
  h->fan_changed.clear();
  h->dirty = false;
}

template <class Map, class IO>
void snap_map_out(IO& io, const Map& mp) {
  io.template pod<uint64_t>(mp.size());
  for (const auto& kv : mp) {
    io.pod(kv.first);
    io.vec(kv.second);
  }
}

template <class Map, class IO>
void snap_map_in(IO& io, Map& mp) {
  uint64_t n = 0;
  io.pod(n);
  for (uint64_t i = 0; io.ok && i < n; ++i) {
    uint32_t k = 0;
    io.pod(k);
    io.vec(mp[k]);
  }
}

}  // namespace
extern "C" {

int emqxgm_snapshot_save(emqxgm_t* h, const char* path) {
  if (!h || !path) return -EINVAL;
  std::unique_lock<std::mutex> lk(h->wmu);
  int rc = 0;
  // the file holds committed state only (and the model of the index readers have)
  if ((h->dirty || h->job) && (rc = commit_locked(h, &lk, true))) return rc;
  if (h->job && (rc = wait_build(h, lk))) return rc;
  if (!h->tm.valid) {
    set_err(h, "no host model to save");
    return -EINVAL;
  }
  FILE* f = fopen(path, "wb");
  if (!f) return -errno;
  SnapOut o{f};
  o.pod(SNAP_MAGIC);
  o.pod(SNAP_VERSION);
  o.pod(h->cfg.word_hash_bits);
  o.pod(h->cfg.full_hash_bits);
  o.vec(h->pool);
  o.vec(h->filters);
  o.pod(h->n_trie_pending);
  o.pod(h->n_route_pending);
  o.pod(h->local_node);
  snap_map_out(o, h->rdest);
  snap_map_out(o, h->lsubs);
  snap_model(o, h->tm);
  o.pod(SNAP_MAGIC);
  const bool ok = o.ok && fflush(f) == 0;
  fclose(f);
  if (!ok) {
    set_err(h, "snapshot write failed");
    return -EIO;
  }
  return 0;
}

int emqxgm_snapshot_load(emqxgm_t* h, const char* path) {
  if (!h || !path) return -EINVAL;
  std::lock_guard<std::mutex> g(h->wmu);
  if (!h->filters.empty() || h->dirty) {
    set_err(h, "snapshot load needs a fresh handle");
    return -EBUSY;
  }
  FILE* f = fopen(path, "rb");
  if (!f) return -errno;
  const auto t0 = std::chrono::steady_clock::now();
  SnapIn in{f};
  uint64_t magic = 0, magic2 = 0;
  uint32_t ver = 0, whb = 0, fhb = 0;
  in.pod(magic);
  in.pod(ver);
  in.pod(whb);
  in.pod(fhb);
  if (!in.ok || magic != SNAP_MAGIC || ver != SNAP_VERSION || whb != h->cfg.word_hash_bits ||
      fhb != h->cfg.full_hash_bits) {
    fclose(f);
    set_err(h, "not a snapshot of this engine configuration");
    return -EINVAL;
  }
  std::vector<uint8_t> pool;
  std::vector<Filter> filters;
  uint64_t ntp = 0, nrp = 0;
  uint32_t local = NONE;
  decltype(h->rdest) rdest;
  decltype(h->lsubs) lsubs;
  TrieModel m;
  in.vec(pool);
  in.vec(filters);
  in.pod(ntp);
  in.pod(nrp);
  in.pod(local);
  snap_map_in(in, rdest);
  snap_map_in(in, lsubs);
  snap_model(in, m);
  in.pod(magic2);
  fclose(f);
  bool sane = in.ok && magic2 == SNAP_MAGIC && filters.size() < NONE;
  for (size_t i = 0; sane && i < filters.size(); ++i)
    sane = filters[i].len <= pool.size() && filters[i].off <= pool.size() - filters[i].len;
  for (const auto& kv : rdest) sane = sane && kv.first < filters.size();
  for (const auto& kv : lsubs) sane = sane && kv.first < filters.size();
  std::string why = "truncated";
  if (!sane || !model_consistent(m, filters.size(), why)) {
    set_err(h, "snapshot corrupt: " + why);
    return -EINVAL;
  }
  // a resync generation belongs to the handle that ran it: a loaded handle's first resync must
  // not take the saved marks for its own (it would keep every key the table lost meanwhile)
  for (Filter& f : filters) f.sync_gen = 0;
  {
    std::unique_lock<std::shared_mutex> pg(h->pmu);
    h->pool.swap(pool);
    h->filters.swap(filters);
    h->slots.clear();
    h->slot_mask = 0;
    if (!h->filters.empty()) slots_grow(h);
  }
  h->n_trie_pending = ntp;
  h->n_route_pending = nrp;
  h->local_node = local;
  h->rdest.swap(rdest);
  h->lsubs.swap(lsubs);
  if (hipSetDevice(h->cfg.device) != hipSuccess) {
    reset_loaded(h);
    return fail(h, hipErrorInvalidDevice, "hipSetDevice");
  }
  int rc = 0;
  h->foff_host.clear();
  h->fver_host.clear();
  if ((rc = patch_wait(h)) || (rc = upload_pool(h, nullptr)) || (rc = fan_full(h)) ||
      (rc = upload_model(h, m))) {
    reset_loaded(h);
    return rc;
  }
  m.valid = true;
  m.n_nodes0 = m.parent.size();  // (headroom counted from the restored index on)
  m.fv_words0 = std::min<uint64_t>(m.fv_cap, (h->filters.size() + 31) / 32 + 1);
  h->tm = std::move(m);
  h->changed.clear();
  h->fan_changed.clear();
  if ((rc = publish_epoch(h, false))) {
    reset_loaded(h);
    return rc;
  }
  h->dirty = false;
  commit_stats(h, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(),
               false);
  return 0;
}

int emqxgm_trie_empty(emqxgm_t* h) {
  if (!h) return -EINVAL;
  return h->cur_trie_empty.load();
}

int emqxgm_trie_member(emqxgm_t* h, const uint8_t* filter, uint32_t len) {
  if (!h || (!filter && len)) return -EINVAL;
  std::shared_lock<std::shared_mutex> g(h->pmu);
  const uint32_t i = find_id(h, filter, len, false);
  return (i != NONE && h->filters[i].trie_committed) ? 1 : 0;
}

int emqxgm_lookup_id(emqxgm_t* h, const uint8_t* filter, uint32_t len, uint32_t* id) {
  if (!h || !id || (!filter && len)) return -EINVAL;
  std::shared_lock<std::shared_mutex> g(h->pmu);
  const uint32_t i = find_id(h, filter, len, false);
  if (i == NONE) return -ENOENT;
  *id = i;
  return 0;
}

int emqxgm_filter_bytes(emqxgm_t* h, uint32_t id, const uint8_t** p, uint32_t* len) {
  if (!h || !p || !len) return -EINVAL;
  std::shared_lock<std::shared_mutex> g(h->pmu);
  if (id >= h->filters.size()) return -ENOENT;
  *p = h->pool.data() + h->filters[id].off;
  *len = h->filters[id].len;
  return 0;
}

int emqxgm_filter_copy(emqxgm_t* h, uint32_t id, uint8_t* buf, uint32_t cap, uint32_t* len) {
  if (!h || !len || (!buf && cap)) return -EINVAL;
  std::shared_lock<std::shared_mutex> g(h->pmu);
  if (id >= h->filters.size()) return -ENOENT;
  const Filter& f = h->filters[id];
  *len = f.len;
  if (f.len > cap) return -ENOSPC;
  if (f.len) memcpy(buf, h->pool.data() + f.off, f.len);
  return 0;
}

int emqxgm_filters_copy(emqxgm_t* h, const uint32_t* ids, uint64_t n, uint8_t* buf, uint64_t cap,
                        uint64_t* offsets) {
  if (!h || !offsets || (n && !ids) || (!buf && cap)) return -EINVAL;
  std::shared_lock<std::shared_mutex> g(h->pmu);
  uint64_t need = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (ids[i] >= h->filters.size()) return -ENOENT;
    need += h->filters[ids[i]].len;
  }
  offsets[0] = 0;
  if (need > cap) {
    offsets[n] = need;
    return -ENOSPC;
  }
  uint64_t o = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const Filter& f = h->filters[ids[i]];
    if (f.len) memcpy(buf + o, h->pool.data() + f.off, f.len);
    o += f.len;
    offsets[i + 1] = o;
  }
  return 0;
}

int emqxgm_match_device(emqxgm_t* h, const uint8_t* d_bytes, const uint32_t* d_offsets, uint32_t n,
                        uint64_t bytes_len, emqxgm_dev_out* out) {
  if (!h || !out || (!d_offsets && n)) return -EINVAL;
  if (int rc = refuse_stale(h)) return rc;
  std::lock_guard<std::mutex> g(h->mmu);
  if (hipSetDevice(h->cfg.device) != hipSuccess) return -EIO;
  uint32_t pairs = 0;
  int rc = run_device(h, h->sync, d_bytes, d_offsets, n, bytes_len, &pairs);
  h->sync.epoch.reset();
  if (rc) return rc;
  out->n = n;
  out->n_pairs = pairs;
  out->row_ptr = h->sync.sc.row;
  out->filter_id = h->sync.sc.out;
  out->exact_id = h->sync.sc.exact_id;
  out->n_words = h->sync.sc.nw;
  return 0;
}

int emqxgm_key_owners(emqxgm_t* h, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                      uint32_t parts, uint32_t* owner) {
  if (!h || !offsets || !owner || parts == 0 || (!bytes && n && offsets[n])) return -EINVAL;
  const uint64_t fmask = h->cfg.full_hash_bits >= 64 ? ~0ull : ((1ull << h->cfg.full_hash_bits) - 1ull);
  for (uint64_t i = 0; i < n; ++i) {
    if (offsets[i + 1] < offsets[i] || offsets[i + 1] - offsets[i] > 65535) return -EINVAL;
    const uint64_t fh = key_hash(bytes + offsets[i], (uint32_t)(offsets[i + 1] - offsets[i]), fmask);
    owner[i] = (uint32_t)(fh >> 32) % parts;
  }
  return 0;
}

int emqxgm_exact_owned_device(emqxgm_t* h, const uint8_t* d_bytes, const uint32_t* d_offsets,
                              uint32_t n, uint32_t parts, uint32_t part, uint32_t* d_out) {
  if (!h || (!d_offsets && n) || (!d_out && n) || parts == 0 || part >= parts) return -EINVAL;
  if (int rc = refuse_stale(h)) return rc;
  std::lock_guard<std::mutex> g(h->mmu);
  if (hipSetDevice(h->cfg.device) != hipSuccess) return -EIO;
  EpochP E;
  {
    std::lock_guard<std::mutex> ge(h->emu);
    E = h->cur;
  }
  hipStream_t st = h->sync.stream;
  if (!E->ready_seen.load(std::memory_order_relaxed)) HIPCHK(h, hipStreamWaitEvent(st, E->ready, 0));
  HIPCHK(h, launch_exact_owned(d_bytes, d_offsets, n, E->ix, parts, part, d_out, st));
  HIPCHK(h, hipStreamSynchronize(st));  // (the epoch is held until its tables were read)
  return 0;
}

int emqxgm_match_device_submit(emqxgm_t* h, const uint8_t* d_bytes, const uint32_t* d_offsets,
                               uint32_t n, uint64_t bytes_len, uint64_t* ticket) {
  if (!h || !ticket || (!d_offsets && n)) return -EINVAL;
  if (int rc = refuse_stale(h)) return rc;
  std::lock_guard<std::mutex> g(h->mmu);
  if (hipSetDevice(h->cfg.device) != hipSuccess) return -EIO;
  const uint64_t tk = h->next_ticket;
  emqxgm::Pipe& p = h->pipes[tk % EMQXGM_PIPES];
  if (p.state == 1) {
    set_err(h, "pipe busy: wait for the ticket submitted EMQXGM_PIPES submissions ago");
    return -EBUSY;
  }
  hipStream_t ps = pipe_stream(h, (uint32_t)(tk % EMQXGM_PIPES));
  if (!ps) {
    set_err(h, "hipStreamCreateWithFlags failed");
    return -EIO;
  }
  int rc = ctx_init(h, p.c, ps);
  p.c.pipelined = true;
  if (rc) return rc;
  rc = pass_prepare(h, p.c, n, bytes_len);
  if (rc < 0) return rc;
  p.d_bytes = d_bytes;
  p.d_off = d_offsets;
  p.n = n;
  p.bytes_len = bytes_len;
  p.pairs = 0;
  if (rc == 2) {
    p.state = 2;  // empty batch: already complete
  } else {
    if ((rc = pass_submit(h, p.c, d_bytes, d_offsets, n, false, false))) return rc;
    p.state = 1;
  }
  p.ticket = tk;
  h->next_ticket += 1;
  *ticket = tk;
  return 0;
}

int emqxgm_match_device_wait(emqxgm_t* h, uint64_t ticket, emqxgm_dev_out* out) {
  if (!h || !out) return -EINVAL;
  std::lock_guard<std::mutex> g(h->mmu);
  RoctxRange rr(h->roctx, "emqxgm.wait");
  if (hipSetDevice(h->cfg.device) != hipSuccess) return -EIO;
  emqxgm::Pipe& p = h->pipes[ticket % EMQXGM_PIPES];
  if (ticket == 0 || p.ticket != ticket || p.state == 0) {
    set_err(h, "unknown ticket, or its result was already taken / overwritten");
    return -ENOENT;
  }
  int rc = pipe_complete(h, p);
  if (rc) return rc;
  p.state = 0;
  out->n = p.n;
  out->n_pairs = p.pairs;
  out->row_ptr = p.c.sc.row;
  out->filter_id = p.c.sc.out;
  out->exact_id = p.c.sc.exact_id;
  out->n_words = p.c.sc.nw;
  return 0;
}

}  // extern "C"
namespace {
int host_pipe_enqueue_gather(emqxgm* h, emqxgm::HostPipe& p);
// The device address of pinned host memory, or null (pageable memory: the failed lookup's error
// is cleared, or the next launch's hipGetLastError would report it)
void* mapped_ptr(const void* host) {
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, const_cast<void*>(host), 0) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return d;
}

int batch_submit(emqxgm* h, const uint8_t* bytes, const uint32_t* offsets, uint32_t n,
                 uint64_t* ticket, bool want_fb, bool trusted = false) {
  if (!h || !ticket || !offsets || offsets[0] != 0 || (!bytes && offsets[n])) return -EINVAL;
  if (n > h->cfg.batch_max) return -E2BIG;
  if (int rc = refuse_stale(h)) return rc;
  // a decreasing offset would make k_tok / k_exact read a topic of ~4 G bytes past the batch
  // (the concurrent entry's windows build theirs increasing: no O(n) scan on their path)
  for (uint32_t i = 0; !trusted && i < n; ++i)
    if (offsets[i + 1] < offsets[i]) return -EINVAL;
  std::lock_guard<std::mutex> g(h->mmu);
  if (hipSetDevice(h->cfg.device) != hipSuccess) return -EIO;
  const uint64_t tk = h->next_hticket;
  emqxgm::HostPipe& p = h->hpipes[tk % EMQXGM_HOST_PIPES];
  if (p.state == 1) {
    set_err(h, "host pipe busy: wait for the ticket submitted EMQXGM_HOST_PIPES submissions ago");
    return -EBUSY;
  }
  const uint64_t nb = offsets[n];
  hipStream_t ps = pipe_stream(h, (uint32_t)(tk % EMQXGM_HOST_PIPES));
  if (!ps) {
    set_err(h, "hipStreamCreateWithFlags failed");
    return -EIO;
  }
  int rc = ctx_init(h, p.c, ps);
  p.c.pipelined = true;
  if (rc) return rc;
  rc = pass_prepare(h, p.c, n, nb);
  if (rc < 0) return rc;
  // the filter-id buffer: the copy kernel (host_out 1) writes up to its capacity behind the pass;
  // the default path copies the ids in _wait, sized then by the pair count (a pinned allocation
  // here would follow every staging growth and stall the stream)
  if ((rc = host_pipe_reserve(h, p, n, std::max<uint64_t>(nb, 1),
                              h->host_out_mode == 1 ? p.c.sc.p_cap : 1)))
    return rc;
  p.n = n;
  p.bytes_len = nb;
  p.pairs = 0;
  p.fb_async = false;
  // small windows in pinned (device-mapped) memory -- the concurrent entry's, a batcher's: no
  // DMA copies (PassCtx src_*); pageable memory has no device pointer and takes the copies
  p.zc = false;
  if (want_fb && n && n <= h->zc_topics && nb <= (8u << 20) && h->host_out_mode == 0 &&
      !((uintptr_t)bytes & 15u)) {
    void* db = mapped_ptr(bytes);
    void* doff = db ? mapped_ptr(offsets) : nullptr;
    p.zc = db && doff;
    if (p.zc) {
      p.c.src_bytes = (const uint8_t*)db;
      p.c.src_off = (const uint32_t*)doff;
    }
  }
  if (n == 0) {
    p.h_row[0] = 0;
    p.state = 2;
  } else {
    if (!p.zc) {
      if (nb) HIPCHK(h, hipMemcpyAsync(p.d_bytes, bytes, nb, hipMemcpyHostToDevice, p.c.stream));
      HIPCHK(h, hipMemcpyAsync(p.d_off, offsets, ((size_t)n + 1) * 4, hipMemcpyHostToDevice, p.c.stream));
    }
    // with the gather behind the pass the row pointers travel in its block (one copy less)
    p.rows_enq = !want_fb || h->host_out_mode == 1;
    rc = pass_submit(h, p.c, p.d_bytes, p.d_off, n, false, false);
    p.c.src_bytes = nullptr;  // (consumed by the enqueue; never left for a later pass)
    p.c.src_off = nullptr;
    if (rc || (p.rows_enq && (rc = host_pipe_copy_out(h, p))) ||
        (want_fb && (rc = host_pipe_enqueue_gather(h, p))))
      return rc;
    if (!p.fin) HIPCHK(h, hipEventCreateWithFlags(&p.fin, hipEventDisableTiming));
    HIPCHK(h, hipEventRecord(p.fin, p.c.stream));
    p.state = 1;
  }
  p.ticket = tk;
  h->next_hticket += 1;
  *ticket = tk;
  return 0;
}

// The pairs' filter bytes gathered behind the pass (its epoch is held until the wait, so the
// device string pool stays) and packed with the byte offsets, the filter ids and the exact ids
// into one block that one copy brings into the pipe's pinned memory, all stream-ordered.  The
// block holds the pairs and bytes the pipe's recent windows suggest for n topics (x1.2); a
// window beyond them is finished in the wait, synchronously (host_pipe_gather).
int host_pipe_enqueue_gather(emqxgm* h, emqxgm::HostPipe& p) {
  const Scratch& s = p.c.sc;
  const DevIndex& ix = p.c.epoch->ix;
  const uint32_t cap = s.p_cap;  // no pass stages more pairs than this (else it is redone)
  const double ppt = p.fb_ppt > 0 ? p.fb_ppt : 4.0, bpp = p.fb_bpp > 0 ? p.fb_bpp : 32.0;
  // (ppt and bpp are decaying maxima of the pipe's recent windows: x1.2 of headroom on top)
  const double exp_p = ppt * p.n;
  const uint32_t want_p = (uint32_t)std::min<uint64_t>(cap, (uint64_t)(1.2 * exp_p) + 256);
  const uint64_t want_b = (uint64_t)(1.2 * bpp * exp_p) + 4096;
  const FbLayout L(p.n, want_p);
  const uint64_t blk = L.bytes + want_b;
  const uint64_t tw = scan_tmp_words(cap);
  const uint64_t words = 2ull * cap + 1 + tw + 2;  // scratch: lengths, offsets, total, scan
  const uint64_t at = ((words * 4 + 255) / 256) * 256;
  int rc = 0;
  if ((rc = grow_dev(h, p.d_fb, at + blk, p.c.stream)) ||
      (rc = pinned_reserve(h, p.h_blk, (size_t)blk, false)))
    return rc;
  uint32_t* len = (uint32_t*)p.d_fb.p;
  uint32_t* ooff = len + cap;
  uint32_t* total = ooff + cap + 1;
  uint32_t* tmp = total + 2;
  uint8_t* block = (uint8_t*)p.d_fb.p + at;
  // a small window's block goes straight into the pinned buffer (no D2H copy behind the pass)
  void* hb = p.zc ? mapped_ptr(p.h_blk.p) : nullptr;
  const bool direct = hb != nullptr;
  if (direct) block = (uint8_t*)hb;
  const uint32_t* npairs = s.ctl + CTL_TOTAL;  // written by the pass's scan
  hipStream_t st = p.c.stream;
  // (sized by the block's pair capacity: a window with more pairs is finished in the wait); a
  // small block in one single-block launch instead of three
  if (want_p <= FB_SMALL_PAIRS) {
    HIPCHK(h, launch_fb_small(s.out, npairs, ix.foff, ix.fbytes, s.exact_id, s.row, p.n, want_p,
                              want_b, block, st));
  } else {
    HIPCHK(h, launch_filter_len_dev(s.out, npairs, want_p, ix.foff, len, ooff, tmp, total, st));
    HIPCHK(h, launch_fb_pack(s.out, npairs, ix.foff, ix.fbytes, ooff, total, s.exact_id, s.row, p.n,
                             want_p, want_b, block, st));
  }
  if (!direct) HIPCHK(h, hipMemcpyAsync(p.h_blk.p, block, (size_t)blk, hipMemcpyDeviceToHost, st));
  p.fb_pairs_copy = want_p;
  p.fb_bytes_copy = want_b;
  p.fb_async = true;
  return 0;
}
}  // namespace
extern "C" {

int emqxgm_match_batch_submit(emqxgm_t* h, const uint8_t* bytes, const uint32_t* offsets,
                              uint32_t n, uint64_t* ticket) {
  return batch_submit(h, bytes, offsets, n, ticket, false);
}

int emqxgm_match_batch_submit_filters(emqxgm_t* h, const uint8_t* bytes, const uint32_t* offsets,
                                      uint32_t n, uint64_t* ticket) {
  return batch_submit(h, bytes, offsets, n, ticket, true);
}

}  // extern "C"
// gm_async.cpp's window submit: emqxgm_match_batch_submit_filters for offsets built increasing
int gm_submit_window(emqxgm_t* h, const uint8_t* bytes, const uint32_t* offsets, uint32_t n,
                     uint64_t* ticket) {
  return batch_submit(h, bytes, offsets, n, ticket, true, true);
}

int gm_stale(emqxgm_t* h) { return h->stale.load(std::memory_order_acquire) != 0; }

// gm_async.cpp at create: every host pipe's buffers sized for windows of n topics / nb bytes
// (and the filter block for the default density estimate), so that no window of a running
// layer reallocates -- a hipFree synchronises the whole device (r04: 8 reallocations in a load
// point's first windows gave its calls a 3-7 ms p99)
int gm_reserve_windows(emqxgm_t* h, uint32_t n, uint64_t nb) {
  if (!h || !n) return -EINVAL;
  std::lock_guard<std::mutex> g(h->mmu);
  if (hipSetDevice(h->cfg.device) != hipSuccess) return -EIO;
  for (uint32_t k = 0; k < EMQXGM_HOST_PIPES; ++k) {
    emqxgm::HostPipe& p = h->hpipes[k];
    if (p.state == 1) continue;  // in flight (a layer on a busy engine): it grows as it goes
    hipStream_t ps = pipe_stream(h, k);
    if (!ps) return -EIO;
    int rc = ctx_init(h, p.c, ps);
    p.c.pipelined = true;
    if (rc || (rc = pass_prepare(h, p.c, n, nb)) < 0 ||
        (rc = host_pipe_reserve(h, p, n, std::max<uint64_t>(nb, 1), 1)))
      return rc < 0 ? rc : 0;
    // the block host_pipe_enqueue_gather asks for at the default estimates
    const uint32_t cap = p.c.sc.p_cap;
    const double exp_p = 4.0 * n;
    const uint32_t want_p = (uint32_t)std::min<uint64_t>(cap, (uint64_t)(1.2 * exp_p) + 256);
    const uint64_t want_b = (uint64_t)(1.2 * 32.0 * exp_p) + 4096;
    const FbLayout L(n, want_p);
    const uint64_t blk = L.bytes + want_b;
    const uint64_t words = 2ull * cap + 1 + scan_tmp_words(cap) + 2;
    const uint64_t at = ((words * 4 + 255) / 256) * 256;
    if ((rc = grow_dev(h, p.d_fb, at + blk, p.c.stream)) ||
        (rc = pinned_reserve(h, p.h_blk, (size_t)blk, false)))
      return rc;
  }
  return 0;
}
extern "C" {

// Blocks until everything ticket's submit enqueued has run, without holding mmu (the stream
// wait of host_pipe_complete is then immediate).  Only the waiter of a ticket changes its pipe's
// state while it is in flight (a resubmit of the pipe needs the ticket waited: -EBUSY).
static int host_pipe_prewait(emqxgm* h, uint64_t ticket) {
  injected_hang(h);
  hipEvent_t ev = nullptr;
  {
    std::lock_guard<std::mutex> g(h->mmu);
    const emqxgm::HostPipe& p = h->hpipes[ticket % EMQXGM_HOST_PIPES];
    if (ticket != 0 && p.ticket == ticket && p.state == 1) ev = p.fin;
  }
  if (!ev) return 0;
  if (hipSetDevice(h->cfg.device) != hipSuccess) return -EIO;
  if (const uint32_t spin = h->spin_us.load(std::memory_order_relaxed)) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const hipError_t q = hipEventQuery(ev);
      if (q == hipSuccess) return 0;
      if (q != hipErrorNotReady ||
          std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin))
        break;  // (an error: the synchronisation below reports it)
      __builtin_ia32_pause();
    }
    (void)hipGetLastError();  // a pending query's "not ready" is not this thread's error
  }
  if (hipEventSynchronize(ev) != hipSuccess) {
    set_err(h, "hipEventSynchronize failed");
    return -EIO;
  }
  return 0;
}

int emqxgm_match_batch_wait(emqxgm_t* h, uint64_t ticket, emqxgm_batch_out* out) {
  if (!h || !out) return -EINVAL;
  if (int rc = host_pipe_prewait(h, ticket)) return rc;
  std::lock_guard<std::mutex> g(h->mmu);
  RoctxRange rr(h->roctx, "emqxgm.host_wait");
  if (hipSetDevice(h->cfg.device) != hipSuccess) return -EIO;
  emqxgm::HostPipe& p = h->hpipes[ticket % EMQXGM_HOST_PIPES];
  if (ticket == 0 || p.ticket != ticket || p.state == 0) {
    set_err(h, "unknown ticket, or its result was already taken / overwritten");
    return -ENOENT;
  }
  int rc = host_pipe_complete(h, p);
  if (rc) return rc;
  p.state = 0;
  out->n = p.n;
  out->n_pairs = p.pairs;
  out->row_ptr = p.h_row;
  out->filter_id = p.h_fid;
  out->exact_id = p.exact_none ? p.h_none : p.h_exact;
  return 0;
}

int emqxgm_match_batch_wait_filters(emqxgm_t* h, uint64_t ticket, emqxgm_batch_out* out,
                                    const uint32_t** foff, const uint8_t** fbytes) {
  if (!h || !out || !foff || !fbytes) return -EINVAL;
  if (int rc = host_pipe_prewait(h, ticket)) return rc;
  std::lock_guard<std::mutex> g(h->mmu);
  if (hipSetDevice(h->cfg.device) != hipSuccess) return -EIO;
  RoctxRange rr(h->roctx, "emqxgm.host_wait_filters");
  emqxgm::HostPipe& p = h->hpipes[ticket % EMQXGM_HOST_PIPES];
  if (ticket == 0 || p.ticket != ticket || p.state == 0) {
    set_err(h, "unknown ticket, or its result was already taken / overwritten");
    return -ENOENT;
  }
  const bool empty = p.state == 2;  // an empty batch: no pass ran
  if (empty) p.fb_fast = false;
  int rc = host_pipe_complete(h, p, true);
  if (rc || (rc = pinned_reserve(h, p.h_fboff, 4, true)) || (rc = pinned_reserve(h, p.h_fb, 1, true)))
    return rc;
  if (empty) ((uint32_t*)p.h_fboff.p)[0] = 0;
  p.state = 0;
  out->n = p.n;
  out->n_pairs = p.pairs;
  out->row_ptr = p.h_row;
  if (p.fb_fast) {  // one block: FbLayout for the pipe's n and copy sizes
    const FbLayout L(p.n, (uint32_t)p.fb_pairs_copy);
    const uint8_t* b = (const uint8_t*)p.h_blk.p;
    out->row_ptr = (const uint32_t*)(b + L.row);
    out->filter_id = (const uint32_t*)(b + L.fid);
    out->exact_id = (const uint32_t*)(b + L.exact);
    *foff = (const uint32_t*)(b + L.ooff);
    *fbytes = b + L.bytes;
    return 0;
  }
  out->filter_id = p.h_fid;
  out->exact_id = p.exact_none ? p.h_none : p.h_exact;
  *foff = (const uint32_t*)p.h_fboff.p;
  *fbytes = (const uint8_t*)p.h_fb.p;
  return 0;
}

int emqxgm_match_batch(emqxgm_t* h, const uint8_t* bytes, const uint32_t* offsets, uint32_t n,
                       emqxgm_out* out) {
  if (!h || !out || (!offsets && n)) return -EINVAL;
  if (int rc = refuse_stale(h)) return rc;
  std::lock_guard<std::mutex> g(h->mmu);
  if (hipSetDevice(h->cfg.device) != hipSuccess) return -EIO;
  PassCtx& c = h->sync;
  // results land in pinned host buffers of the handle by D2H copies (u64 row pointers are built
  // on the device): no host-side conversion or initialisation per topic
  int rc = 0;
  if ((rc = pinned_reserve(h, h->hp_row, ((size_t)n + 1) * 8, false)) ||
      (rc = pinned_reserve(h, h->hp_exact, std::max<size_t>((size_t)n * 4, 4), false)) ||
      (rc = pinned_reserve(h, h->hp_fid, 4, false)))
    return rc;
  uint64_t* row = (uint64_t*)h->hp_row.p;
  row[0] = 0;
  uint64_t total = 0;
  std::vector<uint32_t> loff;
  for (uint32_t i0 = 0; i0 < n; i0 += h->cfg.batch_max) {
    const uint32_t i1 = std::min<uint64_t>((uint64_t)i0 + h->cfg.batch_max, n);
    const uint32_t m = i1 - i0;
    const uint64_t b0 = offsets[i0], b1 = offsets[i1];
    if (b1 < b0) return -EINVAL;
    loff.resize((size_t)m + 1);
    for (uint32_t i = 0; i <= m; ++i) {
      if (offsets[i0 + i] < b0 || (i && offsets[i0 + i] < offsets[i0 + i - 1])) return -EINVAL;
      loff[i] = (uint32_t)(offsets[i0 + i] - b0);
    }
    if ((rc = ensure_input(h, std::max<uint64_t>(b1 - b0, 1), (uint64_t)m + 1))) return rc;
    if (b1 > b0)
      HIPCHK(h, hipMemcpyAsync(h->d_in_bytes, bytes + b0, b1 - b0, hipMemcpyHostToDevice, c.stream));
    HIPCHK(h, hipMemcpyAsync(h->d_in_off, loff.data(), ((size_t)m + 1) * 4, hipMemcpyHostToDevice,
                             c.stream));
    uint32_t pairs = 0;
    rc = run_device(h, c, h->d_in_bytes, h->d_in_off, m, b1 - b0, &pairs);
    c.epoch.reset();
    if (rc) return rc;
    if ((uint64_t)m + 1 > h->row64_cap) {
      if (h->d_row64) (void)hipFree(h->d_row64);
      h->d_row64 = nullptr;
      h->row64_cap = 0;
      HIPCHK(h, hipMalloc((void**)&h->d_row64, ((size_t)m + 1) * 8));
      h->row64_cap = (uint64_t)m + 1;
    }
    if ((rc = pinned_reserve(h, h->hp_fid, std::max<size_t>((total + pairs) * 4, 4), true)))
      return rc;
    HIPCHK(h, launch_row64(c.sc.row, total, h->d_row64, m + 1, c.stream));
    HIPCHK(h, hipMemcpyAsync(row + i0, h->d_row64, ((size_t)m + 1) * 8, hipMemcpyDeviceToHost,
                             c.stream));
    HIPCHK(h, hipMemcpyAsync((uint32_t*)h->hp_exact.p + i0, c.sc.exact_id, (size_t)m * 4,
                             hipMemcpyDeviceToHost, c.stream));
    if (pairs)
      HIPCHK(h, hipMemcpyAsync((uint32_t*)h->hp_fid.p + total, c.sc.out, (size_t)pairs * 4,
                               hipMemcpyDeviceToHost, c.stream));
    HIPCHK(h, hipStreamSynchronize(c.stream));
    total += pairs;
  }
  out->n = n;
  out->n_pairs = total;
  out->row_ptr = row;
  out->filter_id = (const uint32_t*)h->hp_fid.p;
  out->exact_id = (const uint32_t*)h->hp_exact.p;
  return 0;
}

void* emqxgm_host_alloc(emqxgm_t* h, uint64_t bytes) {
  if (!h) return nullptr;
  void* p = nullptr;
  if (hipSetDevice(h->cfg.device) != hipSuccess ||
      hipHostMalloc(&p, std::max<uint64_t>(bytes, 1), hipHostMallocPortable) != hipSuccess)
    return nullptr;
  return p;
}

void emqxgm_host_free(emqxgm_t* h, void* p) {
  if (h && p) (void)hipHostFree(p);
}

int emqxgm_publish_batch(emqxgm_t* h, const uint8_t* bytes, const uint32_t* offsets, uint32_t n,
                         emqxgm_publish_out* out) {
  if (!h || !out || (!offsets && n)) return -EINVAL;
  if (int rc = refuse_stale(h)) return rc;
  injected_hang(h);
  std::lock_guard<std::mutex> g(h->mmu);
  if (hipSetDevice(h->cfg.device) != hipSuccess) return -EIO;
  PassCtx& c = h->sync;
  h->h_rp.assign((size_t)n + 1, 0);
  h->h_dp.assign((size_t)n + 1, 0);
  h->h_rf.clear();
  h->h_rd.clear();
  h->h_df.clear();
  h->h_ds.clear();
  std::vector<uint32_t> loff;
  for (uint32_t i0 = 0; i0 < n; i0 += h->cfg.batch_max) {
    const uint32_t i1 = std::min<uint64_t>((uint64_t)i0 + h->cfg.batch_max, n);
    const uint32_t m = i1 - i0;
    const uint64_t b0 = offsets[i0], b1 = offsets[i1];
    if (b1 < b0) return -EINVAL;
    loff.resize((size_t)m + 1);
    for (uint32_t i = 0; i <= m; ++i) {
      if (offsets[i0 + i] < b0 || (i && offsets[i0 + i] < offsets[i0 + i - 1])) return -EINVAL;
      loff[i] = (uint32_t)(offsets[i0 + i] - b0);
    }
    int rc = ensure_input(h, std::max<uint64_t>(b1 - b0, 1), (uint64_t)m + 1);
    if (rc) return rc;
    if (b1 > b0)
      HIPCHK(h, hipMemcpyAsync(h->d_in_bytes, bytes + b0, b1 - b0, hipMemcpyHostToDevice, c.stream));
    HIPCHK(h, hipMemcpyAsync(h->d_in_off, loff.data(), ((size_t)m + 1) * 4, hipMemcpyHostToDevice,
                             c.stream));
    uint32_t pairs = 0, nr = 0, nd = 0;
    // the match and the fan-out must read one epoch: redo both if a commit came in between
    for (;;) {
      rc = run_device(h, c, h->d_in_bytes, h->d_in_off, m, b1 - b0, &pairs);
      if (!rc) rc = run_fanout(h, m, &nr, &nd);
      if (rc != 1) break;
    }
    c.epoch.reset();
    if (rc) return rc;
    const FanScratch& f = h->fs;
    const uint64_t rbase = h->h_rf.size(), dbase = h->h_df.size();
    h->h_rf.resize(rbase + nr);
    h->h_rd.resize(rbase + nr);
    h->h_df.resize(dbase + nd);
    h->h_ds.resize(dbase + nd);
    std::vector<uint32_t> rp(m + 1), dp(m + 1);
    HIPCHK(h, hipMemcpyAsync(rp.data(), f.rp, ((size_t)m + 1) * 4, hipMemcpyDeviceToHost, c.stream));
    HIPCHK(h, hipMemcpyAsync(dp.data(), f.dp, ((size_t)m + 1) * 4, hipMemcpyDeviceToHost, c.stream));
    if (nr) {
      HIPCHK(h, hipMemcpyAsync(h->h_rf.data() + rbase, f.o_rf, (size_t)nr * 4, hipMemcpyDeviceToHost, c.stream));
      HIPCHK(h, hipMemcpyAsync(h->h_rd.data() + rbase, f.o_rd, (size_t)nr * 4, hipMemcpyDeviceToHost, c.stream));
    }
    if (nd) {
      HIPCHK(h, hipMemcpyAsync(h->h_df.data() + dbase, f.o_df, (size_t)nd * 4, hipMemcpyDeviceToHost, c.stream));
      HIPCHK(h, hipMemcpyAsync(h->h_ds.data() + dbase, f.o_ds, (size_t)nd * 4, hipMemcpyDeviceToHost, c.stream));
    }
    HIPCHK(h, hipStreamSynchronize(c.stream));
    for (uint32_t i = 0; i <= m; ++i) {
      h->h_rp[i0 + i] = rbase + rp[i];
      h->h_dp[i0 + i] = dbase + dp[i];
    }
  }
  out->n = n;
  out->n_routes = h->h_rf.size();
  out->n_deliveries = h->h_df.size();
  out->route_ptr = h->h_rp.data();
  out->route_filter = h->h_rf.data();
  out->route_dest = h->h_rd.data();
  out->deliver_ptr = h->h_dp.data();
  out->deliver_filter = h->h_df.data();
  out->deliver_sub = h->h_ds.data();
  return 0;
}

static int grow_buf(emqxgm* h, DevBuf& b, uint64_t bytes);

int emqxgm_export(emqxgm_t* h, const emqxgm_dev_out* r, const uint32_t* id_map, uint32_t* row,
                  uint32_t* fid, uint32_t* exact) {
  if (!h || !r || !row || (r->n && !exact) || (r->n_pairs && !fid)) return -EINVAL;
  std::lock_guard<std::mutex> g(h->mmu);
  if (hipSetDevice(h->cfg.device) != hipSuccess) return -EIO;
  hipStream_t s = h->sync.stream;
  HIPCHK(h, launch_export(r->row_ptr, r->filter_id, r->exact_id, r->n, r->n_pairs, id_map, row, fid,
                          exact, s));
  HIPCHK(h, hipStreamSynchronize(s));
  return 0;
}

int emqxgm_merge(emqxgm_t* h, uint32_t parts, const uint32_t* const* rows,
                 const uint32_t* const* fids, const uint32_t* const* exacts, uint32_t n,
                 uint32_t* out_row, uint32_t* out_fid, uint32_t* out_exact, uint32_t* n_pairs) {
  if (!h || !out_row || (parts && (!rows || !fids || !exacts)) || (n && !out_exact)) return -EINVAL;
  std::lock_guard<std::mutex> g(h->mmu);
  if (hipSetDevice(h->cfg.device) != hipSuccess) return -EIO;
  hipStream_t s = h->sync.stream;
  const uint64_t tw = scan_tmp_words(std::max<uint32_t>(n, 1));
  const uint64_t need = (3ull * parts + 1) * 8 + ((uint64_t)n + tw + 2) * 4;
  if (int rc = grow_buf(h, h->d_merge, need)) return rc;
  std::vector<const uint32_t*> pp(3ull * parts);
  for (uint32_t i = 0; i < parts; ++i) {
    pp[3 * i] = rows[i];
    pp[3 * i + 1] = fids[i];
    pp[3 * i + 2] = exacts[i];
  }
  uint8_t* d = (uint8_t*)h->d_merge.p;
  uint32_t* cnt = (uint32_t*)(d + (3ull * parts + 1) * 8);
  uint32_t* total = cnt + n;
  uint32_t* tmp = total + 2;
  if (parts) HIPCHK(h, hipMemcpyAsync(d, pp.data(), pp.size() * 8, hipMemcpyHostToDevice, s));
  HIPCHK(h, launch_merge((const uint32_t* const*)d, parts, n, cnt, tmp, out_row, out_fid, out_exact,
                         total, s));
  uint32_t tot = 0;
  if (n) HIPCHK(h, hipMemcpyAsync(&tot, total, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(h, hipStreamSynchronize(s));
  if (n_pairs) *n_pairs = tot;
  return 0;
}

int emqxgm_export_wire(emqxgm_t* h, const emqxgm_dev_out* r, const uint32_t* id_map,
                       uint32_t flags, void* cnt, void* fid, uint32_t* xs, uint32_t* ovf,
                       uint32_t counts[2]) {
  if (!h || !r || !counts || (flags & ~3u) || (r->n && (!cnt || !xs || !ovf)) ||
      (r->n_pairs && !fid))
    return -EINVAL;
  std::lock_guard<std::mutex> g(h->mmu);
  if (hipSetDevice(h->cfg.device) != hipSuccess) return -EIO;
  hipStream_t s = h->sync.stream;
  if (int rc = grow_buf(h, h->d_merge, 16)) return rc;
  uint32_t* ctr = (uint32_t*)h->d_merge.p;
  HIPCHK(h, launch_wire_export(r->row_ptr, r->filter_id, r->exact_id, r->n, r->n_pairs, id_map,
                               flags, (uint8_t*)cnt, (uint8_t*)fid, (uint2*)xs, (uint2*)ovf, ctr, s));
  HIPCHK(h, hipMemcpyAsync(counts, ctr, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(h, hipStreamSynchronize(s));
  return 0;
}

int emqxgm_merge_wire(emqxgm_t* h, uint32_t parts, const uint32_t* flags, const void* const* cnts,
                      const void* const* fids, const uint32_t* n_pairs_part,
                      const uint32_t* const* xss, const uint32_t* n_xs, const uint32_t* const* ovfs,
                      const uint32_t* n_ovf, uint32_t n, uint32_t* out_row, uint32_t* out_fid,
                      uint32_t* out_exact, uint32_t* n_pairs) {
  if (!h || !out_row ||
      (parts && (!flags || !cnts || !fids || !n_pairs_part || !xss || !n_xs || !ovfs || !n_ovf)) ||
      (n && !out_exact))
    return -EINVAL;
  std::lock_guard<std::mutex> g(h->mmu);
  if (hipSetDevice(h->cfg.device) != hipSuccess) return -EIO;
  hipStream_t s = h->sync.stream;
  // scratch: [pointer table 3 x parts | parts x (n+1) row words | widened ids of 24-bit parts |
  //           n count words | total | scan]
  uint64_t wide = 0;
  for (uint32_t r = 0; r < parts; ++r) wide += (flags[r] & 2u) ? n_pairs_part[r] : 0;
  const uint64_t tw = scan_tmp_words(std::max<uint32_t>(n, 1));
  const uint64_t rows_off = (3ull * parts + 1) * 8;
  const uint64_t need = rows_off + ((uint64_t)parts * (n + 1) + wide + n + 2 + tw) * 4;
  if (int rc = grow_buf(h, h->d_merge, need)) return rc;
  uint8_t* d = (uint8_t*)h->d_merge.p;
  uint32_t* prow = (uint32_t*)(d + rows_off);
  uint32_t* pid = prow + (uint64_t)parts * (n + 1);
  uint32_t* cnt = pid + wide;
  uint32_t* total = cnt + n;
  uint32_t* tmp = total + 2;
  std::vector<const uint32_t*> pp(3ull * parts);
  for (uint32_t r = 0; r < parts; ++r) {
    HIPCHK(h, launch_wire_rows((const uint8_t*)cnts[r], flags[r], (const uint2*)ovfs[r], n_ovf[r], n,
                               cnt, tmp, prow + (uint64_t)r * (n + 1), s));
    pp[3 * r] = prow + (uint64_t)r * (n + 1);
    pp[3 * r + 1] = (const uint32_t*)fids[r];
    pp[3 * r + 2] = out_exact;
    if (flags[r] & 2u) {
      HIPCHK(h, launch_wire_ids((const uint8_t*)fids[r], n_pairs_part[r], pid, s));
      pp[3 * r + 1] = pid;
      pid += n_pairs_part[r];
    }
  }
  HIPCHK(h, launch_wire_exact((const uint2* const*)xss, n_xs, parts, n, out_exact, s));
  // then the merge of emqxgm_merge over {part rows, part ids, the merged exact ids}
  if (parts) HIPCHK(h, hipMemcpyAsync(d, pp.data(), pp.size() * 8, hipMemcpyHostToDevice, s));
  HIPCHK(h, launch_merge((const uint32_t* const*)d, parts, n, cnt, tmp, out_row, out_fid, out_exact,
                         total, s));
  uint32_t tot = 0;
  if (n) HIPCHK(h, hipMemcpyAsync(&tot, total, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(h, hipStreamSynchronize(s));
  if (n_pairs) *n_pairs = tot;
  return 0;
}

int emqxgm_walk_census(emqxgm_t* h, const uint8_t* d_bytes, const uint32_t* d_offsets, uint32_t n,
                       uint64_t bytes_len, uint64_t out[6]) {
  if (!h || !out || (!d_offsets && n)) return -EINVAL;
  std::lock_guard<std::mutex> g(h->mmu);
  if (hipSetDevice(h->cfg.device) != hipSuccess) return -EIO;
  uint32_t pairs = 0;
  memset(out, 0, 6 * sizeof(uint64_t));
  int rc = run_device(h, h->sync, d_bytes, d_offsets, n, bytes_len, &pairs, out);
  h->sync.epoch.reset();
  return rc;
}

int emqxgm_walk_census_levels(emqxgm_t* h, uint64_t* out, uint32_t n_out) {
  if (!h || (!out && n_out)) return -EINVAL;
  std::lock_guard<std::mutex> g(h->mmu);
  for (uint32_t i = 0; i < n_out && i < 2 * CENSUS_DEPTHS; ++i) out[i] = h->census_depth[i];
  return (int)(2 * CENSUS_DEPTHS);
}

static int grow_buf(emqxgm* h, DevBuf& b, uint64_t bytes) {
  if (bytes <= b.bytes && b.p) return 0;
  HIPCHK(h, hipStreamSynchronize(h->sync.stream));
  if (b.p) (void)hipFree(b.p);
  b = DevBuf();
  const uint64_t cap = std::max<uint64_t>(bytes + bytes / 2, 4096);
  HIPCHK(h, hipMalloc(&b.p, cap));
  b.bytes = cap;
  return 0;
}

int emqxgm_match_rules(emqxgm_t* h, const uint8_t* name_bytes, const uint32_t* name_offsets,
                       uint32_t n, const uint8_t* rule_bytes, const uint32_t* rule_offsets,
                       const uint32_t* rule_flags, uint32_t n_rules, uint32_t* out) {
  if (!h || !name_offsets || !rule_offsets || (n && !out) || (n_rules && !rule_flags))
    return -EINVAL;
  const uint64_t nb = name_offsets[n], rb = rule_offsets[n_rules];
  if ((nb && !name_bytes) || (rb && !rule_bytes)) return -EINVAL;
  for (uint32_t i = 0; i < n; ++i)
    if (name_offsets[i + 1] < name_offsets[i]) return -EINVAL;
  for (uint32_t i = 0; i < n_rules; ++i)
    if (rule_offsets[i + 1] < rule_offsets[i]) return -EINVAL;
  std::lock_guard<std::mutex> g(h->mmu);
  if (n == 0) return 0;
  if (hipSetDevice(h->cfg.device) != hipSuccess) return -EIO;
  // one device buffer: [names | name offsets | rules | rule offsets | flags | out]
  auto al = [](uint64_t x) { return (x + 15) & ~15ull; };
  const uint64_t o_no = al(nb), o_rb = o_no + al(((uint64_t)n + 1) * 4), o_ro = o_rb + al(rb);
  const uint64_t o_rf = o_ro + al(((uint64_t)n_rules + 1) * 4);
  const uint64_t o_out = o_rf + al((uint64_t)n_rules * 4 + 4);
  const uint64_t total = o_out + (uint64_t)n * 4;
  int rc = grow_buf(h, h->d_rules, total);
  if (rc) return rc;
  uint8_t* d = (uint8_t*)h->d_rules.p;
  hipStream_t s = h->sync.stream;
  if (nb) HIPCHK(h, hipMemcpyAsync(d, name_bytes, nb, hipMemcpyHostToDevice, s));
  HIPCHK(h, hipMemcpyAsync(d + o_no, name_offsets, ((size_t)n + 1) * 4, hipMemcpyHostToDevice, s));
  if (rb) HIPCHK(h, hipMemcpyAsync(d + o_rb, rule_bytes, rb, hipMemcpyHostToDevice, s));
  HIPCHK(h, hipMemcpyAsync(d + o_ro, rule_offsets, ((size_t)n_rules + 1) * 4,
                           hipMemcpyHostToDevice, s));
  if (n_rules)
    HIPCHK(h, hipMemcpyAsync(d + o_rf, rule_flags, (size_t)n_rules * 4, hipMemcpyHostToDevice, s));
  HIPCHK(h, launch_rules(d, (const uint32_t*)(d + o_no), n, d + o_rb, (const uint32_t*)(d + o_ro),
                         (const uint32_t*)(d + o_rf), n_rules, rb, (uint32_t*)(d + o_out), s));
  HIPCHK(h, hipMemcpyAsync(out, d + o_out, (size_t)n * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(h, hipStreamSynchronize(s));
  return 0;
}

int emqxgm_set_profiling(emqxgm_t* h, int on) {
  if (!h) return -EINVAL;
  std::lock_guard<std::mutex> g(h->mmu);
  h->profiling = on != 0;
  return 0;
}

int emqxgm_tune(emqxgm_t* h, const char* key, int64_t value) {
  if (!h || !key) return -EINVAL;
  if (strcmp(key, "walk_wg_per_cu") == 0) {
    if (value < 1 || value > 16) return -EINVAL;
    std::lock_guard<std::mutex> g(h->mmu);
    if (int rc = drain_pipes(h)) return rc;  // in-flight passes use the old geometry
    h->cfg.walk_wg_per_cu = (uint32_t)value;
    h->geom = walk_geometry(h->cfg.device, h->cfg.walk_wg_per_cu);
    h->geom.xrange_bytes = h->xrange_bytes;
    h->geom.pair = h->walk_pair_on;
    set_pipe_geometry(h);
    return 0;  // spill scratch is re-sized by the next match (ensure_scratch)
  }
  if (strcmp(key, "walk_wg_per_cu_pipe") == 0) {  // pipelined passes' walk (never above the other)
    if (value < 1 || value > 16) return -EINVAL;
    std::lock_guard<std::mutex> g(h->mmu);
    if (int rc = drain_pipes(h)) return rc;
    h->pipe_wg_per_cu = (uint32_t)value;
    set_pipe_geometry(h);
    return 0;
  }
  if (strcmp(key, "leaf_prune") == 0) {  // 1 (default): the walk skips leaf-only children
    if (value < 0 || value > 1) return -EINVAL;
    std::lock_guard<std::mutex> g(h->mmu);
    h->leafp_mask = value ? CF_HMASK : 0u;
    return 0;
  }
  if (strcmp(key, "spin_us") == 0) {  // host pipes' waits poll before they block
    if (value < 0 || value > 1000000) return -EINVAL;
    h->spin_us.store((uint32_t)value, std::memory_order_relaxed);
    return 0;
  }
  if (strcmp(key, "zc_topics") == 0) {  // concurrent-entry windows without DMA copies: max topics
    if (value < 0) return -EINVAL;
    std::lock_guard<std::mutex> g(h->mmu);
    h->zc_topics = (uint32_t)value;
    return 0;
  }
  if (strcmp(key, "host_out") == 0) {  // host pipes' result copy: 0 hipMemcpyAsync (default), 1 kernel
    if (value < 0 || value > 1) return -EINVAL;
    std::lock_guard<std::mutex> g(h->mmu);
    for (auto& p : h->hpipes)
      if (p.state == 1) return -EBUSY;
    h->host_out_mode = (uint32_t)value;
    return 0;
  }
  if (strcmp(key, "walk_pair") == 0) {  // 1 (default): two lanes per topic for small batches
    if (value < 0 || value > 2) return -EINVAL;  // (2: every batch, an A/B)
    std::lock_guard<std::mutex> g(h->mmu);
    if (int rc = drain_pipes(h)) return rc;  // in-flight passes read the geometry
    h->walk_pair_on = (uint32_t)value;
    h->geom.pair = h->geom_pipe.pair = h->walk_pair_on;
    return 0;
  }
  if (strcmp(key, "exact_range_kb") == 0) {  // 0 (default): auto; > 0: probe in ranges of v KiB
    if (value < 0 || value > (int64_t)1 << 32) return -EINVAL;
    std::lock_guard<std::mutex> g(h->mmu);
    if (int rc = drain_pipes(h)) return rc;  // in-flight passes read the geometry
    h->xrange_bytes = (uint64_t)value << 10;
    h->geom.xrange_bytes = h->xrange_bytes;
    h->geom_pipe.xrange_bytes = h->xrange_bytes;
    return 0;
  }
  if (strcmp(key, "delta_commit") == 0) {
    if (value < 0 || value > 2) return -EINVAL;
    std::lock_guard<std::mutex> g(h->wmu);
    h->delta_mode = (uint32_t)value;
    return 0;
  }
  if (strcmp(key, "delta_max") == 0) {  // changes a delta commit takes (0: max(4096, keys / 8))
    if (value < 0) return -EINVAL;
    std::lock_guard<std::mutex> g(h->wmu);
    h->delta_max = (uint64_t)value;
    return 0;
  }
  if (strcmp(key, "bg_build") == 0) {  // full builds of >= v filters in the background (0: never)
    if (value < 0) return -EINVAL;
    std::lock_guard<std::mutex> g(h->wmu);
    h->bg_min = (uint64_t)value;
    return 0;
  }
  if (strcmp(key, "bg_delay_ms") == 0) {  // tests: a background build holds its install back
    if (value < 0 || value > 600000) return -EINVAL;
    h->bg_delay_ms.store((uint32_t)value);
    return 0;
  }
  if (strcmp(key, "fail_commits") == 0) {  // tests: the next v commits fail (health, r06)
    if (value < 0 || value > 1000000) return -EINVAL;
    h->inject_commits.store(value);
    return 0;
  }
  if (strcmp(key, "fail_errno") == 0) {  // the errno an injected failure returns (default EIO)
    if (value <= 0 || value > 4095) return -EINVAL;
    h->inject_errno.store((int32_t)value);
    return 0;
  }
  if (strcmp(key, "hang_ms") == 0) {  // tests: host-pipe waits and publish passes stall first
    if (value < 0 || value > 600000) return -EINVAL;
    h->hang_ms.store((uint32_t)value);
    return 0;
  }
  if (strcmp(key, "stage_rank_bits") == 0) {  // tests: cap the packed staging's rank field
    if (value < 0 || value > 31) return -EINVAL;
    h->stage_rank_bits.store((uint32_t)value);
    return 0;
  }
  if (strcmp(key, "probe_ms") == 0) {  // a repair's bounded wait for the device's streams
    if (value < 1 || value > 600000) return -EINVAL;
    std::lock_guard<std::mutex> g(h->wmu);
    h->probe_ms = (uint32_t)value;
    return 0;
  }
  if (strcmp(key, "rebuild") == 0) {  // 1: a full build in the background now (not waited for)
    if (value != 1) return -EINVAL;
    std::lock_guard<std::mutex> g(h->wmu);
    if (h->job) return -EBUSY;
    if (!bg_allowed(h) || !h->tm.valid) return -EINVAL;
    return start_build(h);
  }
  if (strcmp(key, "roctx") == 0) {  // 1: roctx ranges / launch markers (gm_roctx.h)
    if (value < 0 || value > 1) return -EINVAL;
    h->roctx = value != 0;
    return 0;
  }
  if (strcmp(key, "keyed") == 0) {  // token-keyed parents (select_keyed), next full build on
    if (value < 0 || value > 2) return -EINVAL;
    std::unique_lock<std::mutex> g(h->wmu);
    if (h->job) (void)wait_build(h, g);  // (it builds with the old setting)
    if (h->keyed_mode != (uint32_t)value && !h->filters.empty()) {
      h->tm.valid = false;  // the next commit is a full build
      h->dirty = true;
    }
    h->keyed_mode = (uint32_t)value;
    return 0;
  }
  if (strcmp(key, "fat_buckets") == 0) {  // 1 (default) / 0: from the next full build on
    if (value < 0 || value > 1) return -EINVAL;
    std::unique_lock<std::mutex> g(h->wmu);
    if (h->job) (void)wait_build(h, g);
    h->fat_mode = (uint32_t)value;
    h->tm.valid = false;  // the next commit is a full build
    h->dirty = true;
    return 0;
  }
  return -EINVAL;
}

int emqxgm_get_stats(emqxgm_t* h, emqxgm_stats* st) {
  if (!h || !st) return -EINVAL;
  std::lock_guard<std::mutex> g(h->stmu);
  *st = h->st;
  return 0;
}

const char* emqxgm_last_error(emqxgm_t* h) {
  static thread_local std::string copy;
  if (!h) return "null handle";
  std::lock_guard<std::mutex> g(h->errmu);
  copy = h->err;
  return copy.c_str();
}

}  // extern "C"
