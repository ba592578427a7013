// harness.cpp -- TEST INFRASTRUCTURE: the engine's host code under ASan + UBSan on the CPU.
//
// Built by tests/test_host_sanitize.py with g++ -fsanitize=address,undefined against the fake
// HIP runtime of this directory (device memory = host memory, k_patch applied on the CPU).  It
// includes emqx_amd/csrc/gm_engine.cpp itself, so it sees the committed epochs' tables, and it
// links the oracle's C++ restatement (oracle/ref_trie.cpp) as the checker.
//
// A random churn of trie inserts / deletes, route keys, routes and local subscribers (the
// mutations of emqx_trie.erl:113-144, 242-260 and emqx_router_utils.erl:31-71) runs against two
// engines -- one patching its tables by delta commits, one rebuilding at every commit -- and the
// oracle.  After every commit, for every probe topic:
//   * the trie row that the committed device tables give, walked on the CPU exactly as k_walk
//     walks them (gm_walk.inc create/visit: carried '+' children, depth-code pruning, child
//     signatures, multi lists, the '$' rules, the tn side array; pairs of hashed-token filters
//     re-checked with emqx_topic:match/2 as k_verify does), equals the oracle's emqx_trie:match;
//   * the exact route-key probe over the committed exact table (inline key bytes, overflow
//     bits, both regions) equals the oracle's route-key lookup;
// and every filter's fan-out entry in the device tables equals the lists the registry gives.
// Prints "OK <commits> <delta commits> <full commits> <checks>" on success.
#include <stdio.h>

#include <algorithm>
#include <map>
#include <random>
#include <set>
#include <string>
#include <vector>

#include "../../emqx_amd/csrc/gm_engine.cpp"

extern "C" {
void* ref_create(int compact);
void ref_destroy(void* h);
int ref_add_many(void* h, const uint8_t* bytes, const uint64_t* off, uint64_t n, const uint8_t* kind);
int ref_trie_delete(void* h, const uint8_t* p, uint32_t len);
int ref_route_delete(void* h, const uint8_t* p, uint32_t len);
int ref_match_batch(void* h, const uint8_t* tb, const uint32_t* toff, uint64_t n, int threads,
                    uint64_t* row, uint32_t** ids_out, uint64_t* n_ids, uint32_t* exact);
void ref_free(void* p);
}

namespace {

#define CHECK(c, ...)                                             \
  do {                                                            \
    if (!(c)) {                                                   \
      fprintf(stderr, "FAIL %s:%d: %s: ", __FILE__, __LINE__, #c); \
      fprintf(stderr, __VA_ARGS__);                               \
      fprintf(stderr, "\n");                                      \
      exit(1);                                                    \
    }                                                             \
  } while (0)

// emqx_topic:match/2 on bytes (gm_kernels.hip mqtt_match, the '$' clauses included)
bool mqtt_match(const std::string& t, const std::string& f) {
  if (!t.empty() && t[0] == '$' && !f.empty() && (f[0] == '+' || f[0] == '#')) return false;
  std::vector<std::string> tw, fw;
  auto split = [](const std::string& s, std::vector<std::string>& w) {
    size_t a = 0;
    for (size_t i = 0; i <= s.size(); ++i)
      if (i == s.size() || s[i] == '/') {
        w.push_back(s.substr(a, i - a));
        a = i + 1;
      }
  };
  split(t, tw);
  split(f, fw);
  for (size_t i = 0; i < fw.size(); ++i) {
    if (fw[i] == "#" && i + 1 == fw.size()) return true;
    if (i >= tw.size()) return false;
    if (fw[i] != "+" && fw[i] != tw[i]) return false;
  }
  return tw.size() == fw.size();
}

std::string filter_str(emqxgm* h, uint32_t id) {
  const Filter& f = h->filters[id];
  return std::string((const char*)h->pool.data() + f.off, f.len);
}

// The walk of gm_walk.inc over the committed tables, on the CPU.
struct CpuWalk {
  const DevIndex& ix;
  std::vector<uint64_t> toks;
  uint32_t n = 0;
  bool dollar = false;
  std::vector<uint32_t> out;
  std::vector<std::pair<uint32_t, uint32_t>> stk;  // (node | item kind, level)
  static constexpr uint32_t IT_PLUS = 0x80000000u, IT_TN = 0x40000000u;
  static constexpr uint32_t IT_KEYED = IT_PLUS | IT_TN, IT_KIND = IT_PLUS | IT_TN;

  explicit CpuWalk(const DevIndex& x) : ix(x) {}
  void em(uint32_t v) {
    if (v == NONE) return;
    if (v & LIST_MULTI) {
      const uint32_t i = v & ~LIST_MULTI, c = ix.multi[i];
      for (uint32_t j = 0; j < c; ++j) out.push_back(ix.multi[i + 1 + j]);
    } else {
      out.push_back(v);
    }
  }
  uint32_t strip(uint32_t cf, uint32_t d) const {
    const uint32_t h = cf_depth_code(cf & ix.leafp_mask);
    return (h != 0u && (int)(n - d) > (int)h) ? (cf & ~(CF_LIT | CF_PLUS)) : cf;
  }
  void visit(uint32_t cf, uint32_t hf, uint32_t tw, uint32_t d, bool lit, uint32_t kind = 0) {
    if (hf != NONE) em(hf);
    if (d == n) {
      if (cf & CF_TW) em(tw);
      if (lit && (cf & CF_TN) && dollar && n == 1) stk.push_back({IT_TN | (cf & CF_ID_MASK), d});
    } else if (cf & CF_LIT) {
      stk.push_back({(cf & CF_ID_MASK) | kind, d});
    }
  }
  // fat: the state's only literal child comes with it in {h0, h1} (gm_common.h FAT_ID)
  void create(uint32_t cf, uint32_t hf, uint32_t tw, uint32_t sig, uint32_t pcf, uint32_t phf,
              uint32_t d, bool plus_ok, bool lit, bool fat = false, const uint4* h = nullptr) {
    const bool keyed = sig == 0u && (cf & CF_LIT);  // gm_common.h edge_home
    cf = strip(cf, d);
    const uint64_t wtok = d < REC_TOKS ? (d < n ? toks[d] : 0ull) : 0ull;
    const bool fat_go = fat && (cf & CF_LIT) && d < n && d < REC_TOKS &&
                        (uint32_t)wtok == h[0].x && (uint32_t)(wtok >> 32) == h[0].y;
    if (fat || (!keyed && d < REC_TOKS && !(sig & sig_bit(wtok)))) cf &= ~CF_LIT;
    pcf = strip(pcf, d + 1);
    visit(cf, hf, tw, d, lit, keyed ? IT_KEYED : 0u);
    if (fat_go)
      create(h[0].w, h[1].x, h[1].y, h[0].z >> SIG_SHIFT, h[1].z, h[1].w, d + 1, true, true);
    if (!plus_ok || d >= n || !(cf & CF_PLUS)) return;
    const bool ptw = (pcf & CF_PTW) != 0;  // the carried copy holds the child's tw, no hf
    if (d + 1 == n && (pcf & CF_TW) && !ptw) {
      stk.push_back({IT_PLUS | (cf & CF_ID_MASK), d});
      return;
    }
    visit(pcf & ~CF_PTW, ptw ? NONE : phf, ptw ? phf : NONE, d + 1, false);
    if (d + 1 < n && (pcf & CF_PLUS)) stk.push_back({IT_PLUS | (pcf & CF_ID_MASK), d + 1});
  }
  // the edge slot of (node, key): probes buckets like k_walk (a bucket with an empty slot ends)
  // fat: the hit is a bucket's first slot and the second holds its fat half (copied to h)
  bool probe(uint32_t node, uint64_t key, bool keyed, uint4 s[2], bool& fat, uint4 h[2]) const {
    for (uint64_t b = edge_home(node, key, ix.emask, keyed);; b = (b + 1) & ix.emask) {
      bool empty = false;
      for (uint32_t j = 0; j < EBUCKET; ++j) {
        const uint4* q = ix.edges + SLOT_U4 * (EBUCKET * b + j);
        if ((q[0].z & CF_ID_MASK) == node && q[0].x == (uint32_t)key &&
            q[0].y == (uint32_t)(key >> 32)) {
          s[0] = q[0];
          s[1] = q[1];
          fat = j == 0 && (q[SLOT_U4].z & CF_ID_MASK) == FAT_ID;
          if (fat) {
            h[0] = q[SLOT_U4];
            h[1] = q[SLOT_U4 + 1];
          }
          return true;
        }
        empty = empty || q[0].z == NONE;
      }
      if (empty) return false;
    }
  }
  std::vector<uint32_t> run(const std::string& topic, uint64_t test_mask) {
    std::vector<uint8_t> pl, hs;
    bool hashed;
    tokenize((const uint8_t*)topic.data(), (uint32_t)topic.size(), test_mask, toks, pl, hs, hashed);
    n = (uint32_t)toks.size();
    out.clear();
    stk.clear();
    for (size_t i = 0; i < n; ++i)
      if (pl[i] || hs[i]) return out;  // wildcard topic name -> [] (emqx_trie.erl:157-166)
    if (ix.trie_empty) return out;
    dollar = !topic.empty() && topic[0] == '$';
    const uint4 rh[2] = {ix.rh0, ix.rh1};
    create(ix.root_cf, dollar ? NONE : ix.root_hf, NONE, ix.root_sig, ix.root_pcf, ix.root_phf, 0,
           !dollar, false, (ix.rh0.z & CF_ID_MASK) == FAT_ID, rh);
    while (!stk.empty()) {
      const auto it = stk.back();
      stk.pop_back();
      const uint32_t kind = it.first & IT_KIND;
      if (kind == IT_TN) {
        em(ix.tn_of[it.first & CF_ID_MASK]);
        continue;
      }
      const uint32_t node = it.first & CF_ID_MASK, k = it.second;
      const uint64_t key = kind == IT_PLUS ? PLUS_TOK : toks[k];
      uint4 s[2], hh[2];
      bool fat = false;
      const bool hit = probe(node, key, kind == IT_KEYED, s, fat, hh);
      if (getenv("HH_TRACE")) fprintf(stderr, "probe node %u k %u plus %d -> %d fat %d\n", node, k, (it.first & IT_PLUS) ? 1 : 0, hit ? 1 : 0, fat ? 1 : 0);
      if (hit)
        create(s[0].w, s[1].x, s[1].y, s[0].z >> SIG_SHIFT, s[1].z, s[1].w, k + 1, true,
               kind != IT_PLUS, fat, hh);
    }
    return out;
  }
};

// k_exact's lookup over the committed exact table
uint32_t cpu_exact(const DevIndex& ix, const std::string& t, bool wild) {
  if (wild ? ix.wild_empty : ix.plain_empty) return NONE;
  const uint32_t len = (uint32_t)t.size();
  const uint64_t fh = key_hash((const uint8_t*)t.data(), len, ix.full_mask);
  const uint64_t base = wild ? ix.xwbase : 0, mask = wild ? ix.xwmask : ix.xmask;
  uint64_t b = base + exact_slot(fh, mask);
  for (;;) {
    for (uint32_t j = 0; j < XBUCKET; ++j) {
      const uint4* e = ix.exact + XENT_U4 * (XBUCKET * b + j);
      if (e[0].y == NONE) return NONE;
      if (e[0].y == TOMB || e[0].x != (uint32_t)(fh >> 32) || e[0].z != len) continue;
      uint32_t w[5] = {0, 0, 0, 0, 0};
      memcpy(w, t.data(), std::min<uint32_t>(len, XINL));
      const uint32_t inl[5] = {e[0].w, e[1].x, e[1].y, e[1].z, e[1].w};
      if (memcmp(w, inl, sizeof w) != 0) continue;
      const uint8_t* fp = ix.fbytes + ix.foff[e[0].y];
      if (len > XINL && memcmp(fp + XINL, t.data() + XINL, len - XINL) != 0) continue;
      return e[0].y;
    }
    if (!((ix.xovf[b >> 5] >> (b & 31)) & 1u)) return NONE;
    b = base + ((b - base + 1) & mask);
  }
}

struct Oracle {
  void* r = ref_create(1);
  std::vector<std::string> names;  // oracle id -> bytes
  std::set<std::string> known;
  ~Oracle() { ref_destroy(r); }
  void add(const std::string& s, uint8_t kind) {
    if (known.insert(s).second) names.push_back(s);
    const uint64_t off[2] = {0, s.size()};
    ref_add_many(r, (const uint8_t*)s.data(), off, 1, &kind);
  }
};

bool is_wild_s(const std::string& s) { return is_wild((const uint8_t*)s.data(), (uint32_t)s.size()); }

}  // namespace

int main(int argc, char** argv) {
  const uint64_t seed = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1;
  const int rounds = argc > 2 ? atoi(argv[2]) : 30;
  const uint32_t hash_bits = argc > 3 ? (uint32_t)atoi(argv[3]) : 0;
  const int keyed_mode = argc > 5 ? atoi(argv[5]) : 1;  // emqxgm_tune "keyed" (2: every eligible node)
  std::mt19937_64 rng(seed);
  auto rnd = [&](uint64_t k) { return (uint64_t)(rng() % k); };

  const char* vocab[] = {"a", "b", "", "$x", "c", "dd", "sensor", "long-level-name", "device-0001"};
  auto word = [&]() { return std::string(vocab[rnd(9)]); };
  std::vector<std::string> filters, topics;
  std::set<std::string> seen;
  while (filters.size() < 1500) {
    const uint32_t d = 1 + (uint32_t)rnd(6);
    std::string f;
    for (uint32_t i = 0; i < d; ++i) {
      if (i) f += '/';
      const uint64_t r = rnd(100);
      f += (i + 1 == d && r < 15) ? "#" : (r < 40 ? "+" : word());
    }
    if (seen.insert(f).second) filters.push_back(f);
  }
  for (int i = 0; i < 600; ++i) {
    const uint32_t d = 1 + (uint32_t)rnd(7);
    std::string t;
    for (uint32_t k = 0; k < d; ++k) t += (k ? "/" : "") + word();
    topics.push_back(t);
  }
  for (int i = 0; i < 60; ++i) topics.push_back(filters[rnd(filters.size())]);  // exact / wild names
  topics.push_back(std::string(30, 'z'));

  emqxgm_cfg cfg{};
  cfg.word_hash_bits = hash_bits;
  emqxgm_t *hd = nullptr, *hf = nullptr;
  CHECK(emqxgm_create(&cfg, &hd) == 0, "create");
  CHECK(emqxgm_create(&cfg, &hf) == 0, "create");
  CHECK(emqxgm_tune(hf, "delta_commit", 0) == 0, "tune");
  CHECK(emqxgm_tune(hd, "keyed", keyed_mode) == 0 && emqxgm_tune(hf, "keyed", keyed_mode) == 0, "tune");
  CHECK(emqxgm_set_local_node(hd, 1) == 0 && emqxgm_set_local_node(hf, 1) == 0, "node");
  Oracle orc;
  std::set<std::string> in_trie, keyed;
  std::map<std::string, std::vector<std::pair<uint32_t, uint32_t>>> dests;
  uint64_t checks = 0, fat_seen = 0;
  const std::string snap = std::string(argc > 4 ? argv[4] : "/tmp") + "/emqxgm_harness_" +
                           std::to_string(seed) + ".snap";
  for (int round = 0; round < rounds; ++round) {
    if (round == rounds / 2) {
      // snapshot round trip: the restored engine must answer the same and keep delta-committing
      CHECK(emqxgm_snapshot_save(hd, snap.c_str()) == 0, "save: %s", hd->err.c_str());
      emqxgm_destroy(hd);
      hd = nullptr;
      CHECK(emqxgm_create(&cfg, &hd) == 0, "create");
      CHECK(emqxgm_tune(hd, "keyed", keyed_mode) == 0, "tune");
      CHECK(emqxgm_snapshot_load(hd, snap.c_str()) == 0, "load: %s", hd->err.c_str());
      emqxgm_t* other = nullptr;
      CHECK(emqxgm_create(&cfg, &other) == 0, "create");
      CHECK(emqxgm_trie_insert(other, (const uint8_t*)"a", 1, nullptr) == 0, "ins");
      CHECK(emqxgm_snapshot_load(other, snap.c_str()) == -EBUSY, "load into a used handle");
      emqxgm_destroy(other);
      // corrupt copies (flipped bytes, random words, truncations): every load returns an error
      // code or succeeds, never writes out of bounds (ASan), and a failed load leaves the handle
      // fresh: the intact snapshot loads into it afterwards
      {
        FILE* f = fopen(snap.c_str(), "rb");
        CHECK(f != nullptr, "open snap");
        std::string img;
        char buf[1 << 16];
        size_t k;
        while ((k = fread(buf, 1, sizeof buf, f)) > 0) img.append(buf, k);
        fclose(f);
        const std::string bad = snap + ".bad";
        int rejected = 0;
        for (int trial = 0; trial < 48; ++trial) {
          std::string c = img;
          const int kind = trial % 3;
          if (kind == 0) {
            for (int q = 0; q < 4; ++q) c[rnd(c.size())] ^= (char)(1 + rnd(255));
          } else if (kind == 1) {
            const size_t at = rnd(c.size() - 8);
            const uint64_t v = rng() >> rnd(60);
            memcpy(&c[at], &v, 8);
          } else {
            c.resize(rnd(c.size()));
          }
          FILE* g = fopen(bad.c_str(), "wb");
          CHECK(g && fwrite(c.data(), 1, c.size(), g) == c.size(), "write bad snap");
          fclose(g);
          emqxgm_t* t = nullptr;
          CHECK(emqxgm_create(&cfg, &t) == 0, "create");
          const int rc = emqxgm_snapshot_load(t, bad.c_str());
          CHECK(rc == 0 || rc < 0, "load rc");
          if (rc < 0) {
            ++rejected;
            CHECK(emqxgm_snapshot_load(t, snap.c_str()) == 0, "reload after a failed load: %s",
                  t->err.c_str());
          }
          emqxgm_destroy(t);
        }
        CHECK(rejected > 0, "no corrupt snapshot was rejected");
        remove(bad.c_str());
      }
      remove(snap.c_str());
    }
    const int mode = (int)rnd(10);
    CHECK(emqxgm_tune(hd, "delta_commit", mode == 0 ? 0 : mode == 1 ? 2 : 1) == 0, "tune");
    const int ops = (int)(round == 0 ? 3000 : 1 + rnd(120));  // > 1024 filters registered
    for (int k = 0; k < ops; ++k) {
      // filters [0, 1000) take trie / route-key churn, [1000, ...) route + subscriber churn
      const uint64_t op = rnd(6);
      const std::string& f = op < 5 ? filters[rnd(1000)] : filters[1000 + rnd(filters.size() - 1000)];
      const uint8_t* p = (const uint8_t*)f.data();
      const uint32_t len = (uint32_t)f.size();
      switch (op) {
        case 0:
        case 1:  // emqx_trie:insert/1 (any filter: exact ones become tn keys)
          for (emqxgm_t* h : {hd, hf}) CHECK(emqxgm_trie_insert(h, p, len, nullptr) == 0, "ins");
          orc.add(f, 1);
          in_trie.insert(f);
          break;
        case 2:  // emqx_trie:delete/1 (absent: no-op)
          for (emqxgm_t* h : {hd, hf}) CHECK(emqxgm_trie_delete(h, p, len) == 0, "del");
          ref_trie_delete(orc.r, p, len);
          in_trie.erase(f);
          break;
        case 3:  // a route key appears (one ref: the oracle's key set has no counts)
          if (keyed.insert(f).second) {
            for (emqxgm_t* h : {hd, hf}) CHECK(emqxgm_route_ref(h, p, len, nullptr) == 0, "ref");
            orc.add(f, 2);
          }
          break;
        case 4:
          if (keyed.erase(f)) {
            for (emqxgm_t* h : {hd, hf}) CHECK(emqxgm_route_unref(h, p, len) == 0, "unref");
            ref_route_delete(orc.r, p, len);
          }
          break;
        default: {  // routes (emqx_router do_add_route / do_delete_route) and subscribers
          const uint32_t node = 1 + (uint32_t)rnd(3), sub = (uint32_t)rnd(5);
          const uint32_t grp = rnd(3) == 0 ? (uint32_t)rnd(4) : NONE;
          const uint64_t what = rnd(4);
          auto& ds = dests[f];
          const auto d = std::make_pair(node, grp);
          if (what == 0) {
            const bool first = ds.empty(), had = std::count(ds.begin(), ds.end(), d) > 0;
            for (emqxgm_t* h : {hd, hf}) CHECK(emqxgm_route_add(h, p, len, node, grp) == 0, "radd");
            if (!had) ds.push_back(d);
            if (first) orc.add(f, (uint8_t)(2 | (is_wild_s(f) ? 1 : 0)));
          } else if (what == 1) {
            const auto it = std::find(ds.begin(), ds.end(), d);
            for (emqxgm_t* h : {hd, hf}) CHECK(emqxgm_route_delete(h, p, len, node, grp) == 0, "rdel");
            if (it != ds.end()) {
              ds.erase(it);
              if (ds.empty()) {  // the last route: key and trie entry go (emqx_router_utils:57-71)
                ref_route_delete(orc.r, p, len);
                if (is_wild_s(f)) ref_trie_delete(orc.r, p, len);
              }
            }
          } else {
            for (emqxgm_t* h : {hd, hf}) {
              if (what == 2) {
                CHECK(emqxgm_subscriber_add(h, p, len, sub) == 0, "sub");
              } else {
                CHECK(emqxgm_subscriber_delete(h, p, len, sub) == 0, "unsub");
              }
            }
          }
          break;
        }
      }
    }
    for (emqxgm_t* h : {hd, hf}) CHECK(emqxgm_commit(h, nullptr) == 0, "commit: %s", h->err.c_str());
    // the oracle's answers
    std::string tb;
    std::vector<uint32_t> toff(1, 0);
    for (const auto& t : topics) {
      tb += t;
      toff.push_back((uint32_t)tb.size());
    }
    std::vector<uint64_t> row(topics.size() + 1);
    std::vector<uint32_t> rex(topics.size());
    uint32_t* ids = nullptr;
    uint64_t nids = 0;
    ref_match_batch(orc.r, (const uint8_t*)tb.data(), toff.data(), topics.size(), 1, row.data(),
                    &ids, &nids, rex.data());
    for (emqxgm_t* h : {hd, hf}) {
      const DevIndex& ix = h->cur->ix;
      for (uint32_t c : h->tm.fchild) fat_seen += c != 0;
      for (size_t i = 0; i < topics.size(); ++i) {
        const std::string& t = topics[i];
        CpuWalk w(ix);
        std::vector<uint32_t> got = w.run(t, h->test_mask);
        std::vector<std::string> gs, ws;
        for (uint32_t f : got) {
          const bool verify = (ix.fvbits[f >> 5] >> (f & 31)) & 1u;
          const std::string fs = filter_str(h, f);
          if (!verify || mqtt_match(t, fs)) gs.push_back(fs);
        }
        for (uint64_t j = row[i]; j < row[i + 1]; ++j) ws.push_back(orc.names[ids[j]]);
        std::sort(gs.begin(), gs.end());
        std::sort(ws.begin(), ws.end());
        if (gs != ws && getenv("HH_DEBUG")) {
          setenv("HH_TRACE", "1", 1);
          CpuWalk w2(ix);
          w2.run(t, h->test_mask);
          unsetenv("HH_TRACE");
          for (auto& x : gs) fprintf(stderr, "got  %s\n", x.c_str());
          for (auto& x : ws) fprintf(stderr, "want %s\n", x.c_str());
          for (auto& x : ws) {
            if (std::count(gs.begin(), gs.end(), x)) continue;
            std::vector<uint64_t> tk;
            std::vector<uint8_t> pl, hs;
            bool hashed;
            tokenize((const uint8_t*)x.data(), (uint32_t)x.size(), h->test_mask, tk, pl, hs, hashed);
            uint32_t cur = 0;
            TrieModel& m = h->tm;
            fprintf(stderr, "root fchild %u rh0.z %08x\n", m.fchild[0], ix.rh0.z);
            for (size_t w = 0; w + (hs.back() ? 1 : 0) < tk.size(); ++w) {
              const uint32_t* v = m.emap.find(cur, pl[w] ? PLUS_TOK : tk[w]);
              if (!v) { fprintf(stderr, "  no edge at %zu\n", w); break; }
              cur = *v;
              const uint64_t sl = m.slot[cur];
              fprintf(stderr, "  w%zu node %u slot %lld half %u fchild %u nlit %u pchild %u cf %08x", w, cur,
                      (long long)sl, m.half[cur], m.fchild[cur], m.nlit[cur], m.pchild[cur], m.cf(cur));
              if (sl < m.ecap) {
                const uint4* q = ix.edges + SLOT_U4 * sl;
                fprintf(stderr, " dev{%08x %08x %08x %08x}{%08x %08x %08x %08x} next{%08x %08x %08x %08x}", q[0].x, q[0].y, q[0].z, q[0].w,
                        q[1].x, q[1].y, q[1].z, q[1].w, q[2].x, q[2].y, q[2].z, q[2].w);
              }
              fprintf(stderr, "\n");
            }
          }
        }
        CHECK(gs == ws, "round %d (%s) topic '%s': %zu vs %zu filters", round,
              h == hd ? "delta" : "full", t.c_str(), gs.size(), ws.size());
        const uint32_t ex = cpu_exact(ix, t, is_wild_s(t));
        const std::string exs = ex == NONE ? "<none>" : filter_str(h, ex);
        const std::string wex = rex[i] == NONE ? "<none>" : orc.names[rex[i]];
        CHECK(exs == wex, "round %d exact '%s': %s vs %s", round, t.c_str(), exs.c_str(), wex.c_str());
        ++checks;
      }
      // fan-out entries on the device equal the registry's lists
      if (ix.fan) {
        std::vector<uint32_t> rt, dl, groups;
        for (uint32_t id = 0; id < h->filters.size(); ++id) {
          rt.clear();
          dl.clear();
          fan_lists(h, id, rt, dl, groups);
          const uint4 e = ix.fan[id];
          CHECK(e.y == rt.size() && e.w == dl.size(), "fan sizes of %u", id);
          CHECK(std::equal(rt.begin(), rt.end(), ix.rt_dst + e.x), "fan routes of %u", id);
          CHECK(std::equal(dl.begin(), dl.end(), ix.dl_sub + e.z), "fan subs of %u", id);
        }
      }
    }
    ref_free(ids);
  }
  // emqxgm_match_batch_submit rejects malformed offsets on the host, before anything is enqueued
  {
    const uint8_t tb[8] = {'a', '/', 'b', 'c', 'd', 'e', 'f', 'g'};
    uint64_t tk = 0;
    const uint32_t dec[4] = {0, 5, 3, 8};
    CHECK(emqxgm_match_batch_submit(hd, tb, dec, 3, &tk) == -EINVAL, "decreasing offsets");
    const uint32_t nz[3] = {1, 3, 8};
    CHECK(emqxgm_match_batch_submit(hd, tb, nz, 2, &tk) == -EINVAL, "offsets[0] != 0");
  }
  emqxgm_stats sd{}, sf{};
  emqxgm_get_stats(hd, &sd);
  emqxgm_get_stats(hf, &sf);
  CHECK(sf.delta_commits == 0, "the rebuilding engine never patches");
  CHECK(fat_seen > 0, "no fat bucket was ever built");
  printf("OK %d %llu %llu %llu\n", rounds, (unsigned long long)sd.delta_commits,
         (unsigned long long)sd.full_commits, (unsigned long long)checks);
  emqxgm_destroy(hd);
  emqxgm_destroy(hf);
  return 0;
}
