// harness_walk.h -- TEST INFRASTRUCTURE shared by the host harnesses (harness.cpp, bg_harness.cpp):
// the engine's host code itself (gm_engine.cpp, included), the walk of gm_walk.inc and the probe
// of k_exact restated on the CPU over the committed tables, emqx_topic:match/2 on strings, and
// the oracle's C++ restatement (oracle/ref_trie.cpp) as the checker.
#pragma once
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
  // the registry lock, as the engine's readers take it (a commit may move the arrays: r06
  // reserves room for the deltas ahead)
  std::shared_lock<std::shared_mutex> g(h->pmu);
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
