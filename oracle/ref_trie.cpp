// ref_trie.cpp -- TEST INFRASTRUCTURE ONLY: C++ restatement of the reference's trie/router
// match path, used (a) as the large-case parity checker for the GPU engine and (b) as the CPU
// baseline timed by bench.py (cpu_baseline.kind = "port").  Never linked into the product.
//
// It follows the reference function by function (paths relative to the reference checkout):
//   emqx_topic:words/1            apps/emqx/src/emqx_topic.erl:155-169
//   emqx_topic:wildcard/1         apps/emqx/src/emqx_topic.erl:54-64
//   emqx_topic:join/1             apps/emqx/src/emqx_topic.erl:188-204
//   emqx_topic:match/2            apps/emqx/src/emqx_topic.erl:67-89   (brute-force checker)
//   emqx_trie key model           apps/emqx/src/emqx_trie.erl:54-60 -- an ordered set of
//                                 {Binary, 0|1} keys with refcounts, here two std::map
//   insert/delete                 apps/emqx/src/emqx_trie.erl:121-144, 242-260
//   make_keys/do_compact/prefixes apps/emqx/src/emqx_trie.erl:195-240
//   match/do_match                apps/emqx/src/emqx_trie.erl:155-169, 282-297
//   match_no_compact              apps/emqx/src/emqx_trie.erl:299-325
//   match_compact / 'match_#'     apps/emqx/src/emqx_trie.erl:327-348
//   lookup_topic / has_prefix     apps/emqx/src/emqx_trie.erl:264-280
//   emqx_router:match_routes/1    apps/emqx/src/emqx_router.erl:141-157 (exact key lookup)
//
// Like the reference, every probe joins a freshly allocated prefix binary and does an
// O(log N) ordered-set lookup; it is deliberately NOT optimised (it is the baseline).
// Parity pin: tests/test_oracle_cpp.py checks it against tests/golden/reference_vectors.json
// and against the Python restatement oracle/emqx_ref.py.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

enum WordKind { W_BIN = 0, W_EMPTY = 1, W_PLUS = 2, W_HASH = 3 };
struct Word {
  WordKind k;
  std::string b;
};
using Words = std::vector<Word>;

Words words(const char* p, size_t n) {  // emqx_topic:words/1
  Words out;
  size_t s = 0;
  for (size_t i = 0; i <= n; ++i) {
    if (i == n || p[i] == '/') {
      Word w;
      const size_t l = i - s;
      if (l == 0)
        w.k = W_EMPTY;
      else if (l == 1 && p[s] == '+')
        w.k = W_PLUS;
      else if (l == 1 && p[s] == '#')
        w.k = W_HASH;
      else {
        w.k = W_BIN;
        w.b.assign(p + s, l);
      }
      out.push_back(std::move(w));
      s = i + 1;
    }
  }
  return out;
}

bool wildcard(const Words& ws) {  // emqx_topic:wildcard/1
  for (auto& w : ws)
    if (w.k == W_PLUS || w.k == W_HASH) return true;
  return false;
}

std::string bin(const Word& w) {  // emqx_topic.erl:145-149
  switch (w.k) {
    case W_EMPTY: return std::string();
    case W_PLUS: return "+";
    case W_HASH: return "#";
    default: return w.b;
  }
}

// A trie prefix: the atom 'empty' (root) or a binary.
struct Prefix {
  bool root;
  std::string s;
};

std::string tjoin(const Prefix& p, const Word& w) {  // emqx_trie.erl:223-227
  if (p.root) return bin(w);
  return p.s + "/" + bin(w);  // emqx_topic:join([Prefix, Word])
}

// emqx_topic:match/2 on words (for the brute-force checker)
bool match_words(const Words& n, const Words& f) {
  size_t i = 0;
  for (;;) {
    if (i == n.size() && i == f.size()) return true;
    if (i < n.size() && i < f.size() && n[i].k == f[i].k && (n[i].k != W_BIN || n[i].b == f[i].b)) {
      ++i;
      continue;
    }
    if (i < n.size() && i < f.size() && f[i].k == W_PLUS) {
      ++i;
      continue;
    }
    if (f.size() - i == 1 && f[i].k == W_HASH) return true;
    return false;
  }
}

bool match_bin(const std::string& name, const std::string& filt) {  // emqx_topic.erl:67-75
  if (!name.empty() && name[0] == '$' && !filt.empty() && (filt[0] == '+' || filt[0] == '#'))
    return false;
  return match_words(words(name.data(), name.size()), words(filt.data(), filt.size()));
}

struct TopicEntry {
  uint32_t count;
  uint32_t id;
};

struct Ref {
  bool compact = true;
  std::map<std::string, TopicEntry> topics;  // {Topic, 1} keys
  std::map<std::string, uint32_t> prefixes;  // {Prefix, 0} keys
  std::unordered_map<std::string, uint32_t> route_keys;  // emqx_route bag keys -> id
  std::vector<std::string> id_str;
  std::unordered_map<std::string, uint32_t> ids;

  uint32_t id_of(const std::string& s) {
    auto it = ids.find(s);
    if (it != ids.end()) return it->second;
    const uint32_t id = (uint32_t)id_str.size();
    id_str.push_back(s);
    ids.emplace(s, id);
    return id;
  }

  std::vector<std::string> make_prefixes(const Words& ws) const {  // emqx_trie.erl:229-240
    std::vector<std::string> segs;
    if (compact) {  // do_compact 211-221
      Prefix seg{true, ""};
      bool have = false;
      for (auto& w : ws) {
        if (w.k == W_PLUS || w.k == W_HASH) {
          segs.push_back(tjoin(seg, w));
          seg = Prefix{true, ""};
          have = false;
        } else {
          seg = Prefix{false, tjoin(seg, w)};
          have = true;
        }
      }
      if (have) segs.push_back(seg.s);
    } else {
      for (auto& w : ws) segs.push_back(bin(w));
    }
    std::vector<std::string> out;  // longest first, like the reference
    for (size_t i = segs.size(); i-- > 1;) {
      std::string j;
      for (size_t k = 0; k < i; ++k) {
        if (k) j += '/';
        j += segs[k];
      }
      out.push_back(j);
    }
    return out;
  }

  void insert(const std::string& t) {  // emqx_trie.erl:121-127
    if (topics.count(t)) return;
    const Words ws = words(t.data(), t.size());
    topics[t] = TopicEntry{1, id_of(t)};
    for (auto& p : make_prefixes(ws)) prefixes[p] += 1;
  }

  void erase(const std::string& t) {  // emqx_trie.erl:139-144, 252-260
    auto it = topics.find(t);
    if (it == topics.end()) return;
    topics.erase(it);
    const Words ws = words(t.data(), t.size());
    for (auto& p : make_prefixes(ws)) {
      auto pi = prefixes.find(p);
      if (pi == prefixes.end()) continue;
      if (pi->second > 1)
        pi->second -= 1;
      else
        prefixes.erase(pi);
    }
  }

  void lookup_topic(const std::string& t, bool is_wild, std::vector<uint32_t>& acc) const {
    if (!is_wild) return;  // emqx_trie.erl:264
    auto it = topics.find(t);
    if (it != topics.end() && it->second.count > 0) acc.push_back(it->second.id);
  }

  bool has_prefix(const Prefix& p) const {  // emqx_trie.erl:274-280
    if (p.root) return true;
    auto it = prefixes.find(p.s);
    return it != prefixes.end() && it->second > 0;
  }

  void match_hash(const Prefix& p, std::vector<uint32_t>& acc) const {  // 'match_#' 346-348
    Word h{W_HASH, ""};
    lookup_topic(tjoin(p, h), true, acc);
  }

  void match_compact(const Words& ws, size_t i, const Prefix& p, bool is_wild,
                     std::vector<uint32_t>& acc) const {  // emqx_trie.erl:327-344
    if (i == ws.size()) {
      match_hash(p, acc);
      if (!p.root) lookup_topic(p.s, is_wild, acc);
      return;
    }
    match_hash(p, acc);
    match_compact(ws, i + 1, Prefix{false, tjoin(p, ws[i])}, is_wild, acc);
    Word plus{W_PLUS, ""};
    const Prefix wp{false, tjoin(p, plus)};
    if (i + 1 == ws.size() || has_prefix(wp)) match_compact(ws, i + 1, wp, true, acc);
  }

  void match_no_compact(const Words& ws, size_t i, const Prefix& p, bool is_wild,
                        std::vector<uint32_t>& acc) const {  // emqx_trie.erl:299-325
    if (i == ws.size()) {
      match_hash(p, acc);
      if (!p.root) lookup_topic(p.s, is_wild, acc);
      return;
    }
    if (!has_prefix(p)) return;
    match_hash(p, acc);
    Word plus{W_PLUS, ""};
    match_no_compact(ws, i + 1, Prefix{false, tjoin(p, plus)}, true, acc);
    match_no_compact(ws, i + 1, Prefix{false, tjoin(p, ws[i])}, is_wild, acc);
  }

  void match(const char* t, size_t n, std::vector<uint32_t>& acc) const {  // :155-169, 282-297
    const Words ws = words(t, n);
    if (wildcard(ws)) return;
    if (ws[0].k == W_BIN && ws[0].b[0] == '$') {
      if (ws.size() == 1) lookup_topic(ws[0].b, true, acc);
      Words rest(ws.begin() + 1, ws.end());
      const Prefix p{false, ws[0].b};
      if (compact)
        match_compact(rest, 0, p, false, acc);
      else
        match_no_compact(rest, 0, p, false, acc);
      return;
    }
    if (compact)
      match_compact(ws, 0, Prefix{true, ""}, false, acc);
    else
      match_no_compact(ws, 0, Prefix{true, ""}, false, acc);
  }

  uint32_t exact(const char* t, size_t n) const {  // emqx_router:lookup_routes/1 key lookup
    auto it = route_keys.find(std::string(t, n));
    return it == route_keys.end() ? 0xFFFFFFFFu : it->second;
  }
};

}  // namespace

extern "C" {

void* ref_create(int compact) {
  Ref* r = new Ref();
  r->compact = compact != 0;
  return r;
}

void ref_destroy(void* h) { delete (Ref*)h; }

// Register filters in order (ids = first-registration order), then add them to the trie
// (kind bit 1) and/or the route-key set (kind bit 2).
int ref_add_many(void* h, const uint8_t* bytes, const uint64_t* off, uint64_t n,
                 const uint8_t* kind) {
  Ref* r = (Ref*)h;
  for (uint64_t i = 0; i < n; ++i) {
    const std::string s((const char*)bytes + off[i], off[i + 1] - off[i]);
    const uint32_t id = r->id_of(s);
    if (kind[i] & 1) r->insert(s);
    if (kind[i] & 2) r->route_keys.emplace(s, id);
  }
  return 0;
}

int ref_trie_delete(void* h, const uint8_t* p, uint32_t len) {
  ((Ref*)h)->erase(std::string((const char*)p, len));
  return 0;
}

int ref_route_delete(void* h, const uint8_t* p, uint32_t len) {
  ((Ref*)h)->route_keys.erase(std::string((const char*)p, len));
  return 0;
}

int ref_trie_empty(void* h) { return ((Ref*)h)->topics.empty() ? 1 : 0; }

uint64_t ref_n_ids(void* h) { return ((Ref*)h)->id_str.size(); }

// Batch match with `threads` worker threads, each owning a contiguous slice of topics.
// Results: row[n+1] (u64), ids (caller frees with ref_free), exact[n].  Rows are sorted.
int ref_match_batch(void* h, const uint8_t* tb, const uint32_t* toff, uint64_t n, int threads,
                    uint64_t* row, uint32_t** ids_out, uint64_t* n_ids, uint32_t* exact) {
  Ref* r = (Ref*)h;
  if (threads < 1) threads = 1;
  std::vector<std::vector<uint32_t>> part(threads);
  std::vector<std::vector<uint64_t>> cnt(threads);
  std::vector<std::thread> th;
  const uint64_t per = (n + threads - 1) / threads;
  for (int w = 0; w < threads; ++w) {
    th.emplace_back([&, w]() {
      const uint64_t a = std::min<uint64_t>(n, w * per), b = std::min<uint64_t>(n, a + per);
      std::vector<uint32_t> acc;
      for (uint64_t t = a; t < b; ++t) {
        acc.clear();
        const char* p = (const char*)tb + toff[t];
        const size_t len = toff[t + 1] - toff[t];
        if (!r->topics.empty()) r->match(p, len, acc);  // emqx_router:match_trie 149-153
        std::sort(acc.begin(), acc.end());
        part[w].insert(part[w].end(), acc.begin(), acc.end());
        cnt[w].push_back(acc.size());
        if (exact) exact[t] = r->exact(p, len);
      }
    });
  }
  for (auto& x : th) x.join();
  uint64_t total = 0, t = 0;
  row[0] = 0;
  for (int w = 0; w < threads; ++w)
    for (uint64_t c : cnt[w]) {
      total += c;
      row[++t] = total;
    }
  uint32_t* ids = (uint32_t*)malloc(std::max<uint64_t>(total, 1) * 4);
  uint64_t pos = 0;
  for (int w = 0; w < threads; ++w) {
    memcpy(ids + pos, part[w].data(), part[w].size() * 4);
    pos += part[w].size();
  }
  *ids_out = ids;
  *n_ids = total;
  return 0;
}

// Time-only variant for the CPU baseline: matches topics [0,n) `reps` times, returns the
// number of (topic, filter) pairs found (so the work cannot be elided).
uint64_t ref_match_count(void* h, const uint8_t* tb, const uint32_t* toff, uint64_t n, int threads) {
  Ref* r = (Ref*)h;
  if (threads < 1) threads = 1;
  std::vector<uint64_t> found(threads, 0);
  std::vector<std::thread> th;
  const uint64_t per = (n + threads - 1) / threads;
  for (int w = 0; w < threads; ++w) {
    th.emplace_back([&, w]() {
      const uint64_t a = std::min<uint64_t>(n, w * per), b = std::min<uint64_t>(n, a + per);
      std::vector<uint32_t> acc;
      for (uint64_t t = a; t < b; ++t) {
        acc.clear();
        const char* p = (const char*)tb + toff[t];
        const size_t len = toff[t + 1] - toff[t];
        if (!r->topics.empty()) r->match(p, len, acc);
        found[w] += acc.size() + (r->exact(p, len) != 0xFFFFFFFFu);
      }
    });
  }
  for (auto& x : th) x.join();
  uint64_t s = 0;
  for (auto v : found) s += v;
  return s;
}

void ref_free(void* p) { free(p); }

// Brute-force emqx_topic:match/2 over every trie filter (small cases only).
int ref_bruteforce(void* h, const uint8_t* tb, const uint32_t* toff, uint64_t n, uint64_t* row,
                   uint32_t** ids_out, uint64_t* n_ids) {
  Ref* r = (Ref*)h;
  std::vector<uint32_t> all;
  row[0] = 0;
  for (uint64_t t = 0; t < n; ++t) {
    const std::string name((const char*)tb + toff[t], toff[t + 1] - toff[t]);
    const Words nw = words(name.data(), name.size());
    std::vector<uint32_t> acc;
    if (!wildcard(nw)) {
      for (auto& kv : r->topics) {
        const Words fw = words(kv.first.data(), kv.first.size());
        if (wildcard(fw) && match_bin(name, kv.first)) acc.push_back(kv.second.id);
      }
      if (nw.size() == 1 && nw[0].k == W_BIN && nw[0].b[0] == '$') {  // emqx_trie.erl:286-287
        auto it = r->topics.find(name);
        if (it != r->topics.end() && !wildcard(words(name.data(), name.size())))
          acc.push_back(it->second.id);
      }
    }
    std::sort(acc.begin(), acc.end());
    all.insert(all.end(), acc.begin(), acc.end());
    row[t + 1] = all.size();
  }
  uint32_t* ids = (uint32_t*)malloc(std::max<size_t>(all.size(), 1) * 4);
  memcpy(ids, all.data(), all.size() * 4);
  *ids_out = ids;
  *n_ids = all.size();
  return 0;
}

// S(t) of SURVEY 8d: sum over k = 0..n(t) of the number of distinct length-k word prefixes of
// trie wildcard filters that match t's first k levels ('+' matches any level; no root '+' for
// '$' topics).  '#' words are not part of any prefix.  Returns per-topic counts in `states`.
int ref_states(void* h, const uint8_t* tb, const uint32_t* toff, uint64_t n, uint32_t* states,
               int threads) {
  Ref* r = (Ref*)h;
  std::unordered_set<std::string> pre;  // every word prefix ("" = root) of trie filters
  for (auto& kv : r->topics) {
    const Words fw = words(kv.first.data(), kv.first.size());
    std::string acc;
    for (size_t k = 0; k < fw.size(); ++k) {
      if (fw[k].k == W_HASH) break;
      acc += (k ? "/" : "") + bin(fw[k]);
      pre.insert(std::to_string(k + 1) + ":" + acc);
    }
  }
  if (threads < 1) threads = 1;
  std::vector<std::thread> th;
  const uint64_t per = (n + threads - 1) / threads;
  for (int w = 0; w < threads; ++w) {
    th.emplace_back([&, w]() {
      const uint64_t a = std::min<uint64_t>(n, w * per), b = std::min<uint64_t>(n, a + per);
      for (uint64_t t = a; t < b; ++t) {
        const Words ws = words((const char*)tb + toff[t], toff[t + 1] - toff[t]);
        if (wildcard(ws)) {
          states[t] = 0;
          continue;
        }
        const bool dollar = ws[0].k == W_BIN && ws[0].b[0] == '$';
        std::vector<std::string> fr{""}, nx;
        uint32_t s = r->topics.empty() ? 0 : 1;
        for (size_t k = 0; k < ws.size() && !fr.empty() && !r->topics.empty(); ++k) {
          nx.clear();
          for (auto& p : fr) {
            const std::string lit = p + (k ? "/" : "") + bin(ws[k]);
            if (pre.count(std::to_string(k + 1) + ":" + lit)) nx.push_back(lit);
            if (!(k == 0 && dollar)) {
              const std::string pl = p + (k ? "/" : "") + "+";
              if (pre.count(std::to_string(k + 1) + ":" + pl)) nx.push_back(pl);
            }
          }
          s += (uint32_t)nx.size();
          fr.swap(nx);
        }
        states[t] = s;
      }
    });
  }
  for (auto& x : th) x.join();
  return 0;
}

}  // extern "C"
