// gm_retain.cpp -- host side of the retained-topic store (reverse match, gm_retain.inc): the
// registry of retained topics, the store builder run at commit, the batch driver and the
// emqxgm_retain_* C-ABI of include/emqx_gpumatch.h.
//
// Reference: apps/emqx_retainer/src/emqx_retainer_mnesia.erl (store_retained/2 :138-152,
// delete_message/2 :166-180, read_message/2 :182-183 + read_messages/1 :372-382,
// match_messages/3 :185-195 -> search_table/3 :300-330, clean/1, size/1) and the match-spec
// patterns of emqx_retainer_index:condition/1 (emqx_retainer_index.erl:97-112, the full scan)
// and condition/2 (:174-200, the index path of the configured index specs).
#include <errno.h>
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/emqx_gpumatch.h"
#include "gm_common.h"
#include "gm_kernels.h"

using namespace gm;

namespace {

struct Buf {
  void* p = nullptr;
  size_t bytes = 0;
};

struct Topic {
  uint64_t off;
  uint32_t len;
  uint64_t expiry;
  bool alive;
};

constexpr uint32_t RTERM_BIT = 0x80000000u;  // gm_retain.inc RTERM

}  // namespace

// One preorder topic store on the device (gm_retain.inc): the base or the delta.
struct Store {
  RetainDev d;
  std::vector<Buf> bufs;
  std::vector<uint32_t> order;  // topic id per sorted position
};

struct emqxgm_retain {
  std::mutex mu;
  int32_t device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  // registry (pending state)
  std::vector<uint8_t> pool;
  std::vector<Topic> topics;
  std::unordered_map<std::string, uint32_t> ids;
  std::vector<uint32_t> changed;  // ids stored or deleted since the last commit
  bool dirty = false;
  // committed state: base store + delta store of the topics stored since the base was built
  Store base, delta;
  bool built = false;
  std::vector<uint32_t> pos_of;         // per id: sorted position in the base, or NONE
  std::unordered_set<uint32_t> delta_ids;  // live ids not in the base
  std::vector<uint8_t> alive_committed;  // per id
  std::vector<uint64_t> exp_committed;   // per id
  uint64_t n_committed = 0;
  int64_t delta_max = -1;  // delta topics before a full rebuild (-1: max(4096, base / 16))
  // index specs (config_indices/0: sorted); empty = search_table's full scan only.  Default:
  // ?DEFAULT_INDICES of emqx_retainer_schema.erl:24-29
  std::vector<std::vector<uint32_t>> indices{{1, 2, 3}, {1, 3}, {2, 3}, {3}};
  std::vector<uint8_t> h_fb, h_tail;  // planned filters (gm_retain.inc: cut, open tail)
  std::vector<uint32_t> h_fo;
  uint64_t full_builds = 0, delta_builds = 0;
  // batch scratch and host outputs
  std::vector<Buf> sc;
  std::vector<uint64_t> h_ptr;
  std::vector<uint32_t> h_ptr32, h_id;
};

namespace {

enum { S_FB, S_FO, S_FRAMES, S_CNT, S_RBASE, S_RUNS, S_ACNT, S_ABASE, S_OUT, S_PTR, S_TMP, S_CTL,
       S_CNT2, S_PATCH, S_TAIL };

// emqx_retainer_index:index_score/2 (emqx_retainer_index.erl:141-152): index positions with a
// literal word, in order, up to the first index position holding '+' or '#'.
uint32_t index_score(const std::vector<uint32_t>& ix, const std::vector<std::pair<uint32_t, uint32_t>>& w,
                     const uint8_t* f) {
  uint32_t score = 0, i = 0;
  for (uint32_t n = 1; n <= w.size() && i < ix.size(); ++n) {
    if (ix[i] != n) continue;
    const uint32_t b = w[n - 1].first, l = w[n - 1].second;
    if (l == 1 && (f[b] == '+' || f[b] == '#')) return score;
    ++score;
    ++i;
  }
  return score;
}

// search_table/3 (emqx_retainer_mnesia.erl:300-330) for one filter, in the walk's terms
// (gm_retain.inc): select_index/2 (:83-91, 154-165: the first index with the best score > 0,
// none -> the full scan of condition/1, the filter as it is).  On the index path condition/2
// (:174-200) walks the words with the index positions left; matched against a stored topic's
// index key its pattern selects:
//  * at a '#' reached while index positions remain or right as they run out (:174-177): both
//    pattern parts open -- the words before it as a prefix with any tail, i.e. the filter cut
//    after that '#';
//  * once the positions are used up at a word that is not '#' (:178-179): the rest goes through
//    condition/1, together the full scan's pattern -- the filter as it is;
//  * when the filter ends while positions remain (:180-181): the index part open, the other
//    closed -- the topic has the filter's words (with '+') and may go on only through index
//    positions, i.e. up to `tail` more words, tail = the run of positions right after the
//    filter's last word.
// Checked against the restated index search by tests/test_oracle_golden.py (the predicate
// form, R.retained_match_indexed).  Writes the (possibly cut) filter to fb, returns its tail.
uint32_t plan_filter(const std::vector<std::vector<uint32_t>>& indices, const uint8_t* f,
                     uint32_t len, std::vector<uint8_t>& fb) {
  std::vector<std::pair<uint32_t, uint32_t>> w;
  for (uint32_t b = 0, q = 0; q <= len; ++q)
    if (q == len || f[q] == '/') {
      w.emplace_back(b, q - b);
      b = q + 1;
    }
  const std::vector<uint32_t>* sel = nullptr;
  uint32_t best = 0;
  for (const auto& ix : indices) {
    const uint32_t sc = index_score(ix, w, f);
    if (sc > best) {
      best = sc;
      sel = &ix;
    }
  }
  if (!sel) {
    fb.insert(fb.end(), f, f + len);
    return 0;
  }
  size_t i = 0;  // index positions used so far
  for (uint32_t n = 1; n <= w.size(); ++n) {
    if (w[n - 1].second == 1 && f[w[n - 1].first] == '#') {
      fb.insert(fb.end(), f, f + w[n - 1].first + 1);  // ".../#": the words before it + '#'
      return 0;
    }
    if (i == sel->size()) break;  // the full scan's pattern
    if ((*sel)[i] == n) ++i;
  }
  const uint32_t k = (uint32_t)w.size();
  uint32_t tail = 0;
  for (; i < sel->size(); ++i)
    if ((*sel)[i] == k + 1 + tail) ++tail;
  fb.insert(fb.end(), f, f + len);
  return tail;
}

int grow(emqxgm_retain* r, size_t slot, uint64_t bytes);

int rfail(emqxgm_retain* r, hipError_t e, const char* what) {
  r->err = std::string(what) + ": " + hipGetErrorString(e);
  return -EIO;
}

#define RCHK(r, expr)                                 \
  do {                                                \
    hipError_t _e = (expr);                           \
    if (_e != hipSuccess) return rfail(r, _e, #expr); \
  } while (0)

template <class T>
int upload(emqxgm_retain* r, std::vector<Buf>& keep, const std::vector<T>& v, const T** out) {
  Buf b;
  b.bytes = std::max<size_t>(16, v.size() * sizeof(T));
  RCHK(r, hipMalloc(&b.p, b.bytes));
  keep.push_back(b);
  if (!v.empty()) RCHK(r, hipMemcpy(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  *out = (const T*)b.p;
  return 0;
}

void free_all(std::vector<Buf>& v) {
  for (auto& b : v)
    if (b.p) (void)hipFree(b.p);
  v.clear();
}

uint64_t pow2_ge(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

// Word boundaries of a topic: word k is [s[k], s[k+1] - 1).
void word_starts(const uint8_t* p, uint32_t len, std::vector<uint32_t>& s) {
  s.clear();
  s.push_back(0);
  for (uint32_t i = 0; i < len; ++i)
    if (p[i] == '/') s.push_back(i + 1);
  s.push_back(len + 1);
}

// Word-sequence order (a topic before the topics it prefixes): the preorder of the topic trie.
bool word_less(const uint8_t* a, uint32_t al, const uint8_t* b, uint32_t bl) {
  uint32_t i = 0, j = 0;
  for (;;) {
    uint32_t ie = i, je = j;
    while (ie < al && a[ie] != '/') ++ie;
    while (je < bl && b[je] != '/') ++je;
    const uint32_t la = ie - i, lb = je - j;
    const int c = memcmp(a + i, b + j, std::min(la, lb));
    if (c != 0) return c < 0;
    if (la != lb) return la < lb;
    const bool ea = ie >= al, eb = je >= bl;  // last word of a / b
    if (ea || eb) return ea && !eb;
    i = ie + 1;
    j = je + 1;
  }
}

uint64_t word_tok(const uint8_t* p, uint32_t len) {
  uint64_t packed = 0, fnv = FNV_OFF;
  for (uint32_t q = 0; q < len; ++q) {
    if (q < 8) packed |= (uint64_t)p[q] << (8 * q);
    fnv = fnv_step(fnv, p[q]);
  }
  return word_token(packed, fnv, len, 0);
}

// Build a store over the topics `order` (any order in, sorted out) and swap it into st.  The
// store keeps its own packed copy of its topics' bytes.
int build_store(emqxgm_retain* r, std::vector<uint32_t> order, Store& st) {
  const uint8_t* P = r->pool.data();
  std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
    const Topic &a = r->topics[x], &b = r->topics[y];
    return word_less(P + a.off, a.len, P + b.off, b.len);
  });
  const uint32_t N = (uint32_t)order.size();
  std::vector<uint8_t> spool;  // this store's topic bytes, in sorted order
  std::vector<uint64_t> soff(N + 1, 0);
  for (uint32_t i = 0; i < N; ++i) soff[i + 1] = soff[i] + r->topics[order[i]].len;
  if (soff[N] >= 0xFFFFFFFFull) {
    r->err = "retained topic bytes exceed 4 GiB";
    return -E2BIG;
  }
  spool.resize(soff[N]);
  for (uint32_t i = 0; i < N; ++i)
    if (r->topics[order[i]].len)
      memcpy(spool.data() + soff[i], P + r->topics[order[i]].off, r->topics[order[i]].len);
  // ---- topic trie in preorder ----
  std::vector<uint32_t> tb(1, 0), te(1, N), parent(1, NONE), woff(1, 0), wlen(1, 0);
  std::vector<uint8_t> term(1, 0);
  std::vector<uint64_t> tok(1, 0);
  std::vector<uint32_t> path(1, 0);  // node per depth of the previous topic
  std::vector<uint32_t> ws, pws;
  const uint8_t* prev = nullptr;
  for (uint32_t i = 0; i < N; ++i) {
    const Topic& t = r->topics[order[i]];
    const uint8_t* p = P + t.off;
    word_starts(p, t.len, ws);
    const uint32_t nw = (uint32_t)ws.size() - 1;
    uint32_t lcp = 0;  // words shared with the previous topic
    if (prev) {
      const uint32_t pn = (uint32_t)pws.size() - 1;
      while (lcp < nw && lcp < pn) {
        const uint32_t la = ws[lcp + 1] - 1 - ws[lcp], lb = pws[lcp + 1] - 1 - pws[lcp];
        if (la != lb || memcmp(p + ws[lcp], prev + pws[lcp], la) != 0) break;
        ++lcp;
      }
    }
    while (path.size() > lcp + 1) {  // close the previous topic's deeper nodes
      te[path.back()] = i;
      path.pop_back();
    }
    for (uint32_t k = lcp; k < nw; ++k) {  // open this topic's new nodes
      const uint32_t v = (uint32_t)tb.size();
      const uint32_t wl = ws[k + 1] - 1 - ws[k];
      tb.push_back(i);
      te.push_back(N);
      parent.push_back(path.back());
      woff.push_back((uint32_t)(soff[i] + ws[k]));
      wlen.push_back(wl);
      term.push_back(0);
      tok.push_back(word_tok(p + ws[k], wl));
      path.push_back(v);
    }
    term[path.back()] = 1;  // sorted and distinct: the topic's own node is new, first of its run
    prev = p;
    pws.swap(ws);
  }
  while (path.size() > 1) {
    te[path.back()] = N;
    path.pop_back();
  }
  const uint32_t nn = (uint32_t)tb.size();
  // children lists (ascending ids = ascending topic order) by counting parents
  std::vector<uint32_t> c0(nn + 1, 0), rch(nn > 0 ? nn - 1 : 0);
  for (uint32_t v = 1; v < nn; ++v) c0[parent[v] + 1] += 1;
  for (uint32_t v = 0; v < nn; ++v) c0[v + 1] += c0[v];
  {
    std::vector<uint32_t> cur(c0.begin(), c0.end() - 1);
    for (uint32_t v = 1; v < nn; ++v) rch[cur[parent[v]]++] = v;
  }
  std::vector<uint4> rn(nn);
  std::vector<uint2> rw(nn);
  for (uint32_t v = 0; v < nn; ++v) {
    rn[v] = make_uint4(tb[v] | (term[v] ? RTERM_BIT : 0u), te[v], c0[v], c0[v + 1]);
    rw[v] = make_uint2(woff[v], wlen[v]);
  }
  // (parent, token) -> child, 16-B slots, load <= 1/2
  const uint64_t cap = pow2_ge(std::max<uint64_t>(64, (uint64_t)nn * 2));
  std::vector<uint4> edge(cap, make_uint4(0u, 0u, NONE, 0u));
  for (uint32_t v = 1; v < nn; ++v) {
    uint64_t i = edge_slot(parent[v], tok[v], cap - 1);
    while (edge[i].z != NONE) i = (i + 1) & (cap - 1);
    edge[i] = make_uint4((uint32_t)tok[v], (uint32_t)(tok[v] >> 32), parent[v], v);
  }
  std::vector<uint64_t> sexp(N);
  for (uint32_t i = 0; i < N; ++i) sexp[i] = r->topics[order[i]].expiry;
  // ---- upload and swap ----
  if (hipSetDevice(r->device) != hipSuccess) return rfail(r, hipErrorInvalidDevice, "hipSetDevice");
  RCHK(r, hipStreamSynchronize(r->stream));
  std::vector<Buf> nb;
  RetainDev d;
  int rc = 0;
  if ((rc = upload(r, nb, rn, &d.rn)) || (rc = upload(r, nb, edge, &d.redge)) ||
      (rc = upload(r, nb, rch, &d.rch)) || (rc = upload(r, nb, rw, &d.rw)) ||
      (rc = upload(r, nb, spool, &d.pool)) || (rc = upload(r, nb, order, &d.sid)) ||
      (rc = upload(r, nb, sexp, &d.sexp))) {
    free_all(nb);
    return rc;
  }
  d.rmask = cap - 1;
  free_all(st.bufs);
  st.bufs.swap(nb);
  st.d = d;
  st.order.swap(order);
  return 0;
}

void mark_committed(emqxgm_retain* r, uint32_t id) {
  if (r->alive_committed.size() < r->topics.size()) {
    r->alive_committed.resize(r->topics.size(), 0);
    r->exp_committed.resize(r->topics.size(), 0);
  }
  r->alive_committed[id] = r->topics[id].alive;
  r->exp_committed[id] = r->topics[id].expiry;
}

// Full commit: every live topic into a new base, the delta store emptied.
int commit_full(emqxgm_retain* r) {
  std::vector<uint32_t> all;
  for (uint32_t id = 0; id < r->topics.size(); ++id)
    if (r->topics[id].alive) all.push_back(id);
  int rc = build_store(r, std::move(all), r->base);
  if (rc) return rc;
  if ((rc = build_store(r, {}, r->delta))) return rc;
  r->pos_of.assign(r->topics.size(), NONE);
  for (uint32_t i = 0; i < r->base.order.size(); ++i) r->pos_of[r->base.order[i]] = i;
  r->delta_ids.clear();
  r->alive_committed.assign(r->topics.size(), 0);
  r->exp_committed.assign(r->topics.size(), 0);
  for (uint32_t id = 0; id < r->topics.size(); ++id) mark_committed(r, id);
  r->n_committed = r->base.order.size();
  r->built = true;
  r->full_builds += 1;
  return 0;
}

// Delta commit: base topics stored again or deleted patch their expiry word (RDEAD: deleted);
// topics new since the base go to the delta store, rebuilt here.  Too many of them: full.
int commit_store(emqxgm_retain* r) {
  auto& ch = r->changed;
  std::sort(ch.begin(), ch.end());
  ch.erase(std::unique(ch.begin(), ch.end()), ch.end());
  if (!r->built || r->delta_max == 0) {
    ch.clear();
    return commit_full(r);
  }
  r->pos_of.resize(r->topics.size(), NONE);
  std::vector<PatchEnt> ents;
  std::vector<uint32_t> src;
  bool delta_changed = false;
  for (uint32_t id : ch) {
    const Topic& t = r->topics[id];
    const uint32_t p = r->pos_of[id];
    if (p != NONE) {
      const uint64_t e = t.alive ? t.expiry : ~0ull;  // gm_retain.inc RDEAD
      ents.push_back(PatchEnt{(uint64_t)(uintptr_t)(r->base.d.sexp + p), (uint32_t)src.size(), 2u});
      src.push_back((uint32_t)e);
      src.push_back((uint32_t)(e >> 32));
    } else if (t.alive) {
      delta_changed = true;  // (an expiry change of a delta topic too)
      r->delta_ids.insert(id);
    } else if (r->delta_ids.erase(id)) {
      delta_changed = true;
    }
  }
  const uint64_t lim = r->delta_max > 0
                           ? (uint64_t)r->delta_max
                           : std::max<uint64_t>(4096, r->base.order.size() / 16);
  if (r->delta_ids.size() > lim) {
    ch.clear();
    return commit_full(r);
  }
  if (hipSetDevice(r->device) != hipSuccess) return rfail(r, hipErrorInvalidDevice, "hipSetDevice");
  int rc = 0;
  if (!ents.empty()) {
    const uint64_t eb = ents.size() * sizeof(PatchEnt), total = eb + src.size() * 4;
    if ((rc = grow(r, S_PATCH, total))) return rc;
    uint8_t* d = (uint8_t*)r->sc[S_PATCH].p;
    RCHK(r, hipMemcpyAsync(d, ents.data(), eb, hipMemcpyHostToDevice, r->stream));
    RCHK(r, hipMemcpyAsync(d + eb, src.data(), src.size() * 4, hipMemcpyHostToDevice, r->stream));
    RCHK(r, launch_patch((const PatchEnt*)d, (uint32_t)ents.size(), (const uint32_t*)(d + eb),
                         r->stream));
    RCHK(r, hipStreamSynchronize(r->stream));
  }
  if (delta_changed &&
      (rc = build_store(r, std::vector<uint32_t>(r->delta_ids.begin(), r->delta_ids.end()),
                        r->delta)))
    return rc;
  for (uint32_t id : ch) {
    const bool was = id < r->alive_committed.size() && r->alive_committed[id];
    mark_committed(r, id);
    r->n_committed += (uint64_t)r->topics[id].alive - (uint64_t)was;
  }
  ch.clear();
  r->delta_builds += 1;
  return 0;
}

int grow(emqxgm_retain* r, size_t slot, uint64_t bytes) {
  if (r->sc.size() <= slot) r->sc.resize(slot + 1);
  Buf& b = r->sc[slot];
  if (b.p && b.bytes >= bytes) return 0;
  RCHK(r, hipStreamSynchronize(r->stream));
  if (b.p) (void)hipFree(b.p);
  b = Buf();
  const uint64_t cap = std::max<uint64_t>(bytes + bytes / 2, 4096);
  RCHK(r, hipMalloc(&b.p, cap));
  b.bytes = cap;
  return 0;
}



}  // namespace

extern "C" {

int emqxgm_retain_create(int32_t device, emqxgm_retain_t** out) {
  if (!out) return -EINVAL;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return -ENODEV;
  emqxgm_retain* r = new (std::nothrow) emqxgm_retain();
  if (!r) return -ENOMEM;
  r->device = device;
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) != hipSuccess) {
    delete r;
    return -EIO;
  }
  int rc = commit_store(r);
  if (rc) {
    emqxgm_retain_destroy(r);
    return rc;
  }
  *out = r;
  return 0;
}

void emqxgm_retain_destroy(emqxgm_retain_t* r) {
  if (!r) return;
  (void)hipSetDevice(r->device);
  if (r->stream) (void)hipStreamSynchronize(r->stream);
  free_all(r->base.bufs);
  free_all(r->delta.bufs);
  free_all(r->sc);
  if (r->stream) (void)hipStreamDestroy(r->stream);
  delete r;
}

int emqxgm_retain_store(emqxgm_retain_t* r, const uint8_t* topic, uint32_t len,
                        uint64_t expiry_ms, uint32_t* id) {
  if (!r || (!topic && len) || len > 65535) return -EINVAL;
  std::lock_guard<std::mutex> g(r->mu);
  std::string key((const char*)topic, len);
  auto it = r->ids.find(key);
  uint32_t i;
  if (it == r->ids.end()) {
    if (r->topics.size() >= 0x7FFFFFFFu) return -E2BIG;
    i = (uint32_t)r->topics.size();
    r->topics.push_back(Topic{r->pool.size(), len, expiry_ms, true});
    r->pool.insert(r->pool.end(), topic, topic + len);
    r->ids.emplace(std::move(key), i);
  } else {
    i = it->second;
    r->topics[i].alive = true;
    r->topics[i].expiry = expiry_ms;
  }
  r->changed.push_back(i);
  r->dirty = true;
  if (id) *id = i;
  return 0;
}

int emqxgm_retain_delete(emqxgm_retain_t* r, const uint8_t* topic, uint32_t len) {
  if (!r || (!topic && len)) return -EINVAL;
  std::lock_guard<std::mutex> g(r->mu);
  auto it = r->ids.find(std::string((const char*)topic, len));
  if (it != r->ids.end() && r->topics[it->second].alive) {
    r->topics[it->second].alive = false;
    r->changed.push_back(it->second);
    r->dirty = true;
  }
  return 0;
}

int emqxgm_retain_clean(emqxgm_retain_t* r) {
  if (!r) return -EINVAL;
  std::lock_guard<std::mutex> g(r->mu);
  for (Topic& t : r->topics) t.alive = false;
  r->built = false;  // the next commit rebuilds (an empty base)
  r->dirty = true;
  return 0;
}

int emqxgm_retain_commit(emqxgm_retain_t* r) {
  if (!r) return -EINVAL;
  std::lock_guard<std::mutex> g(r->mu);
  return r->dirty ? commit_store(r) : 0;
}

int emqxgm_retain_tune(emqxgm_retain_t* r, const char* key, int64_t value) {
  if (!r || !key) return -EINVAL;
  std::lock_guard<std::mutex> g(r->mu);
  if (strcmp(key, "delta_max") == 0) {
    r->delta_max = value;
    return 0;
  }
  return -EINVAL;
}

int emqxgm_retain_set_indices(emqxgm_retain_t* r, const uint32_t* pos, const uint32_t* offsets,
                              uint32_t n) {
  if (!r || (n && (!pos || !offsets)) || n > 64) return -EINVAL;
  std::vector<std::vector<uint32_t>> ix(n);
  for (uint32_t i = 0; i < n; ++i) {
    if (offsets[i + 1] <= offsets[i] || offsets[i + 1] - offsets[i] > 255) return -EINVAL;
    for (uint32_t q = offsets[i]; q < offsets[i + 1]; ++q) {
      // positions >= 1, strictly ascending (emqx_retainer_schema: an index is a sorted set)
      if (pos[q] == 0 || pos[q] > 65535 || (q > offsets[i] && pos[q] <= pos[q - 1])) return -EINVAL;
      ix[i].push_back(pos[q]);
    }
  }
  std::sort(ix.begin(), ix.end());  // config_indices/0 (emqx_retainer_mnesia.erl) sorts them
  ix.erase(std::unique(ix.begin(), ix.end()), ix.end());
  std::lock_guard<std::mutex> g(r->mu);
  r->indices = std::move(ix);
  return 0;
}

int emqxgm_retain_stats(emqxgm_retain_t* r, uint64_t out[4]) {
  if (!r || !out) return -EINVAL;
  std::lock_guard<std::mutex> g(r->mu);
  out[0] = r->full_builds;
  out[1] = r->delta_builds;
  out[2] = r->base.order.size();
  out[3] = r->delta.order.size();
  return 0;
}

int emqxgm_retain_size(emqxgm_retain_t* r, uint64_t* n) {
  if (!r || !n) return -EINVAL;
  std::lock_guard<std::mutex> g(r->mu);
  *n = r->n_committed;
  return 0;
}

int emqxgm_retain_read(emqxgm_retain_t* r, const uint8_t* topic, uint32_t len, uint64_t now_ms,
                       uint32_t* id) {
  if (!r || (!topic && len)) return -EINVAL;
  std::lock_guard<std::mutex> g(r->mu);
  auto it = r->ids.find(std::string((const char*)topic, len));
  if (it == r->ids.end() || it->second >= r->alive_committed.size() ||
      !r->alive_committed[it->second])
    return 0;
  const uint64_t e = r->exp_committed[it->second];
  if (!(e == 0 || e >= now_ms)) return 0;
  if (id) *id = it->second;
  return 1;
}

int emqxgm_retain_topic(emqxgm_retain_t* r, uint32_t id, const uint8_t** p, uint32_t* len) {
  if (!r || !p || !len) return -EINVAL;
  std::lock_guard<std::mutex> g(r->mu);
  if (id >= r->topics.size()) return -ENOENT;
  *p = r->pool.data() + r->topics[id].off;
  *len = r->topics[id].len;
  return 0;
}

int emqxgm_retain_match(emqxgm_retain_t* r, const uint8_t* bytes, const uint32_t* offsets,
                        uint32_t n, uint64_t now_ms, emqxgm_retain_out* out) {
  if (!r || !out || !offsets || (offsets[n] && !bytes)) return -EINVAL;
  // '+' words per filter bound the DFS frames of a lane
  uint32_t max_plus = 0;
  std::vector<uint32_t> plus_of(n);
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t b = offsets[i], e = offsets[i + 1];
    if (e < b || e - b > 65535) return -EINVAL;
    uint32_t plus = 0, s = b;
    for (uint32_t q = b; q <= e; ++q)
      if (q == e || bytes[q] == '/') {
        plus += (q - s == 1 && bytes[s] == '+');
        s = q + 1;
      }
    plus_of[i] = plus;
  }
  std::lock_guard<std::mutex> g(r->mu);
  // the index path's filter plan (cut after a '#', open tails): the walk's frames per filter
  // are its '+' words plus its tail
  r->h_fb.clear();
  r->h_fo.assign(1, 0u);
  r->h_tail.resize(n);
  bool any_tail = false;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t tl = plan_filter(r->indices, bytes + offsets[i], offsets[i + 1] - offsets[i], r->h_fb);
    r->h_tail[i] = (uint8_t)tl;
    any_tail = any_tail || tl;
    r->h_fo.push_back((uint32_t)r->h_fb.size());
    max_plus = std::max<uint32_t>(max_plus, plus_of[i] + tl);
  }
  bytes = r->h_fb.data();
  offsets = r->h_fo.data();
  out->n = n;
  r->h_ptr.assign((size_t)n + 1, 0);
  r->h_id.clear();
  out->ptr = r->h_ptr.data();
  out->id = r->h_id.data();
  out->n_ids = 0;
  if (n == 0) return 0;
  if (hipSetDevice(r->device) != hipSuccess) return -EIO;
  hipStream_t s = r->stream;
  const uint64_t fbytes = offsets[n];
  int rc = 0;
  if ((rc = grow(r, S_FB, fbytes + 16)) || (rc = grow(r, S_FO, ((uint64_t)n + 1) * 4)) ||
      (rc = grow(r, S_FRAMES, (uint64_t)n * std::max<uint32_t>(max_plus, 1) * 16)) ||
      (rc = grow(r, S_CNT, (uint64_t)n * 4)) || (rc = grow(r, S_RBASE, ((uint64_t)n + 1) * 4)) ||
      (rc = grow(r, S_PTR, ((uint64_t)n + 1) * 4)) || (rc = grow(r, S_CTL, 64)) ||
      (rc = grow(r, S_TMP, (uint64_t)scan_tmp_words(n) * 4)) || (rc = grow(r, S_TAIL, (uint64_t)n + 16)))
    return rc;
  auto B = [&](int k) { return r->sc[k].p; };
  if (any_tail) RCHK(r, hipMemcpyAsync(B(S_TAIL), r->h_tail.data(), n, hipMemcpyHostToDevice, s));
  const uint8_t* tail = any_tail ? (const uint8_t*)B(S_TAIL) : nullptr;
  if (fbytes) RCHK(r, hipMemcpyAsync(B(S_FB), bytes, fbytes, hipMemcpyHostToDevice, s));
  RCHK(r, hipMemcpyAsync(B(S_FO), offsets, ((size_t)n + 1) * 4, hipMemcpyHostToDevice, s));
  const uint8_t* fb = (const uint8_t*)B(S_FB);
  const uint32_t* fo = (const uint32_t*)B(S_FO);
  uint32_t* ctl = (uint32_t*)B(S_CTL);
  uint32_t* cnt = (uint32_t*)B(S_CNT);
  uint32_t* rbase = (uint32_t*)B(S_RBASE);
  // runs per filter (base, then base + delta) -> scan -> runs (base, then delta after them)
  const bool has_delta = !r->delta.order.empty();
  uint32_t* cnt2 = nullptr;
  if (has_delta) {
    if ((rc = grow(r, S_CNT2, (uint64_t)n * 4))) return rc;
    cnt2 = (uint32_t*)B(S_CNT2);
  }
  uint4* frames = (uint4*)B(S_FRAMES);
  RCHK(r, launch_retain_walk(r->base.d, fb, fo, n, tail, frames, max_plus, cnt, nullptr, nullptr, nullptr,
                             false, nullptr, false, s));
  if (has_delta)
    RCHK(r, launch_retain_walk(r->delta.d, fb, fo, n, tail, frames, max_plus, cnt2, cnt, nullptr, nullptr,
                               true, nullptr, false, s));
  RCHK(r, launch_scan(has_delta ? cnt2 : cnt, rbase, n, (uint32_t*)B(S_TMP), ctl, s));
  uint32_t nr = 0;
  RCHK(r, hipMemcpyAsync(&nr, ctl, 4, hipMemcpyDeviceToHost, s));
  RCHK(r, hipStreamSynchronize(s));
  if ((rc = grow(r, S_RUNS, (uint64_t)nr * 8 + 16)) || (rc = grow(r, S_ACNT, (uint64_t)nr * 4 + 4)) ||
      (rc = grow(r, S_ABASE, ((uint64_t)nr + 1) * 4)) ||
      (rc = grow(r, S_TMP, (uint64_t)scan_tmp_words(std::max(n, nr)) * 4)))
    return rc;
  uint2* runs = (uint2*)B(S_RUNS);
  uint32_t* acnt = (uint32_t*)B(S_ACNT);
  uint32_t* abase = (uint32_t*)B(S_ABASE);
  RCHK(r, launch_retain_walk(r->base.d, fb, fo, n, tail, frames, max_plus, nullptr, nullptr, rbase,
                             nullptr, false, runs, true, s));
  if (has_delta)
    RCHK(r, launch_retain_walk(r->delta.d, fb, fo, n, tail, frames, max_plus, nullptr, nullptr, rbase, cnt,
                               true, runs, true, s));
  // live ids per run -> scan -> ids
  unsigned long long* total = (unsigned long long*)(ctl + 4);
  RCHK(r, hipMemsetAsync(total, 0, 8, s));
  RCHK(r, launch_retain_runs(r->base.d, r->delta.d, runs, nr, now_ms, acnt, nullptr, nullptr, total,
                             false, s));
  unsigned long long nid = 0;
  RCHK(r, hipMemcpyAsync(&nid, total, 8, hipMemcpyDeviceToHost, s));
  RCHK(r, hipStreamSynchronize(s));
  if (nid >= 0xFFFFFFFFull) {
    r->err = "retained match selects more than 2^32 ids in one batch";
    return -E2BIG;
  }
  RCHK(r, launch_scan(acnt, abase, nr, (uint32_t*)B(S_TMP), nullptr, s));
  if ((rc = grow(r, S_OUT, nid * 4 + 4))) return rc;
  uint32_t* ids = (uint32_t*)B(S_OUT);
  RCHK(r, launch_retain_runs(r->base.d, r->delta.d, runs, nr, now_ms, acnt, abase, ids, total,
                             true, s));
  uint32_t* ptr = (uint32_t*)B(S_PTR);
  RCHK(r, launch_retain_ptr(rbase, abase, n, ptr, s));
  r->h_ptr32.resize((size_t)n + 1);
  r->h_id.resize(nid);
  RCHK(r, hipMemcpyAsync(r->h_ptr32.data(), ptr, ((size_t)n + 1) * 4, hipMemcpyDeviceToHost, s));
  if (nid) RCHK(r, hipMemcpyAsync(r->h_id.data(), ids, nid * 4, hipMemcpyDeviceToHost, s));
  RCHK(r, hipStreamSynchronize(s));
  for (uint32_t i = 0; i <= n; ++i) r->h_ptr[i] = r->h_ptr32[i];
  out->ptr = r->h_ptr.data();
  out->id = r->h_id.data();
  out->n_ids = nid;
  return 0;
}

}  // extern "C"
