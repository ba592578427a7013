// gm_async.cpp -- the concurrent publish entry (include/emqx_gpumatch.h "concurrent publish
// entry"): any number of threads hand in one topic each, the layer packs them into windows in
// pinned host memory, a flusher thread submits a window when it is full or window_us after its
// first topic (emqxgm_match_batch_submit_filters), and one completer thread per engine handle
// waits for its windows in submission order (emqxgm_match_batch_wait_filters, which waits
// without holding the engine's locks) and hands each completed window to the caller's callback.
// With several handles (one engine per GPU, each holding the whole index: the replica layout of
// DESIGN.md 5) windows go round robin to the handles with a pipe free.
//
// The reference matches each publish inside the publisher's own process, concurrently on every
// scheduler, against read_concurrency ETS tables (emqx_broker:publish/1 ->
// emqx_router:match_routes/1 -> emqx_trie:match/1, apps/emqx/src/emqx_broker.erl:218-232,
// emqx_router.erl:141-157, emqx_trie.erl:70-75, 147-169); the NIF's match_async/3
// (c_src/emqx_trie_gpu_nif.c) is this layer's emqxgm_async_match, called from those processes
// directly, and its callback enif_sends each caller its result.
//
// A call takes no lock: it reserves its place in the open window with one atomic add on the
// window's (calls, bytes) cursor, copies its topic there and counts itself settled.  Places are
// handed out in order, so the reservations that fit are a prefix of the window; the first one
// that does not fit (or the flusher's timer) seals the window: a seal adds SEAL calls to the
// cursor, so every later reservation fails and goes to the next window.  The flusher submits a
// sealed window once every reservation made before the seal has settled.  Only the slow paths
// (a window full or due, no window open, the flusher and completers) take the layer's mutex.
#include <errno.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/emqx_gpumatch.h"

namespace {

uint64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

enum SlotState { FREE, OPEN, READY, SUBMITTING, INFLIGHT, DELIVERING };

constexpr uint64_t CALL1 = 1ull << 32;     // one call in the cursor's high half
constexpr uint32_t SEAL = 1u << 31;        // calls a seal adds: every later reservation fails

static_assert(sizeof(std::atomic<uint64_t>) == sizeof(uint64_t), "tags are read as uint64_t");

// One window: its packed topics in pinned memory (the H2D source of its pass) and the callers.
struct Slot {
  uint8_t* bytes = nullptr;  // pinned [window_bytes]
  uint32_t* off = nullptr;   // pinned [window_topics + 1]
  std::unique_ptr<std::atomic<uint64_t>[]> tag, owner;  // [window_topics]
  std::atomic<uint64_t> cursor{0};    // (calls reserved << 32) | bytes reserved
  std::atomic<uint32_t> settled{0};   // reservations made before the seal that are done
  std::atomic<uint32_t> limit{~0u};   // the first reservation that did not fit
  std::atomic<bool> sealed{false};
  std::atomic<uint64_t> first_ns{0};
  uint32_t reserved = 0;  // calls reserved before the seal (set by the sealer)
  uint32_t n = 0;         // calls in the window (set once they settled)
  int state = FREE;       // guarded by the layer's mutex
  int status = 0;         // a failed submit's error (the completer reports it)
  uint32_t hi = 0;        // handle it went to
  uint64_t ticket = 0, flush_ns = 0;
};

}  // namespace

struct emqxgm_async {
  std::vector<emqxgm_t*> hs;
  emqxgm_async_cfg cfg{};
  emqxgm_async_cb cb = nullptr;
  void* user = nullptr;
  std::vector<std::unique_ptr<Slot>> slots;
  std::vector<int> free_slots;
  std::atomic<int> open{-1};                     // the slot taking calls, or -1
  std::deque<int> ready;                         // sealed windows, oldest first
  std::vector<std::deque<int>> inflight;         // per handle, in submission order
  std::vector<uint32_t> outstanding;             // per handle: submitted and not yet released
  uint32_t rr = 0;                               // next handle to try
  bool stop = false, flusher_done = false;
  std::mutex mu;
  std::condition_variable cv_flush;              // the flusher: a window ready / opened, a pipe free
  std::condition_variable cv_done;               // a window was released (cancel)
  std::vector<std::unique_ptr<std::condition_variable>> cv_comp;  // completer k: work on handle k
  std::thread flusher;
  std::vector<std::thread> completers;
  std::atomic<uint64_t> st_calls{0}, st_busy{0}, st_too_big{0};
  uint64_t st_windows = 0, st_cancelled = 0, st_errors = 0, st_delivered = 0;

  // Seals slot si (with mu held): no reservation after this one succeeds; the window goes to the
  // ready queue (the flusher submits it once its reservations settled) or, empty, back to free.
  void seal(int si) {
    Slot& s = *slots[si];
    if (s.state != OPEN || s.sealed.exchange(true)) return;
    const uint64_t c = s.cursor.fetch_add((uint64_t)SEAL << 32);
    s.reserved = (uint32_t)(c >> 32);
    int expect = si;
    open.compare_exchange_strong(expect, -1);
    s.state = READY;
    ready.push_back(si);
    cv_flush.notify_one();
  }
  // Opens a free slot (with mu held); false: none free.
  bool open_slot() {
    if (free_slots.empty()) return false;
    const int si = free_slots.back();
    free_slots.pop_back();
    Slot& s = *slots[si];
    s.state = OPEN;
    s.n = 0;
    s.reserved = 0;
    s.status = 0;
    s.off[0] = 0;
    s.first_ns.store(0, std::memory_order_relaxed);
    s.settled.store(0, std::memory_order_relaxed);
    s.limit.store(~0u, std::memory_order_relaxed);
    s.sealed.store(false, std::memory_order_relaxed);
    s.cursor.store(0, std::memory_order_release);
    open.store(si, std::memory_order_release);
    return true;
  }
  // The calls of a sealed window, once every reservation made before its seal settled (mu not
  // needed: `reserved` was set under mu before the window became READY).
  bool settled(Slot& s) const {
    return s.settled.load(std::memory_order_acquire) >= s.reserved;
  }
  void finish_window(Slot& s) {
    const uint32_t lim = s.limit.load(std::memory_order_relaxed);
    s.n = std::min({s.reserved, lim, cfg.window_topics});
    // off[i] = start of call i; the end of the last one was stored by it as off[n]
    if (s.n == 0) s.off[0] = 0;
  }

  bool pipe_free() const {
    for (uint32_t v : outstanding)
      if (v < EMQXGM_HOST_PIPES) return true;
    return false;
  }

  // Windows grow while every pipe is busy: the window_us timer seals the open window only when a
  // pipe could take it at once (and nothing sealed is waiting), so an idle broker answers within
  // window_us plus a pass, and a loaded one submits windows as large as the pipes' pace allows
  // (sealing on the timer regardless made windows of a few hundred calls queue behind the busy
  // pipes: r04 nif_concurrent, 3 M calls/s at 330 calls per window).
  void flusher_loop() {
    std::unique_lock<std::mutex> g(mu);
    for (;;) {
      const int oi = open.load(std::memory_order_acquire);
      if (oi >= 0) {
        const uint64_t f = slots[oi]->first_ns.load(std::memory_order_acquire);
        if (stop || (f != 0 && ready.empty() && pipe_free() &&
                     mono_ns() >= f + 1000ull * cfg.window_us))
          seal(oi);
      }
      bool progressed = false;
      while (!ready.empty()) {
        const uint32_t H = (uint32_t)hs.size();
        uint32_t k = H;
        for (uint32_t j = 0; j < H; ++j) {
          const uint32_t c = (rr + j) % H;
          if (outstanding[c] < EMQXGM_HOST_PIPES) {
            k = c;
            break;
          }
        }
        if (k == H) break;  // every pipe busy: a completer's release wakes us
        const int si = ready.front();
        Slot& s = *slots[si];
        if (!settled(s)) {  // a caller is still copying its topic in: a moment
          g.unlock();
          std::this_thread::yield();
          g.lock();
          progressed = true;
          break;
        }
        ready.pop_front();
        finish_window(s);
        if (s.n == 0) {  // sealed before anyone's reservation fit
          s.state = FREE;
          free_slots.push_back(si);
          progressed = true;
          continue;
        }
        rr = (k + 1) % H;
        s.state = SUBMITTING;
        s.hi = k;
        outstanding[k] += 1;
        g.unlock();
        s.flush_ns = mono_ns();
        uint64_t tk = 0;
        // the filter-byte gather and every result copy go behind the pass: one wait
        const int rc = emqxgm_match_batch_submit_filters(hs[k], s.bytes, s.off, s.n, &tk);
        g.lock();
        s.ticket = tk;
        s.status = rc;
        s.state = INFLIGHT;
        inflight[k].push_back(si);
        st_windows += 1;
        cv_comp[k]->notify_one();
        progressed = true;
      }
      if (progressed) continue;
      if (stop && open.load() < 0 && ready.empty()) break;
      const int o2 = open.load(std::memory_order_acquire);
      const uint64_t f = o2 >= 0 ? slots[o2]->first_ns.load(std::memory_order_acquire) : 0;
      if (f != 0 && ready.empty() && pipe_free()) {
        const uint64_t due = f + 1000ull * cfg.window_us, t = mono_ns();
        if (due > t) cv_flush.wait_for(g, std::chrono::nanoseconds(due - t));
      } else {
        cv_flush.wait(g);
      }
    }
    flusher_done = true;
    for (auto& c : cv_comp) c->notify_all();
  }

  void completer_loop(uint32_t k) {
    std::unique_lock<std::mutex> g(mu);
    for (;;) {
      while (inflight[k].empty() && !flusher_done) cv_comp[k]->wait(g);
      if (inflight[k].empty()) break;  // the flusher is done and nothing is left here
      const int si = inflight[k].front();
      Slot& s = *slots[si];
      g.unlock();
      emqxgm_batch_out bo{};
      const uint32_t* foff = nullptr;
      const uint8_t* fb = nullptr;
      int rc = s.status;
      if (rc == 0) rc = emqxgm_match_batch_wait_filters(hs[k], s.ticket, &bo, &foff, &fb);
      const uint64_t done = mono_ns();
      g.lock();
      inflight[k].pop_front();
      s.state = DELIVERING;  // a cancel() of one of its calls waits for the release below
      g.unlock();
      emqxgm_async_window w{};
      w.status = rc;
      w.n = s.n;
      w.tag = reinterpret_cast<const uint64_t*>(s.tag.get());
      w.owner = reinterpret_cast<const uint64_t*>(s.owner.get());
      if (rc == 0) {
        w.n_pairs = bo.n_pairs;
        w.row = bo.row_ptr;
        w.filter_id = bo.filter_id;
        w.foff = foff;
        w.fbytes = fb;
        w.exact_id = bo.exact_id;
      }
      w.device_index = k;
      w.first_ns = s.first_ns.load(std::memory_order_relaxed);
      w.flush_ns = s.flush_ns;
      w.done_ns = done;
      cb(user, &w);
      g.lock();
      st_delivered += s.n;
      if (rc) st_errors += 1;
      s.state = FREE;
      free_slots.push_back(si);
      outstanding[k] -= 1;
      cv_flush.notify_one();
      cv_done.notify_all();
    }
  }
};

extern "C" {

int emqxgm_async_create(emqxgm_t* const* hs, uint32_t n_handles, const emqxgm_async_cfg* cfg,
                        emqxgm_async_cb cb, void* user, emqxgm_async_t** out) {
  if (!hs || !n_handles || !cb || !out) return -EINVAL;
  *out = nullptr;
  for (uint32_t k = 0; k < n_handles; ++k)
    if (!hs[k]) return -EINVAL;
  emqxgm_async* a = new (std::nothrow) emqxgm_async();
  if (!a) return -ENOMEM;
  a->hs.assign(hs, hs + n_handles);
  if (cfg) a->cfg = *cfg;
  if (!a->cfg.window_topics) a->cfg.window_topics = 65536;
  if (!a->cfg.window_bytes) a->cfg.window_bytes = 64u * a->cfg.window_topics;
  if (!a->cfg.window_us) a->cfg.window_us = 50;
  if (!a->cfg.queued_windows) a->cfg.queued_windows = 2;
  if (a->cfg.window_topics >= SEAL || a->cfg.window_bytes >= SEAL) {
    delete a;
    return -EINVAL;
  }
  a->cb = cb;
  a->user = user;
  const uint32_t n_slots = n_handles * EMQXGM_HOST_PIPES + 1 + a->cfg.queued_windows;
  int rc = 0;
  for (uint32_t i = 0; i < n_slots && !rc; ++i) {
    a->slots.emplace_back(new (std::nothrow) Slot());
    Slot* s = a->slots.back().get();
    if (!s) {
      a->slots.pop_back();
      rc = -ENOMEM;
      break;
    }
    // pinned on the handle it most likely goes to (portable: any handle's copies run at speed)
    emqxgm_t* h = a->hs[i % n_handles];
    s->bytes = (uint8_t*)emqxgm_host_alloc(h, a->cfg.window_bytes);
    s->off = (uint32_t*)emqxgm_host_alloc(h, ((uint64_t)a->cfg.window_topics + 1) * 4);
    s->tag.reset(new (std::nothrow) std::atomic<uint64_t>[a->cfg.window_topics]);
    s->owner.reset(new (std::nothrow) std::atomic<uint64_t>[a->cfg.window_topics]);
    if (!s->bytes || !s->off || !s->tag || !s->owner) rc = -ENOMEM;
    else s->off[0] = 0;
    a->free_slots.push_back((int)(n_slots - 1 - i));
  }
  if (rc) {
    for (size_t i = 0; i < a->slots.size(); ++i) {
      emqxgm_host_free(a->hs[i % n_handles], a->slots[i]->bytes);
      emqxgm_host_free(a->hs[i % n_handles], a->slots[i]->off);
    }
    delete a;
    return rc;
  }
  a->inflight.resize(n_handles);
  a->outstanding.assign(n_handles, 0);
  for (uint32_t k = 0; k < n_handles; ++k) a->cv_comp.emplace_back(new std::condition_variable());
  {
    std::lock_guard<std::mutex> g(a->mu);
    a->open_slot();
  }
  a->flusher = std::thread([a] { a->flusher_loop(); });
  for (uint32_t k = 0; k < n_handles; ++k) a->completers.emplace_back([a, k] { a->completer_loop(k); });
  *out = a;
  return 0;
}

void emqxgm_async_destroy(emqxgm_async_t* a) {
  if (!a) return;
  {
    std::lock_guard<std::mutex> g(a->mu);
    a->stop = true;
    a->cv_flush.notify_all();
  }
  a->flusher.join();  // seals and submits what is left, then wakes the completers
  for (auto& t : a->completers) t.join();  // deliver every accepted call
  const uint32_t H = (uint32_t)a->hs.size();
  for (size_t i = 0; i < a->slots.size(); ++i) {
    emqxgm_host_free(a->hs[i % H], a->slots[i]->bytes);
    emqxgm_host_free(a->hs[i % H], a->slots[i]->off);
  }
  delete a;
}

int emqxgm_async_match(emqxgm_async_t* a, const uint8_t* topic, uint32_t len, uint64_t tag,
                       uint64_t owner) {
  if (!a || (!topic && len) || tag == EMQXGM_TAG_CANCELLED) return -EINVAL;
  if (len > a->cfg.window_bytes) return -E2BIG;
  if (a->cfg.max_levels) {
    // emqx_topic:levels/1 = words: separators + 1 (the zone's max_topic_levels, checked here so
    // a caller does not tokenise on the host first)
    uint32_t levels = 1;
    for (const uint8_t* p = topic; (p = (const uint8_t*)memchr(p, '/', topic + len - p)); ++p) ++levels;
    if (levels > a->cfg.max_levels) {
      a->st_too_big.fetch_add(1, std::memory_order_relaxed);
      return -E2BIG;
    }
  }
  const uint32_t WT = a->cfg.window_topics, WB = a->cfg.window_bytes;
  for (;;) {
    const int si = a->open.load(std::memory_order_acquire);
    if (si >= 0) {
      Slot& s = *a->slots[si];
      const uint64_t c = s.cursor.fetch_add(CALL1 | len, std::memory_order_acq_rel);
      const uint32_t n = (uint32_t)(c >> 32), b = (uint32_t)c;
      if (n < SEAL) {  // a reservation made before the window was sealed
        const bool fits = n < WT && (uint64_t)b + len <= WB;
        if (fits) {
          if (len) memcpy(s.bytes + b, topic, len);
          __atomic_store_n(&s.off[n], b, __ATOMIC_RELAXED);
          __atomic_store_n(&s.off[n + 1], b + len, __ATOMIC_RELAXED);
          s.tag[n].store(tag, std::memory_order_relaxed);
          s.owner[n].store(owner, std::memory_order_relaxed);
          if (n == 0) s.first_ns.store(mono_ns(), std::memory_order_release);
        } else {
          // the first reservation that does not fit bounds the window (the later ones cannot
          // fit either: places and bytes are handed out in order)
          uint32_t cur = s.limit.load(std::memory_order_relaxed);
          while (n < cur && !s.limit.compare_exchange_weak(cur, n, std::memory_order_relaxed)) {
          }
        }
        s.settled.fetch_add(1, std::memory_order_release);
        if (fits) {
          a->st_calls.fetch_add(1, std::memory_order_relaxed);
          const bool full = n + 1 == WT || (uint64_t)b + len == WB;
          if (n == 0 || full) {
            std::lock_guard<std::mutex> g(a->mu);
            if (full) a->seal(si);  // no room for the next one
            else a->cv_flush.notify_one();  // arms the flusher's window_us timer
          }
          return 0;
        }
      }
      // the window is full or sealed: seal it (if nobody did) and go to the next one
      std::lock_guard<std::mutex> g(a->mu);
      if (a->stop) return -ESHUTDOWN;
      if (a->open.load() == si) a->seal(si);
      if (a->open.load() < 0 && !a->open_slot()) {
        a->st_busy.fetch_add(1, std::memory_order_relaxed);
        return -EBUSY;  // every window is full or in flight: the caller answers this one itself
      }
      continue;
    }
    std::lock_guard<std::mutex> g(a->mu);
    if (a->stop) return -ESHUTDOWN;
    if (a->open.load() < 0 && !a->open_slot()) {
      a->st_busy.fetch_add(1, std::memory_order_relaxed);
      return -EBUSY;
    }
  }
}

int emqxgm_async_cancel(emqxgm_async_t* a, uint64_t tag, uint64_t owner) {
  if (!a || tag == EMQXGM_TAG_CANCELLED) return -EINVAL;
  std::unique_lock<std::mutex> g(a->mu);
  int delivering = -1;
  for (size_t i = 0; i < a->slots.size() && delivering < 0; ++i) {
    Slot& s = *a->slots[i];
    if (s.state == FREE) continue;
    // an open window's calls: those reserved so far (the caller's own call is complete)
    const uint32_t m = s.state == OPEN || s.state == READY
                           ? std::min<uint32_t>((uint32_t)(s.cursor.load() >> 32), a->cfg.window_topics)
                           : s.n;
    for (uint32_t j = 0; j < m; ++j) {
      if (s.tag[j].load(std::memory_order_relaxed) != tag ||
          s.owner[j].load(std::memory_order_relaxed) != owner)
        continue;
      if (s.state == DELIVERING) {
        delivering = (int)i;
        break;
      }
      s.tag[j].store(EMQXGM_TAG_CANCELLED, std::memory_order_relaxed);  // matched, never reported
      a->st_cancelled += 1;
      return 1;
    }
  }
  if (delivering < 0) return 0;  // already reported (or never accepted)
  // its window is being reported right now: once released, the report has been made
  Slot& d = *a->slots[delivering];
  a->cv_done.wait(g, [&] { return d.state != DELIVERING; });
  return 0;
}

int emqxgm_async_stats(emqxgm_async_t* a, uint64_t out[8]) {
  if (!a || !out) return -EINVAL;
  std::lock_guard<std::mutex> g(a->mu);
  out[0] = a->st_calls.load();
  out[1] = a->st_windows;
  out[2] = a->st_delivered;
  out[3] = a->st_busy.load();
  out[4] = a->st_cancelled;
  out[5] = a->st_too_big.load();
  out[6] = a->st_errors;
  uint64_t q = 0;
  for (auto v : a->outstanding) q += v;
  out[7] = q;
  return 0;
}

}  // extern "C"
