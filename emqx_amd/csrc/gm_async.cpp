// gm_async.cpp -- the concurrent publish entry (include/emqx_gpumatch.h "concurrent publish
// entry"): any number of threads hand in one topic each, the layer packs them into windows in
// pinned host memory, a flusher thread submits a window when it is full or (with a pipe free)
// window_us after its first topic (emqxgm_match_batch_submit_filters), and one completer thread
// per engine handle waits for its windows in submission order (emqxgm_match_batch_wait_filters,
// which waits without holding the engine's locks) and hands each completed window to the
// caller's callback.  With several handles (one engine per GPU, each holding the whole index:
// the replica layout of DESIGN.md 5) windows go round robin to the handles with a pipe free.
//
// The reference matches each publish inside the publisher's own process, concurrently on every
// scheduler, against read_concurrency ETS tables (emqx_broker:publish/1 ->
// emqx_router:match_routes/1 -> emqx_trie:match/1, apps/emqx/src/emqx_broker.erl:218-232,
// emqx_router.erl:141-157, emqx_trie.erl:70-75, 147-169); the NIF's match_async/3
// (c_src/emqx_trie_gpu_nif.c) is this layer's emqxgm_async_match, called from those processes
// directly, and its callback enif_sends each caller its result.
//
// Contention.  A call appends its topic to its own thread's staging chunk (a spinlock nobody else
// takes except the flusher, when it seals a window): no shared cache line per call.  A full chunk
// -- or the flusher, before it seals a window -- moves the chunk into the open window with ONE
// atomic add on the window's (calls, bytes) cursor and one copy.  Places are handed out in
// order, so the reservations that fit are a prefix of the window; the first that does not seals
// it (a seal adds SEAL calls to the cursor: every later reservation fails and goes to the next
// window).  The flusher submits a sealed window once every reservation made before the seal has
// settled.  (r04: one atomic reservation per call put every call on two contended lines and the
// calls' neighbouring tags on shared lines: 4 M calls/s whatever the thread count.)
#include <errno.h>
#include <string.h>
#include <sys/prctl.h>
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
#include "gm_internal.h"

namespace {

uint64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

enum SlotState { FREE, OPEN, READY, SUBMITTING, INFLIGHT, DELIVERING };

constexpr uint32_t SEAL = 1u << 31;        // calls a seal adds: every later reservation fails
constexpr uint32_t CHUNK_CALLS = 64;       // a thread's staging chunk (at most: a window's size)
constexpr uint32_t CHUNK_BYTES = 4096;
#ifndef GM_DELIVER_MIN
#define GM_DELIVER_MIN 1024  // (the host harness builds with a small value to split small windows)
#endif
constexpr uint32_t DELIVER_MIN = GM_DELIVER_MIN;  // calls per part of a window the pool reports

static_assert(sizeof(std::atomic<uint64_t>) == sizeof(uint64_t), "tags are read as uint64_t");

std::atomic<uint64_t> g_layer_ids{1};

// One window: its packed topics in pinned memory (the H2D source of its pass) and the callers.
struct Slot {
  uint8_t* bytes = nullptr;  // pinned [window_bytes]
  uint32_t* off = nullptr;   // pinned [window_topics + 1]
  std::unique_ptr<std::atomic<uint64_t>[]> tag, owner;  // [window_topics]
  alignas(64) std::atomic<uint64_t> cursor{0};  // (calls reserved << 32) | bytes reserved
  alignas(64) std::atomic<uint32_t> settled{0};  // calls of reservations before the seal, done
  std::atomic<uint32_t> limit{~0u};   // the first call of the first reservation that did not fit
  std::atomic<bool> sealed{false};
  std::atomic<uint64_t> first_ns{0};  // its oldest call
  uint32_t reserved = 0;  // calls reserved before the seal (set by the sealer)
  uint32_t n = 0;         // calls in the window (set once they settled)
  int state = FREE;       // guarded by the layer's mutex
  int status = 0;         // a failed submit's error (the completer reports it)
  uint32_t hi = 0;        // handle it went to
  uint64_t ticket = 0, flush_ns = 0;
  uint64_t seq = 0;       // submission order (the handle registry's quiescence marks)
};

// Calls on their way into a window: a thread's staging chunk, or one long call on its own.
struct Span {
  uint32_t k = 0, b = 0;  // calls, bytes
  uint32_t* len = nullptr;
  uint64_t *tag = nullptr, *owner = nullptr;
  const uint8_t* bytes = nullptr;
  uint64_t first_ns = 0;
};

// One producer thread's staging chunk.  Its spinlock is taken by its own thread per call and by
// the flusher when it drains every chunk before a seal.
struct alignas(64) Chunk {
  std::atomic<bool> busy{false};
  std::atomic<uint64_t> first_ns{0};  // its oldest call (0: empty)
  uint32_t k = 0, b = 0;
  uint64_t accepted = 0;  // calls this thread handed in (stats)
  std::unique_ptr<uint32_t[]> len;
  std::unique_ptr<uint64_t[]> tag, owner;
  std::unique_ptr<uint8_t[]> bytes;
  void lock() {
    while (busy.exchange(true, std::memory_order_acquire))
      while (busy.load(std::memory_order_relaxed)) std::this_thread::yield();
  }
  void unlock() { busy.store(false, std::memory_order_release); }
  Span span() {
    Span s;
    s.k = k;
    s.b = b;
    s.len = len.get();
    s.tag = tag.get();
    s.owner = owner.get();
    s.bytes = bytes.get();
    s.first_ns = first_ns.load(std::memory_order_relaxed);
    return s;
  }
  void clear() {
    k = b = 0;
    first_ns.store(0, std::memory_order_relaxed);
  }
};

}  // namespace

struct emqxgm_async {
  uint64_t id = 0;
  std::vector<emqxgm_t*> hs;
  emqxgm_async_cfg cfg{};
  uint32_t chunk_calls = CHUNK_CALLS, chunk_bytes = CHUNK_BYTES;
  emqxgm_async_cb cb = nullptr;
  void* user = nullptr;
  std::vector<std::unique_ptr<Slot>> slots;
  std::vector<int> free_slots;
  std::vector<std::unique_ptr<Chunk>> chunks;    // registered staging chunks (mu)
  std::atomic<int> open{-1};                     // the slot taking calls, or -1
  std::deque<int> ready;                         // sealed windows, oldest first
  std::vector<std::deque<int>> inflight;         // per handle, in submission order
  std::vector<uint32_t> outstanding;             // per handle: submitted and not yet released
  uint32_t rr = 0;                               // next handle to try
  bool stop = false, flusher_done = false;
  std::atomic<int> flusher_idle{0};              // the flusher sleeps with nothing pending
  std::mutex mu;
  std::condition_variable cv_flush;              // the flusher: work, a pipe free
  std::condition_variable cv_done;               // a window was released (cancel)
  std::vector<std::unique_ptr<std::condition_variable>> cv_comp;  // completer k: work on handle k
  std::thread flusher;
  std::vector<std::thread> completers;
  std::atomic<uint64_t> st_direct{0}, st_busy{0}, st_too_big{0};
  // EMQXGM_ASYNC_PUBLISH: per handle, the bytes of a window's route entries' filters
  std::vector<std::vector<uint8_t>> rf_bytes;
  std::vector<std::vector<uint64_t>> rf_off;
  bool publish_mode() const { return (cfg.flags & EMQXGM_ASYNC_PUBLISH) != 0; }
  bool eager() const { return (cfg.flags & EMQXGM_ASYNC_EAGER) != 0; }
  uint64_t st_windows = 0, st_cancelled = 0, st_errors = 0, st_delivered = 0;
  // health (cfg.fail_threshold > 0): consecutive failures -- pending calls cancelled by callers
  // that timed out, windows that failed -- until every handle is marked stale
  std::atomic<uint32_t> fails{0};
  std::atomic<uint64_t> st_timeouts{0}, st_failed{0}, st_stale{0};
  uint64_t submit_seq = 1;  // the next window's submission number (mu)

  // The handle registry's quiescence (emqxgm_handles_*): mark() = the next submission number;
  // passed(m): every window submitted before the mark has been reported (its pass read whatever
  // epoch it took; later windows take epochs published before the mark)
  uint64_t mark() {
    std::lock_guard<std::mutex> g(mu);
    return submit_seq;
  }
  bool passed(uint64_t m) {
    std::lock_guard<std::mutex> g(mu);
    for (auto& sp : slots)
      if ((sp->state == SUBMITTING || sp->state == INFLIGHT || sp->state == DELIVERING) && sp->seq < m)
        return false;
    return true;
  }

  bool all_stale() const {
    for (emqxgm_t* h : hs)
      if (!gm_stale(h)) return false;
    return true;
  }
  // a pending call cancelled: with health counting on, its caller timed out
  void timed_out() {
    if (!cfg.fail_threshold) return;
    st_timeouts.fetch_add(1, std::memory_order_relaxed);
    note_failure(-ETIMEDOUT);
  }
  void note_failure(int err) {
    if (!cfg.fail_threshold) return;
    if (fails.fetch_add(1) + 1 < cfg.fail_threshold) return;
    fails.store(0);
    for (emqxgm_t* h : hs) (void)emqxgm_mark_stale(h, err);
  }

  // ---- delivery: cfg.deliver_threads > 1 splits a large window's reports over a pool (the
  // caller's per-call work -- the NIF builds each call's terms and enif_sends them -- would
  // otherwise run on the one completer thread of the handle and bound the layer's rate) ----
  struct Part {
    emqxgm_async_window w;          // a view of calls [i0, i1) of the window
    std::atomic<uint32_t>* left;    // parts of the window not yet reported
  };
  std::vector<std::thread> dpool;
  std::mutex dmu;
  std::condition_variable dcv, ddone;
  std::deque<Part> dq;
  bool dstop = false;

  static emqxgm_async_window part_view(const emqxgm_async_window& w, uint32_t i0, uint32_t i1) {
    emqxgm_async_window v = w;
    v.n = i1 - i0;
    v.tag = w.tag + i0;
    v.owner = w.owner + i0;
    if (w.row) v.row = w.row + i0;  // (pair indices stay absolute)
    if (w.exact_id) v.exact_id = w.exact_id + i0;
    if (w.route_ptr) v.route_ptr = w.route_ptr + i0;
    if (w.deliver_ptr) v.deliver_ptr = w.deliver_ptr + i0;
    return v;
  }

  void deliver_loop() {
    std::unique_lock<std::mutex> g(dmu);
    for (;;) {
      while (dq.empty() && !dstop) dcv.wait(g);
      if (dq.empty()) return;
      Part pt = dq.front();
      dq.pop_front();
      g.unlock();
      cb(user, &pt.w);
      g.lock();
      if (pt.left->fetch_sub(1) == 1) ddone.notify_all();
    }
  }

  // Reports window w: in parts over the pool when it is large, the completer taking one part.
  void deliver(const emqxgm_async_window& w) {
    const uint32_t k = std::min<uint32_t>((uint32_t)dpool.size() + 1, w.n / DELIVER_MIN);
    if (k <= 1 || w.status) {
      cb(user, &w);
      return;
    }
    std::atomic<uint32_t> left{k - 1};
    {
      std::lock_guard<std::mutex> g(dmu);
      for (uint32_t p = 1; p < k; ++p)
        dq.push_back(Part{part_view(w, (uint32_t)((uint64_t)w.n * p / k), (uint32_t)((uint64_t)w.n * (p + 1) / k)), &left});
    }
    dcv.notify_all();
    const emqxgm_async_window v0 = part_view(w, 0, (uint32_t)((uint64_t)w.n / k));
    cb(user, &v0);
    std::unique_lock<std::mutex> g(dmu);
    ddone.wait(g, [&] { return left.load() == 0; });
  }

  // Seals slot si (with mu held): no reservation after this one succeeds; the window goes to the
  // ready queue (the flusher submits it once its reservations settled).
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
  bool settled(Slot& s) const { return s.settled.load(std::memory_order_acquire) >= s.reserved; }
  void finish_window(Slot& s) {
    const uint32_t lim = s.limit.load(std::memory_order_relaxed);
    s.n = std::min({s.reserved, lim, cfg.window_topics});
    if (s.n == 0) s.off[0] = 0;  // (off[n] was stored by the last reservation that fit)
  }
  bool pipe_free() const {
    for (uint32_t v : outstanding)
      if (v < EMQXGM_HOST_PIPES) return true;
    return false;
  }

  // Moves span x into the open window (opening / sealing windows as they fill).  0, or -EBUSY
  // (no window to take it: every slot full or in flight), -ESHUTDOWN.  Lock-free except when a
  // window fills or none is open.
  int place(const Span& x) {
    const uint32_t WT = cfg.window_topics, WB = cfg.window_bytes;
    for (;;) {
      const int si = open.load(std::memory_order_acquire);
      if (si < 0) {
        std::lock_guard<std::mutex> g(mu);
        if (stop && flusher_done) return -ESHUTDOWN;
        if (open.load() < 0 && !open_slot()) return -EBUSY;
        continue;
      }
      Slot& s = *slots[si];
      const uint64_t c = s.cursor.fetch_add(((uint64_t)x.k << 32) | x.b, std::memory_order_acq_rel);
      const uint32_t n = (uint32_t)(c >> 32), b0 = (uint32_t)c;
      if (n >= SEAL) {  // sealed: the next window
        std::lock_guard<std::mutex> g(mu);
        if (open.load() == si) seal(si);
        if (open.load() < 0 && !open_slot()) return -EBUSY;
        continue;
      }
      const bool fits = (uint64_t)n + x.k <= WT && (uint64_t)b0 + x.b <= WB;
      if (fits) {
        if (x.b) memcpy(s.bytes + b0, x.bytes, x.b);
        uint32_t o = b0;
        for (uint32_t i = 0; i < x.k; ++i) {
          __atomic_store_n(&s.off[n + i], o, __ATOMIC_RELAXED);
          o += x.len[i];
          s.tag[n + i].store(x.tag[i], std::memory_order_relaxed);
          s.owner[n + i].store(x.owner[i], std::memory_order_relaxed);
        }
        __atomic_store_n(&s.off[n + x.k], o, __ATOMIC_RELAXED);
        const uint64_t xf = x.first_ns ? x.first_ns : mono_ns();
        uint64_t f = s.first_ns.load(std::memory_order_relaxed);
        while ((f == 0 || xf < f) &&
               !s.first_ns.compare_exchange_weak(f, xf, std::memory_order_release)) {
        }
      } else {
        // the first reservation that does not fit bounds the window (no later one can fit:
        // places and bytes are handed out in order)
        uint32_t cur = s.limit.load(std::memory_order_relaxed);
        while (n < cur && !s.limit.compare_exchange_weak(cur, n, std::memory_order_relaxed)) {
        }
      }
      s.settled.fetch_add(x.k, std::memory_order_release);
      const bool full = fits && ((uint64_t)n + x.k == WT || (uint64_t)b0 + x.b == WB);
      if (fits && !full) return 0;
      std::lock_guard<std::mutex> g(mu);
      if (open.load() == si) seal(si);
      if (fits) return 0;
      if (open.load() < 0 && !open_slot()) return -EBUSY;
    }
  }

  Chunk* my_chunk() {
    thread_local std::vector<std::pair<uint64_t, Chunk*>> cache;
    for (auto& e : cache)
      if (e.first == id) return e.second;
    std::unique_ptr<Chunk> c(new (std::nothrow) Chunk());
    if (!c) return nullptr;
    c->len.reset(new (std::nothrow) uint32_t[chunk_calls]);
    c->tag.reset(new (std::nothrow) uint64_t[chunk_calls]);
    c->owner.reset(new (std::nothrow) uint64_t[chunk_calls]);
    c->bytes.reset(new (std::nothrow) uint8_t[chunk_bytes]);
    if (!c->len || !c->tag || !c->owner || !c->bytes) return nullptr;
    Chunk* p = c.get();
    {
      std::lock_guard<std::mutex> g(mu);
      chunks.push_back(std::move(c));
    }
    cache.emplace_back(id, p);  // ids are never reused: a destroyed layer's entry never matches
    return p;
  }

  // Every chunk into the windows (the flusher, before it seals; mu not held).  false: a chunk
  // could not be placed (no window free), it stays staged.
  bool drain_all() {
    std::vector<Chunk*> cs;
    {
      std::lock_guard<std::mutex> g(mu);
      for (auto& c : chunks) cs.push_back(c.get());
    }
    bool ok = true;
    for (Chunk* c : cs) {
      if (c->first_ns.load(std::memory_order_acquire) == 0) continue;
      c->lock();
      if (c->k) {
        if (place(c->span()) == 0) c->clear();
        else ok = false;
      }
      c->unlock();
    }
    return ok;
  }
  // The oldest staged call of any chunk (0: none); mu held.
  uint64_t oldest_staged() const {
    uint64_t f = 0;
    for (auto& c : chunks) {
      const uint64_t x = c->first_ns.load(std::memory_order_seq_cst);
      if (x && (!f || x < f)) f = x;
    }
    return f;
  }

  // Windows grow while every pipe is busy: the window_us timer seals the open window (after
  // draining the staging chunks into it) only when a pipe could take it at once and nothing
  // sealed is waiting, so an idle broker answers within window_us plus a pass, and a loaded one
  // submits windows as large as the pipes' pace allows (sealing on the timer regardless made
  // windows of a few hundred calls queue behind the busy pipes, r04).
  void flusher_loop() {
    // the window_us timer: Linux lets a normal thread's timed waits run up to 50 us late (its
    // timer slack), as long as the timer itself at the default window_us
    (void)prctl(PR_SET_TIMERSLACK, 1000ul, 0ul, 0ul, 0ul);
    std::unique_lock<std::mutex> g(mu);
    const uint64_t W = 1000ull * cfg.window_us;
    bool drain_blocked = false;  // staged calls found no window: wait for a release
    for (;;) {
      // Staged calls older than window_us go into the open window now, whether or not a pipe is
      // free: a publisher thread whose chunk stopped filling (its processes all waiting) left
      // them there until the next timer seal, which waits for an idle pipe (r04: p99 ~3 ms under
      // load).  The window itself still seals by size, or by the timer when a pipe is free.
      const uint64_t fc0 = oldest_staged();
      if (fc0 != 0 && !drain_blocked && mono_ns() >= fc0 + W) {
        g.unlock();
        drain_blocked = !drain_all();
        g.lock();
      }
      const int oi = open.load(std::memory_order_acquire);
      const uint64_t fw = oi >= 0 ? slots[oi]->first_ns.load(std::memory_order_acquire) : 0;
      const uint64_t fc = oldest_staged();
      const uint64_t f = (fw && fc) ? std::min(fw, fc) : (fw | fc);
      if (stop || (f != 0 && ready.empty() && pipe_free() && (eager() || mono_ns() >= f + W))) {
        g.unlock();
        const bool drained = drain_all();
        g.lock();
        drain_blocked = !drained;
        const int o2 = open.load();
        if (o2 >= 0 && slots[o2]->cursor.load() != 0) seal(o2);
        if (stop && !drained) {  // staged calls and no window free: wait for a completer
          if (ready.empty()) cv_flush.wait_for(g, std::chrono::microseconds(100));
        }
      }
      bool progressed = false;
      while (!ready.empty()) {
        const uint32_t H = (uint32_t)hs.size();
        // a handle with a pipe free, one whose index is not stale first (a stale one refuses the
        // window: its calls are reported -ESTALE and answered by their callers)
        uint32_t k = H, ks = H;
        for (uint32_t j = 0; j < H; ++j) {
          const uint32_t c = (rr + j) % H;
          if (outstanding[c] >= EMQXGM_HOST_PIPES) continue;
          if (!gm_stale(hs[c])) {
            k = c;
            break;
          }
          if (ks == H) ks = c;
        }
        if (k == H) k = ks;
        if (k == H) break;  // every pipe busy: a completer's release wakes us
        const int si = ready.front();
        Slot& s = *slots[si];
        if (!settled(s)) {  // a caller is still copying its calls in: a moment
          g.unlock();
          std::this_thread::yield();
          g.lock();
          progressed = true;
          break;
        }
        ready.pop_front();
        finish_window(s);
        if (s.n == 0) {  // sealed before any reservation fit
          s.state = FREE;
          free_slots.push_back(si);
          drain_blocked = false;
          progressed = true;
          continue;
        }
        rr = (k + 1) % H;
        s.state = SUBMITTING;
        s.seq = submit_seq++;
        s.hi = k;
        outstanding[k] += 1;
        g.unlock();
        s.flush_ns = mono_ns();
        uint64_t tk = 0;
        // the filter-byte gather and every result copy go behind the pass: one wait (a publish
        // layer's completer runs the whole pass itself)
        const int rc = publish_mode() ? 0 : gm_submit_window(hs[k], s.bytes, s.off, s.n, &tk);
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
      const int o3 = open.load(std::memory_order_acquire);
      const bool window_empty = o3 < 0 || slots[o3]->cursor.load() == 0;
      if (stop && window_empty && ready.empty() && oldest_staged() == 0) break;
      const uint64_t fw2 = o3 >= 0 ? slots[o3]->first_ns.load(std::memory_order_acquire) : 0;
      flusher_idle.store(1, std::memory_order_seq_cst);
      const uint64_t fc2 = oldest_staged();  // (re-read after announcing the idle sleep)
      const uint64_t f2 = (fw2 && fc2) ? std::min(fw2, fc2) : (fw2 | fc2);
      if (f2 != 0) flusher_idle.store(0, std::memory_order_relaxed);
      // the next deadline: the timer seal (a pipe free) or the oldest staged call's drain
      uint64_t due = 0;
      if (f2 != 0 && ready.empty() && pipe_free()) due = eager() ? 1 : f2 + W;  // (1: now)
      if (fc2 != 0 && !drain_blocked && (due == 0 || fc2 + W < due)) due = fc2 + W;
      if (due != 0) {
        const uint64_t t = mono_ns();
        if (due > t) cv_flush.wait_for(g, std::chrono::nanoseconds(due - t));
        drain_blocked = false;  // (a release may have woken us: try again)
      } else {
        // pipes busy (a completer's release wakes us), or nothing pending (a producer's first
        // staged call does)
        cv_flush.wait(g);
        drain_blocked = false;
      }
      flusher_idle.store(0, std::memory_order_relaxed);
    }
    flusher_done = true;
    for (auto& c : cv_comp) c->notify_all();
  }

  // The bytes of every route entry's To of a publish window (one registry copy per window).
  int route_bytes(uint32_t k, const emqxgm_publish_out& po) {
    auto& b = rf_bytes[k];
    auto& o = rf_off[k];
    o.resize(po.n_routes + 1);
    if (b.empty()) b.resize(1u << 16);
    for (;;) {
      const int rc = emqxgm_filters_copy(hs[k], po.route_filter, po.n_routes, b.data(), b.size(), o.data());
      if (rc != -ENOSPC) return rc;
      b.resize(std::max<uint64_t>(o[po.n_routes], 2 * b.size()));
    }
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
      emqxgm_publish_out po{};
      if (rc == 0 && publish_mode()) {
        rc = emqxgm_publish_batch(hs[k], s.bytes, s.off, s.n, &po);
        if (rc == 0) rc = route_bytes(k, po);
      } else if (rc == 0) {
        rc = emqxgm_match_batch_wait_filters(hs[k], s.ticket, &bo, &foff, &fb);
      }
      const uint64_t done = mono_ns();
      if (rc == 0) {
        fails.store(0, std::memory_order_relaxed);
      } else if (rc != -ESTALE) {
        st_failed.fetch_add(1, std::memory_order_relaxed);
        note_failure(rc);
      }
      g.lock();
      inflight[k].pop_front();
      s.state = DELIVERING;  // a cancel() of one of its calls waits for the release below
      g.unlock();
      emqxgm_async_window w{};
      w.status = rc;
      w.n = s.n;
      w.tag = reinterpret_cast<const uint64_t*>(s.tag.get());
      w.owner = reinterpret_cast<const uint64_t*>(s.owner.get());
      if (rc == 0 && publish_mode()) {
        w.n_routes = po.n_routes;
        w.n_deliveries = po.n_deliveries;
        w.route_ptr = po.route_ptr;
        w.route_filter = po.route_filter;
        w.route_dest = po.route_dest;
        w.deliver_ptr = po.deliver_ptr;
        w.deliver_filter = po.deliver_filter;
        w.deliver_sub = po.deliver_sub;
        w.rfoff = rf_off[k].data();
        w.rfbytes = rf_bytes[k].data();
      } else if (rc == 0) {
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
      deliver(w);
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
  a->id = g_layer_ids.fetch_add(1);
  a->hs.assign(hs, hs + n_handles);
  if (cfg) a->cfg = *cfg;
  if (!a->cfg.window_topics) a->cfg.window_topics = 65536;
  if (!a->cfg.window_bytes) a->cfg.window_bytes = 64u * a->cfg.window_topics;
  if (!a->cfg.window_us) a->cfg.window_us = 50;
  if (!a->cfg.queued_windows) a->cfg.queued_windows = 2;
  if (a->cfg.window_topics >= SEAL || a->cfg.window_bytes >= SEAL ||
      (a->cfg.flags & ~(EMQXGM_ASYNC_PUBLISH | EMQXGM_ASYNC_EAGER)) || a->cfg.deliver_threads > 64) {
    delete a;
    return -EINVAL;
  }
  // a chunk always fits an empty window
  a->chunk_calls = std::min(CHUNK_CALLS, a->cfg.window_topics);
  a->chunk_bytes = std::min(CHUNK_BYTES, a->cfg.window_bytes);
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
  // each engine's host pipes at the windows' size now (a reallocation later would stall every
  // pass on the device; a publish layer's passes go through the handle's synchronous context)
  for (uint32_t k = 0; k < n_handles && !rc && !(a->cfg.flags & EMQXGM_ASYNC_PUBLISH); ++k)
    rc = gm_reserve_windows(a->hs[k], a->cfg.window_topics, a->cfg.window_bytes);
  if (rc) {
    for (size_t i = 0; i < a->slots.size(); ++i) {
      emqxgm_host_free(a->hs[i % n_handles], a->slots[i]->bytes);
      emqxgm_host_free(a->hs[i % n_handles], a->slots[i]->off);
    }
    delete a;
    return rc;
  }
  a->inflight.resize(n_handles);
  a->rf_bytes.resize(n_handles);
  a->rf_off.resize(n_handles);
  a->outstanding.assign(n_handles, 0);
  for (uint32_t k = 0; k < n_handles; ++k) a->cv_comp.emplace_back(new std::condition_variable());
  {
    std::lock_guard<std::mutex> g(a->mu);
    a->open_slot();
  }
  for (uint32_t k = 1; k < a->cfg.deliver_threads; ++k) a->dpool.emplace_back([a] { a->deliver_loop(); });
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
  a->flusher.join();  // drains the chunks, seals and submits what is left, wakes the completers
  for (auto& t : a->completers) t.join();  // deliver every accepted call
  {
    std::lock_guard<std::mutex> g(a->dmu);
    a->dstop = true;
  }
  a->dcv.notify_all();
  for (auto& t : a->dpool) t.join();
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
  if (a->all_stale()) {  // no index may answer: the caller's own path (include: "Health")
    a->st_stale.fetch_add(1, std::memory_order_relaxed);
    return -ESTALE;
  }
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
  if (len > a->chunk_bytes) {  // a long topic goes into the window on its own
    Span x;
    x.k = 1;
    x.b = len;
    x.len = &len;
    x.tag = &tag;
    x.owner = &owner;
    x.bytes = topic;
    x.first_ns = mono_ns();
    const int rc = a->place(x);
    if (rc == -EBUSY) a->st_busy.fetch_add(1, std::memory_order_relaxed);
    if (rc == 0) {
      a->st_direct.fetch_add(1, std::memory_order_relaxed);
      // the window may have been empty and the flusher asleep with no deadline: it arms the
      // window_us timer for this call, as a chunk's first call does
      if (a->flusher_idle.load(std::memory_order_seq_cst)) {
        std::lock_guard<std::mutex> g(a->mu);
        a->cv_flush.notify_one();
      }
    }
    return rc;
  }
  Chunk* c = a->my_chunk();
  if (!c) return -ENOMEM;
  c->lock();
  if (c->k == a->chunk_calls || c->b + len > a->chunk_bytes) {
    const int rc = a->place(c->span());
    if (rc) {
      c->unlock();
      if (rc == -EBUSY) a->st_busy.fetch_add(1, std::memory_order_relaxed);
      return rc;  // every window full or in flight: the caller answers this one itself
    }
    c->clear();
  }
  const uint32_t i = c->k;
  if (len) memcpy(c->bytes.get() + c->b, topic, len);
  c->len[i] = len;
  c->tag[i] = tag;
  c->owner[i] = owner;
  c->k = i + 1;
  c->b += len;
  c->accepted += 1;
  const bool first = i == 0;
  if (first) c->first_ns.store(mono_ns(), std::memory_order_seq_cst);
  c->unlock();
  // the chunk's first call: an idle flusher arms its window_us timer
  if (first && a->flusher_idle.load(std::memory_order_seq_cst)) {
    std::lock_guard<std::mutex> g(a->mu);
    a->cv_flush.notify_one();
  }
  return 0;
}

int emqxgm_async_cancel(emqxgm_async_t* a, uint64_t tag, uint64_t owner) {
  if (!a || tag == EMQXGM_TAG_CANCELLED) return -EINVAL;
  // staged calls first, without the layer's mutex (a producer holds its chunk's lock while it
  // places the chunk, which may take the mutex).  A call only ever moves from a chunk into a
  // window, under the chunk's lock: if this scan misses it, the window scan below finds it.
  std::vector<Chunk*> cs;
  {
    std::lock_guard<std::mutex> g(a->mu);
    for (auto& c : a->chunks) cs.push_back(c.get());
  }
  for (Chunk* c : cs) {
    c->lock();
    for (uint32_t j = 0; j < c->k; ++j)
      if (c->tag[j] == tag && c->owner[j] == owner) {
        c->tag[j] = EMQXGM_TAG_CANCELLED;  // still matched, never reported
        c->unlock();
        {
          std::lock_guard<std::mutex> g(a->mu);
          a->st_cancelled += 1;
        }
        a->timed_out();
        return 1;
      }
    c->unlock();
  }
  std::unique_lock<std::mutex> g(a->mu);
  int delivering = -1;
  for (size_t i = 0; i < a->slots.size() && delivering < 0; ++i) {
    Slot& s = *a->slots[i];
    if (s.state == FREE) continue;
    // an open window's calls: the reservations so far that fit (the caller's own call is
    // complete); a sealed one's: those made before the seal that fit.  Places past them hold
    // tags of earlier uses of the slot.
    const uint32_t lim = std::min(s.limit.load(), a->cfg.window_topics);
    const uint32_t m = s.state == OPEN    ? std::min<uint32_t>((uint32_t)(s.cursor.load() >> 32), lim)
                       : s.state == READY ? std::min<uint32_t>(s.reserved, lim)
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
      g.unlock();
      a->timed_out();
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
  std::vector<Chunk*> cs;
  {
    std::lock_guard<std::mutex> g(a->mu);
    for (auto& c : a->chunks) cs.push_back(c.get());
  }
  uint64_t calls = a->st_direct.load();
  for (Chunk* c : cs) {  // (chunk locks never taken under the mutex: see cancel)
    c->lock();
    calls += c->accepted;
    c->unlock();
  }
  std::lock_guard<std::mutex> g(a->mu);
  out[0] = calls;
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

// ---- the handle registry (include/emqx_gpumatch.h "Handle registry") ----
struct emqxgm_handles {
  std::mutex mu;
  std::vector<emqxgm_async*> layers;
  struct Kind {
    uint32_t next = 0;                 // numbers made so far
    std::vector<uint32_t> free_;       // released and quiesced: reused first
    struct Limbo {
      uint32_t h;
      std::vector<uint64_t> marks;     // each layer's mark at the release
    };
    std::deque<Limbo> limbo;           // released, windows from before the release in flight
    std::vector<uint8_t> live;         // per number: 1 allocated, 0 not
    uint64_t n_live = 0;
  } k[EMQXGM_HANDLE_KINDS];

  // limbo entries whose marks every layer has passed become free (in release order: marks only
  // grow, so the first entry not passed stops the scan)
  void promote(Kind& K) {
    while (!K.limbo.empty()) {
      const auto& e = K.limbo.front();
      for (size_t i = 0; i < layers.size(); ++i)
        if (!layers[i]->passed(e.marks[i])) return;
      K.free_.push_back(e.h);
      K.limbo.pop_front();
    }
  }
};

extern "C" {

int emqxgm_handles_create(emqxgm_async_t* const* layers, uint32_t n_layers, emqxgm_handles_t** out) {
  if (!out || (n_layers && !layers)) return -EINVAL;
  *out = nullptr;
  emqxgm_handles* r = new (std::nothrow) emqxgm_handles();
  if (!r) return -ENOMEM;
  for (uint32_t i = 0; i < n_layers; ++i) {
    if (!layers[i]) {
      delete r;
      return -EINVAL;
    }
    r->layers.push_back(layers[i]);
  }
  *out = r;
  return 0;
}

void emqxgm_handles_destroy(emqxgm_handles_t* r) { delete r; }

int emqxgm_handles_alloc(emqxgm_handles_t* r, uint32_t kind, uint32_t* handle) {
  if (!r || !handle || kind >= EMQXGM_HANDLE_KINDS) return -EINVAL;
  std::lock_guard<std::mutex> g(r->mu);
  auto& K = r->k[kind];
  if (K.free_.empty()) r->promote(K);
  uint32_t h;
  if (!K.free_.empty()) {
    h = K.free_.back();
    K.free_.pop_back();
  } else {
    if (K.next >= EMQXGM_HANDLE_MAX) return -E2BIG;
    h = K.next++;
    K.live.push_back(0);
  }
  K.live[h] = 1;
  K.n_live += 1;
  *handle = h;
  return 0;
}

int emqxgm_handles_release(emqxgm_handles_t* r, uint32_t kind, uint32_t handle) {
  if (!r || kind >= EMQXGM_HANDLE_KINDS) return -EINVAL;
  std::lock_guard<std::mutex> g(r->mu);
  auto& K = r->k[kind];
  if (handle >= K.next || !K.live[handle]) return -ENOENT;
  K.live[handle] = 0;
  K.n_live -= 1;
  emqxgm_handles::Kind::Limbo e;
  e.h = handle;
  for (emqxgm_async* a : r->layers) e.marks.push_back(a->mark());
  K.limbo.push_back(std::move(e));
  r->promote(K);
  return 0;
}

int emqxgm_handles_reset(emqxgm_handles_t* r) {
  if (!r) return -EINVAL;
  std::lock_guard<std::mutex> g(r->mu);
  std::vector<uint64_t> marks;
  for (emqxgm_async* a : r->layers) marks.push_back(a->mark());
  for (auto& K : r->k) {
    for (uint32_t h = 0; h < K.next; ++h)
      if (K.live[h]) {
        K.live[h] = 0;
        K.limbo.push_back(emqxgm_handles::Kind::Limbo{h, marks});
      }
    K.n_live = 0;
    r->promote(K);
  }
  return 0;
}

int emqxgm_handles_stats(emqxgm_handles_t* r, uint32_t kind, uint64_t out[4]) {
  if (!r || !out || kind >= EMQXGM_HANDLE_KINDS) return -EINVAL;
  std::lock_guard<std::mutex> g(r->mu);
  auto& K = r->k[kind];
  out[0] = K.next;
  out[1] = K.n_live;
  out[2] = K.limbo.size();
  out[3] = K.free_.size();
  return 0;
}

int emqxgm_async_health(emqxgm_async_t* a, uint64_t out[4]) {
  if (!a || !out) return -EINVAL;
  uint64_t n = 0;
  for (emqxgm_t* h : a->hs) n += gm_stale(h) ? 1 : 0;
  out[0] = n;
  out[1] = a->st_timeouts.load();
  out[2] = a->st_failed.load();
  out[3] = a->st_stale.load();
  return (int)n;
}

}  // extern "C"
