// async_load.cpp -- TEST / BENCH INFRASTRUCTURE: publisher threads driving the concurrent publish
// entry (emqxgm_async_*, include/emqx_gpumatch.h) of the real engine, as the NIF's callers do.
//
// The reference matches each publish in the publisher's own process, all schedulers at once
// (emqx_broker:publish/1 -> emqx_router:match_routes/1 -> emqx_trie:match/1,
// apps/emqx/src/emqx_broker.erl:218-232).  Here T threads stand for T schedulers; each runs P
// publisher "processes": a thread makes one emqxgm_async_match call per topic (one topic a call,
// never batched by the caller) while fewer than P of its calls are outstanding, and a call ends
// when the engine's callback reports it -- call -> result latency is measured per call.
//
// Per call it can record the topic index, the number of trie filters, an order-independent hash
// of their bytes (sum of mix(fnv1a64(filter))) and whether the topic is a route key, so that
// tests/test_gpu_async.py checks every call's answer against the oracle.
//
// Built by __graft_entry__.build() / tests (g++ -shared), linked against the in-tree
// emqx_amd/libemqx_gpumatch.so.
#include <errno.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/emqx_gpumatch.h"

namespace {

uint64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

uint64_t fnv1a(const uint8_t* p, uint32_t n) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (uint32_t i = 0; i < n; ++i) h = (h ^ p[i]) * 0x100000001b3ull;
  return h;
}

// A publisher thread ("scheduler"): its calls outstanding, and where it sleeps when it has P of
// them (a BEAM scheduler whose processes all wait in receive sleeps too; spinning threads would
// take the CPUs the engine's flusher and completer threads need).
struct Pub {
  std::atomic<int64_t> outstanding{0};
  std::mutex m;
  std::condition_variable cv;
};

struct Load {
  uint64_t calls_per_thread = 0;
  std::vector<uint64_t> t0;               // per call: when it was made
  std::vector<uint32_t> lat_us;           // per call: call -> result
  Pub* pubs = nullptr;
  uint32_t threads = 0;
  uint32_t* out_count = nullptr;
  uint64_t* out_hash = nullptr;
  uint8_t* out_exact = nullptr;
  uint32_t report_ns = 0;                 // per call: work standing for the NIF's terms + enif_send
  std::atomic<uint64_t> reported{0}, failed{0};
};

void on_window(void* user, const emqxgm_async_window* w) {
  Load* L = (Load*)user;
  const uint64_t now0 = mono_ns();  // (one clock read per window unless each report costs time)
  // reports per publisher thread, released once per window (one wake-up, not one per call)
  thread_local std::vector<uint32_t> done;
  done.assign(L->threads, 0);
  for (uint32_t i = 0; i < w->n; ++i) {
    const uint64_t c = w->tag[i];
    if (c == EMQXGM_TAG_CANCELLED) continue;
    if (w->status) {
      L->failed++;
    } else if (L->out_count) {
      uint64_t h = 0;
      for (uint32_t j = w->row[i]; j < w->row[i + 1]; ++j)
        h += mix64(fnv1a(w->fbytes + w->foff[j], w->foff[j + 1] - w->foff[j]));
      L->out_count[c] = w->row[i + 1] - w->row[i];
      L->out_hash[c] = h;
      L->out_exact[c] = w->exact_id[i] != EMQXGM_NONE;
    }
    if (L->report_ns) {  // a model of the NIF's per-call report (built terms, a message send)
      const uint64_t until = mono_ns() + L->report_ns;
      while (mono_ns() < until) {
      }
    }
    const uint64_t now = L->report_ns ? mono_ns() : now0;
    L->lat_us[c] = (uint32_t)std::min<uint64_t>((now - L->t0[c]) / 1000, 0xFFFFFFFFu);
    done[w->owner[i]] += 1;
  }
  uint64_t total = 0;
  for (uint32_t k = 0; k < L->threads; ++k) {
    if (!done[k]) continue;
    total += done[k];
    Pub& p = L->pubs[k];
    p.outstanding.fetch_sub(done[k], std::memory_order_release);
    { std::lock_guard<std::mutex> g(p.m); }
    p.cv.notify_one();
  }
  L->reported += total;
}

}  // namespace

extern "C" {

// out_stats: [0] seconds, [1] calls, [2] p50 us, [3] p99 us, [4] p999 us, [5] windows,
// [6] -EBUSY retries, [7] failed calls, [8] mean calls per window, [9] max us
int async_load_run(emqxgm_t* const* hs, uint32_t nh, const emqxgm_async_cfg* cfg,
                   const uint8_t* tb, const uint64_t* toff, uint64_t n_topics, uint32_t threads,
                   uint32_t procs, uint64_t calls_per_thread, uint32_t* out_topic,
                   uint32_t* out_count, uint64_t* out_hash, uint8_t* out_exact,
                   double* out_stats, uint32_t report_ns) {
  if (!hs || !nh || !tb || !toff || !n_topics || !threads || !procs || !out_stats) return -EINVAL;
  Load L;
  const uint64_t total = (uint64_t)threads * calls_per_thread;
  L.calls_per_thread = calls_per_thread;
  L.t0.assign(total, 0);
  L.lat_us.assign(total, 0);
  std::vector<Pub> pubs(threads);
  L.pubs = pubs.data();
  L.threads = threads;
  L.out_count = out_count;
  L.out_hash = out_hash;
  L.out_exact = out_exact;
  L.report_ns = report_ns;
  emqxgm_async_t* a = nullptr;
  int rc = emqxgm_async_create(hs, nh, cfg, on_window, &L, &a);
  if (rc) return rc;
  std::atomic<uint64_t> busy{0};
  std::atomic<int> err{0};
  const uint64_t t_start = mono_ns();
  std::vector<std::thread> th;
  for (uint32_t k = 0; k < threads; ++k) {
    th.emplace_back([&, k] {
      Pub& p = pubs[k];
      for (uint64_t i = 0; i < calls_per_thread; ++i) {
        const uint64_t c = (uint64_t)k * calls_per_thread + i;
        const uint64_t t = c % n_topics;
        if (out_topic) out_topic[c] = (uint32_t)t;
        if (p.outstanding.load(std::memory_order_acquire) >= (int64_t)procs) {
          std::unique_lock<std::mutex> g(p.m);
          p.cv.wait(g, [&] { return p.outstanding.load(std::memory_order_acquire) < (int64_t)procs; });
        }
        p.outstanding.fetch_add(1, std::memory_order_relaxed);
        L.t0[c] = mono_ns();
        for (;;) {
          const int r = emqxgm_async_match(a, tb + toff[t], (uint32_t)(toff[t + 1] - toff[t]), c, k);
          if (r == 0) break;
          if (r != -EBUSY) {
            err.store(r);
            p.outstanding.fetch_sub(1);
            break;
          }
          // every window full or in flight: sleep until one of this thread's calls is reported
          // (or a moment, when none is outstanding)
          busy++;
          const int64_t before = p.outstanding.load();
          std::unique_lock<std::mutex> g(p.m);
          p.cv.wait_for(g, std::chrono::microseconds(50),
                        [&] { return p.outstanding.load() < before; });
        }
        if (err.load()) return;
      }
    });
  }
  for (auto& x : th) x.join();
  // every call made: wait for the last reports (window_us at most, then a pass), then count
  const uint64_t deadline = mono_ns() + 10000000000ull;
  while (!err.load() && L.reported.load() < total && mono_ns() < deadline) std::this_thread::yield();
  const double secs = (mono_ns() - t_start) * 1e-9;
  uint64_t st[8] = {0};
  emqxgm_async_stats(a, st);
  emqxgm_async_destroy(a);  // reports whatever is left
  if (err.load()) return err.load();
  if (L.reported.load() != total) return -ETIMEDOUT;
  std::vector<uint32_t> lat(L.lat_us);
  std::sort(lat.begin(), lat.end());
  auto pct = [&](double p) { return lat.empty() ? 0.0 : (double)lat[std::min<size_t>(lat.size() - 1, (size_t)(p * lat.size()))]; };
  out_stats[0] = secs;
  out_stats[1] = (double)L.reported.load();
  out_stats[2] = pct(0.50);
  out_stats[3] = pct(0.99);
  out_stats[4] = pct(0.999);
  out_stats[5] = (double)st[1];
  out_stats[6] = (double)busy.load();
  out_stats[7] = (double)L.failed.load();
  out_stats[8] = st[1] ? (double)st[0] / (double)st[1] : 0.0;
  out_stats[9] = lat.empty() ? 0.0 : (double)lat.back();
  return 0;
}

}  // extern "C"
