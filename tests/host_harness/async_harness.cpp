// async_harness.cpp -- TEST INFRASTRUCTURE: the concurrent publish entry (emqx_amd/csrc/
// gm_async.cpp) under ThreadSanitizer / AddressSanitizer on the CPU.
//
// gm_async.cpp is a layer over four engine entry points (emqxgm_host_alloc / _free,
// emqxgm_match_batch_submit_filters / _wait_filters).  Here they are a mock engine whose
// "device pass" is the oracle's C++ restatement of emqx_trie:match/1 + the route-key lookup
// (oracle/ref_trie.cpp, emqx_trie.erl:282-348, emqx_router.erl:141-146), with the real engine's
// contract enforced: at most EMQXGM_HOST_PIPES tickets in flight per handle (-EBUSY beyond), a
// result's buffers valid only until ticket + EMQXGM_HOST_PIPES is submitted (the mock then
// poisons them, so a layer that reads a released result reports garbage and fails the check),
// and waits that take a random while.
//
// T publisher threads call emqxgm_async_match one topic at a time with a bounded number of
// calls outstanding each (their "processes"), cancel some of them, and check in the callback:
// every reported call's filter set and exact hit equal the oracle's for its topic; every accepted
// call is reported exactly once unless its cancel returned 1, and never after a cancel that
// returned 1.  Prints "OK <calls> <windows> <cancelled> <busy>".
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/emqx_gpumatch.h"
#include "../../emqx_amd/csrc/gm_internal.h"

extern "C" {
void* ref_create(int compact);
void ref_destroy(void* h);
int ref_add_many(void* h, const uint8_t* bytes, const uint64_t* off, uint64_t n, const uint8_t* kind);
int ref_match_batch(void* h, const uint8_t* tb, const uint32_t* toff, uint64_t n, int threads,
                    uint64_t* row, uint32_t** ids_out, uint64_t* n_ids, uint32_t* exact);
void ref_free(void* p);
}

#define CHECK(c, ...)                                             \
  do {                                                            \
    if (!(c)) {                                                   \
      fprintf(stderr, "FAIL %s:%d: %s: ", __FILE__, __LINE__, #c); \
      fprintf(stderr, __VA_ARGS__);                               \
      fprintf(stderr, "\n");                                      \
      abort();                                                    \
    }                                                             \
  } while (0)

namespace {

std::vector<std::string> g_filters;  // oracle ids = registration order
void* g_ref = nullptr;
std::mutex g_ref_mu;  // ref_match_batch is a reader, but keep the oracle single-threaded

struct MockPipe {
  uint64_t ticket = 0;
  int state = 0;  // 0 free / taken, 1 in flight
  std::vector<uint32_t> row, fid, exact, foff;
  std::vector<uint8_t> fb;
};

}  // namespace

struct emqxgm {
  std::mutex mu;
  MockPipe p[EMQXGM_HOST_PIPES];
  uint64_t next = 1;
  std::atomic<uint64_t> busy{0};
  std::atomic<int> stale{0};     // the engine's health mark (emqxgm_mark_stale)
  std::atomic<int> hang_us{0};   // health mode: waits stall this long (a hung device)
};

extern "C" {

void* emqxgm_host_alloc(emqxgm_t*, uint64_t bytes) { return malloc(bytes ? bytes : 1); }
int emqxgm_mark_stale(emqxgm_t* h, int) {
  h->stale.store(1);
  return 0;
}
void emqxgm_host_free(emqxgm_t*, void* p) { free(p); }

int emqxgm_match_batch_submit_filters(emqxgm_t* h, const uint8_t* bytes, const uint32_t* off,
                                      uint32_t n, uint64_t* ticket) {
  if (h->stale.load()) return -ESTALE;  // the real engine refuses a stale index's windows
  std::lock_guard<std::mutex> g(h->mu);
  const uint64_t tk = h->next;
  MockPipe& p = h->p[tk % EMQXGM_HOST_PIPES];
  if (p.state == 1) {
    h->busy++;
    return -EBUSY;
  }
  // the previous result of this pipe is overwritten now: poison it first (a reader of a released
  // result then sees garbage)
  std::fill(p.row.begin(), p.row.end(), 0xDEADBEEFu);
  std::fill(p.fid.begin(), p.fid.end(), 0xDEADBEEFu);
  std::fill(p.foff.begin(), p.foff.end(), 0xDEADBEEFu);
  std::fill(p.fb.begin(), p.fb.end(), (uint8_t)0xEE);
  CHECK(off[0] == 0, "offsets[0]");
  std::vector<uint64_t> row(n + 1);
  uint32_t* ids = nullptr;
  uint64_t nid = 0;
  p.exact.assign(n, 0);
  {
    std::lock_guard<std::mutex> r(g_ref_mu);
    ref_match_batch(g_ref, bytes, off, n, 1, row.data(), &ids, &nid, p.exact.data());
  }
  p.row.assign(row.begin(), row.end());
  p.fid.assign(ids, ids + nid);
  ref_free(ids);
  p.foff.assign(1, 0);
  p.fb.clear();
  for (uint32_t id : p.fid) {
    p.fb.insert(p.fb.end(), g_filters[id].begin(), g_filters[id].end());
    p.foff.push_back((uint32_t)p.fb.size());
  }
  p.ticket = tk;
  p.state = 1;
  h->next += 1;
  *ticket = tk;
  return 0;
}

}  // extern "C"
int gm_stale(emqxgm_t* h) { return h->stale.load(); }
// the engine's buffers sized for the layer's windows (nothing to size in the mock)
int gm_reserve_windows(emqxgm_t* h, uint32_t n, uint64_t) { return h && n ? 0 : -EINVAL; }
// the layer's window submit (gm_engine.cpp skips the offsets check there; the mock checks them)
int gm_submit_window(emqxgm_t* h, const uint8_t* bytes, const uint32_t* off, uint32_t n,
                     uint64_t* ticket) {
  for (uint32_t i = 0; i < n; ++i) CHECK(off[i + 1] >= off[i], "window offsets increase");
  return emqxgm_match_batch_submit_filters(h, bytes, off, n, ticket);
}
extern "C" {

// publish-mode layers (EMQXGM_ASYNC_PUBLISH) are checked on the GPU (tests/test_gpu_async.py)
int emqxgm_publish_batch(emqxgm_t*, const uint8_t*, const uint32_t*, uint32_t, emqxgm_publish_out*) {
  return -EIO;
}
int emqxgm_filters_copy(emqxgm_t*, const uint32_t*, uint64_t, uint8_t*, uint64_t, uint64_t*) {
  return -EIO;
}

std::atomic<int> g_hang{0};  // health mode: every wait blocks while set (a hung device)

int emqxgm_match_batch_wait_filters(emqxgm_t* h, uint64_t ticket, emqxgm_batch_out* out,
                                    const uint32_t** foff, const uint8_t** fbytes) {
  // the "device" takes a while; the layer must not hold its own lock meanwhile
  thread_local std::mt19937 rng(std::hash<std::thread::id>()(std::this_thread::get_id()));
  std::this_thread::sleep_for(std::chrono::microseconds(rng() % 300));
  while (g_hang.load()) std::this_thread::sleep_for(std::chrono::microseconds(200));
  std::lock_guard<std::mutex> g(h->mu);
  MockPipe& p = h->p[ticket % EMQXGM_HOST_PIPES];
  if (ticket == 0 || p.ticket != ticket || p.state != 1) return -ENOENT;
  p.state = 0;
  out->n = (uint32_t)p.exact.size();
  out->n_pairs = (uint32_t)p.fid.size();
  out->row_ptr = p.row.data();
  out->filter_id = p.fid.data();
  out->exact_id = p.exact.data();
  *foff = p.foff.data();
  *fbytes = p.fb.data();
  return 0;
}

}  // extern "C"

namespace {

// per call: its topic index; reported / cancelled flags
struct CallState {
  std::atomic<int> reported{0};
  std::atomic<int> cancelled{0};
  uint32_t topic = 0;
};

std::vector<std::string> g_topics;
std::vector<std::vector<std::string>> g_want;  // sorted filter strings per topic
std::vector<uint32_t> g_want_exact;
std::vector<CallState>* g_calls = nullptr;
std::atomic<uint64_t> g_reported{0};
std::atomic<int64_t>* g_outstanding = nullptr;  // per thread

void on_window(void* user, const emqxgm_async_window* w) {
  (void)user;
  CHECK(w->status == 0, "window status %d", w->status);
  for (uint32_t i = 0; i < w->n; ++i) {
    if (w->tag[i] == EMQXGM_TAG_CANCELLED) continue;
    CallState& c = (*g_calls)[w->tag[i]];
    CHECK(c.cancelled.load() == 0, "call %llu reported after a successful cancel",
          (unsigned long long)w->tag[i]);
    CHECK(c.reported.fetch_add(1) == 0, "call %llu reported twice", (unsigned long long)w->tag[i]);
    std::vector<std::string> got;
    for (uint32_t j = w->row[i]; j < w->row[i + 1]; ++j)
      got.emplace_back((const char*)w->fbytes + w->foff[j], w->foff[j + 1] - w->foff[j]);
    std::sort(got.begin(), got.end());
    CHECK(got == g_want[c.topic], "call %llu topic %u: %zu filters vs %zu",
          (unsigned long long)w->tag[i], c.topic, got.size(), g_want[c.topic].size());
    CHECK((w->exact_id[i] == EMQXGM_NONE) == (g_want_exact[c.topic] == EMQXGM_NONE),
          "exact hit of topic %u", c.topic);
    g_outstanding[w->owner[i]].fetch_sub(1);
    g_reported++;
  }
}

std::string rand_topic(std::mt19937& rng, bool filter) {
  static const char* W[] = {"a", "b", "c", "dd", "eeeeeeeee", "", "$s"};
  const int n = 1 + rng() % 5;
  std::string t;
  for (int i = 0; i < n; ++i) {
    if (i) t += '/';
    const uint32_t r = rng() % (filter ? 9 : 7);
    if (filter && r == 7) t += '+';
    else if (filter && r == 8) {
      t += '#';
      break;
    } else t += W[r == 6 && i ? 0 : r];
  }
  return t;
}

}  // namespace

// Health mode ("a window that never completes"): publishers that wait for
// their answer with a deadline and cancel on timeout, as src/emqx_trie_gpu.erl does.  Phase 1 the
// device answers; phase 2 it hangs (every wait blocks): the first calls time out, and after
// fail_threshold timeouts the layer marks the handles stale and refuses every call at once
// (-ESTALE) -- the bound checked is that no more than the calls in flight at the hang, plus the
// threshold, ever pay a timeout; phase 3 the device answers again and the handles are repaired:
// calls are accepted and answered correctly again.  Prints "OK <accepted> <reported> <cancelled>
// <busy> <too_deep>" like the main mode.
int health_main(unsigned seed, int threads, int handles, uint32_t window) {
  std::mt19937 rng(seed);
  std::vector<emqxgm> engines(handles);
  std::vector<emqxgm_t*> hs;
  for (auto& e : engines) hs.push_back(&e);
  const uint64_t per_phase = 200;
  std::vector<CallState> calls(3 * threads * per_phase);
  g_calls = &calls;
  std::vector<std::atomic<int64_t>> outstanding(threads);
  g_outstanding = outstanding.data();
  emqxgm_async_cfg cfg{};
  cfg.window_topics = window;
  cfg.window_us = 20;
  cfg.fail_threshold = 3;
  emqxgm_async_t* a = nullptr;
  CHECK(emqxgm_async_create(hs.data(), handles, &cfg, on_window, nullptr, &a) == 0, "create");
  std::atomic<uint64_t> accepted{0}, cancelled{0}, busy{0}, refused{0}, timeouts_paid[3];
  for (auto& t : timeouts_paid) t = 0;
  const auto timeout = std::chrono::milliseconds(20);
  auto run_phase = [&](int phase) {
    std::vector<std::thread> th;
    for (int k = 0; k < threads; ++k) {
      th.emplace_back([&, k, phase] {
        std::mt19937 r(seed * 7919 + k + 1000 * phase);
        for (uint64_t i = 0; i < per_phase; ++i) {
          const uint64_t tag = (uint64_t)phase * threads * per_phase + k * per_phase + i;
          CallState& c = calls[tag];
          c.topic = r() % g_topics.size();
          const std::string& t = g_topics[c.topic];
          outstanding[k].fetch_add(1);
          const int rc = emqxgm_async_match(a, (const uint8_t*)t.data(), (uint32_t)t.size(), tag, k);
          if (rc != 0) {  // the publisher's reference path
            outstanding[k].fetch_sub(1);
            c.cancelled.store(2);
            CHECK(rc == -ESTALE || rc == -EBUSY || rc == -E2BIG, "async_match %d", rc);
            (rc == -ESTALE ? refused : busy)++;
            CHECK(phase == 1 || rc != -ESTALE, "refused -ESTALE in phase %d", phase);
            continue;
          }
          accepted++;
          const auto t0 = std::chrono::steady_clock::now();
          while (c.reported.load() == 0 && std::chrono::steady_clock::now() - t0 < timeout)
            std::this_thread::sleep_for(std::chrono::microseconds(50));
          if (c.reported.load()) continue;
          const int cr = emqxgm_async_cancel(a, tag, k);  // timed out
          CHECK(cr == 0 || cr == 1, "cancel %d", cr);
          if (cr == 1) {
            c.cancelled.store(1);
            cancelled++;
            timeouts_paid[phase]++;
            outstanding[k].fetch_sub(1);
          }
        }
      });
    }
    for (auto& t : th) t.join();
  };
  run_phase(0);
  CHECK(timeouts_paid[0] == 0, "%llu timeouts with a working device",
        (unsigned long long)timeouts_paid[0].load());
  g_hang.store(1);
  run_phase(1);
  uint64_t hv[4];
  CHECK(emqxgm_async_health(a, hv) == handles, "every handle stale after the hang (%llu)",
        (unsigned long long)hv[0]);
  CHECK(refused.load() > 0, "no call refused while the device hung");
  // bounded: the calls in flight when the hang began (one per publisher) and those accepted
  // before the threshold's third timeout
  CHECK(timeouts_paid[1] <= (uint64_t)(2 * threads + cfg.fail_threshold),
        "%llu calls paid a timeout (threads %d)", (unsigned long long)timeouts_paid[1].load(), threads);
  g_hang.store(0);  // the device answers again; the mirror's repair clears the marks
  for (auto& e : engines) e.stale.store(0);
  run_phase(2);
  CHECK(timeouts_paid[2] == 0, "%llu timeouts after the repair",
        (unsigned long long)timeouts_paid[2].load());
  emqxgm_async_destroy(a);
  uint64_t never = 0;
  for (auto& c : calls)
    if (c.cancelled.load() == 0 && c.reported.load() != 1) ++never;
  CHECK(never == 0, "%llu accepted calls never reported", (unsigned long long)never);
  CHECK(g_reported.load() + cancelled.load() == accepted.load(), "report count");
  fprintf(stderr, "timeouts paid %llu, refused %llu\n", (unsigned long long)timeouts_paid[1].load(),
          (unsigned long long)refused.load());
  printf("OK %llu %llu %llu %llu %llu\n", (unsigned long long)accepted.load(),
         (unsigned long long)g_reported.load(), (unsigned long long)cancelled.load(),
         (unsigned long long)busy.load(), 0ull);
  return 0;
}

// Handles mode: the handle registry over a real layer.  A number released
// while a window submitted before the release is still in flight (the device hangs) is not handed
// out again; once that window has been reported it is.  Prints "OK ..." like the main mode.
int handles_main() {
  emqxgm e;
  emqxgm_t* hs[1] = {&e};
  g_calls = new std::vector<CallState>(4);
  std::vector<std::atomic<int64_t>> outstanding(1);
  g_outstanding = outstanding.data();
  emqxgm_async_cfg cfg{};
  cfg.window_topics = 64;
  cfg.window_us = 20;
  emqxgm_async_t* a = nullptr;
  CHECK(emqxgm_async_create(hs, 1, &cfg, on_window, nullptr, &a) == 0, "create");
  emqxgm_handles_t* r = nullptr;
  CHECK(emqxgm_handles_create(&a, 1, &r) == 0, "handles_create");
  uint32_t h0, h1, h2, h3;
  CHECK(emqxgm_handles_alloc(r, 2, &h0) == 0 && emqxgm_handles_alloc(r, 2, &h1) == 0, "alloc");
  CHECK(h0 == 0 && h1 == 1, "fresh numbers %u %u", h0, h1);
  g_hang.store(1);
  (*g_calls)[0].topic = 0;
  outstanding[0].fetch_add(1);
  const std::string& t = g_topics[0];
  CHECK(emqxgm_async_match(a, (const uint8_t*)t.data(), (uint32_t)t.size(), 0, 0) == 0, "match");
  // wait until the window is submitted (its wait is blocked on the hang)
  uint64_t st[8];
  for (int i = 0; i < 2000; ++i) {
    emqxgm_async_stats(a, st);
    if (st[1] >= 1) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  CHECK(st[1] >= 1, "the window was never submitted");
  CHECK(emqxgm_handles_release(r, 2, h0) == 0, "release");
  CHECK(emqxgm_handles_release(r, 2, h0) == -ENOENT, "double release");
  CHECK(emqxgm_handles_alloc(r, 2, &h2) == 0 && h2 == 2, "a number released under a window in "
        "flight was reused: %u", h2);
  uint64_t hv[4];
  emqxgm_handles_stats(r, 2, hv);
  CHECK(hv[0] == 3 && hv[1] == 2 && hv[2] == 1 && hv[3] == 0, "stats %llu %llu %llu %llu",
        (unsigned long long)hv[0], (unsigned long long)hv[1], (unsigned long long)hv[2],
        (unsigned long long)hv[3]);
  g_hang.store(0);
  while ((*g_calls)[0].reported.load() == 0) std::this_thread::sleep_for(std::chrono::milliseconds(1));
  // reported: released before the report's release of its slot?  wait for the slot to free
  for (int i = 0; i < 2000; ++i) {
    emqxgm_async_stats(a, st);
    if (st[7] == 0) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  CHECK(emqxgm_handles_alloc(r, 2, &h3) == 0 && h3 == h0, "the quiesced number %u was not reused "
        "(got %u)", h0, h3);
  CHECK(emqxgm_handles_reset(r) == 0, "reset");
  emqxgm_handles_stats(r, 2, hv);
  CHECK(hv[1] == 0 && hv[0] == 3, "after reset %llu live", (unsigned long long)hv[1]);
  emqxgm_handles_destroy(r);
  emqxgm_async_destroy(a);
  delete g_calls;
  printf("OK 1 1 0 0 0\n");
  return 0;
}

int main(int argc, char** argv) {
  const unsigned seed = argc > 1 ? atoi(argv[1]) : 1;
  const int threads = argc > 2 ? atoi(argv[2]) : 16;
  const int handles = argc > 3 ? atoi(argv[3]) : 2;
  const uint32_t window = argc > 4 ? atoi(argv[4]) : 64;
  const uint64_t calls_per_thread = argc > 5 ? atoll(argv[5]) : 3000;
  const uint32_t cancel_every = argc > 6 ? (uint32_t)atoi(argv[6]) : 17;  // 0: no cancels
  const bool health = argc > 7 && strcmp(argv[7], "health") == 0;
  std::mt19937 rng(seed);
  // the index: random filters (trie + route keys) and some exact keys
  std::vector<uint8_t> fb;
  std::vector<uint64_t> fo{0};
  std::vector<uint8_t> kind;
  std::unordered_map<std::string, int> seen;
  for (int i = 0; i < 400; ++i) {
    std::string f = rand_topic(rng, true);
    if (seen.count(f)) continue;
    seen[f] = 1;
    const bool wild = f.find('+') != std::string::npos || f.find('#') != std::string::npos;
    g_filters.push_back(f);
    fb.insert(fb.end(), f.begin(), f.end());
    fo.push_back(fb.size());
    kind.push_back(wild ? 3 : 2);
  }
  g_ref = ref_create(1);
  ref_add_many(g_ref, fb.data(), fo.data(), g_filters.size(), kind.data());
  for (int i = 0; i < 300; ++i) g_topics.push_back(rand_topic(rng, false));
  {  // expected answers, one oracle call per topic
    std::vector<uint8_t> tb;
    std::vector<uint32_t> to{0};
    for (auto& t : g_topics) {
      tb.insert(tb.end(), t.begin(), t.end());
      to.push_back((uint32_t)tb.size());
    }
    std::vector<uint64_t> row(g_topics.size() + 1);
    uint32_t* ids = nullptr;
    uint64_t nid = 0;
    g_want_exact.assign(g_topics.size(), 0);
    ref_match_batch(g_ref, tb.data(), to.data(), g_topics.size(), 1, row.data(), &ids, &nid,
                    g_want_exact.data());
    for (size_t t = 0; t < g_topics.size(); ++t) {
      std::vector<std::string> v;
      for (uint64_t j = row[t]; j < row[t + 1]; ++j) v.push_back(g_filters[ids[j]]);
      std::sort(v.begin(), v.end());
      g_want.push_back(v);
    }
    ref_free(ids);
  }
  if (argc > 7 && strcmp(argv[7], "handles") == 0) {
    const int rc = handles_main();
    ref_destroy(g_ref);
    return rc;
  }
  if (health) {
    const int rc = health_main(seed, threads, handles, window);
    ref_destroy(g_ref);
    return rc;
  }
  std::vector<emqxgm> engines(handles);
  std::vector<emqxgm_t*> hs;
  for (auto& e : engines) hs.push_back(&e);
  std::vector<CallState> calls(threads * calls_per_thread);
  g_calls = &calls;
  std::vector<std::atomic<int64_t>> outstanding(threads);
  g_outstanding = outstanding.data();
  emqxgm_async_cfg cfg{};
  cfg.window_topics = window;
  cfg.window_bytes = 64 * window;
  cfg.window_us = 20 + seed % 100;
  cfg.max_levels = 4;
  cfg.deliver_threads = 1 + seed % 4;  // windows reported in parts by a pool (GM_DELIVER_MIN=4)
  cfg.flags = seed % 2 == 0 ? EMQXGM_ASYNC_EAGER : 0u;  // even seeds: windows out as pipes free
  emqxgm_async_t* a = nullptr;
  CHECK(emqxgm_async_create(hs.data(), handles, &cfg, on_window, nullptr, &a) == 0, "create");
  std::atomic<uint64_t> accepted{0}, cancelled{0}, busy{0}, too_deep{0};
  const auto t_start = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int k = 0; k < threads; ++k) {
    th.emplace_back([&, k] {
      std::mt19937 r(seed * 7919 + k);
      const int64_t procs = 1 + r() % 48;  // this "scheduler"'s publisher processes
      for (uint64_t i = 0; i < calls_per_thread; ++i) {
        const uint64_t tag = k * calls_per_thread + i;
        CallState& c = calls[tag];
        c.topic = r() % g_topics.size();
        while (outstanding[k].load() >= procs) std::this_thread::yield();
        outstanding[k].fetch_add(1);
        const std::string& t = g_topics[c.topic];
        const int rc = emqxgm_async_match(a, (const uint8_t*)t.data(), (uint32_t)t.size(), tag, k);
        if (rc == -EBUSY || rc == -E2BIG) {
          outstanding[k].fetch_sub(1);
          c.cancelled.store(2);  // never accepted
          (rc == -EBUSY ? busy : too_deep)++;
          if (rc == -E2BIG) {
            const long levels = std::count(t.begin(), t.end(), '/') + 1;
            CHECK(levels > 4, "E2BIG for a %ld-level topic", levels);
          }
          continue;
        }
        CHECK(rc == 0, "async_match %d", rc);
        accepted++;
        if (cancel_every && r() % cancel_every == 0) {  // a caller that gives up at once
          // mark first: the callback must not report it once the cancel succeeds
          const int cr = emqxgm_async_cancel(a, tag, k);
          CHECK(cr == 0 || cr == 1, "cancel %d", cr);
          if (cr == 1) {
            c.cancelled.store(1);
            cancelled++;
            outstanding[k].fetch_sub(1);
          } else {
            CHECK(c.reported.load() == 1, "cancel returned 0 but call %llu not reported",
                  (unsigned long long)tag);
          }
        }
      }
    });
  }
  for (auto& t : th) t.join();
  emqxgm_async_destroy(a);  // reports every accepted call
  uint64_t never = 0;
  for (auto& c : calls) {
    if (c.cancelled.load() == 2) continue;
    if (c.cancelled.load() == 1) {
      CHECK(c.reported.load() == 0, "cancelled call reported");
      continue;
    }
    if (c.reported.load() != 1) ++never;
  }
  CHECK(never == 0, "%llu accepted calls never reported", (unsigned long long)never);
  CHECK(g_reported.load() + cancelled.load() == accepted.load(), "report count");
  uint64_t eb = 0;
  for (auto& e : engines) eb += e.busy.load();
  CHECK(eb == 0, "the layer overran a handle's pipes (%llu -EBUSY)", (unsigned long long)eb);
  ref_destroy(g_ref);
  fprintf(stderr, "calls/s %.0f\n", accepted.load() / std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count());
  printf("OK %llu %llu %llu %llu %llu\n", (unsigned long long)accepted.load(),
         (unsigned long long)g_reported.load(), (unsigned long long)cancelled.load(),
         (unsigned long long)busy.load(), (unsigned long long)too_deep.load());
  return 0;
}
