// bg_harness.cpp -- TEST INFRASTRUCTURE: subscribe-then-publish visibility while full builds run
// in the background (r05), on the CPU under a sanitizer (tests/test_host_sanitize.py builds it
// with ThreadSanitizer and with ASan + UBSan against the fake HIP runtime).
//
// The reference adds a subscriber's route inside the broker-pool call before SUBACK
// (emqx_broker.erl:163-168, 484-486 -> emqx_router.erl:124-138), so the node's next publish sees
// it.  Here the writing node's hook is emqxgm_route_set_batch(.., EMQXGM_SET_COMMIT).  Every
// check walks the tables of the epoch readers have right after the call returns, on the CPU
// exactly as k_walk does (harness_walk.h), and compares the row with emqx_topic:match/2 over the
// set of filters that must be visible at that moment:
//   A. a bulk subscribe of `bulk` filters commits through emqxgm_commit on another thread; its
//      full build runs in the background (held back by tune "bg_delay_ms").  Meanwhile single
//      subscribes and unsubscribes commit with EMQXGM_SET_COMMIT: each one is visible at once
//      (and the bulk is not, until its commit returns); then everything is.
//   B. a build started because the tables are nearly full (no commit waits for it), with
//      subscribes during it, each visible at once.
//   C. during a build, a batch too large for a delta: that commit waits for the install, which
//      includes it.
// Prints "OK <checks> <bg_builds> <bg_waits> <p50_us> <p99_us>" (latency of the single
// subscribes during builds) on success.
#include <thread>

#include "harness_walk.h"

namespace {

struct Vis {
  emqxgm* h;
  std::set<std::string> vis;  // filters that must be visible (route key + wildcard trie member)
  uint64_t checks = 0;
  std::mt19937_64& rng;
  Vis(emqxgm* hh, std::mt19937_64& r) : h(hh), rng(r) {}

  // the current epoch, and whether every background build started so far is installed in it
  // (read together: installs publish under the writer lock)
  EpochP now(bool& installed) {
    std::lock_guard<std::mutex> w(h->wmu);
    std::lock_guard<std::mutex> g(h->emu);
    installed = h->builds_done >= h->builds_started;
    return h->cur;
  }
  // the row the current epoch gives for topic t (wildcard filters, byte-checked like k_verify),
  // and its exact route key, against the visible set -- plus `pend` once the build in flight is
  // installed
  void check(const std::string& t, const char* what, const std::set<std::string>* pend = nullptr) {
    bool installed = false;
    EpochP e = now(installed);
    std::set<std::string> both;
    const std::set<std::string>* want = &vis;
    if (pend && installed) {
      both = vis;
      both.insert(pend->begin(), pend->end());
      want = &both;
    }
    const DevIndex& ix = e->ix;
    CpuWalk w(ix);
    std::vector<uint32_t> got = w.run(t, h->test_mask);
    std::vector<std::string> gs, ws;
    for (uint32_t f : got) {
      const bool verify = (ix.fvbits[f >> 5] >> (f & 31)) & 1u;
      const std::string fs = filter_str(h, f);
      if (!verify || mqtt_match(t, fs)) gs.push_back(fs);
    }
    if (!is_wild_s(t))  // a wildcard name matches no trie filter (emqx_trie.erl:157-166)
      for (const std::string& f : *want)
        if (is_wild_s(f) && mqtt_match(t, f)) ws.push_back(f);
    std::sort(gs.begin(), gs.end());
    std::sort(ws.begin(), ws.end());
    CHECK(gs == ws, "%s: topic '%s': %zu filters visible, %zu expected", what, t.c_str(), gs.size(),
          ws.size());
    const uint32_t ex = cpu_exact(ix, t, is_wild_s(t));
    const bool wk = want->count(t) > 0;
    CHECK((ex != NONE) == wk, "%s: route key '%s' %s", what, t.c_str(), wk ? "missing" : "present");
    ++checks;
  }
};

}  // namespace

int main(int argc, char** argv) {
  const uint64_t seed = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1;
  // a delta commit takes at most delta_max changes (tune "delta_max"; 0: the default bound)
  const uint32_t delta_max = argc > 2 ? (uint32_t)atoi(argv[2]) : 0;
  const uint32_t bulk = delta_max ? 2 * delta_max : 6000;  // more than a delta takes
  std::mt19937_64 rng(seed);
  auto rnd = [&](uint64_t k) { return (uint64_t)(rng() % k); };
  const char* vocab[] = {"a", "b", "", "c", "dd", "sensor", "long-level-name", "device-0001", "x", "y"};
  auto word = [&]() { return std::string(vocab[rnd(10)]); };
  std::set<std::string> used;
  auto filter = [&]() {
    for (;;) {
      const uint32_t d = 1 + (uint32_t)rnd(5);
      std::string f;
      for (uint32_t i = 0; i < d; ++i) {
        if (i) f += '/';
        const uint64_t r = rnd(100);
        f += (i + 1 == d && r < 20) ? "#" : (r < 35 ? "+" : word() + std::to_string(rnd(40)));
      }
      if (used.insert(f).second) return f;
    }
  };
  // a topic that f matches ('+' a word, '#' zero to two words), or a random one
  auto topic_for = [&](const std::string& f) {
    std::string t;
    size_t a = 0;
    bool first = true;
    for (size_t i = 0; i <= f.size(); ++i) {
      if (i < f.size() && f[i] != '/') continue;
      const std::string w = f.substr(a, i - a);
      a = i + 1;
      if (w == "#") {
        for (uint64_t k = rnd(3); k-- > 0;) t += (first ? "" : "/") + word(), first = false;
        break;
      }
      t += (first ? "" : "/") + (w == "+" ? word() + std::to_string(rnd(40)) : w);
      first = false;
    }
    return t;
  };

  emqxgm_cfg cfg{};
  emqxgm_t* h = nullptr;
  CHECK(emqxgm_create(&cfg, &h) == 0, "create");
  CHECK(emqxgm_tune(h, "bg_build", 1) == 0 && emqxgm_tune(h, "delta_max", delta_max) == 0, "tune");
  Vis V(h, rng);
  std::vector<double> lat_us;
  auto set1 = [&](const std::string& f, bool present) {
    const uint64_t off[2] = {0, f.size()};
    const uint8_t pr = present ? 1 : 0;
    const auto t0 = std::chrono::steady_clock::now();
    CHECK(emqxgm_route_set_batch(h, (const uint8_t*)f.data(), off, &pr, 1, EMQXGM_SET_COMMIT, nullptr) == 0,
          "set_batch: %s", h->err.c_str());
    lat_us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    if (present)
      V.vis.insert(f);
    else
      V.vis.erase(f);
  };
  auto in_flight = [&]() {
    std::lock_guard<std::mutex> g(h->wmu);
    return h->builds_done < h->builds_started;
  };

  // a committed base index
  std::vector<std::string> base;
  for (uint32_t i = 0; i < std::min<uint32_t>(600, bulk / 2); ++i) {
    base.push_back(filter());
    set1(base.back(), true);
  }
  for (int i = 0; i < 30; ++i) V.check(topic_for(base[rnd(base.size())]), "base");

  // ---- A: a bulk subscribe whose full build runs in the background ----
  CHECK(emqxgm_tune(h, "bg_delay_ms", 400) == 0, "tune");
  std::vector<std::string> bulk_f;
  std::string bb;
  std::vector<uint64_t> bo(1, 0);
  for (uint32_t i = 0; i < bulk; ++i) {
    bulk_f.push_back(filter());
    bb += bulk_f.back();
    bo.push_back(bb.size());
  }
  CHECK(emqxgm_route_set_many(h, (const uint8_t*)bb.data(), bo.data(), bulk, 1) == 0, "set_many");
  const std::set<std::string> bulk_s(bulk_f.begin(), bulk_f.end());
  std::atomic<bool> bulk_done{false};
  std::thread committer([&] {
    CHECK(emqxgm_commit(h, nullptr) == 0, "bulk commit: %s", h->err.c_str());
    bulk_done = true;
  });
  for (int k = 0; !in_flight(); ++k) {
    CHECK(!bulk_done && k < 200000, "the bulk commit did not build in the background");
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  int during = 0;
  std::vector<std::string> mine;
  for (int i = 0; i < 200 && !bulk_done; ++i) {
    if (!mine.empty() && rnd(4) == 0) {  // an unsubscribe: gone from the next publish on
      const size_t k = rnd(mine.size());
      const std::string f = mine[k];
      mine.erase(mine.begin() + k);
      set1(f, false);
      V.check(topic_for(f), "A unsubscribe during the build", &bulk_s);
    } else {
      const std::string f = filter();
      mine.push_back(f);
      set1(f, true);
      V.check(topic_for(f), "A subscribe during the build", &bulk_s);
      V.check(f, "A route key during the build", &bulk_s);
    }
    // the bulk is visible exactly once its build is installed
    V.check(topic_for(bulk_f[rnd(bulk)]), "A bulk visible with its install", &bulk_s);
    during += 1;
  }
  CHECK(during > 20, "the build finished before the subscribes ran (%d)", during);
  committer.join();
  for (const auto& f : bulk_f) V.vis.insert(f);
  for (int i = 0; i < 200; ++i) V.check(topic_for(bulk_f[rnd(bulk)]), "A after the install");
  for (const auto& f : mine) V.check(topic_for(f), "A subscribes after the install");
  emqxgm_stats st{};
  emqxgm_get_stats(h, &st);
  CHECK(st.bg_builds >= 1 && st.catchup_changes > 0, "A: builds %llu catch-up %llu",
        (unsigned long long)st.bg_builds, (unsigned long long)st.catchup_changes);
  const std::vector<double> lat_a(lat_us.end() - during, lat_us.end());

  // ---- B: single subscribes until the tables are nearly full: a build starts that nobody waits
  // for; the subscribes during it are visible at once ----
  CHECK(emqxgm_tune(h, "bg_delay_ms", 200) == 0, "tune");
  const uint64_t b0 = st.bg_builds;
  int b_during = 0;
  for (int i = 0; i < 200000 && b_during < 60; ++i) {
    const std::string f = filter();
    set1(f, true);
    if (in_flight()) {
      V.check(topic_for(f), "B subscribe during a build");
      b_during += 1;
    }
  }
  emqxgm_get_stats(h, &st);
  CHECK(st.bg_builds > b0 && b_during > 0, "B: no build started by the tables' load");
  CHECK(emqxgm_commit(h, nullptr) == 0, "commit");

  // ---- C: during a build, a batch too large for a delta waits for the install ----
  CHECK(emqxgm_tune(h, "bg_delay_ms", 300) == 0, "tune");
  std::vector<std::string> more;
  bb.clear();
  bo.assign(1, 0);
  emqxgm_get_stats(h, &st);
  // more changes than a delta takes (commit_delta: max(4096, (trie members + route keys) / 8))
  const uint32_t nmore = delta_max ? 2 * delta_max
                                   : (uint32_t)std::max<uint64_t>(bulk, (st.n_trie_filters + st.n_route_keys) / 8 + 1000);
  for (uint32_t i = 0; i < nmore; ++i) {
    more.push_back(filter());
    bb += more.back();
    bo.push_back(bb.size());
  }
  CHECK(emqxgm_route_set_many(h, (const uint8_t*)bb.data(), bo.data(), nmore, 1) == 0, "set_many");
  std::atomic<bool> c2_done{false};
  std::thread c2([&] {
    CHECK(emqxgm_commit(h, nullptr) == 0, "commit");
    c2_done = true;
  });
  for (int k = 0; !in_flight(); ++k) {
    CHECK(!c2_done && k < 200000, "C: the commit did not build in the background");
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  const uint64_t w0 = st.bg_waits;
  std::vector<std::string> big;
  bb.clear();
  bo.assign(1, 0);
  const uint32_t nbig = nmore;
  for (uint32_t i = 0; i < nbig; ++i) {
    big.push_back(filter());
    bb += big.back();
    bo.push_back(bb.size());
  }
  std::vector<uint8_t> pr(nbig, 1);
  CHECK(emqxgm_route_set_batch(h, (const uint8_t*)bb.data(), bo.data(), pr.data(), nbig,
                               EMQXGM_SET_COMMIT, nullptr) == 0, "big batch");
  // it waited for the install, which publishes the build's own changes too
  for (const auto& f : big) V.vis.insert(f);
  for (const auto& f : more) V.vis.insert(f);
  for (int i = 0; i < 50; ++i) V.check(topic_for(big[rnd(nbig)]), "C big batch after its commit");
  c2.join();
  emqxgm_get_stats(h, &st);
  CHECK(st.bg_waits > w0, "C: the big batch did not wait");
  for (int i = 0; i < 300; ++i) {
    const auto& pool = rnd(2) ? more : big;
    V.check(topic_for(pool[rnd(pool.size())]), "C after both");
  }
  for (int i = 0; i < 100; ++i) V.check(word() + "/" + word(), "C random");

  // ---- D: another caller's bulk left pending (a resync's chunks, not committed yet): a single
  // subscribe commits its own change alone -- no build, no wait -- and the bulk stays pending
  // until its own commit ----
  {
    emqxgm_get_stats(h, &st);
    const uint64_t builds0 = st.bg_builds, waits0 = st.bg_waits, full0 = st.full_commits;
    std::vector<std::string> pend;
    bb.clear();
    bo.assign(1, 0);
    for (uint32_t i = 0; i < nmore; ++i) {
      pend.push_back(filter());
      bb += pend.back();
      bo.push_back(bb.size());
    }
    CHECK(emqxgm_route_set_many(h, (const uint8_t*)bb.data(), bo.data(), nmore, 1) == 0, "set_many");
    for (int i = 0; i < 40; ++i) {
      const std::string f = filter();
      set1(f, true);
      V.check(topic_for(f), "D subscribe beside a pending bulk");
      V.check(topic_for(pend[rnd(pend.size())]), "D pending bulk not visible");
    }
    emqxgm_get_stats(h, &st);
    CHECK(st.bg_builds == builds0 && st.bg_waits == waits0 && st.full_commits == full0,
          "D: a single subscribe built or waited");
    CHECK(emqxgm_commit(h, nullptr) == 0, "commit");
    for (const auto& f : pend) V.vis.insert(f);
    for (int i = 0; i < 100; ++i) V.check(topic_for(pend[rnd(pend.size())]), "D bulk after its commit");
  }

  std::vector<double> s = lat_a;
  std::sort(s.begin(), s.end());
  const double p50 = s[s.size() / 2], p99 = s[std::min(s.size() - 1, s.size() * 99 / 100)];
  printf("OK %llu %llu %llu %.1f %.1f\n", (unsigned long long)V.checks,
         (unsigned long long)st.bg_builds, (unsigned long long)st.bg_waits, p50, p99);
  emqxgm_destroy(h);
  return 0;
}
