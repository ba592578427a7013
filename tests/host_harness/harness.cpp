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
#include "harness_walk.h"

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
  // the delta-committing engine builds in the background at every size (r05): its full builds'
  // installs replay the changes since they read the registry
  CHECK(emqxgm_tune(hd, "bg_build", 1) == 0, "tune");
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
      CHECK(emqxgm_tune(hd, "keyed", keyed_mode) == 0 && emqxgm_tune(hd, "bg_build", 1) == 0, "tune");
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
