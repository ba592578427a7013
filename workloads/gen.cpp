// gen.cpp -- deterministic synthetic workloads of SURVEY.md 8d (cfg1..cfg4) for the parity
// tests and bench.py.  Not part of the engine: it only produces filter and topic byte sets.
//
// Reference patterns: the in-tree bench renders "device/{{id}}/+/{{num}}/#" subscriptions and
// "device/{{id}}/foo/{{num}}/bar/1/2/3/4/5" publishes (apps/emqx/src/emqx_broker_bench.erl:25-35);
// the configs below scale that idea to the BASELINE.json workloads.
//
// Every draw goes through xoshiro256** seeded by splitmix64 (no std::distribution), so the byte
// sets are identical on every machine.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <cmath>
#include <string>
#include <unordered_set>
#include <vector>

namespace {

bool g_topics_only = false;  // wl_generate_topics: skip the filter draws

struct Rng {
  uint64_t s[4];
  explicit Rng(uint64_t seed) {
    uint64_t x = seed;
    for (auto& v : s) {
      x += 0x9e3779b97f4a7c15ull;
      uint64_t z = x;
      z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
      z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
      v = z ^ (z >> 31);
    }
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return r;
  }
  double uni() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  uint64_t below(uint64_t n) { return n ? next() % n : 0; }
};

struct Zipf {
  std::vector<double> cdf;
  Zipf(uint64_t n, double s) {
    cdf.resize(n);
    double acc = 0;
    for (uint64_t i = 0; i < n; ++i) {
      acc += 1.0 / std::pow((double)(i + 1), s);
      cdf[i] = acc;
    }
    for (auto& c : cdf) c /= acc;
  }
  uint64_t draw(Rng& r) const {
    const double u = r.uni();
    uint64_t lo = 0, hi = cdf.size() - 1;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) / 2;
      if (cdf[mid] < u)
        lo = mid + 1;
      else
        hi = mid;
    }
    return lo;
  }
};

struct Packed {
  std::vector<uint8_t> bytes;
  std::vector<uint64_t> off{0};
  std::vector<uint8_t> wild;
  void add(const std::string& s, bool w) {
    bytes.insert(bytes.end(), s.begin(), s.end());
    off.push_back(bytes.size());
    wild.push_back(w ? 1 : 0);
  }
  size_t size() const { return wild.size(); }
};

bool is_wild(const std::string& s) {
  size_t st = 0;
  for (size_t i = 0; i <= s.size(); ++i)
    if (i == s.size() || s[i] == '/') {
      if (i - st == 1 && (s[st] == '+' || s[st] == '#')) return true;
      st = i + 1;
    }
  return false;
}

std::string vw(int level, uint64_t i) { return "l" + std::to_string(level) + "w" + std::to_string(i); }

// cfg1: 10k wildcard filters, exactly 4 levels, vocab [8,32,128,512] Zipf 1.1, '+' p=.25 per
// level, last level '#' p=.25; 100k topics of depth {3,4,5}, 5th level x{0..63}, 2% '$SYS'.
void gen_cfg1(uint64_t nf, uint64_t nt, uint64_t sf, uint64_t st, Packed& F, Packed& T) {
  const uint64_t vs[4] = {8, 32, 128, 512};
  std::vector<Zipf> z;
  for (auto v : vs) z.emplace_back(v, 1.1);
  Zipf zx(64, 1.1);
  Rng rf(sf);
  std::unordered_set<std::string> seen;
  while (!g_topics_only && F.size() < nf) {
    std::string s;
    for (int k = 0; k < 4; ++k) {
      if (k) s += '/';
      const double u = rf.uni();
      if (k == 3 && u < 0.25)
        s += '#';
      else if (rf.uni() < 0.25)
        s += '+';
      else
        s += vw(k, z[k].draw(rf));
    }
    if (!is_wild(s) || !seen.insert(s).second) continue;
    F.add(s, true);
  }
  Rng rt(st);
  for (uint64_t i = 0; i < nt; ++i) {
    const int depth = 3 + (int)rt.below(3);
    std::string s;
    for (int k = 0; k < depth; ++k) {
      if (k) s += '/';
      s += (k < 4) ? vw(k, z[k].draw(rt)) : ("x" + std::to_string(zx.draw(rt)));
    }
    if (rt.uni() < 0.02) s = "$SYS" + s.substr(s.find('/'));
    T.add(s, false);
  }
}

// cfg2: 1M filters, 6 levels, vocab [4,16,64,256,1024,4096] Zipf 1.0, '+' p=.2 per level, last
// level '#' p=.05; non-wildcard draws are exact route keys.  Topics: depth 6 (80%), 5 (10%),
// 7 (10%, 7th level x{0..63}); 1% '$SYS' first level.
void gen_cfg2(uint64_t nf, uint64_t nt, uint64_t sf, uint64_t st, Packed& F, Packed& T) {
  const uint64_t vs[6] = {4, 16, 64, 256, 1024, 4096};
  std::vector<Zipf> z;
  for (auto v : vs) z.emplace_back(v, 1.0);
  Zipf zx(64, 1.0);
  Rng rf(sf);
  std::unordered_set<std::string> seen;
  seen.reserve(nf * 2);
  while (!g_topics_only && F.size() < nf) {
    std::string s;
    for (int k = 0; k < 6; ++k) {
      if (k) s += '/';
      if (k == 5 && rf.uni() < 0.05)
        s += '#';
      else if (rf.uni() < 0.20)
        s += '+';
      else
        s += vw(k, z[k].draw(rf));
    }
    if (!seen.insert(s).second) continue;
    F.add(s, is_wild(s));
  }
  Rng rt(st);
  for (uint64_t i = 0; i < nt; ++i) {
    const double u = rt.uni();
    const int depth = u < 0.8 ? 6 : (u < 0.9 ? 5 : 7);
    std::string s;
    for (int k = 0; k < depth; ++k) {
      if (k) s += '/';
      s += (k < 6) ? vw(k, z[k].draw(rt)) : ("x" + std::to_string(zx.draw(rt)));
    }
    if (rt.uni() < 0.01) s = "$SYS" + s.substr(s.find('/'));
    T.add(s, false);
  }
}

// cfg3: IoT tree over 10,000 sites x 1,000 devices (global device ids s*1000+j), sites Zipf 0.8.
// Draw probabilities 70/10/10/5/5 over
//   site/{s}/device/{d}/#, site/{s}/device/+/{m}, site/+/device/{d}/#, site/{s}/+/+/{m},
//   site/{s}/device/{d}/+/{k}        (m in 32 metric names, k in 0..15)
// until nf distinct filters (patterns 2 and 4 saturate at 320k distinct values each, the draw
// simply continues).  Topics: site/{s}/device/{d}/{m}/{k}.
void gen_cfg3(uint64_t nf, uint64_t nt, uint64_t sf, uint64_t st, Packed& F, Packed& T) {
  const uint64_t SITES = 10000, DEV = 1000;
  Zipf zs(SITES, 0.8);
  auto metric = [](uint64_t m) { return "m" + std::to_string(m); };
  Rng rf(sf);
  std::unordered_set<std::string> seen;
  seen.reserve(nf * 2);
  while (!g_topics_only && F.size() < nf) {
    const uint64_t s = zs.draw(rf);
    const uint64_t d = s * DEV + rf.below(DEV);
    const double u = rf.uni();
    std::string f;
    const std::string site = "site/" + std::to_string(s);
    if (u < 0.70)
      f = site + "/device/" + std::to_string(d) + "/#";
    else if (u < 0.80)
      f = site + "/device/+/" + metric(rf.below(32));
    else if (u < 0.90)
      f = "site/+/device/" + std::to_string(d) + "/#";
    else if (u < 0.95)
      f = site + "/+/+/" + metric(rf.below(32));
    else
      f = site + "/device/" + std::to_string(d) + "/+/" + std::to_string(rf.below(16));
    if (!seen.insert(f).second) continue;
    F.add(f, true);
  }
  Rng rt(st);
  for (uint64_t i = 0; i < nt; ++i) {
    const uint64_t s = zs.draw(rt);
    const uint64_t d = s * DEV + rt.below(DEV);
    std::string t = "site/" + std::to_string(s) + "/device/" + std::to_string(d) + "/" +
                    metric(rt.below(32)) + "/" + std::to_string(rt.below(16));
    T.add(t, false);
  }
}

std::string id9(uint64_t id) {
  char b[32];
  snprintf(b, sizeof b, "%09llu", (unsigned long long)id);
  return b;
}

// cfg4: n_exact exact "dev/{id:09}/state" + n_wild wildcards (dev/{id:09}/+,
// fleet/+/dev/{id:09}/#, fleet/{f}/#; 1/3 each); topics 90% exact hits, 10% misses.
void gen_cfg4(uint64_t nf, uint64_t nt, uint64_t sf, uint64_t st, Packed& F, Packed& T) {
  const uint64_t n_wild = nf / 101, n_exact = nf - n_wild;
  for (uint64_t i = 0; !g_topics_only && i < n_exact; ++i) F.add("dev/" + id9(i) + "/state", false);
  Rng rf(sf);
  std::unordered_set<std::string> seen;
  while (!g_topics_only && F.size() < nf) {
    const double u = rf.uni();
    std::string f;
    if (u < 1.0 / 3)
      f = "dev/" + id9(rf.below(n_exact)) + "/+";
    else if (u < 2.0 / 3)
      f = "fleet/+/dev/" + id9(rf.below(n_exact)) + "/#";
    else
      f = "fleet/" + std::to_string(rf.below(n_exact / 100 + 1)) + "/#";
    if (!seen.insert(f).second) continue;
    F.add(f, true);
  }
  Rng rt(st);
  for (uint64_t i = 0; i < nt; ++i) {
    const bool hit = rt.uni() < 0.9;
    const uint64_t id = hit ? rt.below(n_exact) : n_exact + rt.below(n_exact);
    T.add("dev/" + id9(id) + "/state", false);
  }
}

}  // namespace

extern "C" {

typedef struct wl_set {
  uint8_t* fbytes;
  uint64_t* foff;
  uint8_t* fwild;
  uint64_t nf;
  uint8_t* tbytes;
  uint32_t* toff;
  uint64_t nt;
  uint64_t fbytes_len, tbytes_len;
} wl_set;

int wl_generate(int cfg, uint64_t nf, uint64_t nt, uint64_t seed_f, uint64_t seed_t, wl_set* out) {
  if (!out) return -1;
  memset(out, 0, sizeof *out);
  Packed F, T;
  switch (cfg) {
    case 1: gen_cfg1(nf, nt, seed_f, seed_t, F, T); break;
    case 2: gen_cfg2(nf, nt, seed_f, seed_t, F, T); break;
    case 3: gen_cfg3(nf, nt, seed_f, seed_t, F, T); break;
    case 4: gen_cfg4(nf, nt, seed_f, seed_t, F, T); break;
    default: return -2;
  }
  if (T.bytes.size() > 0xFFFFFFFFull) return -3;
  out->nf = F.size();
  out->nt = T.size();
  out->fbytes_len = F.bytes.size();
  out->tbytes_len = T.bytes.size();
  out->fbytes = (uint8_t*)malloc(F.bytes.size() + 1);
  out->foff = (uint64_t*)malloc(F.off.size() * 8);
  out->fwild = (uint8_t*)malloc(F.wild.size() + 1);
  out->tbytes = (uint8_t*)malloc(T.bytes.size() + 1);
  out->toff = (uint32_t*)malloc(T.off.size() * 4);
  if (!out->fbytes || !out->foff || !out->fwild || !out->tbytes || !out->toff) return -4;
  memcpy(out->fbytes, F.bytes.data(), F.bytes.size());
  memcpy(out->foff, F.off.data(), F.off.size() * 8);
  memcpy(out->fwild, F.wild.data(), F.wild.size());
  memcpy(out->tbytes, T.bytes.data(), T.bytes.size());
  for (size_t i = 0; i < T.off.size(); ++i) out->toff[i] = (uint32_t)T.off[i];
  return 0;
}

// the topics of wl_generate(cfg, nf, nt, seed_f, seed_t) without the filters (bench.py draws
// several distinct batches against one index)
int wl_generate_topics(int cfg, uint64_t nf, uint64_t nt, uint64_t seed_f, uint64_t seed_t,
                       wl_set* out) {
  g_topics_only = true;
  const int rc = wl_generate(cfg, nf, nt, seed_f, seed_t, out);
  g_topics_only = false;
  return rc;
}

void wl_free(wl_set* s) {
  if (!s) return;
  free(s->fbytes);
  free(s->foff);
  free(s->fwild);
  free(s->tbytes);
  free(s->toff);
  memset(s, 0, sizeof *s);
}

}  // extern "C"
