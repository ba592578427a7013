// gm_kernels.hip -- gfx950 (MI355X, CDNA4) kernels of the batched MQTT publish-match pipeline.
//
// Pipeline for one batch of N published topics (DESIGN.md "Kernels"):
//   k_tok_count      levels per topic (emqx_topic:tokens/1, emqx_topic.erl:155-159)
//   k_scan_*         exclusive scan -> word base of each topic
//   k_tok_hash       level-token hashes (emqx_topic:words/1, :162-169), wildcard flag
//                    (emqx_topic:wildcard/1, :54-64), '$' flag, and the exact route-key probe
//                    with byte verification (emqx_router:lookup_routes/1, emqx_router.erl:155-157)
//   k_walk           persistent trie walk: one lane owns one topic at a time and walks the
//                    frontier depth-first (literal edge, '+' edge, '#' filter, terminal filters)
//                    -- emqx_trie:match_compact/5 (emqx_trie.erl:327-348) restated over a
//                    hashed CSR/hash trie; matches compacted with wave ballot + mbcnt into
//                    wave-private chunks of a staging buffer
//   k_scan_*         exclusive scan of per-topic match counts -> CSR row pointers
//   k_verify_scatter every staged (topic, filter) pair is re-checked bytewise against the
//                    string pool with the MQTT predicate (emqx_topic:match/2, :67-89), so a
//                    level-token hash collision can never change a result; scattered to CSR
//   k_fix_* (rare)   compaction when verification rejected pairs
#include <hip/hip_runtime.h>

#include "gm_common.h"
#include "gm_kernels.h"

namespace gm {

namespace {

constexpr uint32_t WG = 256;
constexpr uint32_t STK = 8;       // LDS stack entries per lane (deeper entries spill to HBM)
constexpr uint32_t CH = 1024;     // staged-pair slots reserved per wave per atomic
constexpr uint32_t TBLK = 128;    // topics claimed per wave per atomic
constexpr uint32_t SCAN_ITEMS = 16;
constexpr uint32_t SCAN_TILE = WG * SCAN_ITEMS;

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint64_t tag_of(const uint4& s) { return ((uint64_t)s.y << 32) | s.x; }

__device__ __forceinline__ bool bytes_equal(const uint8_t* a, const uint8_t* b, uint32_t len) {
  for (uint32_t i = 0; i < len; ++i)
    if (a[i] != b[i]) return false;
  return true;
}

// emqx_topic:match/2 (emqx_topic.erl:67-89) on raw bytes, for a NON-wildcard topic name T
// (the trie never returns anything for wildcard names, emqx_trie.erl:157-166).
__device__ bool mqtt_match(const uint8_t* T, uint32_t tl, const uint8_t* F, uint32_t fl) {
  if (tl > 0 && T[0] == '$' && fl > 0 && (F[0] == '+' || F[0] == '#')) return false;  // :70-73
  uint32_t i = 0, j = 0;  // start of the current topic / filter word
  for (;;) {
    uint32_t je = j;
    while (je < fl && F[je] != '/') ++je;
    const bool flast = (je == fl);
    const uint32_t flen = je - j;
    const bool fplus = (flen == 1 && F[j] == '+');
    const bool fhash = (flen == 1 && F[j] == '#');
    if (fhash && flast) return true;  // match(_, ['#']) -> true
    if (i > tl) return false;         // match([], [_|_]) -> false
    uint32_t ie = i;
    while (ie < tl && T[ie] != '/') ++ie;
    if (fplus || (flen == ie - i && bytes_equal(T + i, F + j, flen))) {
      i = ie + 1;
      j = je + 1;
      if (flast) return i > tl;  // match([], []) -> true ; match([_|_], []) -> false
      continue;
    }
    return false;
  }
}

// ----------------------------------------------------------------------------------------
// tokenizer
// ----------------------------------------------------------------------------------------

__global__ __launch_bounds__(WG) void k_tok_count(const uint8_t* __restrict__ bytes,
                                                  const uint32_t* __restrict__ off, uint32_t n,
                                                  uint32_t* __restrict__ nw) {
  for (uint32_t t = blockIdx.x * WG + threadIdx.x; t < n; t += gridDim.x * WG) {
    const uint32_t b = off[t], e = off[t + 1];
    uint32_t c = 1;
    for (uint32_t i = b; i < e; ++i) c += (bytes[i] == '/');
    nw[t] = c;
  }
}

struct TokArgs {
  const uint8_t* bytes;
  const uint32_t* off;
  uint32_t n;
  const uint32_t* wbase;
  uint32_t* wh;
  uint4* rec;
  uint32_t* exact_id;
  const uint4* exact;
  uint64_t xmask;
  const uint8_t* fbytes;
  const uint64_t* foff;
  uint32_t word_mask;
  uint64_t full_mask;
  bool exact_empty;
};

__global__ __launch_bounds__(WG) void k_tok_hash(TokArgs A) {
  for (uint32_t t = blockIdx.x * WG + threadIdx.x; t < A.n; t += gridDim.x * WG) {
    const uint32_t b = A.off[t], e = A.off[t + 1];
    const uint32_t wb = A.wbase[t];
    uint64_t hw = FNV_OFF, hall = FNV_OFF;
    uint32_t k = 0, wlen = 0, flags = 0, h0 = 0, c0 = 0;
    if (e > b && A.bytes[b] == '$') flags |= T_DOLLAR;
    for (uint32_t i = b; i < e; ++i) {
      const uint32_t c = A.bytes[i];
      hall = fnv_step(hall, c);
      if (c == '/') {
        if (wlen == 1 && (c0 == '+' || c0 == '#')) flags |= T_WILD;
        const uint32_t h = word_hash(hw, A.word_mask);
        if (k == 0) h0 = h;
        A.wh[wb + k] = h;
        ++k;
        hw = FNV_OFF;
        wlen = 0;
      } else {
        if (wlen == 0) c0 = c;
        hw = fnv_step(hw, c);
        ++wlen;
      }
    }
    if (wlen == 1 && (c0 == '+' || c0 == '#')) flags |= T_WILD;
    const uint32_t h = word_hash(hw, A.word_mask);
    if (k == 0) h0 = h;
    A.wh[wb + k] = h;
    ++k;
    A.rec[t] = make_uint4(wb, k, flags, h0);

    // exact route key (all route keys, wildcard strings included: emqx_router.erl:143,157)
    uint32_t hit = NONE;
    if (!A.exact_empty) {
      const uint64_t fh = full_hash(hall, A.full_mask);
      const uint32_t len = e - b;
      uint64_t i = exact_slot(fh, A.xmask);
      for (;;) {
        const uint4 s = A.exact[i];
        if (s.z == NONE) break;
        if (tag_of(s) == fh && s.w == len) {
          const uint64_t fo = A.foff[s.z];
          if (bytes_equal(A.bytes + b, A.fbytes + fo, len)) {
            hit = s.z;
            break;
          }
        }
        i = (i + 1) & A.xmask;
      }
    }
    A.exact_id[t] = hit;
  }
}

// ----------------------------------------------------------------------------------------
// exclusive scan (u32), reduce-then-scan over tiles of SCAN_TILE elements
// ----------------------------------------------------------------------------------------

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_w, uint32_t& total) {
  const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  uint32_t woff = 0, tot = 0;
#pragma unroll
  for (uint32_t i = 0; i < WG / 64; ++i) {
    const uint32_t sv = s_w[i];
    woff += (i < w) ? sv : 0u;
    tot += sv;
  }
  __syncthreads();
  total = tot;
  return woff + x - v;
}

__global__ __launch_bounds__(WG) void k_scan_partials(const uint32_t* __restrict__ in, uint32_t n,
                                                      uint32_t* __restrict__ part) {
  __shared__ uint32_t s_w[WG / 64];
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
  uint32_t acc = 0;
  for (uint32_t j = 0; j < SCAN_ITEMS; ++j) {
    const uint64_t i = base + (uint64_t)j * WG + threadIdx.x;
    acc += (i < n) ? in[i] : 0u;
  }
  uint32_t tot;
  block_excl_scan(acc, s_w, tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ __launch_bounds__(WG) void k_scan_top(uint32_t* __restrict__ part, uint32_t np,
                                                 uint32_t* __restrict__ out_n,
                                                 uint32_t* __restrict__ total_dst) {
  __shared__ uint32_t s_w[WG / 64];
  uint32_t carry = 0;
  for (uint32_t b = 0; b < np; b += WG) {
    const uint32_t i = b + threadIdx.x;
    const uint32_t v = (i < np) ? part[i] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl_scan(v, s_w, tot);
    if (i < np) part[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) {
    *out_n = carry;
    if (total_dst) *total_dst = carry;
  }
}

__global__ __launch_bounds__(WG) void k_scan_final(const uint32_t* __restrict__ in, uint32_t n,
                                                   const uint32_t* __restrict__ part,
                                                   uint32_t* __restrict__ out) {
  __shared__ uint32_t s_w[WG / 64];
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
  uint32_t carry = part[blockIdx.x];
  for (uint32_t j = 0; j < SCAN_ITEMS; ++j) {
    const uint64_t i = base + (uint64_t)j * WG + threadIdx.x;
    const uint32_t v = (i < n) ? in[i] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl_scan(v, s_w, tot);
    if (i < n) out[i] = carry + ex;
    carry += tot;
  }
}

// ----------------------------------------------------------------------------------------
// trie walk
// ----------------------------------------------------------------------------------------

struct WalkArgs {
  const uint4* rec;
  const uint32_t* wh;
  const uint4* edges;
  uint64_t emask;
  const uint32_t* node_tw;
  const uint32_t* node_tn;
  const uint32_t* multi;
  uint32_t root_cf, root_hf;
  uint32_t n;
  uint32_t* ctl;
  uint32_t* cnt;
  uint32_t* pt;
  uint32_t* pf;
  uint32_t* pr;
  uint32_t pcap;
  uint4* spill;
  uint32_t lanes;
  unsigned long long* census;  // [0] trie states matched (S(t) summed), [1] edge-slot loads
};

struct WaveOut {  // wave-uniform cursor into this wave's reserved chunk of staged pairs
  uint32_t pos, end;
};

// One emission round: each lane with `v` appends (t, f, rank) to the wave's chunk.
__device__ __forceinline__ void emit1(bool v, uint32_t t, uint32_t f, uint32_t& rank, WaveOut& o,
                                      const WalkArgs& A) {
  const uint64_t m = __ballot(v);
  if (m == 0) return;
  const uint32_t c = (uint32_t)__popcll(m);
  if (o.pos + c > o.end) {
    for (uint32_t i = o.pos + lane_id(); i < o.end && i < A.pcap; i += 64) A.pt[i] = NONE;
    uint32_t base = 0;
    if (lane_id() == 0) base = atomicAdd(&A.ctl[CTL_PAIR_TOP], CH);
    base = __shfl(base, 0, 64);
    o.pos = base;
    o.end = base + CH;
  }
  if (v) {
    const uint32_t i = o.pos + mbcnt64(m);
    if (i < A.pcap) {
      A.pt[i] = t;
      A.pf[i] = f;
      A.pr[i] = rank;
    }
    ++rank;
  }
  o.pos += c;
}

// Emit a filter list: a single id, or (multi) an index into the multi[] pool.
__device__ __forceinline__ void emit_list(bool has, uint32_t val, bool multi, uint32_t t,
                                          uint32_t& rank, WaveOut& o, const WalkArgs& A) {
  emit1(has && !multi, t, val, rank, o, A);
  const bool mh = has && multi;
  if (__ballot(mh) != 0) {
    const uint32_t cntm = mh ? A.multi[val] : 0u;
    for (uint32_t j = 0; __ballot(mh && j < cntm) != 0; ++j) {
      const bool v = mh && j < cntm;
      const uint32_t f = v ? A.multi[val + 1 + j] : 0u;
      emit1(v, t, f, rank, o, A);
    }
  }
}

// CENSUS=true is a diagnostic build that also counts, per batch, the trie states matched
// (SURVEY 8d's S(t), summed) and the edge slots loaded; it feeds the roofline's algorithmic
// bytes and is checked against the oracle's S(t).  The production launch is CENSUS=false.
template <bool CENSUS>
__global__ __launch_bounds__(WG) void k_walk(WalkArgs A) {
  __shared__ uint32_t s_cf[STK][WG];
  __shared__ uint32_t s_k[STK][WG];
  __shared__ uint32_t s_h[STK][WG];
  const uint32_t tid = threadIdx.x;
  const uint32_t gl = blockIdx.x * WG + tid;
  const uint4 EMPTY4 = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0u, NONE);

  uint32_t t = NONE, n = 0, wb = 0, fl = 0, cf = 0, k = 0, hk = 0, rank = 0, sp = 0;
  uint32_t q_next = 0, q_end = 0;
  bool done = false;
  WaveOut o{0u, 0u};
  uint32_t c_states = 0, c_loads = 0;

  for (;;) {
    // ---- refill idle lanes from the wave's topic block (wave-uniform bookkeeping) ----
    bool fresh = false;
    uint64_t mi = __ballot(t == NONE);
    while (mi != 0 && !done) {
      const uint32_t avail = q_end - q_next;
      if (avail == 0) {
        uint32_t base = 0;
        if (lane_id() == 0) base = atomicAdd(&A.ctl[CTL_TOPIC_CTR], TBLK);
        base = __shfl(base, 0, 64);
        if (base >= A.n) {
          done = true;
          break;
        }
        q_next = base;
        q_end = min(base + TBLK, A.n);
        continue;
      }
      const uint32_t r = mbcnt64(mi);
      if (t == NONE && r < avail) {
        t = q_next + r;
        fresh = true;
      }
      q_next += min((uint32_t)__popcll(mi), avail);
      mi = __ballot(t == NONE);
    }
    if (fresh) {
      const uint4 r = A.rec[t];
      wb = r.x;
      n = r.y;
      fl = r.z;
      hk = r.w;
      cf = A.root_cf;
      k = 0;
      rank = 0;
      sp = 0;
      if (fl & T_WILD) {  // emqx_trie.erl:157-166: wildcard topic name -> []
        A.cnt[t] = 0;
        t = NONE;
        fresh = false;
      } else if (CENSUS) {
        c_states += 1;  // the root
      }
    }
    // root '#' filter (emqx_trie.erl:334 at the root; skipped for '$' topics, :282-289)
    emit_list(fresh && !(fl & T_DOLLAR) && A.root_hf != NONE, A.root_hf,
              (A.root_cf & CF_HFM) != 0, t, rank, o, A);

    const bool active = (t != NONE);
    if (__ballot(active) == 0) {
      if (done) break;
      continue;
    }

    // ---- expand the lane's current state (cf at depth k, level token hk) ----
    const bool root_dollar = (k == 0) && (fl & T_DOLLAR);
    const bool do_lit = active && (cf & CF_LIT);
    const bool do_plus = active && (cf & CF_PLUS) && !root_dollar;
    const uint32_t cur = cf & CF_ID_MASK;
    const uint64_t tag_a = edge_tag(cur, hk), tag_b = edge_tag(cur, PLUS_WH);
    uint64_t ia = edge_slot(tag_a, A.emask), ib = edge_slot(tag_b, A.emask);
    uint4 sa = do_lit ? A.edges[ia] : EMPTY4;
    uint4 sb = do_plus ? A.edges[ib] : EMPTY4;
    const bool more = active && (k + 1 < n);
    const uint32_t hn = more ? A.wh[wb + k + 1] : 0u;
    bool fa = false, fb = false;
    if (do_lit) {
      for (;;) {
        if (CENSUS) ++c_loads;
        const uint64_t st = tag_of(sa);
        if (st == tag_a) { fa = true; break; }
        if (st == EMPTY_TAG) break;
        ia = (ia + 1) & A.emask;
        sa = A.edges[ia];
      }
    }
    if (do_plus) {
      for (;;) {
        if (CENSUS) ++c_loads;
        const uint64_t st = tag_of(sb);
        if (st == tag_b) { fb = true; break; }
        if (st == EMPTY_TAG) break;
        ib = (ib + 1) & A.emask;
        sb = A.edges[ib];
      }
    }
    if (CENSUS) c_states += (fa ? 1u : 0u) + (fb ? 1u : 0u);

    // '#' filters of the children: "child_path/#" matches every remaining suffix
    emit_list(fa && sa.w != NONE, sa.w, (sa.z & CF_HFM) != 0, t, rank, o, A);
    emit_list(fb && sb.w != NONE, sb.w, (sb.z & CF_HFM) != 0, t, rank, o, A);
    // terminal filters at the last level (emqx_trie.erl:327-332); non-wildcard trie keys only
    // for a single-level '$' topic (lookup_topic at :287)
    const bool last = active && (k + 1 == n);
    const bool qn = (fl & T_DOLLAR) && n == 1;
    const bool twa = fa && last && (sa.z & CF_TW);
    const bool twb = fb && last && (sb.z & CF_TW);
    const bool tna = fa && last && qn && (sa.z & CF_TN);
    const uint32_t va = twa ? A.node_tw[sa.z & CF_ID_MASK] : 0u;
    const uint32_t vb = twb ? A.node_tw[sb.z & CF_ID_MASK] : 0u;
    const uint32_t vn = tna ? A.node_tn[sa.z & CF_ID_MASK] : 0u;
    emit_list(twa, va & ~LIST_MULTI, (va & LIST_MULTI) != 0, t, rank, o, A);
    emit_list(twb, vb & ~LIST_MULTI, (vb & LIST_MULTI) != 0, t, rank, o, A);
    emit_list(tna, vn & ~LIST_MULTI, (vn & LIST_MULTI) != 0, t, rank, o, A);

    // ---- continue depth-first: literal child first, '+' child pushed ----
    const bool ca = fa && more && (sa.z & (CF_LIT | CF_PLUS));
    const bool cb = fb && more && (sb.z & (CF_LIT | CF_PLUS));
    if (ca && cb) {
      if (sp < STK) {
        s_cf[sp][tid] = sb.z;
        s_k[sp][tid] = k + 1;
        s_h[sp][tid] = hn;
      } else {
        A.spill[(uint64_t)(sp - STK) * A.lanes + gl] = make_uint4(sb.z, k + 1, hn, 0u);
      }
      ++sp;
    }
    if (ca) {
      cf = sa.z;
      ++k;
      hk = hn;
    } else if (cb) {
      cf = sb.z;
      ++k;
      hk = hn;
    } else if (active) {
      if (sp > 0) {
        --sp;
        if (sp < STK) {
          cf = s_cf[sp][tid];
          k = s_k[sp][tid];
          hk = s_h[sp][tid];
        } else {
          const uint4 e = A.spill[(uint64_t)(sp - STK) * A.lanes + gl];
          cf = e.x;
          k = e.y;
          hk = e.z;
        }
      } else {
        A.cnt[t] = rank;
        t = NONE;
      }
    }
  }
  for (uint32_t i = o.pos + lane_id(); i < o.end && i < A.pcap; i += 64) A.pt[i] = NONE;
  if (CENSUS) {
    atomicAdd(&A.census[0], (unsigned long long)c_states);
    atomicAdd(&A.census[1], (unsigned long long)c_loads);
  }
}

// ----------------------------------------------------------------------------------------
// verify + scatter to CSR
// ----------------------------------------------------------------------------------------

struct VerifyArgs {
  const uint8_t* tbytes;
  const uint32_t* toff;
  const uint8_t* fbytes;
  const uint64_t* foff;
  const uint32_t* pt;
  const uint32_t* pf;
  const uint32_t* pr;
  uint32_t pcap;
  const uint32_t* row;
  uint32_t* out;
  uint32_t ocap;
  uint32_t* rej;
  uint32_t* ctl;
};

__global__ __launch_bounds__(WG) void k_verify_scatter(VerifyArgs A) {
  const uint32_t top = min(A.ctl[CTL_PAIR_TOP], A.pcap);
  for (uint32_t i = blockIdx.x * WG + threadIdx.x; i < top; i += gridDim.x * WG) {
    const uint32_t t = A.pt[i];
    if (t == NONE) continue;
    const uint32_t f = A.pf[i];
    const uint32_t r = A.pr[i];
    const uint32_t tb = A.toff[t], te = A.toff[t + 1];
    const uint64_t fb = A.foff[f], fe = A.foff[f + 1];
    const bool ok = mqtt_match(A.tbytes + tb, te - tb, A.fbytes + fb, (uint32_t)(fe - fb));
    const uint32_t pos = A.row[t] + r;
    if (pos < A.ocap) A.out[pos] = ok ? f : NONE;  // beyond ocap only on an overflowed pass
    if (!ok) {
      atomicAdd(&A.rej[t], 1u);
      A.ctl[CTL_ANY_REJ] = 1u;
    }
  }
}

__global__ __launch_bounds__(WG) void k_fix_counts(uint32_t* __restrict__ cnt,
                                                   const uint32_t* __restrict__ rej, uint32_t n) {
  for (uint32_t t = blockIdx.x * WG + threadIdx.x; t < n; t += gridDim.x * WG) cnt[t] -= rej[t];
}

__global__ __launch_bounds__(WG) void k_compact_rows(const uint32_t* __restrict__ row,
                                                     const uint32_t* __restrict__ out,
                                                     const uint32_t* __restrict__ row2,
                                                     uint32_t* __restrict__ out2, uint32_t n) {
  for (uint32_t t = blockIdx.x * WG + threadIdx.x; t < n; t += gridDim.x * WG) {
    uint32_t d = row2[t];
    for (uint32_t i = row[t]; i < row[t + 1]; ++i) {
      const uint32_t f = out[i];
      if (f != NONE) out2[d++] = f;
    }
  }
}

uint32_t grid_for(uint64_t items, uint32_t cap_blocks) {
  uint64_t b = (items + WG - 1) / WG;
  if (b == 0) b = 1;
  return (uint32_t)(b < cap_blocks ? b : cap_blocks);
}

}  // namespace

WalkGeom walk_geometry(int device, uint32_t wg_per_cu) {
  hipDeviceProp_t p;
  WalkGeom g;
  int cus = 256;
  if (hipGetDeviceProperties(&p, device) == hipSuccess && p.multiProcessorCount > 0)
    cus = p.multiProcessorCount;
  g.blocks = (uint32_t)cus * (wg_per_cu ? wg_per_cu : 4u);
  g.lanes = g.blocks * WG;
  return g;
}

hipError_t launch_tok_count(const uint8_t* bytes, const uint32_t* off, uint32_t n, uint32_t* nw,
                            hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_tok_count, dim3(grid_for(n, 8192)), dim3(WG), 0, s, bytes, off, n, nw);
  return hipGetLastError();
}

uint32_t scan_tmp_words(uint32_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE + 1; }

hipError_t launch_scan(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* tmp,
                       uint32_t* total_dst, hipStream_t s) {
  const uint32_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (nb > 0) hipLaunchKernelGGL(k_scan_partials, dim3(nb), dim3(WG), 0, s, in, n, tmp);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(WG), 0, s, tmp, nb, out + n, total_dst);
  if (nb > 0) hipLaunchKernelGGL(k_scan_final, dim3(nb), dim3(WG), 0, s, in, n, tmp, out);
  return hipGetLastError();
}

hipError_t launch_tok_hash(const uint8_t* bytes, const uint32_t* off, uint32_t n,
                           const DevIndex& ix, Scratch& sc, hipStream_t s) {
  if (n == 0) return hipSuccess;
  TokArgs a;
  a.bytes = bytes;
  a.off = off;
  a.n = n;
  a.wbase = sc.wbase;
  a.wh = sc.wh;
  a.rec = sc.rec;
  a.exact_id = sc.exact_id;
  a.exact = ix.exact;
  a.xmask = ix.xmask;
  a.fbytes = ix.fbytes;
  a.foff = ix.foff;
  a.word_mask = ix.word_mask;
  a.full_mask = ix.full_mask;
  a.exact_empty = ix.exact_empty;
  hipLaunchKernelGGL(k_tok_hash, dim3(grid_for(n, 8192)), dim3(WG), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_walk(const DevIndex& ix, Scratch& sc, uint32_t n, const WalkGeom& g,
                       hipStream_t s, unsigned long long* census) {
  WalkArgs a;
  a.rec = sc.rec;
  a.wh = sc.wh;
  a.edges = ix.edges;
  a.emask = ix.emask;
  a.node_tw = ix.node_tw;
  a.node_tn = ix.node_tn;
  a.multi = ix.multi;
  a.root_cf = ix.root_cf;
  a.root_hf = ix.root_hf;
  a.n = n;
  a.ctl = sc.ctl;
  a.cnt = sc.cnt;
  a.pt = sc.pt;
  a.pf = sc.pf;
  a.pr = sc.pr;
  a.pcap = sc.p_cap;
  a.spill = sc.spill;
  a.lanes = g.lanes;
  a.census = census;
  if (census)
    hipLaunchKernelGGL(k_walk<true>, dim3(g.blocks), dim3(WG), 0, s, a);
  else
    hipLaunchKernelGGL(k_walk<false>, dim3(g.blocks), dim3(WG), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_verify_scatter(const uint8_t* bytes, const uint32_t* off, const DevIndex& ix,
                                 Scratch& sc, uint32_t n, hipStream_t s) {
  (void)n;
  VerifyArgs a;
  a.tbytes = bytes;
  a.toff = off;
  a.fbytes = ix.fbytes;
  a.foff = ix.foff;
  a.pt = sc.pt;
  a.pf = sc.pf;
  a.pr = sc.pr;
  a.pcap = sc.p_cap;
  a.row = sc.row;
  a.out = sc.out;
  a.ocap = sc.o_cap;
  a.rej = sc.rej;
  a.ctl = sc.ctl;
  hipLaunchKernelGGL(k_verify_scatter, dim3(grid_for(sc.p_cap, 4096)), dim3(WG), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_fixup(Scratch& sc, uint32_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_fix_counts, dim3(grid_for(n, 4096)), dim3(WG), 0, s, sc.cnt, sc.rej, n);
  hipError_t e = launch_scan(sc.cnt, sc.row2, n, sc.scan_tmp, sc.ctl + CTL_TOTAL, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_compact_rows, dim3(grid_for(n, 4096)), dim3(WG), 0, s, sc.row, sc.out,
                     sc.row2, sc.out2, n);
  return hipGetLastError();
}

}  // namespace gm
