// gm_kernels.hip -- gfx950 (MI355X, CDNA4) kernels of the batched MQTT publish-match pipeline.
//
// Pipeline for one batch of N published topics (DESIGN.md "Kernels"):
//   k_tok_count      levels per topic (emqx_topic:tokens/1, emqx_topic.erl:155-159)
//   k_scan_*         exclusive scan -> word base of each topic
//   k_tok_hash       level tokens (emqx_topic:words/1, :162-169), wildcard flag
//                    (emqx_topic:wildcard/1, :54-64), '$' flag, and the exact route-key probe
//                    with byte verification (emqx_router:lookup_routes/1, emqx_router.erl:155-157)
//                    Both tokenizer kernels stage a 256-topic tile of packed bytes in LDS with
//                    coalesced 16-B loads and then work lane-per-topic out of LDS.
//   k_walk           persistent trie walk: one lane owns one topic at a time and walks its
//                    frontier depth-first over the hashed trie (literal edge, '+' edge, '#'
//                    filter, terminal filters) -- emqx_trie:match_compact/5 (emqx_trie.erl:
//                    327-348) restated; matches are compacted with wave ballot + mbcnt into
//                    wave-private chunks of a staging buffer
//   k_verify         every staged (topic, filter) pair is re-checked bytewise (LDS-staged) with
//                    the MQTT predicate (emqx_topic:match/2, :67-89) against the filter's 64-B
//                    verification record, so a level-token hash collision can never change a
//                    result; rejects are subtracted from the per-topic counts
//   k_scan_*         exclusive scan of per-topic match counts -> CSR row pointers
//   k_scatter        staged pairs -> CSR rows (deterministic order: walk order within a row)
//   legacy (rare)    verify+scatter then compaction, when too many pairs were rejected for the
//                    in-line rank adjustment of k_scatter
#include <hip/hip_runtime.h>

#include "gm_common.h"
#include "gm_kernels.h"

namespace gm {

namespace {

constexpr uint32_t WG = 256;
constexpr uint32_t CH = 1024;     // staged-pair slots reserved per wave per atomic
constexpr uint32_t TBLK = 128;    // topics claimed per wave per atomic
constexpr uint32_t SCAN_ITEMS = 16;
constexpr uint32_t SCAN_TILE = WG * SCAN_ITEMS;
constexpr uint32_t TILE_BYTES = 16384;  // tokenizer LDS tile (256 topics)
constexpr uint32_t TILE_CHUNKS = TILE_BYTES / 16 + 2;

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint64_t tag_of(const uint4& s) { return ((uint64_t)s.y << 32) | s.x; }

template <class PA, class PB>
__device__ __forceinline__ bool bytes_equal(PA a, PB b, uint32_t len) {
  for (uint32_t i = 0; i < len; ++i)
    if (a[i] != b[i]) return false;
  return true;
}

// emqx_topic:match/2 (emqx_topic.erl:67-89) on raw bytes, for a NON-wildcard topic name T
// (the trie never returns anything for wildcard names, emqx_trie.erl:157-166).  T and F are
// byte accessors over LDS or global memory.
template <class PT, class PF>
__device__ __forceinline__ bool mqtt_match(PT T, uint32_t tl, PF F, uint32_t fl) {
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
    bool eq = fplus;
    if (!eq && flen == ie - i) {
      eq = true;
      for (uint32_t q = 0; q < flen; ++q)
        if (T[i + q] != F[j + q]) {
          eq = false;
          break;
        }
    }
    if (!eq) return false;
    i = ie + 1;
    j = je + 1;
    if (flast) return i > tl;  // match([], []) -> true ; match([_|_], []) -> false
  }
}

// ----------------------------------------------------------------------------------------
// tokenizer (LDS-tiled)
// ----------------------------------------------------------------------------------------

// Stages the packed bytes [B0, B1) into s_buf with coalesced 16-B loads; returns false when the
// tile does not fit (the caller then reads global memory).  `sh` = offset of B0 in s_buf.
__device__ __forceinline__ bool stage_tile(const uint8_t* bytes, uint32_t B0, uint32_t B1,
                                           uint4* s_buf, uint32_t& sh) {
  const uintptr_t p0 = (uintptr_t)(bytes + B0);
  sh = (uint32_t)(p0 & 15u);
  const uint32_t nch = (sh + (B1 - B0) + 15u) >> 4;
  if (nch > TILE_CHUNKS) return false;
  const uint4* q = (const uint4*)(bytes + B0 - sh);  // keep the global address space
  for (uint32_t c = threadIdx.x; c < nch; c += WG) s_buf[c] = q[c];
  return true;
}

__global__ __launch_bounds__(WG) void k_tok_count(const uint8_t* __restrict__ bytes,
                                                  const uint32_t* __restrict__ off, uint32_t n,
                                                  uint32_t* __restrict__ nw) {
  __shared__ uint4 s_buf[TILE_CHUNKS];
  for (uint32_t t0 = blockIdx.x * WG; t0 < n; t0 += gridDim.x * WG) {
    const uint32_t t1 = min(t0 + WG, n);
    const uint32_t B0 = off[t0], B1 = off[t1];
    uint32_t sh;
    const bool tiled = stage_tile(bytes, B0, B1, s_buf, sh);
    __syncthreads();
    const uint32_t t = t0 + threadIdx.x;
    if (t < t1) {
      const uint32_t b = off[t], e = off[t + 1];
      uint32_t c = 1;
      if (tiled) {
        const uint8_t* p = (const uint8_t*)s_buf + sh + (b - B0);
        for (uint32_t i = 0; i < e - b; ++i) c += (p[i] == '/');
      } else {
        for (uint32_t i = b; i < e; ++i) c += (bytes[i] == '/');
      }
      nw[t] = c;
    }
    __syncthreads();
  }
}

struct TokArgs {
  const uint8_t* bytes;
  const uint32_t* off;
  uint32_t n;
  const uint32_t* wbase;
  uint64_t* wh;
  uint4* rec;
  uint32_t* exact_id;
  const uint4* exact;
  uint64_t xmask;
  const uint8_t* fbytes;
  const uint64_t* foff;
  const uint4* fver;
  uint64_t word_mask;
  uint64_t full_mask;
  bool exact_empty;
};

template <class P>
__device__ __forceinline__ void tok_one(const TokArgs& A, uint32_t t, P p, uint32_t len) {
  const uint32_t wb = A.wbase[t];
  uint64_t hw = FNV_OFF, hall = FNV_OFF, h0 = 0;
  uint32_t k = 0, wlen = 0, flags = 0, c0 = 0;
  if (len > 0 && p[0] == '$') flags |= T_DOLLAR;
  for (uint32_t i = 0; i < len; ++i) {
    const uint32_t c = p[i];
    hall = fnv_step(hall, c);
    if (c == '/') {
      if (wlen == 1 && (c0 == '+' || c0 == '#')) flags |= T_WILD;
      const uint64_t h = word_hash(hw, A.word_mask);
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
  const uint64_t h = word_hash(hw, A.word_mask);
  if (k == 0) h0 = h;
  A.wh[wb + k] = h;
  ++k;
  A.rec[t] = make_uint4(wb, k, flags | ((uint32_t)(h0 >> 32) << 8), (uint32_t)h0);

  // exact route key (all route keys, wildcard strings included: emqx_router.erl:143,157)
  uint32_t hit = NONE;
  if (!A.exact_empty) {
    const uint64_t fh = full_hash(hall, A.full_mask);
    uint64_t i = exact_slot(fh, A.xmask);
    for (;;) {
      const uint4 s = A.exact[i];
      if (s.z == NONE) break;
      if (tag_of(s) == fh && s.w == len) {
        const uint8_t* fp = len <= VINL ? (const uint8_t*)(A.fver + (uint64_t)s.z * 4) + 4
                                        : A.fbytes + A.foff[s.z];
        if (bytes_equal(p, fp, len)) {
          hit = s.z;
          break;
        }
      }
      i = (i + 1) & A.xmask;
    }
  }
  A.exact_id[t] = hit;
}

__global__ __launch_bounds__(WG) void k_tok_hash(TokArgs A) {
  __shared__ uint4 s_buf[TILE_CHUNKS];
  for (uint32_t t0 = blockIdx.x * WG; t0 < A.n; t0 += gridDim.x * WG) {
    const uint32_t t1 = min(t0 + WG, A.n);
    const uint32_t B0 = A.off[t0], B1 = A.off[t1];
    uint32_t sh;
    const bool tiled = stage_tile(A.bytes, B0, B1, s_buf, sh);
    __syncthreads();
    const uint32_t t = t0 + threadIdx.x;
    if (t < t1) {
      const uint32_t b = A.off[t], e = A.off[t + 1];
      if (tiled)
        tok_one(A, t, (const uint8_t*)s_buf + sh + (b - B0), e - b);
      else
        tok_one(A, t, A.bytes + b, e - b);
    }
    __syncthreads();
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

#include "gm_walk.inc"

// ----------------------------------------------------------------------------------------
// verify (flags + counts) and deferred scatter
// ----------------------------------------------------------------------------------------

struct VerifyArgs {
  const uint8_t* tbytes;
  const uint32_t* toff;
  const uint8_t* fbytes;
  const uint64_t* foff;
  const uint4* fver;
  const uint32_t* pt;
  const uint32_t* pf;
  uint32_t* pr;
  uint32_t pcap;
  uint32_t* cnt;
  uint32_t* rej;
  uint2* rlist;
  uint32_t rcap;
  uint32_t* ctl;
};

constexpr uint32_t TWIN = 5;  // 16-B chunks of topic window per lane (topics <= 64 B in LDS)

// Byte view of one lane's chunk-major LDS window: chunk c of lane `tid` lives at
// base[c * WG * 16], so the 16-B stores of a wave are bank-conflict free.
struct LdsWin {
  const uint8_t* base;
  uint32_t sh;
  __device__ __forceinline__ uint8_t operator[](uint32_t x) const {
    const uint32_t y = x + sh;
    return base[(y >> 4) * (WG * 16) + (y & 15u)];
  }
};

__global__ __launch_bounds__(WG) void k_verify(VerifyArgs A) {
  __shared__ uint4 s_tw[TWIN][WG];
  __shared__ uint4 s_fr[4][WG];
  const uint32_t tid = threadIdx.x;
  const uint32_t top = min(A.ctl[CTL_PAIR_TOP], A.pcap);
  for (uint32_t i = blockIdx.x * WG + tid; i < top; i += gridDim.x * WG) {
    const uint32_t t = A.pt[i];
    if (t == NONE) continue;
    const uint32_t f = A.pf[i];
    const uint32_t tb0 = A.toff[t], tl = A.toff[t + 1] - tb0;
    const uint4* rp = A.fver + (uint64_t)f * 4;
    const uint4 r0 = rp[0], r1 = rp[1], r2 = rp[2], r3 = rp[3];
    const uint32_t fl = r0.x;
    bool ok;
    if (tl <= 64 && fl <= VINL) {
      const uintptr_t p = (uintptr_t)(A.tbytes + tb0);
      const uint32_t sh = (uint32_t)(p & 15u);
      const uint4* q = (const uint4*)(A.tbytes + tb0 - sh);  // global address space kept
      const uint32_t nch = (sh + tl + 15u) >> 4;
#pragma unroll
      for (uint32_t c = 0; c < TWIN; ++c)
        if (c < nch) s_tw[c][tid] = q[c];
      s_fr[0][tid] = r0;
      s_fr[1][tid] = r1;
      s_fr[2][tid] = r2;
      s_fr[3][tid] = r3;
      const LdsWin T{(const uint8_t*)&s_tw[0][tid], sh};
      const LdsWin F{(const uint8_t*)&s_fr[0][tid], 4u};
      ok = mqtt_match(T, tl, F, fl);
    } else {
      const uint64_t fo = A.foff[f];
      ok = mqtt_match(A.tbytes + tb0, tl, A.fbytes + fo, fl);
    }
    if (!ok) {
      const uint32_t r = A.pr[i];
      A.pr[i] = r | REJ_BIT;
      atomicSub(&A.cnt[t], 1u);
      atomicAdd(&A.rej[t], 1u);
      A.ctl[CTL_ANY_REJ] = 1u;
      const uint32_t j = atomicAdd(&A.ctl[CTL_NREJ], 1u);
      if (j < A.rcap) A.rlist[j] = make_uint2(t, r);
    }
  }
}

struct ScatterArgs {
  const uint32_t* pt;
  const uint32_t* pf;
  const uint32_t* pr;
  uint32_t pcap;
  const uint32_t* row;
  const uint32_t* rej;
  const uint2* rlist;
  uint32_t rcap;
  uint32_t* out;
  uint32_t ocap;
  uint32_t* ctl;
};

__global__ __launch_bounds__(WG) void k_scatter(ScatterArgs A) {
  const uint32_t top = min(A.ctl[CTL_PAIR_TOP], A.pcap);
  const uint32_t nrej = A.ctl[CTL_NREJ];
  const bool inline_adj = nrej <= min(A.rcap, REJ_SCAN_MAX);
  for (uint32_t i = blockIdx.x * WG + threadIdx.x; i < top; i += gridDim.x * WG) {
    const uint32_t t = A.pt[i];
    if (t == NONE) continue;
    const uint32_t r = A.pr[i];
    if (r & REJ_BIT) continue;
    uint32_t adj = 0;
    if (nrej && A.rej[t]) {
      if (!inline_adj) {
        A.ctl[CTL_LEGACY] = 1u;
        continue;
      }
      for (uint32_t j = 0; j < nrej; ++j) {
        const uint2 e = A.rlist[j];
        adj += (e.x == t && e.y < r) ? 1u : 0u;
      }
    }
    const uint32_t pos = A.row[t] + r - adj;
    if (pos < A.ocap) A.out[pos] = A.pf[i];
  }
}

// ---- legacy path: verify + scatter with holes, then compaction ----

struct VerifyScatterArgs {
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

__global__ __launch_bounds__(WG) void k_verify_scatter(VerifyScatterArgs A) {
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
  g.cus = (uint32_t)cus;
  // 6 x 256-thread workgroups per CU = 24 waves: k_walk's SGPR count (~106) admits 6 per CU
  // (MI355X_MICROARCH "Residency"), its 16 KiB of LDS 10, its VGPRs 7 waves per SIMD.
  g.blocks = (uint32_t)cus * (wg_per_cu ? wg_per_cu : 6u);
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
  a.fver = ix.fver;
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

hipError_t launch_verify(const uint8_t* bytes, const uint32_t* off, const DevIndex& ix,
                         Scratch& sc, uint32_t n, const WalkGeom& g, hipStream_t s) {
  (void)n;
  VerifyArgs a;
  a.tbytes = bytes;
  a.toff = off;
  a.fbytes = ix.fbytes;
  a.foff = ix.foff;
  a.fver = ix.fver;
  a.pt = sc.pt;
  a.pf = sc.pf;
  a.pr = sc.pr;
  a.pcap = sc.p_cap;
  a.cnt = sc.cnt;
  a.rej = sc.rej;
  a.rlist = sc.rlist;
  a.rcap = sc.r_cap;
  a.ctl = sc.ctl;
  hipLaunchKernelGGL(k_verify, dim3(grid_for(sc.p_cap, g.cus * 8)), dim3(WG), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_scatter(Scratch& sc, uint32_t n, const WalkGeom& g, hipStream_t s) {
  (void)n;
  ScatterArgs a;
  a.pt = sc.pt;
  a.pf = sc.pf;
  a.pr = sc.pr;
  a.pcap = sc.p_cap;
  a.row = sc.row;
  a.rej = sc.rej;
  a.rlist = sc.rlist;
  a.rcap = sc.r_cap;
  a.out = sc.out;
  a.ocap = sc.o_cap;
  a.ctl = sc.ctl;
  hipLaunchKernelGGL(k_scatter, dim3(grid_for(sc.p_cap, g.cus * 8)), dim3(WG), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_verify_scatter(const uint8_t* bytes, const uint32_t* off, const DevIndex& ix,
                                 Scratch& sc, uint32_t n, hipStream_t s) {
  (void)n;
  VerifyScatterArgs a;
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
