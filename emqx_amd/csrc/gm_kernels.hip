// gm_kernels.hip -- gfx950 (MI355X, CDNA4) kernels of the batched MQTT publish-match pipeline.
//
// Pipeline for one batch of N published topics (DESIGN.md "Kernels"):
//   k_tok            levels, level tokens, wildcard/'$' flags (one pass per 256-topic tile)
//   k_exact          exact route-key probe of every name, when there are plain route keys
//                                                                                (gm_tok.inc)
//   k_walk           persistent trie walk, matches staged as (topic, filter, rank) (gm_walk.inc)
//   k_verify         byte re-check of pairs whose filter has a hashed token   (gm_verify.inc)
//   k_scan_*         per-topic match counts -> CSR row pointers
//   k_scatter        staged pairs -> CSR rows                                  (gm_verify.inc)
//   legacy (rare)    verify+scatter then compaction, when too many pairs were rejected
#include <hip/hip_runtime.h>

#include "gm_common.h"
#include "gm_kernels.h"

namespace gm {

namespace {

constexpr uint32_t WG = 256;
constexpr uint32_t CH = STAGE_CHUNK;  // staged-pair slots reserved per wave per atomic
constexpr uint32_t TBLK = 128;  // topics claimed per wave per atomic (r02: 64 / 256 no better)
constexpr uint32_t SCAN_ITEMS = 16;
constexpr uint32_t SCAN_TILE = WG * SCAN_ITEMS;
static_assert(FB_SMALL_PAIRS == SCAN_TILE, "k_fb_small scans one tile");
static_assert(SCATTER_SCAN_MAX == SCAN_TILE, "k_scatter<true> scans one tile");
constexpr uint32_t TILE_BYTES = 16384;  // tokenizer LDS tile (256 topics)
constexpr uint32_t TILE_CHUNKS = TILE_BYTES / 16 + 2;
// The route-key probe over a table beyond the TLB's reach: random lines over an 8 GiB table come
// at a third of the 2 GiB rate (profiles/r02/gather_tlb.txt), and at the 2 GiB rate again when
// each workgroup draws from one range of at most ~2 GiB (profiles/r05/gather_part.txt).  Three
// ways to give cfg4's probe (100M keys, 8.6 GB, 1M names) that shape were measured, and all are
// slower than one plain pass (k_exact: 0.088 ms at r05):
//   * one pass per 2-GiB range (r02): 0.015 + 5 x 0.031 ms (each pass re-read every name and
//     probed at a fifth of the lanes);
//   * names binned by range, then probed in that order (r02): 0.170 ms (random per-name gathers);
//   * one partitioned launch (r05, k_exact_part): k_xhash + k_exact_part 0.110 ms.  Each wave
//     queues its range's names and probes them.  The added round trips per name (its hash,
//     then its bytes, then the bucket) cost more than the faster bucket lines save
//     (profiles/r05/ab_xpart/).
// k_exact_part stays as an option (emqxgm_tune("exact_range_kb"), tested); the default never
// chooses it (XRANGE_MIN_TABLE).
constexpr uint64_t XRANGE_MIN_TABLE = ~0ull;
constexpr uint32_t XRANGE_MIN_NAMES = 65536;
constexpr uint64_t XRANGE_DEFAULT = 2ull << 30;
constexpr uint32_t XPART_BLOCKS = 2048;  // k_exact_part workgroups (8 per CU)

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <class PA, class PB>
__device__ __forceinline__ bool bytes_equal(PA a, PB b, uint32_t len) {
  for (uint32_t i = 0; i < len; ++i)
    if (a[i] != b[i]) return false;
  return true;
}

// emqx_topic:match/2 (emqx_topic.erl:67-89) on raw bytes.  T and F are byte accessors over LDS
// or global memory.  A '+'/'#' word of T is compared literally, as match/2 does for wildcard
// names.  DOLLAR: the binary clauses (:70-73, a '$' name never matches a root wildcard); false
// for match/2 called on word lists, which skips them (emqx_authz_rule.erl:213-214).
template <bool DOLLAR = true, class PT, class PF>
__device__ __forceinline__ bool mqtt_match(PT T, uint32_t tl, PF F, uint32_t fl) {
  if (DOLLAR && tl > 0 && T[0] == '$' && fl > 0 && (F[0] == '+' || F[0] == '#')) return false;
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

// Thread-sequential tiles: thread i of a block owns items [16 i, 16 i + 16) of the block's
// SCAN_TILE, read and written as four 16-B vectors (the arrays are 256-B aligned); a ragged
// tail falls back to scalar accesses.
__device__ __forceinline__ void load16(const uint32_t* in, uint64_t i0, uint32_t n, uint32_t v[16]) {
  if (i0 + 16 <= n) {
    const uint4* q = (const uint4*)(in + i0);
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      const uint4 x = q[j];
      v[4 * j] = x.x, v[4 * j + 1] = x.y, v[4 * j + 2] = x.z, v[4 * j + 3] = x.w;
    }
  } else {
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) v[j] = (i0 + j < n) ? in[i0 + j] : 0u;
  }
}

// n_dev (optional): the element count is min(*n_dev, n), read on the device (n is then the
// capacity the grid was sized for); blocks past the last tile return at once.
__device__ __forceinline__ uint32_t scan_count(uint32_t n, const uint32_t* n_dev) {
  return n_dev ? min(*n_dev, n) : n;
}

__global__ __launch_bounds__(WG) void k_scan_partials(const uint32_t* __restrict__ in, uint32_t n,
                                                      uint32_t* __restrict__ part,
                                                      const uint32_t* __restrict__ n_dev) {
  __shared__ uint32_t s_w[WG / 64];
  n = scan_count(n, n_dev);
  if (blockIdx.x > 0 && (uint64_t)blockIdx.x * SCAN_TILE >= n) return;
  uint32_t v[16];
  load16(in, (uint64_t)blockIdx.x * SCAN_TILE + 16ull * threadIdx.x, n, v);
  uint32_t acc = 0;
#pragma unroll
  for (uint32_t j = 0; j < 16; ++j) acc += v[j];
  uint32_t tot;
  block_excl_scan(acc, s_w, tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// Each block adds up the partials of the blocks before it itself (a few hundred words), so the
// scan is two launches.  The last block writes the grand total to out_n (and total_dst).
__global__ __launch_bounds__(WG) void k_scan_final(const uint32_t* __restrict__ in, uint32_t n,
                                                   const uint32_t* __restrict__ part, uint32_t nb,
                                                   uint32_t* __restrict__ out,
                                                   uint32_t* __restrict__ total_dst,
                                                   const uint32_t* __restrict__ n_dev,
                                                   const uint32_t* __restrict__ ctl_src = nullptr,
                                                   uint32_t* __restrict__ ctl_dst = nullptr) {
  __shared__ uint32_t s_w[WG / 64];
  if (n_dev) {
    n = scan_count(n, n_dev);
    nb = n ? (n + SCAN_TILE - 1) / SCAN_TILE : 1u;
    if (blockIdx.x >= nb) return;
  }
  uint32_t* const out_n = out + n;
  uint32_t pre = 0;
  for (uint32_t i = threadIdx.x; i < blockIdx.x; i += WG) pre += part[i];
  uint32_t carry;
  block_excl_scan(pre, s_w, carry);  // carry = sum of part[0 .. blockIdx)
  const uint64_t i0 = (uint64_t)blockIdx.x * SCAN_TILE + 16ull * threadIdx.x;
  uint32_t v[16];
  load16(in, i0, n, v);
  uint32_t acc = 0;
#pragma unroll
  for (uint32_t j = 0; j < 16; ++j) acc += v[j];
  uint32_t tot;
  uint32_t x = carry + block_excl_scan(acc, s_w, tot);
#pragma unroll
  for (uint32_t j = 0; j < 16; ++j) {
    const uint32_t e = x;
    x += v[j];
    v[j] = e;
  }
  if (i0 + 16 <= n) {
    uint4* q = (uint4*)(out + i0);
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) q[j] = make_uint4(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]);
  } else {
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j)
      if (i0 + j < n) out[i0 + j] = v[j];
  }
  if (blockIdx.x == nb - 1 && threadIdx.x == 0) {
    *out_n = carry + tot;
    if (total_dst) *total_dst = carry + tot;
  }
  // a pass's row scan: its last block also copies the control words to the host mirror (every
  // kernel that writes them has finished but k_scatter, which mirrors its one word itself);
  // CTL_TOTAL is this block's own result
  if (ctl_dst && blockIdx.x == nb - 1)
    for (uint32_t i = threadIdx.x; i < CTL_N; i += WG)
      ctl_dst[i] = i == CTL_TOTAL ? carry + tot : ctl_src[i];
}

// Staged pairs (StgFmt, gm_kernels.h): the packed word and back; rank carries REJ_BIT when the
// pair was rejected, as the wide layout's z does.
__device__ __forceinline__ uint64_t stg_pack(const StgFmt& F, uint32_t t, uint32_t f, uint32_t r) {
  return ((uint64_t)t << F.tsh) | ((uint64_t)f << F.fsh) | ((uint64_t)(r & F.rmask) << 1) |
         ((r & REJ_BIT) ? 1ull : 0ull);
}
__device__ __forceinline__ uint3 stg_unpack(const StgFmt& F, uint64_t w) {
  return make_uint3((uint32_t)(w >> F.tsh), (uint32_t)(w >> F.fsh) & F.fmask,
                    ((uint32_t)(w >> 1) & F.rmask) | ((w & 1ull) ? REJ_BIT : 0u));
}
template <bool PK>
__device__ __forceinline__ uint3 stg_load(const uint3* stg, const StgFmt& F, uint64_t i) {
  if constexpr (PK) return stg_unpack(F, ((const uint64_t*)stg)[i]);
  else return stg[i];
}

#include "gm_tok.inc"
#include "gm_walk.inc"
#include "gm_verify.inc"
#include "gm_fanout.inc"
#include "gm_rules.inc"
#include "gm_retain.inc"

__global__ __launch_bounds__(WG) void k_row64(const uint32_t* row, uint64_t base, uint64_t* out,
                                              uint32_t m) {
  for (uint32_t i = blockIdx.x * WG + threadIdx.x; i < m; i += gridDim.x * WG) out[i] = base + row[i];
}

// Three result arrays into pinned host memory (blockIdx.y picks one): 16-B stores over the
// body, the ragged tail by the first block.
__global__ __launch_bounds__(WG) void k_ctl_out(const uint32_t* ctl, uint32_t* dst) {
  for (uint32_t i = threadIdx.x; i < CTL_N; i += WG) dst[i] = ctl[i];
}

__global__ __launch_bounds__(WG) void k_copy_out(CopyOut a0, CopyOut a1, CopyOut a2) {
  const CopyOut d = blockIdx.y == 0 ? a0 : blockIdx.y == 1 ? a1 : a2;
  const uint32_t n = d.n_dev ? min(*d.n_dev, d.cap) : d.n;
  const uint32_t nv = n >> 2;
  const uint4* s4 = (const uint4*)d.src;
  uint4* d4 = (uint4*)d.dst;
  for (uint32_t i = blockIdx.x * WG + threadIdx.x; i < nv; i += gridDim.x * WG) d4[i] = s4[i];
  if (blockIdx.x == 0 && threadIdx.x < (n & 3u)) d.dst[4 * nv + threadIdx.x] = d.src[4 * nv + threadIdx.x];
}

// ---- filter-sharded layout: results of one shard exported with global ids, and the
// shards' rows merged topic by topic (the shards are disjoint: nothing to dedupe) ----

__global__ __launch_bounds__(WG) void k_export(const uint32_t* row, const uint32_t* fid,
                                               const uint32_t* exact, uint32_t n, uint32_t pairs,
                                               const uint32_t* map, uint32_t* orow,
                                               uint32_t* ofid, uint32_t* oexact) {
  const uint32_t m = max(n + 1, pairs);
  for (uint32_t i = blockIdx.x * WG + threadIdx.x; i < m; i += gridDim.x * WG) {
    if (i <= n) orow[i] = row[i];
    if (i < n) {
      const uint32_t e = exact[i];
      oexact[i] = (map && e != NONE) ? map[e] : e;
    }
    if (i < pairs) ofid[i] = map ? map[fid[i]] : fid[i];
  }
}

// parts[3 * r + {0, 1, 2}] = shard r's {row, fid, exact}
__global__ __launch_bounds__(WG) void k_merge_count(const uint32_t* const* parts, uint32_t np,
                                                    uint32_t n, uint32_t* cnt, uint32_t* exact) {
  for (uint32_t t = blockIdx.x * WG + threadIdx.x; t < n; t += gridDim.x * WG) {
    uint32_t c = 0, e = NONE;
    for (uint32_t r = 0; r < np; ++r) {
      const uint32_t* row = parts[3 * r];
      c += row[t + 1] - row[t];
      e = min(e, parts[3 * r + 2][t]);  // a route key lives on exactly one shard
    }
    cnt[t] = c;
    exact[t] = e;
  }
}

__global__ __launch_bounds__(WG) void k_merge_fill(const uint32_t* const* parts, uint32_t np,
                                                   uint32_t n, const uint32_t* orow,
                                                   uint32_t* ofid) {
  for (uint32_t t = blockIdx.x * WG + threadIdx.x; t < n; t += gridDim.x * WG) {
    uint32_t d = orow[t];
    for (uint32_t r = 0; r < np; ++r) {
      const uint32_t* row = parts[3 * r];
      const uint32_t* fid = parts[3 * r + 1];
      for (uint32_t i = row[t], e = row[t + 1]; i < e; ++i) ofid[d++] = fid[i];
    }
  }
}

// ---- the compact wire form of a shard's result (filter-sharded layout over xGMI): per-topic
// pair counts (u8, or with WIRE_CNT2 two bit planes of 64 topics -- 2 bits a topic), the pairs'
// global ids (u32, or with WIRE_ID24 a u16 low half + a u8 high byte), and sparse lists of
// (topic, exact id) and (topic, count) for the counts the width cannot hold (>= 255 / >= 3).
// Sparse entries are appended with one atomic per wave (their order is free: the root
// scatters them). ----
constexpr uint32_t WIRE_CNT2 = 1u, WIRE_ID24 = 2u;  // include/emqx_gpumatch.h EMQXGM_WIRE_*

__device__ __forceinline__ uint32_t wave_append(bool v, uint32_t* ctr) {
  const uint64_t m = __ballot(v);
  uint32_t base = 0;
  if (lane_id() == 0 && m) base = atomicAdd(ctr, (uint32_t)__popcll(m));
  base = __shfl(base, 0, 64);
  return base + mbcnt64(m);
}

__global__ __launch_bounds__(WG) void k_wire_export(const uint32_t* row, const uint32_t* fid,
                                                    const uint32_t* exact, uint32_t n,
                                                    uint32_t pairs, const uint32_t* map,
                                                    uint32_t flags, uint8_t* cnt, uint8_t* ofid,
                                                    uint2* xs, uint2* ovf, uint32_t* ctr) {
  const uint32_t stride = gridDim.x * WG;
  const bool c2 = (flags & WIRE_CNT2) != 0;
  const uint32_t cap = c2 ? 3u : 255u;
  // topics in wave-aligned groups of 64 (a count plane word is one wave's ballot); every lane
  // of a block runs the same trip count (wave_append is a wave-wide ballot)
  const uint32_t n64 = (n + 63u) & ~63u;
  for (uint32_t base = blockIdx.x * WG; base < n64; base += stride) {
    const uint32_t i = base + threadIdx.x;
    const bool tv = i < n;
    const uint32_t c = tv ? row[i + 1] - row[i] : 0u;
    const uint32_t e = tv ? exact[i] : NONE;
    if (c2) {
      const uint32_t code = min(c, 3u);
      const uint64_t p0 = __ballot(code & 1u), p1 = __ballot((code >> 1) & 1u);
      if (lane_id() == 0 && i < n64 && i - lane_id() < n) {
        uint64_t* pl = (uint64_t*)cnt + 2ull * (i >> 6);
        pl[0] = p0;
        pl[1] = p1;
      }
    } else if (tv) {
      cnt[i] = (uint8_t)min(c, 255u);
    }
    const bool big = tv && c >= cap, hit = tv && e != NONE;
    const uint32_t po = wave_append(big, &ctr[1]);
    if (big) ovf[po] = make_uint2(i, c);
    const uint32_t px = wave_append(hit, &ctr[0]);
    if (hit) xs[px] = make_uint2(i, map ? map[e] : e);
  }
  for (uint32_t j = blockIdx.x * WG + threadIdx.x; j < pairs; j += stride) {
    const uint32_t id = map ? map[fid[j]] : fid[j];
    if (flags & WIRE_ID24) {
      ((uint16_t*)ofid)[j] = (uint16_t)id;
      ofid[2ull * pairs + j] = (uint8_t)(id >> 16);
    } else {
      ((uint32_t*)ofid)[j] = id;
    }
  }
}

// one part's counts from its wire form (counts its width cannot hold are patched in from the
// overflow list by k_wire_patch)
__global__ __launch_bounds__(WG) void k_wire_counts(const uint8_t* cnt, uint32_t flags, uint32_t n,
                                                    uint32_t* out) {
  for (uint32_t i = blockIdx.x * WG + threadIdx.x; i < n; i += gridDim.x * WG) {
    if (flags & WIRE_CNT2) {
      const uint64_t* pl = (const uint64_t*)cnt + 2ull * (i >> 6);
      const uint32_t b = i & 63u;
      out[i] = (uint32_t)((pl[0] >> b) & 1ull) | ((uint32_t)((pl[1] >> b) & 1ull) << 1);
    } else {
      out[i] = cnt[i];
    }
  }
}

// a part's 24-bit ids widened to u32
__global__ __launch_bounds__(WG) void k_wire_ids(const uint8_t* fid, uint32_t pairs, uint32_t* out) {
  for (uint32_t j = blockIdx.x * WG + threadIdx.x; j < pairs; j += gridDim.x * WG)
    out[j] = (uint32_t)((const uint16_t*)fid)[j] | ((uint32_t)fid[2ull * pairs + j] << 16);
}

// dst[e.x] = e.y for the m sparse entries (overflow counts; exact ids)
__global__ __launch_bounds__(WG) void k_wire_patch(const uint2* ent, uint32_t m, uint32_t* dst) {
  for (uint32_t i = blockIdx.x * WG + threadIdx.x; i < m; i += gridDim.x * WG) {
    const uint2 e = ent[i];
    dst[e.x] = e.y;
  }
}

__global__ __launch_bounds__(WG) void k_fill_u32(uint32_t* dst, uint32_t n, uint32_t v) {
  for (uint32_t i = blockIdx.x * WG + threadIdx.x; i < n; i += gridDim.x * WG) dst[i] = v;
}

// ---- the matched filters' bytes for the host (the NIF's filter binaries): lengths from the
// device copy of the string pool's offsets, a scan, then each pair's bytes gathered ----
__global__ __launch_bounds__(WG) void k_filter_len(const uint32_t* fid, uint32_t pairs,
                                                   const uint64_t* foff, uint32_t* len,
                                                   const uint32_t* pairs_dev) {
  pairs = pairs_dev ? min(*pairs_dev, pairs) : pairs;
  for (uint32_t j = blockIdx.x * WG + threadIdx.x; j < pairs; j += gridDim.x * WG) {
    const uint32_t f = fid[j];
    len[j] = (uint32_t)(foff[f + 1] - foff[f]);
  }
}

// Bytes [0, n) of the pool from byte s into d: aligned dword loads, eight (plus one) in flight
// per step, funnel-shifted into bytes (a byte-by-byte loop waited on every load: 28 round trips
// for a 28-B filter).  Reads only the dwords that hold the filter's bytes.
__device__ __forceinline__ void copy_filter(const uint8_t* __restrict__ pool, uint64_t s, uint32_t n,
                                            uint8_t* __restrict__ d) {
  if (n == 0) return;
  const uint32_t* w = (const uint32_t*)(pool + (s & ~3ull));
  const uint32_t sh = (uint32_t)(s & 3u), last = (sh + n - 1) >> 2;
  for (uint32_t i = 0; i < n; i += 32) {
    const uint32_t w0 = i >> 2;
    uint32_t v[9];
#pragma unroll
    for (uint32_t k = 0; k < 9; ++k) v[k] = w[min(w0 + k, last)];
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
      const uint32_t x = __builtin_amdgcn_alignbyte(v[k + 1], v[k], sh);
#pragma unroll
      for (uint32_t b = 0; b < 4; ++b)
        if (i + 4 * k + b < n) d[i + 4 * k + b] = (uint8_t)(x >> (8 * b));
    }
  }
}

// one lane per pair
__global__ __launch_bounds__(WG) void k_filter_gather(const uint32_t* __restrict__ fid, uint32_t pairs,
                                                      const uint64_t* __restrict__ foff,
                                                      const uint8_t* __restrict__ pool,
                                                      const uint32_t* __restrict__ ooff,
                                                      uint8_t* __restrict__ out) {
  for (uint32_t j = blockIdx.x * WG + threadIdx.x; j < pairs; j += gridDim.x * WG) {
    const uint32_t o = ooff[j];
    copy_filter(pool, foff[fid[j]], ooff[j + 1] - o, out + o);
  }
}

// A host window's whole result in one block for one D2H copy (emqxgm_match_batch_submit_filters):
// {byte total, byte offsets [pairs+1], filter ids [pairs], exact ids [n], bytes}, at offsets the
// host chose for cap_p pairs and cap_b bytes.  The pair count and the byte total are read on the
// device; a window beyond the caps writes only its total (the host finishes it synchronously).
struct FbPack {
  const uint32_t* fid;
  const uint32_t* pairs_dev;
  const uint64_t* foff;
  const uint8_t* pool;
  const uint32_t* ooff;   // the scan of the pairs' filter lengths (pairs + 1 entries)
  const uint32_t* total;  // bytes of all pairs
  const uint32_t* exact;
  const uint32_t* row;    // the pass's row pointers (n + 1)
  uint32_t n, cap_p;
  uint64_t cap_b;
  uint32_t* b_total;
  uint32_t* b_ooff;
  uint32_t* b_fid;
  uint32_t* b_exact;
  uint32_t* b_row;
  uint8_t* b_bytes;
};

__global__ __launch_bounds__(WG) void k_fb_pack(FbPack A) {
  const uint32_t pairs = *A.pairs_dev, total = *A.total;
  if (blockIdx.x == 0 && threadIdx.x == 0) *A.b_total = total;
  if (pairs > A.cap_p || total > A.cap_b) return;
  const uint32_t m = max(pairs, A.n) + 1;
  for (uint32_t i = blockIdx.x * WG + threadIdx.x; i < m; i += gridDim.x * WG) {
    if (i < A.n) A.b_exact[i] = A.exact[i];
    if (i <= A.n) A.b_row[i] = A.row[i];
    if (i <= pairs) A.b_ooff[i] = A.ooff[i];
    if (i < pairs) {
      const uint32_t f = A.fid[i], o = A.ooff[i];
      A.b_fid[i] = f;
      copy_filter(A.pool, A.foff[f], A.ooff[i + 1] - o, A.b_bytes + o);
    }
  }
}

// The whole filter-byte gather of a small window in one block (k_filter_len + the length scan +
// k_fb_pack in one launch, r04): every pair's filter length, their exclusive scan in LDS, then
// the packed block as k_fb_pack writes it.  For a block of at most SCAN_TILE pairs (cap_p).
__global__ __launch_bounds__(WG) void k_fb_small(FbPack A) {
  __shared__ uint32_t s_w[WG / 64];
  __shared__ uint32_t s_off[SCAN_TILE + 1];
  const uint32_t pairs = *A.pairs_dev;
  const uint32_t c = min(pairs, A.cap_p);  // (a window beyond cap_p is finished by the host)
  uint32_t len[SCAN_ITEMS];
  uint32_t acc = 0;
#pragma unroll
  for (uint32_t k = 0; k < SCAN_ITEMS; ++k) {
    const uint32_t j = threadIdx.x * SCAN_ITEMS + k;
    uint32_t l = 0;
    if (j < c) {
      const uint32_t f = A.fid[j];
      l = (uint32_t)(A.foff[f + 1] - A.foff[f]);
    }
    len[k] = l;
    acc += l;
  }
  uint32_t total;
  uint32_t x = block_excl_scan(acc, s_w, total);
#pragma unroll
  for (uint32_t k = 0; k < SCAN_ITEMS; ++k) {
    s_off[threadIdx.x * SCAN_ITEMS + k] = x;
    x += len[k];
  }
  if (threadIdx.x == 0) {
    s_off[c] = total;
    *A.b_total = total;
  }
  __syncthreads();
  if (pairs > A.cap_p || total > A.cap_b) return;
  const uint32_t m = max(pairs, A.n) + 1;
  for (uint32_t i = threadIdx.x; i < m; i += WG) {
    if (i < A.n) A.b_exact[i] = A.exact[i];
    if (i <= A.n) A.b_row[i] = A.row[i];
    if (i <= pairs) A.b_ooff[i] = s_off[i];
    if (i < pairs) {
      const uint32_t f = A.fid[i], o = s_off[i];
      A.b_fid[i] = f;
      copy_filter(A.pool, A.foff[f], s_off[i + 1] - o, A.b_bytes + o);
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
  // default 3 x 256-thread workgroups per CU: the walk is bounded by the random line rate of
  // HBM/MALL (tools/gather_bench: ~54 G lines/s), and more resident waves only thrash the L2
  // (measured sweep in profiles/r01/sweep_v3.txt)
  g.blocks = (uint32_t)cus * (wg_per_cu ? wg_per_cu : 4u);
  g.lanes = g.blocks * WG;
  return g;
}

uint32_t scan_tmp_words(uint32_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE + 1; }

hipError_t launch_scan_ctl(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* tmp,
                           uint32_t* total_dst, const uint32_t* ctl, uint32_t* ctl_host_dev,
                           hipStream_t s) {
  const uint32_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (nb == 0) return hipErrorInvalidValue;  // a pass has topics
  // one tile: k_scan_final's block 0 needs no partials (a launch less for small windows)
  if (nb > 1)
    hipLaunchKernelGGL(k_scan_partials, dim3(nb), dim3(WG), 0, s, in, n, tmp, (const uint32_t*)nullptr);
  hipLaunchKernelGGL(k_scan_final, dim3(nb), dim3(WG), 0, s, in, n, tmp, nb, out, total_dst,
                     (const uint32_t*)nullptr, ctl, ctl_host_dev);
  return hipGetLastError();
}

hipError_t launch_scan(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* tmp,
                       uint32_t* total_dst, hipStream_t s) {
  const uint32_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (nb == 0) {
    // empty input: out[0] = 0 (and the total) without a kernel
    hipError_t e = hipMemsetAsync(out, 0, 4, s);
    if (e == hipSuccess && total_dst) e = hipMemsetAsync(total_dst, 0, 4, s);
    return e;
  }
  if (nb > 1)
    hipLaunchKernelGGL(k_scan_partials, dim3(nb), dim3(WG), 0, s, in, n, tmp, (const uint32_t*)nullptr);
  hipLaunchKernelGGL(k_scan_final, dim3(nb), dim3(WG), 0, s, in, n, tmp, nb, out, total_dst,
                     (const uint32_t*)nullptr);
  return hipGetLastError();
}

static ExactArgs exact_args(const DevIndex& ix, uint32_t xseq) {
  ExactArgs x;
  x.xseq = xseq;
  x.exact = ix.exact;
  x.xovf = ix.xovf;
  x.xmask = ix.xmask;
  x.xwbase = ix.xwbase;
  x.xwmask = ix.xwmask;
  x.fbytes = ix.fbytes;
  x.foff = ix.foff;
  x.full_mask = ix.full_mask;
  return x;
}

hipError_t launch_tok(const uint8_t* bytes, const uint32_t* off, uint32_t n, const DevIndex& ix,
                      Scratch& sc, hipStream_t s, uint32_t pair_top0, bool zero_rej,
                      const uint32_t* claim0, const uint8_t* src_bytes, const uint32_t* src_off) {
  if (n == 0) return hipSuccess;
  TokArgs a;
  a.ctl_host = sc.ctl_host_dev;
  a.cp_bytes = src_bytes ? const_cast<uint8_t*>(bytes) : nullptr;
  a.cp_off = src_off ? const_cast<uint32_t*>(off) : nullptr;
  if (src_bytes) bytes = src_bytes;
  if (src_off) off = src_off;
  for (uint32_t cs = 0; cs < WALK_SHARDS; ++cs) a.claim0[cs] = claim0 ? claim0[cs] : 0u;
  a.pair_top0 = pair_top0;
  a.rej = zero_rej ? sc.rej : nullptr;
  a.bytes = bytes;
  a.off = off;
  a.n = n;
  a.nw = sc.nw;
  a.wh = sc.wh;
  a.rec = sc.rec;
  a.exact_id = sc.exact_id;
  a.ctl = sc.ctl;
  a.test_mask = ix.test_mask;
  a.wild_empty = ix.wild_empty;
  a.nt_rec = n >= TOK_NT_MIN;
  const dim3 grid(grid_for(n, 8192));
  const ExactArgs X = exact_args(ix, sc.xseq);
  if (a.cp_bytes) {
    if (ix.plain_empty)
      hipLaunchKernelGGL((k_tok<false, true>), grid, dim3(WG), 0, s, a, X);
    else
      hipLaunchKernelGGL((k_tok<true, true>), grid, dim3(WG), 0, s, a, X);
  } else if (ix.plain_empty) {
    hipLaunchKernelGGL((k_tok<false, false>), grid, dim3(WG), 0, s, a, X);
  } else {
    hipLaunchKernelGGL((k_tok<true, false>), grid, dim3(WG), 0, s, a, X);
  }
  return hipGetLastError();
}

hipError_t launch_exact(const uint8_t* bytes, const uint32_t* off, uint32_t n, const DevIndex& ix,
                        Scratch& sc, const WalkGeom& g, hipStream_t s) {
  if (n == 0 || ix.plain_empty) return hipSuccess;
  const uint64_t buckets = ix.xwbase + ix.xwmask + 1;
  const bool forced = g.xrange_bytes != 0;
  const uint64_t rb = std::max<uint64_t>(1, (forced ? g.xrange_bytes : XRANGE_DEFAULT) / 64);
  if ((!forced && (buckets * 64ull <= XRANGE_MIN_TABLE || n < XRANGE_MIN_NAMES)) ||
      buckets >= NONE) {
    hipLaunchKernelGGL(k_exact, dim3(grid_for(n, 1u << 20)), dim3(WG), 0, s, bytes, off, n,
                       sc.exact_id, exact_args(ix, sc.xseq), ix.wild_empty, sc.ctl);
    return hipGetLastError();
  }
  const ExactArgs X = exact_args(ix, sc.xseq);
  hipLaunchKernelGGL(k_xhash, dim3(grid_for(n, 1u << 20)), dim3(WG), 0, s, bytes, off, n,
                     sc.exact_id, X, ix.wild_empty, sc.xh);
  // R equal ranges of at most rb buckets; G name slices per range
  const uint64_t R = (buckets + std::max<uint64_t>(rb, buckets >> 16) - 1) / std::max<uint64_t>(rb, buckets >> 16);
  const uint64_t rbe = (buckets + R - 1) / R;
  const uint64_t G = std::max<uint64_t>(1, std::min<uint64_t>(XPART_BLOCKS / R, (n + 511) / 512));
  hipLaunchKernelGGL(k_exact_part, dim3((uint32_t)(R * G)), dim3(WG), 0, s, bytes, off, n,
                     sc.exact_id, X, (const uint2*)sc.xh, (uint32_t)R, (uint32_t)rbe, sc.ctl);
  return hipGetLastError();
}

hipError_t launch_exact_owned(const uint8_t* bytes, const uint32_t* off, uint32_t n,
                              const DevIndex& ix, uint32_t parts, uint32_t part, uint32_t* out,
                              hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (ix.plain_empty) return hipMemsetAsync(out, 0xFF, (size_t)n * 4, s);
  hipLaunchKernelGGL(k_exact_owned, dim3(grid_for(n, 1u << 20)), dim3(WG), 0, s, bytes, off, n,
                     out, exact_args(ix, 0), parts, part);
  return hipGetLastError();
}

// Workgroups of one walk launch.  The deep-stack variants fit fewer blocks per CU (LDS): only
// as many are launched as are resident at once, so that no block of the persistent grid starts
// after the others have drained.  A batch that gives the grid less than one topic per lane
// launches only the blocks it fills: the waves a full grid adds only queue
// failed claims on the exhausted shard counters (r03: a cfg3 walk took 79 us at 64k topics and
// 80 us at 262k).
// Resident walk blocks: LDS-bound (all) or also bound by the geometry (wg_per_cu).
static uint32_t walk_cap_blocks(const WalkGeom& g, uint32_t level, bool lds_only = false) {
  constexpr uint32_t LDS_CU = 160u * 1024u;
  const uint32_t lds = level >= WALK_SPILL ? walk_lds_bytes(WALK_STK_SPILL)
                       : level == WALK_DEEP ? walk_lds_bytes(WALK_STK_DEEP, WALK_CPT)
                                            : walk_lds_bytes(WALK_STK_SHALLOW, WALK_CPT);
  return lds_only ? g.cus * (LDS_CU / lds) : std::min<uint32_t>(g.blocks, g.cus * (LDS_CU / lds));
}

// A pair walk may use every block LDS allows, also in the pipelined passes' geometry (three
// workgroups per CU, which leaves room for the other pass's kernels): a batch this small has
// little of them to run beside it, and 100k topics need 782 blocks, just past 768.
// Pairs also for large batches (claims past the grid's lanes) once an index's walks outgrew the
// shallow stack with one lane per topic (WALK_PAIRED and up): its searches are bushy, and two
// lanes share them, each with a shallower stack (r05, cfg2 1M topics: walk 1.207 -> 1.017 ms in
// the shallow stack instead of the deep one, verify+scan+scatter 0.224 -> 0.170 ms).  A narrow
// search (cfg3) only loses lanes to it: walk 0.33 -> 0.58 ms.  pair = 2 (A/B): every batch.
bool walk_pair(const WalkGeom& g, uint32_t n, uint32_t level) {
  if (!g.pair || !WALK_CPT || level >= WALK_SPILL || n == 0) return false;
  return g.pair == 2 || level >= WALK_PAIRED ||
         2ull * n <= (uint64_t)walk_cap_blocks(g, level, true) * WG;
}

// topics' lanes: two per topic for a pair walk
static uint64_t walk_lanes(const WalkGeom& g, uint32_t n, uint32_t level) {
  return walk_pair(g, n, level) ? 2ull * n : (uint64_t)n;
}

uint32_t walk_blocks(const WalkGeom& g, uint32_t n, uint32_t level) {
  // (a static pair walk may use every block LDS allows; a claiming one keeps the geometry)
  const bool pair = walk_pair(g, n, level);
  const uint32_t blocks = walk_cap_blocks(g, level, pair && 2ull * n <= (uint64_t)walk_cap_blocks(g, level, true) * WG);
  // one topic per lane (static_one), or per pair of lanes: only the blocks that hold topics
  // (r04: a 16-topic window launched one block per CU, all but one of them empty)
  const uint64_t lanes = walk_lanes(g, n, level);
  return std::min<uint32_t>(blocks, std::max<uint32_t>((uint32_t)((lanes + WG - 1) / WG), 1u));
}

// Topics per claim: a batch too small to give every wave TBLK topics is spread over all of them
// (a 100k-topic batch would otherwise keep 3 in 4 waves idle).
static uint32_t walk_tblk(uint32_t blocks, uint32_t n) {
  const uint32_t waves = blocks * (WG / 64);
  const uint32_t per_wave = waves ? (n + waves - 1) / waves : TBLK;
  return per_wave >= TBLK ? TBLK : ((per_wave + 7) & ~7u) < 8 ? 8 : ((per_wave + 7) & ~7u);
}

// Static first claims: wave r of shard cs's blocks (block b walks shard b % 8 first) owns the
// shard's topic block r without an atomic; the shard's counter starts past them (set by k_tok).
// Every wave claims at the start of a pass, ~500 atomics on each counter at once (r03).
// claim0[cs] = the counter's start value (0: none).
void walk_claim_init(const WalkGeom& g, uint32_t n, uint32_t level, uint32_t claim0[WALK_SHARDS]) {
  const uint32_t blocks = walk_blocks(g, n, level);
  const uint32_t tblk = walk_tblk(blocks, n);
  // exactly the walk's condition: claims at all (not static_one), static first ones
  const bool on = walk_lanes(g, n, level) > (uint64_t)blocks * WG;
  for (uint32_t cs = 0; cs < WALK_SHARDS; ++cs) {
    const uint32_t lo = (uint32_t)((uint64_t)n * cs / WALK_SHARDS);
    const uint32_t hi = (uint32_t)((uint64_t)n * (cs + 1) / WALK_SHARDS);
    const uint64_t waves = (uint64_t)(blocks > cs ? (blocks - cs + WALK_SHARDS - 1) / WALK_SHARDS : 0) * (WG / 64);
    claim0[cs] = on ? (uint32_t)std::min<uint64_t>(waves * tblk, hi - lo) : 0u;
  }
}

// Staged-pair chunks handed out before the walk starts: wave w of the launch owns chunk w from
// its first flush on (only later chunks take an atomic on CTL_PAIR_TOP, which k_tok sets to the
// end of the static ones).  0 when the staging buffer cannot hold one chunk per wave.
uint32_t walk_static_chunks(const WalkGeom& g, uint32_t n, uint32_t level, uint32_t pcap) {
  const uint64_t waves = (uint64_t)walk_blocks(g, n, level) * (WG / 64);
  return waves * CH <= pcap ? (uint32_t)waves : 0u;
}

hipError_t launch_walk(const DevIndex& ix, Scratch& sc, uint32_t n, const WalkGeom& g,
                       hipStream_t s, unsigned long long* census, uint32_t level,
                       uint32_t stat_chunks) {
  WalkArgs a;
  a.rec = sc.rec;
  a.wh = sc.wh;
  a.edges = ix.edges;
  a.emask = ix.emask;
  a.multi = ix.multi;
  a.root_cf = ix.root_cf;
  a.root_hf = ix.root_hf;
  a.root_pcf = ix.root_pcf;
  a.root_phf = ix.root_phf;
  a.tn_of = ix.tn_of;
  a.n = n;
  a.ctl = sc.ctl;
  a.cnt = sc.cnt;
  a.stg = sc.stg;
  a.fmt = sc.fmt;
  a.chk = sc.chk;
  a.pcap = sc.p_cap;
  a.spill = sc.spill;
  a.spill_items = sc.spill_items;
  a.lanes = g.lanes;
  constexpr uint32_t SH = WALK_STK_SHALLOW, DP = WALK_STK_DEEP, SP = WALK_STK_SPILL;
  constexpr bool C = WALK_CPT;
  const uint32_t blocks = walk_blocks(g, n, level);
  // a batch too small to give every wave TBLK topics is spread over all of them instead
  // (a 100k-topic batch would otherwise keep 3 in 4 waves idle)
  a.tblk = walk_tblk(blocks, n);
  // at most one topic per lane of the launched grid: lane gl walks topic gl, no claims (r03:
  // the failed claims of every wave on the exhausted counters dominated small batches)
  const bool pair = !census && walk_pair(g, n, level);
  a.static_one = (pair ? 2ull * n : (uint64_t)n) <= (uint64_t)blocks * WG ? 1u : 0u;
  a.stat_chunks = stat_chunks;
  a.static_claim = 1;
  a.census = census;
  a.leafp_mask = ix.leafp_mask;
  a.root_sig = ix.root_sig;
  a.rh0 = ix.rh0;
  a.rh1 = ix.rh1;
  const dim3 grid(blocks);
  if (census) {
    if (level >= WALK_SPILL)
      hipLaunchKernelGGL((k_walk<true, true, SP>), grid, dim3(WG), 0, s, a);
    else if (level == WALK_DEEP)
      hipLaunchKernelGGL((k_walk<true, false, DP, C>), grid, dim3(WG), 0, s, a);
    else
      hipLaunchKernelGGL((k_walk<true, false, SH, C>), grid, dim3(WG), 0, s, a);
  } else {
    if (level >= WALK_SPILL)
      hipLaunchKernelGGL((k_walk<false, true, SP>), grid, dim3(WG), 0, s, a);
    else if (level == WALK_DEEP && pair)
      hipLaunchKernelGGL((k_walk<false, false, DP, C, true>), grid, dim3(WG), 0, s, a);
    else if (level == WALK_DEEP)
      hipLaunchKernelGGL((k_walk<false, false, DP, C>), grid, dim3(WG), 0, s, a);
    else if (pair)
      hipLaunchKernelGGL((k_walk<false, false, SH, C, true>), grid, dim3(WG), 0, s, a);
    else
      hipLaunchKernelGGL((k_walk<false, false, SH, C>), grid, dim3(WG), 0, s, a);
  }
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
  a.fvbits = ix.fvbits;
  a.stg = sc.stg;
  a.fmt = sc.fmt;
  a.chk = sc.chk;
  a.pcap = sc.p_cap;
  a.cnt = sc.cnt;
  a.rej = sc.rej;
  a.rlist = sc.rlist;
  a.rcap = sc.r_cap;
  a.ctl = sc.ctl;
  // a wave per staging chunk, every block resident at once (k_verify: 4 blocks per CU by LDS)
  const dim3 grid(std::min<uint32_t>((sc.p_cap / CH + 3) / 4, g.cus * 4));
  if (sc.fmt.pk)
    hipLaunchKernelGGL(k_verify<true>, grid, dim3(WG), 0, s, a);
  else
    hipLaunchKernelGGL(k_verify<false>, grid, dim3(WG), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_scatter(Scratch& sc, uint32_t n, const WalkGeom& g, hipStream_t s,
                          bool mirror_ctl, bool fuse_scan) {
  ScatterArgs a;
  a.cnt = sc.cnt;
  a.n = n;
  a.row_out = sc.row;
  a.ctl_host = mirror_ctl ? sc.ctl_host_dev : nullptr;
  a.stg = sc.stg;
  a.fmt = sc.fmt;
  a.chk = sc.chk;
  a.pcap = sc.p_cap;
  a.row = sc.row;
  a.rej = sc.rej;
  a.rlist = sc.rlist;
  a.rcap = sc.r_cap;
  a.out = sc.out;
  a.ocap = sc.o_cap;
  a.ctl = sc.ctl;
  if (fuse_scan) {
    if (n > SCAN_TILE || !sc.ctl_host_dev) return hipErrorInvalidValue;
    a.ctl_host = sc.ctl_host_dev;
    // (a small batch's chunks are few: 128 blocks stride over them; the full grid was
    // thousands of blocks with nothing to do)
    const dim3 grid(std::min<uint32_t>(grid_for(sc.p_cap, g.cus * 8), 128u));
    if (sc.fmt.pk)
      hipLaunchKernelGGL((k_scatter<true, true>), grid, dim3(WG), 0, s, a);
    else
      hipLaunchKernelGGL((k_scatter<true, false>), grid, dim3(WG), 0, s, a);
  } else {
    const dim3 grid(grid_for(sc.p_cap, g.cus * 8));
    // (EMQXGM_SCATTER_DIRECT: the ungrouped stores, for A/B runs)
    static const bool direct = getenv("EMQXGM_SCATTER_DIRECT") != nullptr;
    if (direct) {
      if (sc.fmt.pk)
        hipLaunchKernelGGL((k_scatter<false, true>), grid, dim3(WG), 0, s, a);
      else
        hipLaunchKernelGGL((k_scatter<false, false>), grid, dim3(WG), 0, s, a);
    } else {
      if (sc.fmt.pk)
        hipLaunchKernelGGL(k_scatter_grp<true>, grid, dim3(WG), 0, s, a);
      else
        hipLaunchKernelGGL(k_scatter_grp<false>, grid, dim3(WG), 0, s, a);
    }
  }
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
  a.fvbits = ix.fvbits;
  a.stg = sc.stg;
  a.chk = sc.chk;
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

hipError_t launch_export(const uint32_t* row, const uint32_t* fid, const uint32_t* exact, uint32_t n,
                         uint32_t pairs, const uint32_t* map, uint32_t* orow, uint32_t* ofid,
                         uint32_t* oexact, hipStream_t s) {
  hipLaunchKernelGGL(k_export, dim3(grid_for((uint64_t)n + 1 + pairs, 8192)), dim3(WG), 0, s, row,
                     fid, exact, n, pairs, map, orow, ofid, oexact);
  return hipGetLastError();
}

hipError_t launch_merge(const uint32_t* const* parts, uint32_t np, uint32_t n, uint32_t* cnt,
                        uint32_t* tmp, uint32_t* orow, uint32_t* ofid, uint32_t* oexact,
                        uint32_t* total, hipStream_t s) {
  if (n == 0) return hipMemsetAsync(orow, 0, 4, s);
  hipLaunchKernelGGL(k_merge_count, dim3(grid_for(n, 8192)), dim3(WG), 0, s, parts, np, n, cnt,
                     oexact);
  hipError_t e = launch_scan(cnt, orow, n, tmp, total, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_merge_fill, dim3(grid_for(n, 8192)), dim3(WG), 0, s, parts, np, n, orow,
                     ofid);
  return hipGetLastError();
}

hipError_t launch_wire_export(const uint32_t* row, const uint32_t* fid, const uint32_t* exact,
                              uint32_t n, uint32_t pairs, const uint32_t* map, uint32_t flags,
                              uint8_t* cnt, uint8_t* ofid, uint2* xs, uint2* ovf, uint32_t* ctr,
                              hipStream_t s) {
  hipError_t e = hipMemsetAsync(ctr, 0, 8, s);
  if (e != hipSuccess) return e;
  const uint64_t m = std::max<uint64_t>((n + 63ull) & ~63ull, pairs);
  if (m == 0) return hipSuccess;
  hipLaunchKernelGGL(k_wire_export, dim3(grid_for(m, 8192)), dim3(WG), 0, s, row, fid, exact, n,
                     pairs, map, flags, cnt, ofid, xs, ovf, ctr);
  return hipGetLastError();
}

hipError_t launch_wire_rows(const uint8_t* cnt, uint32_t flags, const uint2* ovf, uint32_t novf,
                            uint32_t n, uint32_t* counts, uint32_t* tmp, uint32_t* row,
                            hipStream_t s) {
  if (n) {
    hipLaunchKernelGGL(k_wire_counts, dim3(grid_for(n, 8192)), dim3(WG), 0, s, cnt, flags, n,
                       counts);
    if (novf)
      hipLaunchKernelGGL(k_wire_patch, dim3(grid_for(novf, 8192)), dim3(WG), 0, s, ovf, novf,
                         counts);
  }
  return launch_scan(counts, row, n, tmp, nullptr, s);
}

hipError_t launch_wire_ids(const uint8_t* fid, uint32_t pairs, uint32_t* out, hipStream_t s) {
  if (pairs)
    hipLaunchKernelGGL(k_wire_ids, dim3(grid_for(pairs, 8192)), dim3(WG), 0, s, fid, pairs, out);
  return hipGetLastError();
}

hipError_t launch_wire_exact(const uint2* const* xs, const uint32_t* nx, uint32_t parts, uint32_t n,
                             uint32_t* exact, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_fill_u32, dim3(grid_for(n, 8192)), dim3(WG), 0, s, exact, n, NONE);
  for (uint32_t r = 0; r < parts; ++r)
    if (nx[r])
      hipLaunchKernelGGL(k_wire_patch, dim3(grid_for(nx[r], 8192)), dim3(WG), 0, s, xs[r], nx[r],
                         exact);
  return hipGetLastError();
}

hipError_t launch_filter_len(const uint32_t* fid, uint32_t pairs, const uint64_t* foff,
                             uint32_t* len, uint32_t* ooff, uint32_t* tmp, uint32_t* total,
                             hipStream_t s) {
  if (pairs)
    hipLaunchKernelGGL(k_filter_len, dim3(grid_for(pairs, 8192)), dim3(WG), 0, s, fid, pairs, foff,
                       len, (const uint32_t*)nullptr);
  return launch_scan(len, ooff, pairs, tmp, total, s);
}

hipError_t launch_filter_len_dev(const uint32_t* fid, const uint32_t* pairs_dev, uint32_t cap,
                                 const uint64_t* foff, uint32_t* len, uint32_t* ooff, uint32_t* tmp,
                                 uint32_t* total, hipStream_t s) {
  const uint32_t c = std::max<uint32_t>(cap, 1);
  hipLaunchKernelGGL(k_filter_len, dim3(grid_for(c, 1024)), dim3(WG), 0, s, fid, c, foff, len, pairs_dev);
  const uint32_t nb = (c + SCAN_TILE - 1) / SCAN_TILE;
  if (nb > 1)
    hipLaunchKernelGGL(k_scan_partials, dim3(nb), dim3(WG), 0, s, (const uint32_t*)len, c, tmp, pairs_dev);
  hipLaunchKernelGGL(k_scan_final, dim3(nb), dim3(WG), 0, s, (const uint32_t*)len, c, (const uint32_t*)tmp,
                     nb, ooff, total, pairs_dev);
  return hipGetLastError();
}

hipError_t launch_filter_gather(const uint32_t* fid, uint32_t pairs, const uint64_t* foff,
                                const uint8_t* pool, const uint32_t* ooff, uint8_t* out,
                                hipStream_t s) {
  if (pairs)
    hipLaunchKernelGGL(k_filter_gather, dim3(grid_for(pairs, 8192)), dim3(WG), 0, s, fid, pairs,
                       foff, pool, ooff, out);
  return hipGetLastError();
}

hipError_t launch_fb_pack(const uint32_t* fid, const uint32_t* pairs_dev, const uint64_t* foff,
                          const uint8_t* pool, const uint32_t* ooff, const uint32_t* total,
                          const uint32_t* exact, const uint32_t* row, uint32_t n, uint32_t cap_p,
                          uint64_t cap_b, uint8_t* block, hipStream_t s) {
  const FbLayout L(n, cap_p);
  FbPack a;
  a.fid = fid;
  a.pairs_dev = pairs_dev;
  a.foff = foff;
  a.pool = pool;
  a.ooff = ooff;
  a.total = total;
  a.exact = exact;
  a.row = row;
  a.n = n;
  a.cap_p = cap_p;
  a.cap_b = cap_b;
  a.b_total = (uint32_t*)(block + L.total);
  a.b_ooff = (uint32_t*)(block + L.ooff);
  a.b_fid = (uint32_t*)(block + L.fid);
  a.b_exact = (uint32_t*)(block + L.exact);
  a.b_row = (uint32_t*)(block + L.row);
  a.b_bytes = block + L.bytes;
  hipLaunchKernelGGL(k_fb_pack, dim3(grid_for(std::max<uint32_t>(cap_p, n) + 1, 2048)), dim3(WG), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_fb_small(const uint32_t* fid, const uint32_t* pairs_dev, const uint64_t* foff,
                           const uint8_t* pool, const uint32_t* exact, const uint32_t* row,
                           uint32_t n, uint32_t cap_p, uint64_t cap_b, uint8_t* block, hipStream_t s) {
  if (cap_p > SCAN_TILE) return hipErrorInvalidValue;
  const FbLayout L(n, cap_p);
  FbPack a;
  a.fid = fid;
  a.pairs_dev = pairs_dev;
  a.foff = foff;
  a.pool = pool;
  a.ooff = nullptr;
  a.total = nullptr;
  a.exact = exact;
  a.row = row;
  a.n = n;
  a.cap_p = cap_p;
  a.cap_b = cap_b;
  a.b_total = (uint32_t*)(block + L.total);
  a.b_ooff = (uint32_t*)(block + L.ooff);
  a.b_fid = (uint32_t*)(block + L.fid);
  a.b_exact = (uint32_t*)(block + L.exact);
  a.b_row = (uint32_t*)(block + L.row);
  a.b_bytes = block + L.bytes;
  hipLaunchKernelGGL(k_fb_small, dim3(1), dim3(WG), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_ctl_out(const uint32_t* ctl, uint32_t* ctl_host_dev, hipStream_t s) {
  hipLaunchKernelGGL(k_ctl_out, dim3(1), dim3(WG), 0, s, ctl, ctl_host_dev);
  return hipGetLastError();
}

hipError_t launch_copy_out(const CopyOut& a, const CopyOut& b, const CopyOut& c, hipStream_t s) {
  hipLaunchKernelGGL(k_copy_out, dim3(512, 3), dim3(WG), 0, s, a, b, c);
  return hipGetLastError();
}

hipError_t launch_row64(const uint32_t* row, uint64_t base, uint64_t* out, uint32_t m,
                        hipStream_t s) {
  if (m == 0) return hipSuccess;
  hipLaunchKernelGGL(k_row64, dim3(grid_for(m, 4096)), dim3(WG), 0, s, row, base, out, m);
  return hipGetLastError();
}

hipError_t launch_fanout(const DevIndex& ix, const Scratch& sc, FanScratch& fs, uint32_t n, bool fill,
                         hipStream_t s) {
  if (n == 0) return hipSuccess;
  FanArgs a;
  a.n = n;
  a.row = sc.row;
  a.fid = sc.out;
  a.exact_id = sc.exact_id;
  a.fan = ix.fan;
  a.rt_dst = ix.rt_dst;
  a.dl_sub = ix.dl_sub;
  a.nf = ix.fan_nf;
  a.cr = fs.cr;
  a.cd = fs.cd;
  a.rp = fs.rp;
  a.dp = fs.dp;
  a.o_rf = fs.o_rf;
  a.o_rd = fs.o_rd;
  a.o_df = fs.o_df;
  a.o_ds = fs.o_ds;
  if (fill)
    hipLaunchKernelGGL(k_fanout<true>, dim3(grid_for(n, 8192)), dim3(WG), 0, s, a);
  else
    hipLaunchKernelGGL(k_fanout<false>, dim3(grid_for(n, 8192)), dim3(WG), 0, s, a);
  return hipGetLastError();
}

// Delta commit (gm_engine.cpp PatchList): entry e copies ents[e].w (<= 64) dwords from
// src + ents[e].s to the device address ents[e].dst, lane j of wave e copying dword j.  Every
// table a commit touches (edge slots, exact entries, node side array, verify bits, pools,
// fan-out entries) goes in one list: one upload and one launch per commit.
__global__ void k_patch(const PatchEnt* __restrict__ ents, uint32_t n,
                        const uint32_t* __restrict__ src) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t e = i >> 6;
  const uint32_t j = (uint32_t)(i & 63);
  if (e >= n) return;
  const PatchEnt p = ents[e];
  if (j < p.w) ((uint32_t*)p.dst)[j] = src[p.s + j];
}

hipError_t launch_patch(const PatchEnt* ents, uint32_t n, const uint32_t* src, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t lanes = (uint64_t)n * 64;
  hipLaunchKernelGGL(k_patch, dim3((uint32_t)((lanes + WG - 1) / WG)), dim3(WG), 0, s, ents, n,
                     src);
  return hipGetLastError();
}

hipError_t launch_rules(const uint8_t* nb, const uint32_t* no, uint32_t n, const uint8_t* rb,
                        const uint32_t* ro, const uint32_t* rf, uint32_t nr, uint64_t rbytes,
                        uint32_t* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  RuleArgs a{nb, no, n, rb, ro, rf, nr, out};
  const dim3 grid(grid_for(n, 8192));
  if (rbytes <= RULE_LDS && nr <= RULE_LDS_N)
    hipLaunchKernelGGL(k_rules<true>, grid, dim3(WG), 0, s, a);
  else
    hipLaunchKernelGGL(k_rules<false>, grid, dim3(WG), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_retain_walk(const RetainDev& st, const uint8_t* fb, const uint32_t* fo, uint32_t n,
                              const uint8_t* tail, uint4* frames, uint32_t max_plus, uint32_t* cnt,
                              const uint32_t* cnt_in, const uint32_t* rbase,
                              const uint32_t* rshift, bool delta, uint2* runs, bool fill,
                              hipStream_t s) {
  if (n == 0) return hipSuccess;
  RetainArgs a{fb, fo, n, st.rn, st.redge, st.rmask, st.rch, st.rw, st.pool, tail, frames, max_plus,
               cnt, cnt_in, rbase, rshift, delta ? RUN_DELTA : 0u, runs};
  const dim3 grid((n + WG - 1) / WG);
  if (fill)
    hipLaunchKernelGGL(k_retain_walk<true>, grid, dim3(WG), 0, s, a);
  else
    hipLaunchKernelGGL(k_retain_walk<false>, grid, dim3(WG), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_retain_runs(const RetainDev& base, const RetainDev& delta, const uint2* runs,
                              uint32_t nr, uint64_t now, uint32_t* acnt, const uint32_t* abase,
                              uint32_t* out, unsigned long long* total, bool fill, hipStream_t s) {
  if (nr == 0) return hipSuccess;
  RunArgs a{runs, nr, base.sexp, base.sid, delta.sexp, delta.sid, now, acnt, abase, out, total};
  const dim3 grid(grid_for((uint64_t)nr * 64, 8192));
  if (fill)
    hipLaunchKernelGGL(k_retain_runs<true>, grid, dim3(WG), 0, s, a);
  else
    hipLaunchKernelGGL(k_retain_runs<false>, grid, dim3(WG), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_retain_ptr(const uint32_t* rbase, const uint32_t* abase, uint32_t n,
                             uint32_t* ptr, hipStream_t s) {
  hipLaunchKernelGGL(k_retain_ptr, dim3(n / WG + 1), dim3(WG), 0, s, rbase, abase, n, ptr);
  return hipGetLastError();
}

}  // namespace gm
