// gm_common.h -- layout constants and hash functions shared by the host index builder and
// the gfx950 kernels.  The device index layout is described in DESIGN.md "Data layout".
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define GM_HD __host__ __device__ __forceinline__
#else
#define GM_HD static inline
#endif

namespace gm {

constexpr uint32_t NONE = 0xFFFFFFFFu;

// Level tokens are 37-bit hashes of one topic level; the all-ones token is reserved for '+'.
constexpr uint32_t WH_BITS = 37;
constexpr uint64_t WH_MASK = (1ull << WH_BITS) - 1;
constexpr uint64_t PLUS_WH = WH_MASK;
constexpr uint64_t EMPTY_TAG = ~0ull;  // parent id 2^27-1 is never assigned

// Edge slot (32 B = 2 x uint4):
//   a = {tag.lo, tag.hi, cf, hf}, b = {tw, tn, 0, 0}
//   tag = (parent_node << 37) | level_token        (exact key on (parent, token))
//   cf  = child node id (27 bits) | child flags (5 bits)
//   hf  = filter id of "child_path/#", NONE, or (CF_HFM) index into the multi[] list pool
//   tw  = wildcard filter(s) ending exactly at the child (fid, or LIST_MULTI|multi index)
//   tn  = non-wildcard trie key(s) ending at the child (same encoding)
constexpr uint32_t CF_ID_BITS = 27;
constexpr uint32_t CF_ID_MASK = (1u << CF_ID_BITS) - 1;
constexpr uint32_t MAX_NODES = CF_ID_MASK;  // ids 0 .. 2^27-2
constexpr uint32_t CF_LIT = 1u << 27;   // child has literal (non-'+') children
constexpr uint32_t CF_PLUS = 1u << 28;  // child has a '+' child
constexpr uint32_t CF_HFM = 1u << 29;   // hf is a multi[] index
constexpr uint32_t CF_TW = 1u << 30;    // child terminates >=1 wildcard filter
constexpr uint32_t CF_TN = 1u << 31;    // child terminates >=1 non-wildcard trie key
constexpr uint32_t LIST_MULTI = 0x80000000u;  // tw/tn value is a multi[] index

// Filter verification record (64 B per filter id): {u32 len, 60 bytes of the filter}; the
// bytes of longer filters are read from the string pool.
constexpr uint32_t VREC = 64;
constexpr uint32_t VINL = 60;

// Per-topic record written by the tokenizer (uint4): {wbase, n_words, flags|tok0_hi<<8, tok0_lo}
constexpr uint32_t T_WILD = 1u;    // some level is exactly '+' or '#'  -> trie result []
constexpr uint32_t T_DOLLAR = 2u;  // first byte is '$' -> no root '+'/'#' (emqx_trie.erl:282)

constexpr uint64_t FNV_OFF = 0xcbf29ce484222325ull;
constexpr uint64_t FNV_PRIME = 0x100000001b3ull;

GM_HD uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

GM_HD uint64_t fnv_step(uint64_t h, uint32_t b) { return (h ^ b) * FNV_PRIME; }

// Level token of one word (from its FNV-1a state after the word's bytes); `mask` keeps
// WH_BITS bits in production and fewer only to force collisions in tests.
GM_HD uint64_t word_hash(uint64_t fnv_state, uint64_t mask) {
  const uint64_t h = fmix64(fnv_state) & mask;
  return h == PLUS_WH ? PLUS_WH - 1 : h;
}

// Whole-topic hash (exact route table key).
GM_HD uint64_t full_hash(uint64_t fnv_state, uint64_t mask) {
  return fmix64(fnv_state ^ 0x9e3779b97f4a7c15ull) & mask;
}

GM_HD uint64_t edge_tag(uint32_t parent, uint64_t wh) { return ((uint64_t)parent << WH_BITS) | wh; }
GM_HD uint64_t edge_slot(uint64_t tag, uint64_t mask) { return fmix64(tag * 0x9e3779b97f4a7c15ull) & mask; }
GM_HD uint64_t exact_slot(uint64_t fh, uint64_t mask) { return fmix64(fh + 0x632be59bd9b4e019ull) & mask; }

}  // namespace gm
