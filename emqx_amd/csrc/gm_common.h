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
constexpr uint32_t PLUS_WH = 0xFFFFFFFFu;  // level-token hash reserved for the '+' edge
constexpr uint64_t EMPTY_TAG = ~0ull;      // edge slot never written (parent id 0xFFFFFFFF)

// Edge slot (16 B, uint4): {tag.lo, tag.hi, cf, hf}
//   tag = (parent_node << 32) | level_token_hash      (exact key: no cross-parent aliasing)
//   cf  = child node id (27 bits) | child flags (5 bits)
//   hf  = filter id of "child_path/#", NONE, or (CF_HFM) index into the multi[] list pool
constexpr uint32_t CF_ID_BITS = 27;
constexpr uint32_t CF_ID_MASK = (1u << CF_ID_BITS) - 1;
constexpr uint32_t CF_LIT = 1u << 27;   // child has literal (non-'+') children
constexpr uint32_t CF_PLUS = 1u << 28;  // child has a '+' child
constexpr uint32_t CF_HFM = 1u << 29;   // hf is a multi[] index
constexpr uint32_t CF_TW = 1u << 30;    // child terminates >=1 wildcard filter   (node_tw)
constexpr uint32_t CF_TN = 1u << 31;    // child terminates >=1 non-wildcard trie key (node_tn)
constexpr uint32_t LIST_MULTI = 0x80000000u;  // node_tw/node_tn value is a multi[] index

// Per-topic record written by the tokenizer (uint4): {wbase, n_words, flags, wh[0]}
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

// Level-token hash of one word (its FNV-1a state after the word's bytes).
GM_HD uint32_t word_hash(uint64_t fnv_state, uint32_t mask) {
  uint32_t h = (uint32_t)fmix64(fnv_state) & mask;
  return h == PLUS_WH ? 0xFFFFFFFEu : h;
}

// Whole-topic hash (exact route table key).
GM_HD uint64_t full_hash(uint64_t fnv_state, uint64_t mask) { return fmix64(fnv_state ^ 0x9e3779b97f4a7c15ull) & mask; }

GM_HD uint64_t edge_tag(uint32_t parent, uint32_t wh) { return ((uint64_t)parent << 32) | wh; }
GM_HD uint64_t edge_slot(uint64_t tag, uint64_t mask) { return fmix64(tag * 0x9e3779b97f4a7c15ull) & mask; }
GM_HD uint64_t exact_slot(uint64_t fh, uint64_t mask) { return fmix64(fh + 0x632be59bd9b4e019ull) & mask; }

}  // namespace gm
