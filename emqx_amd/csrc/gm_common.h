// gm_common.h -- layout constants and token/hash functions shared by the host index builder
// and the gfx950 kernels.  The device index layout is described in DESIGN.md "Data layout".
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define GM_HD __host__ __device__ __forceinline__
#else
#define GM_HD static inline
#endif

namespace gm {

constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t TOMB = 0xFFFFFFFEu;  // deleted slot / exact entry (delta commits)

// ---- level tokens ---------------------------------------------------------------------
// A level token identifies one topic level (emqx_topic:words/1 element).  A word of at most
// 7 bytes is packed injectively: bytes little-endian in bits 0..55, length in bits 56..62,
// bit 63 clear -- two different short words can never share a token, so trie edges over
// short words are exact.  A longer word gets bit 63 set and a 63-bit hash; only filters with
// such a word need the byte verification pass.  '+' has a token no word can have.
constexpr uint64_t TOK_HASHED = 1ull << 63;
constexpr uint64_t PLUS_TOK = 0x7FFFFFFFFFFFFFFFull;  // length field 127: impossible for a word
constexpr uint32_t TOK_INLINE_MAX = 7;

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

// Token of a finished word: `packed` = its first bytes little-endian, `fnv` = FNV-1a state
// over all its bytes, `len` = its length.  `test_mask` != 0 selects the collision-test mode in
// which every word is hashed and only the masked bits of the hash are kept.
GM_HD uint64_t word_token(uint64_t packed, uint64_t fnv, uint32_t len, uint64_t test_mask) {
  if (test_mask) return TOK_HASHED | (fmix64(fnv) & test_mask);
  if (len <= TOK_INLINE_MAX) return packed | ((uint64_t)len << 56);
  return TOK_HASHED | (fmix64(fnv) >> 1);
}

// Route-key hash (exact table): over the key's bytes taken as little-endian 32-bit words, the
// last one zero-padded, in two 32-bit multiply-rotate lanes folded through fmix64.  It needs
// only the bytes (not the level tokens), so the device issues the table probe before it
// tokenises.  `mask` keeps fewer bits in the collision tests.
GM_HD void key_hash_init(uint32_t len, uint32_t& a, uint32_t& b) {
  a = 0x9747b28cu ^ len;
  b = 0x85ebca6bu + len;
}
GM_HD void key_hash_word(uint32_t w, uint32_t& a, uint32_t& b) {
  a ^= w * 0xcc9e2d51u;
  a = ((a << 15) | (a >> 17)) * 5u + 0xe6546b64u;
  b += w * 0x1b873593u;
  b = ((b << 13) | (b >> 19)) * 0x85ebca6bu ^ 0xc2b2ae35u;
}
GM_HD uint64_t key_hash_final(uint32_t a, uint32_t b, uint64_t mask) {
  return fmix64(((uint64_t)a << 32) | b) & mask;
}
GM_HD uint64_t key_hash(const uint8_t* p, uint32_t len, uint64_t mask) {
  uint32_t a, b;
  key_hash_init(len, a, b);
  for (uint32_t i = 0; i < len; i += 4) {
    uint32_t w = 0;
    for (uint32_t j = 0; j < 4 && i + j < len; ++j) w |= (uint32_t)p[i + j] << (8 * j);
    key_hash_word(w, a, b);
  }
  return key_hash_final(a, b, mask);
}

// ---- edge slots -------------------------------------------------------------------------
// 32 B per slot, 2 x uint4, one slot per trie edge (parent --level token--> child C):
//   s0 = {tok.lo, tok.hi, parent, cf}       key = (parent node id, level token), exact
//   s1 = {hf, tw, p.cf, p.hf}
//   cf  = C's node id (26 bits) | C's flags (4 bits) | C's depth code (2 bits)
//   hf  = filter id of "C_path/#", NONE, or LIST_MULTI | index into the multi[] list pool
//   tw  = wildcard filter(s) ending exactly at C (fid, or LIST_MULTI|multi index)
//   p   = C's '+' child {cf, hf} (cf = 0 if there is none; node 0 is the root, never a child),
//         carried so that the walk expands it without a probe.  The rest of p (its terminal
//         filters, its own '+' child) comes from the (C, '+') slot when the walk needs it.
// Non-wildcard trie keys ending at a node (only single-level '$' topics read them,
// emqx_trie.erl:287) live in a per-node side array.  An empty slot has parent == NONE; a slot
// freed by a delta commit has parent == TOMB (never a node id, not empty: lookups go on).
// Slots come in 64-B buckets of EBUCKET (one line: a probe loads and checks both slots, so a
// collision inside the bucket costs no extra round trip); an edge goes to the first free slot
// of its home bucket (edge_slot) or of the buckets after it, and a lookup stops at a bucket
// with a free slot.
constexpr uint32_t SLOT_U4 = 2;
constexpr uint32_t EBUCKET = 2;
constexpr uint32_t EDGE_SLACK = 4;  // slots >= 4 x edges (load <= 1/4): fewer bucket overflows
constexpr uint32_t CF_ID_BITS = 26;
constexpr uint32_t CF_ID_MASK = (1u << CF_ID_BITS) - 1;
constexpr uint32_t MAX_NODES = CF_ID_MASK - 2;  // ids stay below FAT_ID and TOMB's / NONE's low 26 bits
// Fat buckets (path compression of single-literal-child nodes).  A node C at depth 2, 4 or 6,
// reached by a literal edge, whose only literal child is G, takes a whole bucket: C's slot in
// the bucket's first half and G's slot in its second half, whose parent word is FAT_ID | G's
// signature (FAT_ID is never a node id, so no key probe matches the half).  G has no slot at
// its own hash position: a walk that resolves C finds G in the line it already loaded and, when
// the topic's word equals G's token, creates G's state in the same round trip; otherwise C has
// no matching literal child.  The root's only literal child, when it has one, is carried in
// the kernel arguments the same way.  A delta commit that gives a fat node a second literal
// child moves the half to its own hash position (the half's slot becomes TOMB), so a bucket
// holds a half exactly when its first node's literal children are that half alone.
constexpr uint32_t FAT_ID = CF_ID_MASK - 2;  // = MAX_NODES: no id; TOMB and NONE have low bits ..FE, ..FF
constexpr uint32_t FAT_MAX_DEPTH = 6;  // C's word (level depth(C)) is a record token (< REC_TOKS)
// Child signature: the top 6 bits of a slot's parent word (parent ids use 26) hold a 1-bit-per-
// class summary of the child's literal children's level tokens (class = sig_bit(token)); the
// walk does not probe a literal child whose token's class bit is clear.  Bits are only ever
// added (a delta commit ORs a new child in, deletions leave them), so a clear bit is exact.
constexpr uint32_t SIG_SHIFT = CF_ID_BITS;
GM_HD uint32_t sig_bit(uint64_t tok) {
  return 1u << (uint32_t)(((((tok * 0x9E3779B97F4A7C15ull) >> 32) & 0xFFFFFFFFull) * 6ull) >> 32);
}
// Depth code h of the child C (bits CF_H0 | CF_H1 = h & 1, h & 2): every filter strictly below
// C ends within h levels of C and none of them is a '#' filter, so a topic with more than h
// words left after C cannot match anything below it and the walk does not expand C's children.
// h = 0: unbounded (a '#' below, deeper filters, or unknown).  Exact at a full build; a delta
// commit only ever resets codes to 0.
constexpr uint32_t CF_H0 = 1u << 26;
constexpr uint32_t CF_LIT = 1u << 27;   // child has literal (non-'+') children
constexpr uint32_t CF_PLUS = 1u << 28;  // child has a '+' child
constexpr uint32_t CF_H1 = 1u << 29;
constexpr uint32_t CF_HMASK = CF_H0 | CF_H1;
GM_HD uint32_t cf_depth_code(uint32_t cf) { return ((cf >> 26) & 1u) | ((cf >> 28) & 2u); }
GM_HD uint32_t cf_with_depth_code(uint32_t cf, uint32_t h) {
  return (cf & ~CF_HMASK) | ((h & 1u) << 26) | ((h & 2u) << 28);
}
constexpr uint32_t CF_TW = 1u << 30;    // child terminates >=1 wildcard filter
constexpr uint32_t CF_TN = 1u << 31;    // child terminates >=1 non-wildcard trie key
// In the carried copy of a '+' child's cf (p.cf) bit 31 means something else: a '+' node never
// ends a non-wildcard key (a path through '+' is a wildcard filter), so CF_TN is free there and
// CF_PTW says "p.hf holds the child's terminal filters (tw), it has no '#' filter": the walk then
// emits them without a '+' probe.
constexpr uint32_t CF_PTW = 1u << 31;
constexpr uint32_t LIST_MULTI = 0x80000000u;  // tw/tn value is a multi[] index

GM_HD uint64_t edge_slot(uint32_t parent, uint64_t tok, uint64_t mask) {
  return fmix64(tok ^ ((uint64_t)parent * 0x9e3779b97f4a7c15ull)) & mask;
}
// Token-keyed parents.  The home bucket of a child edge (P, t) is edge_slot(P, t) -- or, when P
// is KEYED and t a literal word (not '+'), a hash of t alone, so the edges of the parents that share a child token share a
// line: on cfg3 site/S/device/D and site/+/device/D (D a global device id, one site's) sit in
// one bucket, and the walk's second probe of D is an L1/L2 hit instead of an HBM miss (r04).
// A full build keys the parents with many literal children whose every child token is the child
// of at most EBUCKET keyed parents (tune "keyed"); a node reached by a '+' edge or the root is
// never keyed (the walk creates those states without their slot).  The flag travels in the
// parent's slot as an impossible signature: CF_LIT with sig 0 (every literal child of an
// unkeyed node sets its class bit), so a keyed node's children are never filtered by class.
GM_HD uint64_t edge_home(uint32_t parent, uint64_t tok, uint64_t mask, bool keyed) {
  return keyed ? (fmix64(tok + 0x5851f42d4c957f2dull) & mask) : edge_slot(parent, tok, mask);
}
// Exact route-key table: 64-B buckets (one line) of XBUCKET 32-B entries, filled in order
// (linear probing over buckets); exact_slot gives the home bucket.  An entry carries the key's
// first XINL bytes, so a probe for a key of up to XINL bytes is decided by the one line it loads
// (no dependent load of a verification record):
//   e0 = {h32 (high half of the key hash), fid, len, key bytes 0..3}
//   e1 = {key bytes 4..7, 8..11, 12..15, 16..19}   (zero past len)
// A longer key's inline prefix and hash filter the candidates and its full bytes (verification
// record / string pool) confirm.  An empty entry has fid == NONE, a deleted one fid == TOMB.
// A bit per bucket (xovf) says whether some key whose probe passed it was placed beyond it: a
// probe that finds neither its key nor an empty entry in a bucket goes on only if the bit is
// set, so a miss costs its home bucket's line (plus the bit word, loaded beside it) even when
// that bucket is full.  Bits are only set (a delta commit may leave one set after deletions).
constexpr uint32_t XBUCKET = 2;
constexpr uint32_t XENT_U4 = 2;
constexpr uint32_t XINL = 20;
GM_HD uint64_t exact_slot(uint64_t fh, uint64_t mask) { return fmix64(fh + 0x632be59bd9b4e019ull) & mask; }
// k_tok's exact_id marker for a wildcard name whose route-key probe k_exact still has to run
constexpr uint32_t X_WILDPEND = 0xFFFFFFFDu;

// Filter verification record (64 B per filter id): {u32 len, 60 bytes of the filter}; the
// bytes of longer filters are read from the string pool.
constexpr uint32_t VREC = 64;
constexpr uint32_t VINL = 60;

// Per-topic record written by the tokenizer, 64 B = REC_U4 x uint4:
//   {wbase, n_words | flags << 24, tok0.lo, tok0.hi} {tok1, tok2} {tok3, tok4} {tok5, tok6}
// (tokens past the last level are 0); level tokens from REC_TOKS on are read from the token
// array at wbase.  Topics have at most 32,768 levels (65,535 bytes).  Stored in blocks of
// REC_BLOCK topics, part-major within a block (r06): part c of topic t at uint4 index
// (t / 64) * 256 + c * 64 + t % 64, so a wave's lanes, holding consecutive topics, read and write
// whole lines per 16-B access, and one address with immediate offsets of 1 KB reaches every part.
// A scratch of n topics holds ceil(n / 64) whole blocks.
constexpr uint32_t REC_U4 = 4;
constexpr uint32_t REC_BLOCK = 64;
constexpr uint32_t REC_TOKS = 7;
template <class T>
GM_HD T* rec_at(T* rec, uint32_t t) {
  return rec + (uint64_t)(t / REC_BLOCK) * (REC_BLOCK * REC_U4) + (t % REC_BLOCK);
}
constexpr uint32_t T_WILD = 1u;    // some level is exactly '+' or '#'  -> trie result []
constexpr uint32_t T_DOLLAR = 2u;  // first byte is '$' -> no root '+'/'#' (emqx_trie.erl:282)

}  // namespace gm
