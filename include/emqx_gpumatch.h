/*
 * emqx_gpumatch.h -- C-ABI of the MI355X-native batched MQTT topic-matching engine.
 *
 * This is the drop-in boundary for the publish-time match path of EMQX 5.0.14
 * (fengyangdi/emqx).  Plain pointers and sizes only; no torch/HIP types.  Each entry point
 * names the reference interface it replaces (paths relative to the reference checkout):
 *
 *   emqxgm_trie_insert   <- emqx_trie:insert/1        apps/emqx/src/emqx_trie.erl:113-127
 *   emqxgm_trie_delete   <- emqx_trie:delete/1        apps/emqx/src/emqx_trie.erl:130-144
 *   emqxgm_trie_empty    <- emqx_trie:empty/0         apps/emqx/src/emqx_trie.erl:172-178
 *   emqxgm_trie_member   <- emqx_trie:lookup_topic/2  apps/emqx/src/emqx_trie.erl:267-271
 *   emqxgm_route_ref     <- route-bag key insert      apps/emqx/src/emqx_router_utils.erl:31-39
 *   emqxgm_route_unref   <- route-bag key delete      apps/emqx/src/emqx_router_utils.erl:48-71
 *   emqxgm_route_set     <- the same membership rule as a state, for a mirror of the committed
 *                           route table (emqx_router_utils.erl:34-39, 57-71; emqx_router.erl:72-92)
 *   emqxgm_async_match   <- emqx_trie:match/1 called from every publisher process at once
 *                           (emqx_broker.erl:218-232 -> emqx_router.erl:141-153, read_concurrency
 *                           tables emqx_trie.erl:70-75): the NIF's match_async/3
 *   emqxgm_commit        <- mnesia/mria commit point  (snapshot swap; readers never see partial
 *                           state; emqx_router_utils.erl:74-135 is where writes commit)
 *   emqxgm_match_batch   <- emqx_trie:match/1 + emqx_router:match_routes/1 over a batch of
 *                           published topics        apps/emqx/src/emqx_trie.erl:147-169,
 *                                                    apps/emqx/src/emqx_router.erl:141-157,
 *                           tokenising per emqx_topic:words/1 (emqx_topic.erl:155-169)
 *   emqxgm_match_device  <- the same with topic bytes / results resident in HBM
 *   emqxgm_filter_bytes  <- filter id -> filter binary (the trie returns binaries)
 *   emqxgm_route_add     <- emqx_router:do_add_route/2    apps/emqx/src/emqx_router.erl:124-138
 *   emqxgm_route_delete  <- emqx_router:do_delete_route/2 apps/emqx/src/emqx_router.erl:171-179
 *   emqxgm_subscriber_add/delete <- the local emqx_subscriber bag (emqx_broker.erl:150-214)
 *   emqxgm_publish_batch <- emqx_broker:publish/1 -> route(aggre(match_routes(Topic)))
 *                           apps/emqx/src/emqx_broker.erl:218-300, dispatch/2 :326-355
 *
 * Result semantics (bit-exact with the reference, SURVEY.md 8a/8a'):
 *   for topic t, trie row = { f in trie : emqx_trie:match(t) returns f }  (no duplicates;
 *   [] for a wildcard topic name), exact_id[t] = id of the route key equal to t's bytes (or
 *   EMQXGM_NONE).  match_routes(t) = routes(exact) ++ routes(row).  Row order is
 *   deterministic for a given committed index, but callers should treat it as a set, as the
 *   reference tests do (lists:sort).
 *
 * Return codes: 0 on success, or a negative errno: -EINVAL (bad argument), -ENOMEM (host or
 * device allocation failed), -EIO (device/HIP failure), -ENOENT (unknown id), -E2BIG (index
 * exceeds the device layout limits: 2^27 trie nodes, 2^31 filters).  There is no CPU fallback:
 * a device failure is reported, never silently recomputed on the host.
 *
 * Ownership: input buffers are borrowed for the duration of the call (the pipelined forms:
 * until the matching _wait returns).  Output arrays in emqxgm_out / emqxgm_dev_out are owned by
 * the engine and stay valid until the next match call on the same handle or emqxgm_destroy;
 * pipelined results as documented at their _submit.  Device inputs (emqxgm_match_device*) must
 * be complete in HBM when the call is made: the engine's streams do not wait for the caller's
 * (synchronise the stream that produced them first); the host-in forms copy their input
 * themselves.
 *
 * Threading (the reference reads with read_concurrency while writers commit in mria
 * transactions, emqx_trie.erl:70-75, emqx_router_utils.erl:74-135):
 *   - writers (insert/delete/route/subscriber calls, emqxgm_commit) are serialised by one writer
 *     lock; a full build of a large registry runs in a background thread without it (r05):
 *     meanwhile commits are delta patches of the current index, emqxgm_commit returns once the
 *     build is installed (changes made before it started show with it), and
 *     emqxgm_route_set_batch(.., EMQXGM_SET_COMMIT) returns as soon as its own changes show;
 *   - every match call reads the last committed epoch and never waits for a writer: a commit
 *     builds the next index beside the current one (a full build: seconds at 10M filters) and
 *     swaps it in atomically; a small delta is patched in place on the device, ordered on the GPU
 *     after the passes already enqueued and before every later one.  A pass that started before
 *     the swap completes against the epoch it started on;
 *   - match calls serialise among themselves (one pass context per call kind); filter_bytes,
 *     filter_copy, lookup_id, trie_member and trie_empty only take a shared read lock.
 */
#ifndef EMQX_GPUMATCH_H
#define EMQX_GPUMATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EMQXGM_NONE 0xFFFFFFFFu
#define EMQXGM_DEST_GROUP 0x80000000u /* dest handle bit: a shared-subscription group */
#define EMQXGM_RULE_EQ 1u    /* rule flag: {eq, Filter} -- the name must equal the filter */
#define EMQXGM_RULE_WORDS 2u /* rule flag: match/2 on word lists (no '$' clauses) */
#define EMQXGM_ABI_VERSION 5
#define EMQXGM_SET_COMMIT 1u /* emqxgm_route_set_batch: visible before the call returns */

typedef struct emqxgm emqxgm_t;

typedef struct emqxgm_cfg {
  int32_t device;          /* HIP device ordinal */
  uint32_t word_hash_bits; /* bits kept of each 37-bit level token (0 = 37, production);
                              small values only to force collisions in tests */
  uint32_t full_hash_bits; /* bits kept of the 64-bit whole-topic hash (exact table); 64 */
  uint32_t batch_max;      /* topics per device pass of emqxgm_match_batch (0 = 4Mi) */
  uint32_t walk_wg_per_cu; /* persistent walk workgroups per CU (0 = default) */
  uint32_t reject_cap;     /* verification rejects handled in-line per batch (0 = 1Mi);
                              beyond it a batch is redone on the compaction path */
  uint32_t reserved[2];
} emqxgm_cfg;

typedef struct emqxgm_out { /* host-resident result of emqxgm_match_batch */
  uint32_t n;               /* topics */
  uint64_t n_pairs;         /* total trie matches */
  const uint64_t* row_ptr;  /* [n+1] CSR offsets into filter_id */
  const uint32_t* filter_id;/* [n_pairs] matched trie filter ids */
  const uint32_t* exact_id; /* [n] route key equal to the topic, or EMQXGM_NONE */
} emqxgm_out;

typedef struct emqxgm_dev_out { /* device-resident result of emqxgm_match_device */
  uint32_t n;
  uint32_t n_pairs;
  const uint32_t* row_ptr;  /* device [n+1] */
  const uint32_t* filter_id;/* device [n_pairs] */
  const uint32_t* exact_id; /* device [n] */
  const uint32_t* n_words;  /* device [n] level count per topic (emqx_topic:levels/1) */
} emqxgm_dev_out;

typedef struct emqxgm_stats {
  uint64_t epoch;
  uint64_t n_filters;       /* ids ever assigned */
  uint64_t n_trie_filters;  /* committed trie members */
  uint64_t n_route_keys;    /* committed route keys */
  uint64_t n_nodes;         /* trie nodes (incl. root) */
  uint64_t n_edges;
  uint64_t edge_slots;
  uint64_t exact_slots;
  uint64_t device_bytes;    /* bytes of the committed device index */
  uint32_t max_depth;       /* deepest trie filter (levels) */
  uint32_t legacy_batches;  /* batches redone on the compaction path (many rejects) */
  uint64_t batches, topics, pairs;
  uint64_t rejected_pairs;  /* staged pairs rejected by byte verification (hash collisions) */
  uint64_t reruns;          /* passes redone (staging growth or legacy path) */
  double walk_ms;           /* summed walk-kernel time (HIP events), if profiling is on */
  uint64_t walk_launches;
  double total_ms;          /* summed device time of whole match passes, if profiling is on */
  uint64_t full_commits;    /* commits that rebuilt the device index */
  uint64_t delta_commits;   /* commits that patched it in place (small deltas) */
  double last_commit_ms;    /* host wall time of the last commit (build/patch + upload) */
  double tok_ms;            /* summed tokenizer-kernel time (HIP events), if profiling is on */
  uint64_t tok_launches;
  double exact_ms;          /* summed exact route-key probe time (k_exact; 0 without plain keys) */
  uint64_t keyed_nodes;     /* trie nodes whose literal children are placed by token */
  uint64_t buffer_grows;    /* pass scratch / host-pipe buffers reallocated (each a stall) */
  uint64_t sync_gathers;    /* host windows whose filter block outgrew its estimate (finished
                               synchronously in the wait) */
  uint64_t bg_builds;       /* full builds run in the background, beside the writers (r05) */
  uint64_t bg_waits;        /* commits that waited for one: the current tables could not take
                               their delta */
  double last_build_ms;     /* wall time of the last full build (background: start to ready) */
  uint64_t catchup_changes; /* filters replayed onto the last background build at its install */
} emqxgm_stats;

int emqxgm_abi_version(void);
int emqxgm_create(const emqxgm_cfg* cfg, emqxgm_t** out);
void emqxgm_destroy(emqxgm_t* h);

/* Index mutation (applies to the pending state; visible to match after emqxgm_commit). */
int emqxgm_trie_insert(emqxgm_t* h, const uint8_t* filter, uint32_t len, uint32_t* id);
int emqxgm_trie_delete(emqxgm_t* h, const uint8_t* filter, uint32_t len);
int emqxgm_route_ref(emqxgm_t* h, const uint8_t* filter, uint32_t len, uint32_t* id);
int emqxgm_route_unref(emqxgm_t* h, const uint8_t* filter, uint32_t len);
/* Bulk forms: n filters packed in bytes, filter i = bytes[offsets[i] .. offsets[i+1]). */
int emqxgm_trie_insert_many(emqxgm_t* h, const uint8_t* bytes, const uint64_t* offsets,
                            uint64_t n, uint32_t* ids /* nullable */);
int emqxgm_route_ref_many(emqxgm_t* h, const uint8_t* bytes, const uint64_t* offsets,
                          uint64_t n, uint32_t* ids /* nullable */);
int emqxgm_commit(emqxgm_t* h, uint64_t* epoch /* nullable */);
/* Health of the index (r06; SURVEY 5 "Failure detection").  The reference's route writes abort in
 * the caller when they fail (mria transactions, emqx_router_utils.erl:114-118); here the caller's
 * tables already hold a change when the device refuses it, so the engine fails CLOSED: a commit
 * that fails (emqxgm_commit, or the commit of an EMQXGM_SET_COMMIT set), a set that fails half-way
 * (-E2BIG) and emqxgm_mark_stale (the host saw a timeout or a failed window) mark the index
 * STALE, and every match entry (emqxgm_match_batch*, _match_device*, emqxgm_publish_batch, the
 * windows of the concurrent entry) returns -ESTALE until a repair -- the caller answers from its
 * own tables (the reference path) meanwhile, so no answer ever comes from an index that lacks a
 * change the caller made.  Repair: a successful emqxgm_commit clears the mark when no mark came
 * during it, every EMQXGM_STALE_RESYNC mark has a full resync (emqxgm_route_sync_begin .. _end)
 * begun after it, and an event on each of the engine's streams completes within "probe_ms"
 * (emqxgm_tune, 2000 default).  emqxgm_commit returns -ESTALE (-ETIMEDOUT: the probe) while the
 * index stays stale after its commit.  emqxgm_get_health returns the stale bits (0 = healthy). */
#define EMQXGM_STALE_COMMIT 1u /* a commit failed: the pending registry holds the change */
#define EMQXGM_STALE_RESYNC 2u /* the registry may lack changes: a full resync must follow */
typedef struct emqxgm_health_s {
  uint32_t stale;     /* EMQXGM_STALE_* bits; 0 = healthy */
  int32_t last_error; /* the last mark's errno (negative) */
  uint64_t marks;     /* times marked */
  uint64_t repairs;   /* times a repair cleared the marks */
  uint64_t refused;   /* match calls refused with -ESTALE */
} emqxgm_health_t;
int emqxgm_get_health(emqxgm_t* h, emqxgm_health_t* out);
/* The host's report (a window that timed out or failed): EMQXGM_STALE_RESYNC with errno err. */
int emqxgm_mark_stale(emqxgm_t* h, int err);
/* Index snapshot (the reference rebuilds its ram_copies route tables at start,
 * emqx_router.erl:78-92): _save commits pending changes and writes the committed registry (filter
 * strings, trie / route-key membership, routes, subscribers) and the host model of the device
 * index to `path`; _load restores them into a fresh handle of the same configuration and
 * publishes the index without rebuilding it (the device tables are generated from the model).
 * -EBUSY: the handle is not fresh; -EINVAL: not a snapshot of this configuration. */
int emqxgm_snapshot_save(emqxgm_t* h, const char* path);
int emqxgm_snapshot_load(emqxgm_t* h, const char* path);
/* Level-triggered route-key membership, for a mirror of the committed route table (the NIF's sync
 * process): present != 0 makes `filter` a route key and, when it is a wildcard filter
 * (emqx_topic:wildcard/1), a trie member; present == 0 removes both -- the state
 * emqx_router_utils.erl:34-39, 57-71 keeps (a route key exists while its filter has a route, a
 * wildcard filter is in the trie while it has one).  Idempotent: the index converges to the
 * route table's state whatever the number and order of the calls that told it so.  It overrides
 * the refcount emqxgm_route_ref / _unref keep: a mirror uses this call alone.  Visible after
 * emqxgm_commit. */
int emqxgm_route_set(emqxgm_t* h, const uint8_t* filter, uint32_t len, int present);
int emqxgm_route_set_many(emqxgm_t* h, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                          int present);
/* The same for n filters at once, each with its own state (present[i] != 0; present == NULL: all
 * present), and with flags EMQXGM_SET_COMMIT a commit that makes them visible to every match
 * started after the call returns: the writing node's subscribe / unsubscribe path (SURVEY 8b's
 * post-maybe_trans hook: the reference's subscriber has its route before SUBACK,
 * emqx_broker.erl:163-168, 484-486 -> emqx_router.erl:124-138) and the mirror's batched events.
 * It never waits for a full build: while one runs in the background, the changes are patched
 * into the index the readers have now (a delta commit) and replayed onto the new index when it
 * is installed.  It waits only when the current tables cannot take the delta (a table at its
 * load bound while the rebuild that grows it runs; emqxgm_stats.bg_waits counts them).  Full
 * builds of registries of at least emqxgm_tune("bg_build") filters run in the background. */
int emqxgm_route_set_batch(emqxgm_t* h, const uint8_t* bytes, const uint64_t* offsets,
                           const uint8_t* present, uint64_t n, uint32_t flags, uint64_t* epoch);
/* A full resync (the mirror's start and its periodic anti-entropy pass): _begin starts generation
 * *gen; every emqxgm_route_set(.., 1) until _end marks its filter; _end(gen) sets every route key
 * that was not marked absent (*removed of them).  -ESTALE if another _begin came in between. */
int emqxgm_route_sync_begin(emqxgm_t* h, uint32_t* gen);
int emqxgm_route_sync_end(emqxgm_t* h, uint32_t gen, uint64_t* removed /* nullable */);
/* 1 if `filter` is a committed route key (emqx_router:has_routes/1 of the committed index), 0 if
 * not. */
int emqxgm_route_member(emqxgm_t* h, const uint8_t* filter, uint32_t len);
/* 1 if the committed trie holds no filter, 0 otherwise (emqx_trie:empty/0). */
int emqxgm_trie_empty(emqxgm_t* h);
/* 1 if the committed trie holds exactly this filter key (emqx_trie:lookup_topic/2,
 * emqx_trie.erl:267-271), 0 otherwise. */
int emqxgm_trie_member(emqxgm_t* h, const uint8_t* filter, uint32_t len);

int emqxgm_lookup_id(emqxgm_t* h, const uint8_t* filter, uint32_t len, uint32_t* id);
/* Pointer to filter id's bytes in the engine's registry: valid until the next call that adds a
 * filter string or commits (insert / route / subscriber calls may grow the registry, and a commit
 * reserves room for the deltas ahead).  Prefer the copies. */
int emqxgm_filter_bytes(emqxgm_t* h, uint32_t id, const uint8_t** p, uint32_t* len);
/* Copy of filter id's bytes into buf (cap bytes): *len = its length; -ENOSPC if cap < *len. */
int emqxgm_filter_copy(emqxgm_t* h, uint32_t id, uint8_t* buf, uint32_t cap, uint32_t* len);
/* The filters ids[0..n) packed into buf: filter i = buf[offsets[i] .. offsets[i+1]) (offsets has
 * n+1 entries).  -ENOSPC if cap is too small (offsets[n] = the bytes needed). */
int emqxgm_filters_copy(emqxgm_t* h, const uint32_t* ids, uint64_t n, uint8_t* buf, uint64_t cap,
                        uint64_t* offsets);

/* Match n topics: topic i = bytes[offsets[i] .. offsets[i+1]), offsets has n+1 entries. */
int emqxgm_match_batch(emqxgm_t* h, const uint8_t* bytes, const uint32_t* offsets, uint32_t n,
                       emqxgm_out* out);
/* Same, with bytes/offsets already in HBM on the handle's device; results stay in HBM.
 * bytes_len = offsets[n] (passed so the engine never has to read it back). */
int emqxgm_match_device(emqxgm_t* h, const uint8_t* d_bytes, const uint32_t* d_offsets,
                        uint32_t n, uint64_t bytes_len, emqxgm_dev_out* out);

/* Pipelined form of emqxgm_match_device for a stream of batches (the reference's publishers
 * call match_routes concurrently, emqx_broker.erl:231; a batcher in front of the NIF hands the
 * engine one batch after another).  _submit enqueues the whole pass for one batch and returns
 * at once with a ticket; _wait(ticket) completes it (redoing it synchronously in the rare case
 * of a staging overflow or deep walk) and returns the device-resident result.  Up to
 * EMQXGM_PIPES passes are in flight per handle, each on its own HIP stream and scratch, so one
 * batch's walk tail overlaps the next batch's tokenizer and walk.  Ticket k's result lives in
 * pipe k % EMQXGM_PIPES and stays valid until ticket k + EMQXGM_PIPES is submitted; submitting
 * it before ticket k was waited for returns -EBUSY.  The caller keeps d_bytes/d_offsets alive
 * until the wait.  A commit first completes every pass in flight (results stay retrievable).
 * Results are identical to emqxgm_match_device's. */
#ifndef EMQXGM_PIPES
#define EMQXGM_PIPES 2
#endif
/* EMQXGM_PIPES of the library's build (a caller compiled against another header asks). */
int emqxgm_device_pipes(void);

/* Pinned (page-locked) host memory on the handle's device, for the caller's topic staging: a
 * batcher that packs its window into it gets full-speed H2D copies from emqxgm_match_batch.
 * NULL on failure.  emqxgm_host_free releases it. */
void* emqxgm_host_alloc(emqxgm_t* h, uint64_t bytes);
void emqxgm_host_free(emqxgm_t* h, void* p);
int emqxgm_match_device_submit(emqxgm_t* h, const uint8_t* d_bytes, const uint32_t* d_offsets,
                               uint32_t n, uint64_t bytes_len, uint64_t* ticket);
int emqxgm_match_device_wait(emqxgm_t* h, uint64_t ticket, emqxgm_dev_out* out);

/* Pipelined host-in / host-out form of emqxgm_match_batch: the call a NIF batcher makes (the
 * reference's publishers call match_routes concurrently from every scheduler,
 * emqx_broker.erl:231).  _submit enqueues, on one of EMQXGM_HOST_PIPES streams, the copy of the
 * batch into HBM, the whole device pass and the copy of its result into pinned host memory, and
 * returns at once; _wait(ticket) completes it.  With several tickets in flight one batch's
 * upload, another's pass and a third's download overlap.  The batch: n <= cfg.batch_max topics,
 * topic i = bytes[offsets[i] .. offsets[i+1]), offsets[0] == 0 and non-decreasing (-EINVAL
 * otherwise, checked on the host before anything is enqueued); bytes and
 * offsets stay untouched until the wait (pinned memory from emqxgm_host_alloc gives full-speed
 * copies).  The result (batch-local u32 row pointers, trie filter ids, exact ids) lives in
 * pinned buffers of the pipe and stays valid until ticket + EMQXGM_HOST_PIPES is submitted;
 * submitting that ticket before this one was waited for returns -EBUSY.  When no topic of the
 * batch equals a route key, exact_id points at an all-EMQXGM_NONE buffer of the pipe (same
 * lifetime) and no exact id crossed PCIe.  Results are identical to emqxgm_match_batch's. */
#define EMQXGM_HOST_PIPES 3
typedef struct emqxgm_batch_out {
  uint32_t n;
  uint32_t n_pairs;
  const uint32_t* row_ptr;   /* [n+1] offsets into filter_id */
  const uint32_t* filter_id; /* [n_pairs] matched trie filter ids */
  const uint32_t* exact_id;  /* [n] route key equal to the topic, or EMQXGM_NONE */
} emqxgm_batch_out;
int emqxgm_match_batch_submit(emqxgm_t* h, const uint8_t* bytes, const uint32_t* offsets,
                              uint32_t n, uint64_t* ticket);
int emqxgm_match_batch_wait(emqxgm_t* h, uint64_t ticket, emqxgm_batch_out* out);
/* _wait, plus the bytes of every matched pair's filter, gathered on the device from its copy of
 * the string pool and copied into pinned buffers of the pipe (same lifetime as the result): pair
 * j's filter is fbytes[foff[j] .. foff[j+1]), foff has n_pairs + 1 entries.  What a NIF needs to
 * build each caller's filter binaries without touching the host registry per pair. */
int emqxgm_match_batch_wait_filters(emqxgm_t* h, uint64_t ticket, emqxgm_batch_out* out,
                                    const uint32_t** foff, const uint8_t** fbytes);
/* _submit for a ticket that will be completed with _wait_filters: the filter-byte gather and the
 * copies of every result array (filter ids, byte offsets, bytes, exact ids) are enqueued behind
 * the pass -- packed on the device into one block that one copy brings into pinned memory --
 * sized by the pairs and bytes per topic of the pipe's recent windows (x1.2), so that
 * _wait_filters takes one stream synchronisation instead of four; a window beyond those sizes is
 * finished there synchronously.  Same arguments, errors and results as _submit + _wait_filters
 * (the NIF batcher core submits its windows this way).  A window of at most "zc_topics" topics
 * (emqxgm_tune; 65536 default) and 8 MiB whose bytes and offsets are pinned memory
 * (emqxgm_host_alloc) goes without DMA copies: the tokenizer reads it over PCIe and the result
 * block is written straight into the pipe's pinned buffer (r04: 16k-topic windows 150 -> 114 us
 * one at a time).  Either way bytes / offsets stay untouched until the wait. */
int emqxgm_match_batch_submit_filters(emqxgm_t* h, const uint8_t* bytes, const uint32_t* offsets,
                                      uint32_t n, uint64_t* ticket);

/* ---- publish fan-out (emqx_broker.erl:218-355) -------------------------------------------
 * Routes with dest identity: a plain route {Filter, Node} passes group = EMQXGM_NONE; a shared-
 * subscription route {Filter, {Group, Node}} passes both (handles < 2^31, chosen by the caller).
 * Like emqx_router:do_add_route/do_delete_route, the first route of a wildcard filter inserts it
 * into the trie and its last one removes it, the route key exists while the filter has a route
 * (the same refcount as emqxgm_route_ref), and adding an existing route or deleting an absent
 * one is a no-op.  Visible after emqxgm_commit, like every mutation. */
int emqxgm_route_add(emqxgm_t* h, const uint8_t* filter, uint32_t len, uint32_t node,
                     uint32_t group);
int emqxgm_route_delete(emqxgm_t* h, const uint8_t* filter, uint32_t len, uint32_t node,
                        uint32_t group);
/* node() of this broker: aggre entries {To, local_node} are dispatched to local subscribers. */
int emqxgm_set_local_node(emqxgm_t* h, uint32_t node);
/* The local subscriber bag (filter -> subscriber handle); duplicates / absent deletes: no-op. */
int emqxgm_subscriber_add(emqxgm_t* h, const uint8_t* filter, uint32_t len, uint32_t sub);
int emqxgm_subscriber_delete(emqxgm_t* h, const uint8_t* filter, uint32_t len, uint32_t sub);
/* Level-triggered forms for a mirror of the committed tables (the NIF's sync process and the
 * writing node's hook, r05): filter i = bytes[offsets[i] .. offsets[i+1]) gets exactly the dests
 * (node[j], group[j]) for j in [dptr[i], dptr[i+1]) -- its rows of the emqx_route bag,
 * emqx_router.erl:72-92: group = EMQXGM_NONE for a node dest, else the {Group, Node} dest --
 * and its route key / wildcard trie membership while it has any (emqxgm_route_set's rule);
 * or exactly the local subscribers subs[sptr[i] .. sptr[i+1]) (the emqx_subscriber bag,
 * emqx_broker.erl:150-214, 546-552).  Duplicates are ignored.  flags EMQXGM_SET_COMMIT: visible
 * before the call returns, as emqxgm_route_set_batch. */
int emqxgm_route_dests_batch(emqxgm_t* h, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                             const uint32_t* dptr, const uint32_t* node, const uint32_t* group,
                             uint32_t flags, uint64_t* epoch);
int emqxgm_subscribers_batch(emqxgm_t* h, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                             const uint32_t* sptr, const uint32_t* subs, uint32_t flags,
                             uint64_t* epoch);

typedef struct emqxgm_publish_out { /* host-resident result of emqxgm_publish_batch */
  uint32_t n;
  uint64_t n_routes;              /* aggre entries of the whole batch */
  uint64_t n_deliveries;          /* local dispatches of the whole batch */
  const uint64_t* route_ptr;      /* [n+1] topic i's entries: [route_ptr[i], route_ptr[i+1]) */
  const uint32_t* route_filter;   /* To of each entry (filter id) */
  const uint32_t* route_dest;     /* node handle, or EMQXGM_DEST_GROUP | group handle */
  const uint64_t* deliver_ptr;    /* [n+1] topic i's local dispatches */
  const uint32_t* deliver_filter; /* the filter (To) a dispatch goes through */
  const uint32_t* deliver_sub;    /* the subscriber it reaches */
} emqxgm_publish_out;

/* emqx_broker:publish/1 for a batch of topics: the aggre/1 entries of match_routes(Topic)
 * (node dests as {To, Node}, shared dests as {To, Group} with each group once per filter) and
 * the local dispatches of the entries {To, local_node} (every subscriber of To).  Entries of a
 * topic come in match_routes order (exact key first, then the trie row); callers treat them as
 * the set the reference's route/2 folds over. */
int emqxgm_publish_batch(emqxgm_t* h, const uint8_t* bytes, const uint32_t* offsets, uint32_t n,
                         emqxgm_publish_out* out);

/* First rule matching each name, for the scalar emqx_topic:match/2 loops outside the router:
 * emqx_authz_rule:match_topics/3 (apps/emqx_authz/src/emqx_authz_rule.erl:201-214: rules in
 * order, {eq, F} by equality, others by match/2 on word lists -> EMQXGM_RULE_WORDS) and
 * emqx_rewrite:match_and_rewrite/3 (apps/emqx_modules/src/emqx_rewrite.erl:145-150: match/2 on
 * binaries, flags 0).  names / rules: packed bytes + [n+1] / [n_rules+1] offsets on the host;
 * out[i] = index of the first matching rule, or EMQXGM_NONE.  Independent of the index. */
int emqxgm_match_rules(emqxgm_t* h, const uint8_t* name_bytes, const uint32_t* name_offsets,
                       uint32_t n, const uint8_t* rule_bytes, const uint32_t* rule_offsets,
                       const uint32_t* rule_flags, uint32_t n_rules, uint32_t* out);

/* ---- retained-message store: reverse match (filter -> stored topics) ----
 * The retainer's mnesia backend (apps/emqx_retainer/src/emqx_retainer_mnesia.erl) on the
 * device: topics of retained messages (the messages stay with the caller) with their expiry
 * times, and match_messages/3 (:185-195) for batches of subscription filters.  The selected set
 * is search_table/3's (:300-330): with index specs configured (emqxgm_retain_set_indices; the
 * default is the reference's ?DEFAULT_INDICES [[1,2,3],[1,3],[2,3],[3]],
 * emqx_retainer_schema.erl:24-29) the index path of the best-scoring index (select_index/2 and
 * condition/2, emqx_retainer_index.erl:83-91, 141-200), including its open index tail (a/+
 * also selects a/x/y under [1,2,3]); with none, or when no index scores, the full scan of
 * condition/1 (:97-112: '+' any word, a last '#' any tail).  No '$' rule; expiry 0 or > now.
 * Mutations are visible after emqxgm_retain_commit. */
typedef struct emqxgm_retain emqxgm_retain_t;
int emqxgm_retain_create(int32_t device, emqxgm_retain_t** out);
void emqxgm_retain_destroy(emqxgm_retain_t* r);
/* store_retained/2 (:138-152): insert or overwrite; expiry_ms 0 = never; *id = stable id */
int emqxgm_retain_store(emqxgm_retain_t* r, const uint8_t* topic, uint32_t len,
                        uint64_t expiry_ms, uint32_t* id);
/* delete_message/2 of one topic (:166-170, delete_message_by_topic/2 :345-349); absent: no-op */
int emqxgm_retain_delete(emqxgm_retain_t* r, const uint8_t* topic, uint32_t len);
int emqxgm_retain_clean(emqxgm_retain_t* r); /* clean/1 (:241-244) */
int emqxgm_retain_commit(emqxgm_retain_t* r);
/* Committed state = a base store plus a small delta store of the topics stored since the base
 * was built; re-storing or deleting a base topic patches it in place.  "delta_max": delta topics
 * before a commit rebuilds the base (-1 = max(4096, base / 16), 0 = rebuild at every commit). */
int emqxgm_retain_tune(emqxgm_retain_t* r, const char* key, int64_t value);
/* The retainer's index specs (retainer.backend.index_specs, config_indices/0 of
 * emqx_retainer_mnesia.erl:424-425): spec i = positions pos[offsets[i] .. offsets[i+1]), each
 * >= 1 and strictly ascending; n = 0 selects the full scan only (index_specs = []).  -EINVAL on a
 * malformed spec (then the specs are unchanged).  Applies to the next emqxgm_retain_match. */
int emqxgm_retain_set_indices(emqxgm_retain_t* r, const uint32_t* pos, const uint32_t* offsets,
                              uint32_t n);
/* out = {full rebuilds, delta commits, base topics (incl. deleted), delta topics} */
int emqxgm_retain_stats(emqxgm_retain_t* r, uint64_t out[4]);
/* size/1 (:246-247): committed topics */
int emqxgm_retain_size(emqxgm_retain_t* r, uint64_t* n);
/* read_message/2 (:182-183, read_messages/1 :372-382: expiry 0 or >= now), committed state:
 * 1 and *id if the topic is stored and live, 0 if not */
int emqxgm_retain_read(emqxgm_retain_t* r, const uint8_t* topic, uint32_t len, uint64_t now_ms,
                       uint32_t* id);
int emqxgm_retain_topic(emqxgm_retain_t* r, uint32_t id, const uint8_t** p, uint32_t* len);
typedef struct emqxgm_retain_out { /* host-resident, valid until the next call on r */
  uint32_t n;
  uint64_t n_ids;
  const uint64_t* ptr; /* [n+1]: filter i selects id[ptr[i] .. ptr[i+1]) */
  const uint32_t* id;  /* topic ids: a filter's base-store topics, then its delta-store topics,
                          each ascending in topic word order */
} emqxgm_retain_out;
/* match_messages/3 for a batch of filters (packed bytes + [n+1] offsets on the host) */
int emqxgm_retain_match(emqxgm_retain_t* r, const uint8_t* bytes, const uint32_t* offsets,
                        uint32_t n, uint64_t now_ms, emqxgm_retain_out* out);

/* ---- single-driver batcher core: publish windows over the host pipes ---------------------
 * A caller that batches topics itself (one thread adding, flushing and collecting; bench.py's
 * window sweep) packs them into a window in pinned host memory, submits a full window (or one
 * that is due) with emqxgm_match_batch_submit_filters, and on collection reads every topic's trie
 * row with its filter bytes (gathered on the device).  Up to EMQXGM_HOST_PIPES windows are in
 * flight; a window's result stays valid until that many more windows are flushed.  Collect waits
 * without the batcher's lock.  The NIF uses the concurrent entry below (emqxgm_async_*), which
 * any number of threads call one topic at a time (emqx_broker.erl:218-232,
 * emqx_trie.erl:147-169). */
typedef struct emqxgm_batcher emqxgm_batcher_t;
typedef struct emqxgm_batcher_cfg {
  uint32_t window_topics; /* topics per window (0 = 65,536; <= the engine's batch_max) */
  uint32_t window_bytes;  /* topic bytes per window (0 = 64 x window_topics) */
  uint32_t window_us;     /* a non-empty window is due this long after its first topic (0 = 50) */
  uint32_t reserved;
} emqxgm_batcher_cfg;
typedef struct emqxgm_window_out {
  uint32_t n;                 /* topics in the window, in the order they were added */
  uint32_t n_pairs;
  const uint64_t* tag;        /* [n] the caller's tag of each topic (e.g. its waiter) */
  const uint32_t* row;        /* [n+1] topic i's trie filters are pairs row[i] .. row[i+1] */
  const uint32_t* filter_id;  /* [n_pairs] */
  const uint32_t* foff;       /* [n_pairs + 1] pair j's filter bytes: fbytes[foff[j] .. foff[j+1]) */
  const uint8_t* fbytes;
  const uint32_t* exact_id;   /* [n] route key equal to the topic, or EMQXGM_NONE */
  uint64_t flush_ns, done_ns; /* CLOCK_MONOTONIC at the flush and when the result was complete */
} emqxgm_window_out;
int emqxgm_batcher_create(emqxgm_t* h, const emqxgm_batcher_cfg* cfg, emqxgm_batcher_t** out);
void emqxgm_batcher_destroy(emqxgm_batcher_t* b);
/* Appends a topic to the open window (*slot = its index there).  Returns 1 when the window is
 * now full (flush it before the next add), 0 otherwise; -E2BIG for a topic longer than a window,
 * -ENOSPC when the open window is full, -EINVAL. */
int emqxgm_batcher_add(emqxgm_batcher_t* b, const uint8_t* topic, uint32_t len, uint64_t tag,
                       uint32_t* slot);
/* Appends topics bytes[offsets[i] .. offsets[i+1]) for i in [0, n) (tag tag0 + i) until the
 * open window is full; returns how many were added (>= 0), or -EINVAL / -E2BIG as _add.  A
 * batcher process that drains several callers at once packs them with one call. */
int emqxgm_batcher_add_many(emqxgm_batcher_t* b, const uint8_t* bytes, const uint32_t* offsets,
                            uint32_t n, uint64_t tag0);
/* 1 when the open window holds topics and its first one was added window_us or more before
 * now_ns (CLOCK_MONOTONIC), else 0. */
int emqxgm_batcher_due(emqxgm_batcher_t* b, uint64_t now_ns);
/* Submits the open window and opens an empty one; *window = the window's id (0: it was empty,
 * nothing submitted).  -EBUSY when EMQXGM_HOST_PIPES windows are flushed and not collected. */
int emqxgm_batcher_flush(emqxgm_batcher_t* b, uint64_t* window);
/* Completes window `window` (flushed; the oldest first is cheapest) and returns its result,
 * read in place from the host pipe's pinned buffers: valid until EMQXGM_HOST_PIPES more windows
 * are flushed (collecting it again before that returns the same result). */
int emqxgm_batcher_collect(emqxgm_batcher_t* b, uint64_t window, emqxgm_window_out* out);

/* ---- concurrent publish entry: one topic per call from any number of threads ------------------
 * The reference matches every publish in the publisher's own process, on every scheduler at once
 * (emqx_broker:publish/1 -> emqx_router:match_routes/1 -> emqx_trie:match/1,
 * emqx_broker.erl:218-232, emqx_router.erl:141-153, read_concurrency ETS emqx_trie.erl:70-75).
 * emqxgm_async_match is what those processes call through the NIF (match_async/3): it appends the
 * topic to the open window in pinned memory and returns at once; a flusher thread submits a
 * window when it is full or window_us after its first topic, over the handles' host pipes (round
 * robin over the handles with a pipe free: one handle per GPU, each holding the whole index), and
 * one completer thread per handle waits for its windows in order and calls `cb` once per window
 * (from that thread; the windows of different handles concurrently).  The window passed to `cb`
 * is valid during the call only.  Every accepted call is reported exactly once, unless cancelled
 * first.  Errors of emqxgm_async_match: -E2BIG (longer than a window, or more than max_levels
 * levels), -EBUSY (every window full or in flight), -ESTALE (every handle's index is stale: see
 * "Health"), -EINVAL: the caller answers those itself.  Windows go to handles that are not stale;
 * a window whose handle is (or becomes) stale is reported with status -ESTALE.
 * A layer created with EMQXGM_ASYNC_PUBLISH answers each call with emqx_broker:publish/1's
 * routing instead (emqx_broker.erl:218-300: the aggre/1 entries of match_routes(Topic) and the
 * local dispatches, dispatch/2 :326-355, from the engine's fan-out tables): the completer runs
 * emqxgm_publish_batch for the window (the handle's publish results are then reused by it, so a
 * handle serves one publish layer). */
#define EMQXGM_TAG_CANCELLED 0xFFFFFFFFFFFFFFFFull /* never a caller's tag */
typedef struct emqxgm_async emqxgm_async_t;
typedef struct emqxgm_async_cfg {
  uint32_t window_topics;  /* topics per window (0 = 65,536; <= every handle's batch_max) */
  uint32_t window_bytes;   /* topic bytes per window (0 = 64 x window_topics) */
  uint32_t window_us;      /* a window is submitted at most this long after its first topic (0 = 50) */
  uint32_t max_levels;     /* calls for topics with more levels: -E2BIG (0 = no limit) */
  uint32_t queued_windows; /* full windows that may wait for a pipe (0 = 2) */
  uint32_t flags;          /* EMQXGM_ASYNC_PUBLISH: windows are answered with the publish
                              fan-out (emqxgm_publish_batch) instead of trie rows */
  uint32_t deliver_threads;/* 0 or 1: each completer calls cb once per window; k > 1: a window
                              of at least 2,048 calls is reported in up to k parts of >= 1,024
                              calls, `cb` running concurrently on the completer and k - 1 pool
                              threads (a view per part: n, tag, owner, row / exact_id /
                              route_ptr / deliver_ptr offset to the part; pair and entry indices
                              stay absolute).  For a caller whose per-call report is costly (the
                              NIF: terms + enif_send), so one thread does not bound the rate */
  uint32_t fail_threshold; /* 0: no health counting (the default); k > 0: k consecutive failures
                              -- calls cancelled while still pending (a caller that timed out) or
                              windows that failed other than -ESTALE -- mark every handle stale
                              (emqxgm_mark_stale), so a hung GPU costs the callers in flight one
                              timeout each and every later call is refused at once (-ESTALE) until
                              the index is repaired.  A window answered resets the count. */
} emqxgm_async_cfg;
#define EMQXGM_ASYNC_PUBLISH 1u
/* flags: a window is sealed and submitted as soon as a pipe is free and no sealed window waits,
 * instead of window_us after its first call.  An idle layer then answers a call in one pass; a
 * loaded one still grows its windows while every pipe is busy (the pipes' pace sets their size). */
#define EMQXGM_ASYNC_EAGER 2u
typedef struct emqxgm_async_window {
  int status;               /* 0, or the negative errno the window's pass failed with (no result) */
  uint32_t n;               /* calls in the window, in the order they were made */
  uint32_t n_pairs;
  uint32_t device_index;    /* the handle that matched it */
  const uint64_t* tag;      /* [n] each call's tag (EMQXGM_TAG_CANCELLED: cancelled, skip it) */
  const uint64_t* owner;    /* [n] each call's owner (e.g. the calling process) */
  const uint32_t* row;      /* [n+1] call i's trie filters are pairs row[i] .. row[i+1] */
  const uint32_t* filter_id;/* [n_pairs] */
  const uint32_t* foff;     /* [n_pairs + 1] pair j's filter bytes: fbytes[foff[j] .. foff[j+1]) */
  const uint8_t* fbytes;
  const uint32_t* exact_id; /* [n] route key equal to the topic, or EMQXGM_NONE */
  uint64_t first_ns, flush_ns, done_ns; /* CLOCK_MONOTONIC: first call, submit, result complete */
  /* EMQXGM_ASYNC_PUBLISH layers (row .. exact_id are then unset): the window's
   * emqxgm_publish_batch result -- call i's aggre/1 entries are [route_ptr[i], route_ptr[i+1])
   * (filter id To, dest handle), its local dispatches [deliver_ptr[i], deliver_ptr[i+1])
   * (filter id To, subscriber handle) -- and the bytes of each entry's To:
   * rfbytes[rfoff[j] .. rfoff[j+1]) (rfoff has n_routes + 1 entries) */
  uint64_t n_routes, n_deliveries;
  const uint64_t* route_ptr;
  const uint32_t* route_filter;
  const uint32_t* route_dest;
  const uint64_t* deliver_ptr;
  const uint32_t* deliver_filter;
  const uint32_t* deliver_sub;
  const uint64_t* rfoff;
  const uint8_t* rfbytes;
} emqxgm_async_window;
typedef void (*emqxgm_async_cb)(void* user, const emqxgm_async_window* w);
int emqxgm_async_create(emqxgm_t* const* hs, uint32_t n_handles, const emqxgm_async_cfg* cfg,
                        emqxgm_async_cb cb, void* user, emqxgm_async_t** out);
/* Stops taking calls, submits and reports every accepted one, then frees the layer. */
void emqxgm_async_destroy(emqxgm_async_t* a);
int emqxgm_async_match(emqxgm_async_t* a, const uint8_t* topic, uint32_t len, uint64_t tag,
                       uint64_t owner);
/* 1: the call (tag, owner) was still pending and will never be reported; 0: it was reported
 * already (when its window is being reported right now, this waits until that is done) or is
 * unknown.  A caller that timed out cancels, and on 0 finds the report delivered. */
int emqxgm_async_cancel(emqxgm_async_t* a, uint64_t tag, uint64_t owner);
/* out = {calls accepted, windows submitted, calls reported, -EBUSY refusals, cancelled, -E2BIG
 * refusals (levels), windows failed, windows outstanding} */
int emqxgm_async_stats(emqxgm_async_t* a, uint64_t out[8]);
/* out = {handles stale now, timeouts counted (pending calls cancelled), failed windows counted,
 * calls refused with -ESTALE}.  Returns out[0]. */
int emqxgm_async_health(emqxgm_async_t* a, uint64_t out[4]);

/* ---- handle registry: the 32-bit names of dest and subscriber terms, reused (r06) ----------
 * The engine's fan-out tables name nodes, shared-subscription groups and subscribers by handles
 * the caller chooses (emqxgm_route_dests_batch / _subscribers_batch); the NIF maps them back to
 * terms.  A broker whose clients reconnect sees a new subscriber pid per connection, so handles
 * must be reused or the tables grow without bound (the reference's subscriber_down/1 removes every
 * trace of a pid, emqx_broker.erl:361-380, emqx_broker_helper.erl:133-165).  A handle may be
 * reused only when no answer can still name it for its old term: the caller releases it after the
 * commit that removed it from every list (its lists were set without it and committed), and the
 * registry hands it out again only once every window the layers had submitted before the release
 * has been reported (windows submitted later read an epoch without it).  _alloc: a quiesced
 * released handle of `kind`, else the next never-used number (-E2BIG past EMQXGM_HANDLE_MAX);
 * _release: -ENOENT if not allocated; _stats: {numbers made, allocated, released and waiting for
 * their windows, free}.  Thread-safe.  A released subscriber's lists must all have been committed
 * without it; a full resync (emqxgm_route_sync_begin .. _end) clears every subscriber list it did
 * not set, so a topic whose last subscriber left cannot keep a reused number. */
#define EMQXGM_HANDLE_KINDS 3 /* 0 node, 1 group, 2 subscriber */
#define EMQXGM_HANDLE_MAX 0x7FFFFFFFu
typedef struct emqxgm_handles emqxgm_handles_t;
int emqxgm_handles_create(emqxgm_async_t* const* layers, uint32_t n_layers, emqxgm_handles_t** out);
void emqxgm_handles_destroy(emqxgm_handles_t* r);
int emqxgm_handles_alloc(emqxgm_handles_t* r, uint32_t kind, uint32_t* handle);
int emqxgm_handles_release(emqxgm_handles_t* r, uint32_t kind, uint32_t handle);
int emqxgm_handles_stats(emqxgm_handles_t* r, uint32_t kind, uint64_t out[4]);
/* every allocated handle of every kind released at once (a restarted mirror whose own table of
 * them was lost; its resync then rewrites every list) */
int emqxgm_handles_reset(emqxgm_handles_t* r);

/* ---- filter-sharded layout over several GPUs (the subscription set partitioned by
 * filter, the topic batch broadcast, the per-GPU match lists gathered to one GPU) ----
 * emqxgm_export copies a device-resident result (emqxgm_match_device / _wait) into the caller's
 * device buffers (row [n+1], fid [n_pairs], exact [n]), mapping filter and exact ids through
 * id_map (device u32 array, local id -> global id; NULL = identity; NONE stays NONE).
 * emqxgm_merge merges `parts` such results of one batch (rows/fids/exacts: host arrays of device
 * pointers) into one CSR on the handle's device: topic t's row is shard 0's row, then shard 1's,
 * ...; its exact id the one shard's that has it.  out_fid holds the sum of the parts' pairs;
 * *n_pairs = that sum.  Both calls return when the device work is complete. */
int emqxgm_export(emqxgm_t* h, const emqxgm_dev_out* r, const uint32_t* id_map, uint32_t* row,
                  uint32_t* fid, uint32_t* exact);
int emqxgm_merge(emqxgm_t* h, uint32_t parts, const uint32_t* const* rows,
                 const uint32_t* const* fids, const uint32_t* const* exacts, uint32_t n,
                 uint32_t* out_row, uint32_t* out_fid, uint32_t* out_exact, uint32_t* n_pairs);

/* The key-partitioned layout of a route-key-heavy index (cfg4: 100M exact keys, DESIGN.md 5,
 * SURVEY 8e's alternative): the plain route keys are split over `parts` engines by key hash
 * (emqxgm_key_owners: owner[i] of packed key i, a function of its bytes and the engine's
 * full_hash_bits only), each engine also holding every wildcard filter.  A batch's names are
 * probed each by its owner only: emqxgm_exact_owned_device writes to d_out (device, n u32) the
 * owned names' route-key ids and EMQXGM_NONE for the others, without a probe (the trie walk of a
 * topic and its wildcard-key probe are its topic block's, emqxgm_match_device on that block). */
int emqxgm_key_owners(emqxgm_t* h, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                      uint32_t parts, uint32_t* owner);
int emqxgm_exact_owned_device(emqxgm_t* h, const uint8_t* d_bytes, const uint32_t* d_offsets,
                              uint32_t n, uint32_t parts, uint32_t part, uint32_t* d_out);

/* The compact wire form of a shard's result for the exchange to the root:
 *   cnt  per-topic pair counts: n u8 (255 = in ovf), or with EMQXGM_WIRE_CNT2 two bit planes per
 *        64 topics (16 B per 64 topics, 2 bits a topic; 3 = in ovf) -- for sparse results;
 *   fid  the pairs' ids mapped through id_map (NULL = identity): n_pairs u32, or with
 *        EMQXGM_WIRE_ID24 (every id < 2^24) n_pairs u16 low halves then n_pairs u8 high bytes;
 *   xs   (topic, exact id) u32 pairs of the topics that equal a route key;
 *   ovf  (topic, count) u32 pairs of the counts the count width cannot hold.
 * xs and ovf are device arrays of 2 x n u32; counts[0] / counts[1] = their entries.
 * emqxgm_merge_wire merges `parts` such results (host arrays of device pointers, flags and
 * lengths) into one CSR exactly as emqxgm_merge does.  Both return when the device work is
 * complete. */
#define EMQXGM_WIRE_CNT2 1u
#define EMQXGM_WIRE_ID24 2u
int emqxgm_export_wire(emqxgm_t* h, const emqxgm_dev_out* r, const uint32_t* id_map,
                       uint32_t flags, void* cnt, void* fid, uint32_t* xs, uint32_t* ovf,
                       uint32_t counts[2]);
int emqxgm_merge_wire(emqxgm_t* h, uint32_t parts, const uint32_t* flags, const void* const* cnts,
                      const void* const* fids, const uint32_t* n_pairs_part,
                      const uint32_t* const* xss, const uint32_t* n_xs, const uint32_t* const* ovfs,
                      const uint32_t* n_ovf, uint32_t n, uint32_t* out_row, uint32_t* out_fid,
                      uint32_t* out_exact, uint32_t* n_pairs);

/* Diagnostic pass (instrumented walk kernel, not the production launch): runs the device
 * match and returns out[0] = trie states matched (SURVEY 8d S(t) summed over the batch),
 * out[1] = edge slots loaded, out[2] = pairs, out[3] = levels (words) in the batch,
 * out[4] = walk iterations summed over busy lanes, out[5] = walk iterations summed over
 * wavefronts (one memory round trip each). */
int emqxgm_walk_census(emqxgm_t* h, const uint8_t* d_bytes, const uint32_t* d_offsets,
                       uint32_t n, uint64_t bytes_len, uint64_t out[6]);
/* The last census pass's edge-bucket loads by probed level: out[d] literal probes of level d,
 * out[16 + d] '+' probes (levels >= 15 lumped into 15).  Returns the number of counters (32). */
int emqxgm_walk_census_levels(emqxgm_t* h, uint64_t* out, uint32_t n_out);

int emqxgm_set_profiling(emqxgm_t* h, int on);
/* Runtime tuning knobs: "walk_wg_per_cu" (persistent walk workgroups per CU); "leaf_prune"
 * (1 default: depth-code pruning in the walk, 0 off); "host_out" (host pipes copy results to the
 * host with hipMemcpyAsync, 0 default, or with a kernel writing host memory, 1);
 * "walk_pair" (1 default: a batch of at most half the walk grid's lanes is walked by two lanes
 * per topic; 0: one lane per topic); "exact_range_kb" (0 default: one route-key probe pass over the whole table; > 0: the probe
 * runs in passes over bucket ranges of that many KiB, so that the lines in flight share page
 * translations -- measured slower on a 100M-key table, kept as an option); "delta_commit": 0 = every commit rebuilds the index, 1 = small deltas are patched in place
 * (default), 2 = every delta that fits the tables' load bounds is patched in place; "delta_max":
 * the changes a delta commit takes in mode 1 (0 default = max(4096, (trie members + route keys)
 * / 8));
 * "fat_buckets": 1 (default) = single-literal-child nodes keep their child in their own bucket
 * line, 0 = none (A/B runs), from the next full build on (the next commit);
 * "roctx": 1 = roctx ranges around passes, waits and commits and a marker at each kernel launch
 * (rocprofv3 --marker-trace; also EMQXGM_ROCTX=1 at create), 0 (default) = none;
 * "keyed": token-keyed trie parents from the next full build: 1 (default) =
 * automatic, 0 = none, 2 = every eligible node (tests); "zc_topics": the largest pinned window
 * of _submit_filters that goes without DMA copies (65536 default, 0 = always copies); "spin_us":
 * host pipes' waits poll the pass's completion for up to this long before they block (200
 * default, 0 = block at once); "bg_build": full builds of registries of at least this many
 * filters run in a background thread while commits keep patching the current index (16384
 * default, 0 = every full build blocks the writers, as before r05); "bg_delay_ms": a background
 * build holds its install back this long (tests: a build in flight on demand); "rebuild" (1):
 * start a background full build of the registry now without waiting for it (-EBUSY: one is in
 * flight; it also compacts the tables' deleted slots); "probe_ms": a repair's bounded wait for
 * the engine's streams (2000 default).  Fault injection (tests of "Health"): "fail_commits" (n):
 * the next n commits fail before they change anything, with errno "fail_errno" (EIO default);
 * "hang_ms": every host-pipe wait and publish pass stalls this long first (0 default).
 * "stage_rank_bits": caps the rank field of the packed pair staging (tests of the wide redo a
 * topic with more pairs than the field holds takes; 0 default = as wide as fits). */
int emqxgm_tune(emqxgm_t* h, const char* key, int64_t value);
int emqxgm_get_stats(emqxgm_t* h, emqxgm_stats* st);
/* Last HIP error string seen by the handle (for diagnostics). */
const char* emqxgm_last_error(emqxgm_t* h);

#ifdef __cplusplus
}
#endif
#endif /* EMQX_GPUMATCH_H */
