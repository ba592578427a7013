/*
 * emqx_trie_gpu_nif.c -- the Erlang NIF over libemqx_gpumatch.so (include/emqx_gpumatch.h).
 *
 * Loaded by src/emqx_trie_gpu_nif.erl.  It replaces the publish-time match path of EMQX
 * 5.0.14: emqx_trie:match/1 (apps/emqx/src/emqx_trie.erl:147-169) as called by
 * emqx_router:match_routes/1 (apps/emqx/src/emqx_router.erl:141-157) from
 * emqx_broker:publish/1 (apps/emqx/src/emqx_broker.erl:218-232).  Topics of concurrent
 * publishers go through one batcher process (src/emqx_trie_gpu_batcher.erl), which calls
 * add/3 per topic, flush/1 per window and collect/2 per completed window here; the writes of
 * committed route changes (src/emqx_trie_gpu_sync.erl) call trie_insert/trie_delete/route_ref/
 * route_unref/commit.
 *
 * Compiled only where erl_nif.h exists (c_src/Makefile); this image has no Erlang runtime,
 * so the C-ABI below it is tested through ctypes (tests/test_gpu_batcher.py drives the same
 * emqxgm_batcher_* sequence this file does).
 */
#include <erl_nif.h>
#include <errno.h>
#include <string.h>
#include <time.h>

#include "emqx_gpumatch.h"

typedef struct {
  emqxgm_t* h;
  emqxgm_batcher_t* b;
} gm_res;

static ErlNifResourceType* RT;
static ERL_NIF_TERM A_OK, A_ERROR, A_FULL, A_EMPTY, A_TRUE, A_FALSE;

static void gm_res_dtor(ErlNifEnv* env, void* obj) {
  gm_res* r = (gm_res*)obj;
  (void)env;
  if (r->b) emqxgm_batcher_destroy(r->b); /* completes windows still in flight */
  if (r->h) emqxgm_destroy(r->h);
  r->b = NULL;
  r->h = NULL;
}

static ERL_NIF_TERM err_term(ErlNifEnv* env, int rc) {
  const char* a;
  switch (-rc) {
    case EINVAL: a = "einval"; break;
    case ENOMEM: a = "enomem"; break;
    case E2BIG: a = "e2big"; break;
    case ENOSPC: a = "enospc"; break;
    case EBUSY: a = "ebusy"; break;
    case ENOENT: a = "enoent"; break;
    case ENODEV: a = "enodev"; break;
    default: a = "eio"; break;
  }
  return enif_make_tuple2(env, A_ERROR, enif_make_atom(env, a));
}

static int get_res(ErlNifEnv* env, ERL_NIF_TERM t, gm_res** r) {
  return enif_get_resource(env, t, RT, (void**)r) && (*r)->h;
}

/* open(Device, WindowTopics, WindowBytes, WindowUs) -> {ok, Handle} | {error, Reason}
 * broker.perf.gpu_match.{devices, batch_max, batch_window_us} (src/emqx_trie_gpu_schema.erl) */
static ERL_NIF_TERM nif_open(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  int dev;
  unsigned wt, wb, wus;
  (void)argc;
  if (!enif_get_int(env, argv[0], &dev) || !enif_get_uint(env, argv[1], &wt) ||
      !enif_get_uint(env, argv[2], &wb) || !enif_get_uint(env, argv[3], &wus))
    return enif_make_badarg(env);
  emqxgm_cfg cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.device = dev;
  cfg.full_hash_bits = 64;
  cfg.batch_max = wt; /* one window is one engine batch */
  gm_res* r = enif_alloc_resource(RT, sizeof(gm_res));
  r->h = NULL;
  r->b = NULL;
  int rc = emqxgm_create(&cfg, &r->h);
  if (rc == 0) {
    emqxgm_batcher_cfg bc;
    memset(&bc, 0, sizeof bc);
    bc.window_topics = wt;
    bc.window_bytes = wb;
    bc.window_us = wus;
    rc = emqxgm_batcher_create(r->h, &bc, &r->b);
  }
  if (rc) {
    enif_release_resource(r); /* the destructor frees what was made */
    return err_term(env, rc);
  }
  ERL_NIF_TERM t = enif_make_resource(env, r);
  enif_release_resource(r);
  return enif_make_tuple2(env, A_OK, t);
}

typedef int (*filter_op)(emqxgm_t*, const uint8_t*, uint32_t);

static int op_insert(emqxgm_t* h, const uint8_t* p, uint32_t n) { return emqxgm_trie_insert(h, p, n, NULL); }
static int op_route_ref(emqxgm_t* h, const uint8_t* p, uint32_t n) { return emqxgm_route_ref(h, p, n, NULL); }

static ERL_NIF_TERM do_filter_op(ErlNifEnv* env, const ERL_NIF_TERM argv[], filter_op op) {
  gm_res* r;
  ErlNifBinary bin;
  if (!get_res(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &bin) || bin.size > 65535)
    return enif_make_badarg(env);
  const int rc = op(r->h, bin.data, (uint32_t)bin.size);
  return rc ? err_term(env, rc) : A_OK;
}

/* emqx_trie:insert/1 / delete/1 (emqx_trie.erl:113-144) of a committed change; route-bag key
 * refcounts (emqx_router_utils.erl:31-71).  Visible after commit/1. */
static ERL_NIF_TERM nif_trie_insert(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  return do_filter_op(env, argv, op_insert);
}
static ERL_NIF_TERM nif_trie_delete(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  return do_filter_op(env, argv, emqxgm_trie_delete);
}
static ERL_NIF_TERM nif_route_ref(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  return do_filter_op(env, argv, op_route_ref);
}
static ERL_NIF_TERM nif_route_unref(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  return do_filter_op(env, argv, emqxgm_route_unref);
}

/* commit(H) -> {ok, Epoch}: the atomic epoch swap (a delta patch or a full build; dirty CPU) */
static ERL_NIF_TERM nif_commit(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  uint64_t epoch = 0;
  (void)argc;
  if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
  const int rc = emqxgm_commit(r->h, &epoch);
  return rc ? err_term(env, rc) : enif_make_tuple2(env, A_OK, enif_make_uint64(env, epoch));
}

/* empty(H) -> boolean(): emqx_trie:empty/0 (emqx_trie.erl:172-178) of the committed index */
static ERL_NIF_TERM nif_empty(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  (void)argc;
  if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
  const int rc = emqxgm_trie_empty(r->h);
  return rc < 0 ? err_term(env, rc) : (rc ? A_TRUE : A_FALSE);
}

/* add(H, Topic, Tag) -> ok | full | {error, enospc | e2big}: the topic joins the open window;
 * full = flush it before the next add */
static ERL_NIF_TERM nif_add(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  ErlNifBinary bin;
  ErlNifUInt64 tag;
  uint32_t slot;
  (void)argc;
  if (!get_res(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &bin) ||
      !enif_get_uint64(env, argv[2], &tag) || bin.size > 65535)
    return enif_make_badarg(env);
  const int rc = emqxgm_batcher_add(r->b, bin.data, (uint32_t)bin.size, tag, &slot);
  return rc < 0 ? err_term(env, rc) : (rc ? A_FULL : A_OK);
}

/* due(H) -> boolean(): the open window's first topic is batch_window_us old */
static ERL_NIF_TERM nif_due(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  struct timespec ts;
  (void)argc;
  if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
  clock_gettime(CLOCK_MONOTONIC, &ts);
  const uint64_t now = (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
  return emqxgm_batcher_due(r->b, now) == 1 ? A_TRUE : A_FALSE;
}

/* flush(H) -> {ok, WindowId} | empty | {error, ebusy} */
static ERL_NIF_TERM nif_flush(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  uint64_t w = 0;
  (void)argc;
  if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
  const int rc = emqxgm_batcher_flush(r->b, &w);
  if (rc) return err_term(env, rc);
  return w ? enif_make_tuple2(env, A_OK, enif_make_uint64(env, w)) : A_EMPTY;
}

/* collect(H, WindowId) -> {ok, [{Tag, [Filter], ExactHit}]} in add order (dirty IO: waits for
 * the window's pass).  [Filter] is emqx_trie:match(Topic) -- a set, [] for a wildcard name;
 * ExactHit = whether the topic itself is a route key (emqx_router.erl:143-144). */
static ERL_NIF_TERM nif_collect(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  ErlNifUInt64 wid;
  emqxgm_window_out o;
  (void)argc;
  if (!get_res(env, argv[0], &r) || !enif_get_uint64(env, argv[1], &wid))
    return enif_make_badarg(env);
  const int rc = emqxgm_batcher_collect(r->b, wid, &o);
  if (rc) return err_term(env, rc);
  ERL_NIF_TERM list = enif_make_list(env, 0);
  for (uint32_t i = o.n; i-- > 0;) {
    ERL_NIF_TERM row = enif_make_list(env, 0);
    for (uint32_t j = o.row[i + 1]; j-- > o.row[i];) {
      const size_t len = (size_t)(o.foff[j + 1] - o.foff[j]);
      ERL_NIF_TERM b;
      unsigned char* p = enif_make_new_binary(env, len, &b);
      if (len) memcpy(p, o.fbytes + o.foff[j], len);
      row = enif_make_list_cell(env, b, row);
    }
    ERL_NIF_TERM ent = enif_make_tuple3(env, enif_make_uint64(env, o.tag[i]), row,
                                        o.exact_id[i] == EMQXGM_NONE ? A_FALSE : A_TRUE);
    list = enif_make_list_cell(env, ent, list);
  }
  return enif_make_tuple2(env, A_OK, list);
}

/* tune(H, Key, Value) -> ok | {error, einval}: emqxgm_tune knobs */
static ERL_NIF_TERM nif_tune(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  char key[64];
  ErlNifSInt64 v;
  (void)argc;
  if (!get_res(env, argv[0], &r) || enif_get_atom(env, argv[1], key, sizeof key, ERL_NIF_LATIN1) <= 0 ||
      !enif_get_int64(env, argv[2], &v))
    return enif_make_badarg(env);
  const int rc = emqxgm_tune(r->h, key, v);
  return rc ? err_term(env, rc) : A_OK;
}

static int load(ErlNifEnv* env, void** priv, ERL_NIF_TERM info) {
  (void)priv;
  (void)info;
  RT = enif_open_resource_type(env, NULL, "emqx_trie_gpu", gm_res_dtor, ERL_NIF_RT_CREATE, NULL);
  if (!RT || emqxgm_abi_version() != EMQXGM_ABI_VERSION) return -1;
  A_OK = enif_make_atom(env, "ok");
  A_ERROR = enif_make_atom(env, "error");
  A_FULL = enif_make_atom(env, "full");
  A_EMPTY = enif_make_atom(env, "empty");
  A_TRUE = enif_make_atom(env, "true");
  A_FALSE = enif_make_atom(env, "false");
  return 0;
}

static ErlNifFunc funcs[] = {
    {"open", 4, nif_open, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"trie_insert", 2, nif_trie_insert, 0},
    {"trie_delete", 2, nif_trie_delete, 0},
    {"route_ref", 2, nif_route_ref, 0},
    {"route_unref", 2, nif_route_unref, 0},
    {"commit", 1, nif_commit, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"empty", 1, nif_empty, 0},
    {"add", 3, nif_add, 0},
    {"due", 1, nif_due, 0},
    {"flush", 1, nif_flush, 0},
    {"collect", 2, nif_collect, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"tune", 3, nif_tune, 0},
};

ERL_NIF_INIT(emqx_trie_gpu_nif, funcs, load, NULL, NULL, NULL)
