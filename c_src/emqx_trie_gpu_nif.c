/*
 * emqx_trie_gpu_nif.c -- the Erlang NIF over libemqx_gpumatch.so (include/emqx_gpumatch.h).
 *
 * Loaded by src/emqx_trie_gpu_nif.erl.  It replaces the publish-time match path of EMQX
 * 5.0.14: emqx_trie:match/1 and match_session/1 (apps/emqx/src/emqx_trie.erl:147-169) as called
 * by emqx_router:match_routes/1 (apps/emqx/src/emqx_router.erl:141-157) and
 * emqx_session_router:match_routes/1 (emqx_session_router.erl:145-159) from
 * emqx_broker:publish/1 (apps/emqx/src/emqx_broker.erl:218-232).
 *
 * One resource = one index (the route table's trie + route keys, or the session router's) held
 * by one engine per GPU of broker.perf.gpu_match.devices (every engine the whole index: the
 * replica layout of DESIGN.md 5) plus the concurrent publish entry over them
 * (emqxgm_async_*).  Publisher processes call match_async/3 themselves, concurrently, on their
 * own schedulers; the engine's completer threads send each caller
 *     {emqx_trie_gpu, Id, [Filter]}  or  {emqx_trie_gpu, Id, {error, Reason}}
 * (src/emqx_trie_gpu.erl waits for it, and falls back to the reference's own emqx_trie:match/1
 * on an error or a timeout).  The mirror of the committed route table
 * (src/emqx_trie_gpu_sync.erl) calls route_set/3, sync_begin/1, sync_end/2 and commit/1.
 *
 * Compiled only where erl_nif.h exists (c_src/Makefile); this image has no Erlang runtime, so
 * the C-ABI below it is tested through ctypes and the C harness of tests/host_harness
 * (tests/test_gpu_async.py drives emqxgm_async_* from 16 and 64 threads as publishers do).
 */
#include <erl_nif.h>
#include <errno.h>
#include <string.h>

#include "emqx_gpumatch.h"

#define GM_MAX_DEVICES 16

typedef struct {
  unsigned nh;
  emqxgm_t* h[GM_MAX_DEVICES];
  emqxgm_async_t* a;
} gm_res;

static ErlNifResourceType* RT;
static ERL_NIF_TERM A_OK, A_ERROR, A_TRUE, A_FALSE, A_MOD;

/* An ErlNifPid is one term word: it travels through the engine as the call's owner. */
typedef char gm_pid_fits_owner[sizeof(ErlNifPid) <= sizeof(uint64_t) ? 1 : -1];

static void gm_res_dtor(ErlNifEnv* env, void* obj) {
  gm_res* r = (gm_res*)obj;
  (void)env;
  if (r->a) emqxgm_async_destroy(r->a); /* reports every accepted call first */
  for (unsigned k = 0; k < r->nh; ++k)
    if (r->h[k]) emqxgm_destroy(r->h[k]);
  r->a = NULL;
  r->nh = 0;
}

static ERL_NIF_TERM errno_atom(ErlNifEnv* env, int rc) {
  const char* a;
  switch (-rc) {
    case EINVAL: a = "einval"; break;
    case ENOMEM: a = "enomem"; break;
    case E2BIG: a = "e2big"; break;
    case ENOSPC: a = "enospc"; break;
    case EBUSY: a = "ebusy"; break;
    case ENOENT: a = "enoent"; break;
    case ESTALE: a = "estale"; break;
    case ESHUTDOWN: a = "eshutdown"; break;
    default: a = "eio"; break;
  }
  return enif_make_atom(env, a);
}

static ERL_NIF_TERM err_term(ErlNifEnv* env, int rc) {
  return enif_make_tuple2(env, A_ERROR, errno_atom(env, rc));
}

static int get_res(ErlNifEnv* env, ERL_NIF_TERM t, gm_res** r) {
  return enif_get_resource(env, t, RT, (void**)r) && (*r)->nh > 0;
}

/* The completer thread of one engine handle: every caller of a completed window gets its
 * message.  One process-independent environment per window (enif_send clears it each time). */
static void on_window(void* user, const emqxgm_async_window* w) {
  (void)user;
  ErlNifEnv* env = enif_alloc_env();
  if (!env) return;
  for (uint32_t i = 0; i < w->n; ++i) {
    if (w->tag[i] == EMQXGM_TAG_CANCELLED) continue; /* the caller timed out and cancelled */
    ErlNifPid pid;
    memcpy(&pid, &w->owner[i], sizeof pid);
    ERL_NIF_TERM res;
    if (w->status) {
      res = err_term(env, w->status);
    } else {
      res = enif_make_list(env, 0);
      for (uint32_t j = w->row[i + 1]; j-- > w->row[i];) {
        const size_t len = (size_t)(w->foff[j + 1] - w->foff[j]);
        ERL_NIF_TERM b;
        unsigned char* p = enif_make_new_binary(env, len, &b);
        if (len) memcpy(p, w->fbytes + w->foff[j], len);
        res = enif_make_list_cell(env, b, res);
      }
    }
    ERL_NIF_TERM msg = enif_make_tuple3(env, A_MOD, enif_make_uint64(env, w->tag[i]), res);
    enif_send(NULL, &pid, env, msg);
  }
  enif_free_env(env);
}

/* open(Devices, WindowTopics, WindowBytes, WindowUs, MaxLevels) -> {ok, Res} | {error, Reason}
 * broker.perf.gpu_match.{devices, batch_max, batch_window_us, max_levels}
 * (src/emqx_trie_gpu_schema.erl): one engine per device, windows of WindowTopics topics */
static ERL_NIF_TERM nif_open(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  unsigned ndev, wt, wb, wus, ml;
  ERL_NIF_TERM list = argv[0], head;
  (void)argc;
  if (!enif_get_list_length(env, list, &ndev) || ndev == 0 || ndev > GM_MAX_DEVICES ||
      !enif_get_uint(env, argv[1], &wt) || !enif_get_uint(env, argv[2], &wb) ||
      !enif_get_uint(env, argv[3], &wus) || !enif_get_uint(env, argv[4], &ml))
    return enif_make_badarg(env);
  gm_res* r = enif_alloc_resource(RT, sizeof(gm_res));
  memset(r, 0, sizeof *r);
  int rc = 0;
  for (unsigned k = 0; k < ndev && !rc; ++k) {
    int dev;
    if (!enif_get_list_cell(env, list, &head, &list) || !enif_get_int(env, head, &dev)) {
      enif_release_resource(r);
      return enif_make_badarg(env);
    }
    emqxgm_cfg cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.device = dev;
    cfg.full_hash_bits = 64;
    cfg.batch_max = wt; /* one window is one engine batch */
    rc = emqxgm_create(&cfg, &r->h[k]);
    if (!rc) r->nh = k + 1;
  }
  if (!rc) {
    emqxgm_async_cfg ac;
    memset(&ac, 0, sizeof ac);
    ac.window_topics = wt;
    ac.window_bytes = wb;
    ac.window_us = wus;
    ac.max_levels = ml;
    rc = emqxgm_async_create(r->h, r->nh, &ac, on_window, NULL, &r->a);
  }
  if (rc) {
    enif_release_resource(r); /* the destructor frees what was made */
    return err_term(env, rc);
  }
  ERL_NIF_TERM t = enif_make_resource(env, r);
  enif_release_resource(r);
  return enif_make_tuple2(env, A_OK, t);
}

/* route_set(Res, Filter, Present) -> ok | {error, Reason}: the route-key / trie membership of
 * Filter in every engine (emqxgm_route_set: a state, not a count; emqx_router_utils.erl:34-71).
 * Visible after commit/1. */
static ERL_NIF_TERM nif_route_set(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  ErlNifBinary bin;
  (void)argc;
  if (!get_res(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &bin) || bin.size > 65535 ||
      (argv[2] != A_TRUE && argv[2] != A_FALSE))
    return enif_make_badarg(env);
  for (unsigned k = 0; k < r->nh; ++k) {
    const int rc = emqxgm_route_set(r->h[k], bin.data, (uint32_t)bin.size, argv[2] == A_TRUE);
    if (rc) return err_term(env, rc);
  }
  return A_OK;
}

/* sync_begin(Res) -> {ok, Gen}: a full resync starts (emqxgm_route_sync_begin on every engine;
 * their generations advance together) */
static ERL_NIF_TERM nif_sync_begin(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  uint32_t gen = 0;
  (void)argc;
  if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
  for (unsigned k = 0; k < r->nh; ++k) {
    uint32_t g;
    const int rc = emqxgm_route_sync_begin(r->h[k], &g);
    if (rc) return err_term(env, rc);
    if (k == 0) gen = g;
    else if (g != gen) return err_term(env, -ESTALE);
  }
  return enif_make_tuple2(env, A_OK, enif_make_uint(env, gen));
}

/* sync_end(Res, Gen) -> {ok, Removed}: every route key not set present since sync_begin goes
 * (dirty CPU: one pass over the registry) */
static ERL_NIF_TERM nif_sync_end(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  unsigned gen;
  uint64_t removed = 0;
  (void)argc;
  if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &gen)) return enif_make_badarg(env);
  for (unsigned k = 0; k < r->nh; ++k) {
    uint64_t n = 0;
    const int rc = emqxgm_route_sync_end(r->h[k], gen, &n);
    if (rc) return err_term(env, rc);
    if (k == 0) removed = n;
  }
  return enif_make_tuple2(env, A_OK, enif_make_uint64(env, removed));
}

/* commit(Res) -> {ok, Epoch}: the atomic epoch swap on every engine (a delta patch or a full
 * build; dirty CPU) */
static ERL_NIF_TERM nif_commit(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  uint64_t epoch = 0;
  (void)argc;
  if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
  for (unsigned k = 0; k < r->nh; ++k) {
    uint64_t e = 0;
    const int rc = emqxgm_commit(r->h[k], &e);
    if (rc) return err_term(env, rc);
    if (k == 0) epoch = e;
  }
  return enif_make_tuple2(env, A_OK, enif_make_uint64(env, epoch));
}

/* empty(Res) -> boolean(): emqx_trie:empty/0 (emqx_trie.erl:172-178) of the committed index
 * (an atomic read: never waits for a commit) */
static ERL_NIF_TERM nif_empty(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  (void)argc;
  if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
  const int rc = emqxgm_trie_empty(r->h[0]);
  return rc < 0 ? err_term(env, rc) : (rc ? A_TRUE : A_FALSE);
}

typedef int (*member_fn)(emqxgm_t*, const uint8_t*, uint32_t);

static ERL_NIF_TERM do_member(ErlNifEnv* env, const ERL_NIF_TERM argv[], member_fn f) {
  gm_res* r;
  ErlNifBinary bin;
  if (!get_res(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &bin) || bin.size > 65535)
    return enif_make_badarg(env);
  const int rc = f(r->h[0], bin.data, (uint32_t)bin.size);
  return rc < 0 ? err_term(env, rc) : (rc ? A_TRUE : A_FALSE);
}

/* trie_member(Res, Filter) -> boolean(): emqx_trie:lookup_topic/2 (emqx_trie.erl:267-271) */
static ERL_NIF_TERM nif_trie_member(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  return do_member(env, argv, emqxgm_trie_member);
}

/* route_member(Res, Filter) -> boolean(): whether Filter is a committed route key */
static ERL_NIF_TERM nif_route_member(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  return do_member(env, argv, emqxgm_route_member);
}

/* match_async(Res, Topic, Id) -> ok | {error, e2big | ebusy | eshutdown}: Topic joins the open
 * window; the caller (self()) later receives {emqx_trie_gpu, Id, Result}.  Id: a unique
 * non-negative integer (erlang:unique_integer([positive])).  Runs on the caller's own scheduler
 * (a copy into pinned memory under a short lock). */
static ERL_NIF_TERM nif_match_async(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  ErlNifBinary bin;
  ErlNifUInt64 id;
  ErlNifPid self;
  uint64_t owner = 0;
  (void)argc;
  if (!get_res(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &bin) ||
      !enif_get_uint64(env, argv[2], &id) || id == EMQXGM_TAG_CANCELLED || bin.size > 65535 ||
      !enif_self(env, &self))
    return enif_make_badarg(env);
  memcpy(&owner, &self, sizeof self);
  const int rc = emqxgm_async_match(r->a, bin.data, (uint32_t)bin.size, id, owner);
  return rc ? err_term(env, rc) : A_OK;
}

/* cancel(Res, Id) -> true | false: true = the call will never be answered; false = its answer
 * is already in the caller's mailbox.  Dirty IO: may wait while the call's window is reported. */
static ERL_NIF_TERM nif_cancel(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  ErlNifUInt64 id;
  ErlNifPid self;
  uint64_t owner = 0;
  (void)argc;
  if (!get_res(env, argv[0], &r) || !enif_get_uint64(env, argv[1], &id) || !enif_self(env, &self))
    return enif_make_badarg(env);
  memcpy(&owner, &self, sizeof self);
  const int rc = emqxgm_async_cancel(r->a, id, owner);
  return rc < 0 ? err_term(env, rc) : (rc ? A_TRUE : A_FALSE);
}

/* tune(Res, Key, Value) -> ok | {error, einval}: emqxgm_tune knobs on every engine */
static ERL_NIF_TERM nif_tune(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  char key[64];
  ErlNifSInt64 v;
  (void)argc;
  if (!get_res(env, argv[0], &r) || enif_get_atom(env, argv[1], key, sizeof key, ERL_NIF_LATIN1) <= 0 ||
      !enif_get_int64(env, argv[2], &v))
    return enif_make_badarg(env);
  for (unsigned k = 0; k < r->nh; ++k) {
    const int rc = emqxgm_tune(r->h[k], key, v);
    if (rc) return err_term(env, rc);
  }
  return A_OK;
}

/* stats(Res) -> #{calls, windows, reported, busy, cancelled, too_deep, failed, outstanding} */
static ERL_NIF_TERM nif_stats(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  static const char* keys[8] = {"calls", "windows", "reported", "busy",
                                "cancelled", "too_deep", "failed", "outstanding"};
  gm_res* r;
  uint64_t v[8];
  (void)argc;
  if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
  const int rc = emqxgm_async_stats(r->a, v);
  if (rc) return err_term(env, rc);
  ERL_NIF_TERM m = enif_make_new_map(env);
  for (int i = 0; i < 8; ++i)
    enif_make_map_put(env, m, enif_make_atom(env, keys[i]), enif_make_uint64(env, v[i]), &m);
  return m;
}

static int load(ErlNifEnv* env, void** priv, ERL_NIF_TERM info) {
  (void)priv;
  (void)info;
  RT = enif_open_resource_type(env, NULL, "emqx_trie_gpu", gm_res_dtor, ERL_NIF_RT_CREATE, NULL);
  if (!RT || emqxgm_abi_version() != EMQXGM_ABI_VERSION) return -1;
  A_OK = enif_make_atom(env, "ok");
  A_ERROR = enif_make_atom(env, "error");
  A_TRUE = enif_make_atom(env, "true");
  A_FALSE = enif_make_atom(env, "false");
  A_MOD = enif_make_atom(env, "emqx_trie_gpu");
  return 0;
}

static ErlNifFunc funcs[] = {
    {"open", 5, nif_open, ERL_NIF_DIRTY_JOB_IO_BOUND},
    /* the writer lock: held through a commit's full build (seconds at 10M filters) */
    {"route_set", 3, nif_route_set, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"sync_begin", 1, nif_sync_begin, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"sync_end", 2, nif_sync_end, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"commit", 1, nif_commit, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"empty", 1, nif_empty, 0},
    {"trie_member", 2, nif_trie_member, 0},
    {"route_member", 2, nif_route_member, 0},
    {"match_async", 3, nif_match_async, 0},
    {"cancel", 2, nif_cancel, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"tune", 3, nif_tune, ERL_NIF_DIRTY_JOB_IO_BOUND},  /* some keys drain the passes in flight */
    {"stats", 1, nif_stats, 0},
};

ERL_NIF_INIT(emqx_trie_gpu_nif, funcs, load, NULL, NULL, NULL)
