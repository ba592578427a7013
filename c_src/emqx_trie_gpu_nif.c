/*
 * emqx_trie_gpu_nif.c -- the Erlang NIF over libemqx_gpumatch.so (include/emqx_gpumatch.h).
 *
 * Loaded by src/emqx_trie_gpu_nif.erl.  It replaces the publish-time routing path of EMQX
 * 5.0.14: emqx_trie:match/1 and match_session/1 (apps/emqx/src/emqx_trie.erl:147-169), the route
 * lookups of emqx_router:match_routes/1 (apps/emqx/src/emqx_router.erl:141-157) and the aggre /
 * local dispatch of emqx_broker:publish/1 (apps/emqx/src/emqx_broker.erl:218-300, 546-579).
 *
 * One resource = one index (the route table's trie, route keys, dests and local subscribers, or
 * the session router's) held by one engine per GPU of broker.perf.gpu_match.devices (every engine
 * the whole index: the replica layout of DESIGN.md 5) plus the concurrent entries over them
 * (emqxgm_async_*).  Publisher processes call match_async/3 or publish_async/3 themselves,
 * concurrently, on their own schedulers, with a fresh reference (make_ref/0, so the receive
 * skips the mailbox), and get back {ok, Call}; an engine completer thread sends each caller
 *     {emqx_trie_gpu, Ref, Filters, ExactHit}                  (match_async)
 *     {emqx_trie_gpu, Ref, {routes, Entries, Deliveries}}      (publish_async)
 *     {emqx_trie_gpu, Ref, {error, Reason}}
 * (src/emqx_trie_gpu.erl waits for it and takes the reference's own path on an error or a
 * timeout, after cancel/2).  Each accepted call is a small resource holding its own environment
 * with the caller's reference: it lives until the call is answered or cancelled.
 *
 * The mirror of the committed tables (src/emqx_trie_gpu_sync.erl and the writing node's hook in
 * emqx_trie_gpu) calls route_sync/2 (membership, committed before it returns), route_dests/3,
 * subscribers/3, register/3 and set_local_node/2 (the fan-out tables, the terms behind their
 * handles), and route_set_many/3 + sync_begin/1 + sync_end/2 + commit/1 for a resync.
 *
 * Compiled only where erl_nif.h exists (c_src/Makefile); this image has no Erlang runtime, so
 * the C-ABI below it is tested through ctypes and the C harness of tests/host_harness
 * (tests/test_gpu_async.py drives emqxgm_async_* from 16 and 64 threads as publishers do).
 */
#include <erl_nif.h>
#include <errno.h>
#include <stdint.h>
#include <string.h>

#include "emqx_gpumatch.h"

#define GM_MAX_DEVICES 16
#define GM_MAX_TOPIC 65535 /* emqx_topic.erl:47 ?MAX_TOPIC_LEN */

/* The terms the engine's 32-bit handles stand for (node atoms, shared-subscription groups,
 * subscriber pids), registered by the mirror: the engine's fan-out answers in handles, a
 * publisher gets the terms.  Each slot holds its copy in an environment of its own, freed when
 * the handle is released (r06: handles are reused, emqxgm_handles_*, so the table stays as large
 * as the live subscribers, not as every pid ever seen). */
typedef struct {
  ErlNifEnv* env; /* NULL: no term */
  ERL_NIF_TERM t;
} term_slot;
typedef struct {
  ErlNifRWLock* lk;
  term_slot* v;
  unsigned n;     /* handles [0, n) have a slot */
} term_tab;

typedef struct {
  unsigned nh;
  emqxgm_t* h[GM_MAX_DEVICES];
  emqxgm_async_t* a;  /* match_async */
  emqxgm_async_t* ap; /* publish_async (open option publish) */
  emqxgm_handles_t* hr; /* the handle numbers (node 0, group 1, sub 2), reused after quiescence */
  uint64_t next_tag;  /* call tags: unique per resource, so a stale one never matches a cancel */
  term_tab nodes, groups, subs;
} gm_res;

/* One accepted call until its answer is sent or it is cancelled. */
typedef struct {
  ErlNifEnv* env; /* the message is built here and sent from the completer thread */
  ERL_NIF_TERM ref;
  ErlNifPid pid;
  uint64_t tag;
  int publish;
} gm_call;

static ErlNifResourceType *RT, *CALL_RT, *RETAIN_RT;
static ERL_NIF_TERM A_OK, A_ERROR, A_TRUE, A_FALSE, A_MOD, A_ROUTES, A_NONE, A_NODE, A_GROUP, A_SUB,
    A_SPIN_US, A_BG_BUILD, A_PUBLISH, A_UNDEFINED, A_REPORT_THREADS, A_EQ, A_WORDS, A_BINARY,
    A_FAIL_THRESHOLD, A_EAGER;

static int tab_init(term_tab* t, char* name) {
  t->lk = enif_rwlock_create(name);
  t->v = NULL;
  t->n = 0;
  return t->lk != NULL;
}

static void tab_free(term_tab* t) {
  if (t->lk) enif_rwlock_destroy(t->lk);
  for (unsigned i = 0; i < t->n; ++i)
    if (t->v[i].env) enif_free_env(t->v[i].env);
  enif_free(t->v);
  memset(t, 0, sizeof *t);
}

/* the term behind handle h copied into env, or `undefined` (caller holds the read lock) */
static ERL_NIF_TERM tab_get(ErlNifEnv* env, const term_tab* t, uint32_t h) {
  return (h < t->n && t->v[h].env) ? enif_make_copy(env, t->v[h].t) : A_UNDEFINED;
}

static void gm_res_dtor(ErlNifEnv* env, void* obj) {
  gm_res* r = (gm_res*)obj;
  (void)env;
  if (r->hr) emqxgm_handles_destroy(r->hr);
  r->hr = NULL;
  if (r->a) emqxgm_async_destroy(r->a); /* reports every accepted call first */
  if (r->ap) emqxgm_async_destroy(r->ap);
  for (unsigned k = 0; k < r->nh; ++k)
    if (r->h[k]) emqxgm_destroy(r->h[k]);
  tab_free(&r->nodes);
  tab_free(&r->groups);
  tab_free(&r->subs);
  r->a = r->ap = NULL;
  r->nh = 0;
}

static void gm_call_dtor(ErlNifEnv* env, void* obj) {
  gm_call* c = (gm_call*)obj;
  (void)env;
  if (c->env) enif_free_env(c->env);
  c->env = NULL;
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
    case ETIMEDOUT: a = "etimedout"; break;
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

/* Sends call c its message (built in its own environment) and lets the call go. */
static void answer(gm_call* c, ERL_NIF_TERM result) {
  ERL_NIF_TERM msg = enif_make_tuple3(c->env, A_MOD, c->ref, result);
  enif_send(NULL, &c->pid, c->env, msg);
  enif_free_env(c->env);
  c->env = NULL;
  enif_release_resource(c); /* the in-flight reference */
}

static ERL_NIF_TERM bytes_term(ErlNifEnv* env, const uint8_t* p, size_t len) {
  ERL_NIF_TERM b;
  unsigned char* d = enif_make_new_binary(env, len, &b);
  if (len) memcpy(d, p, len);
  return b;
}

/* The completer thread of one engine handle: every caller of a completed window gets its
 * message (cancelled calls were released by their cancel). */
static void on_window(void* user, const emqxgm_async_window* w) {
  gm_res* r = (gm_res*)user;
  for (uint32_t i = 0; i < w->n; ++i) {
    if (w->tag[i] == EMQXGM_TAG_CANCELLED) continue;
    gm_call* c = (gm_call*)(uintptr_t)w->owner[i];
    ErlNifEnv* env = c->env;
    ERL_NIF_TERM res;
    if (w->status) {
      res = err_term(env, w->status);
    } else if (!c->publish) {
      ERL_NIF_TERM fl = enif_make_list(env, 0);
      for (uint32_t j = w->row[i + 1]; j-- > w->row[i];)
        fl = enif_make_list_cell(env, bytes_term(env, w->fbytes + w->foff[j], w->foff[j + 1] - w->foff[j]), fl);
      /* the topic itself is a route key: match_routes/1 looks it up (emqx_router.erl:143-144) */
      const ERL_NIF_TERM hit = w->exact_id[i] != EMQXGM_NONE ? A_TRUE : A_FALSE;
      ERL_NIF_TERM msg = enif_make_tuple4(env, A_MOD, c->ref, fl, hit);
      enif_send(NULL, &c->pid, env, msg);
      enif_free_env(env);
      c->env = NULL;
      enif_release_resource(c);
      continue;
    } else {
      /* aggre/1 entries {To, Node} | {To, Group} (emqx_broker.erl:284-300) and the local
       * dispatches {To, SubPid} of the {To, node()} entries (dispatch/2, :326-355) */
      const uint64_t a = w->route_ptr[i], b = w->route_ptr[i + 1];
      ERL_NIF_TERM ents = enif_make_list(env, 0), dels = enif_make_list(env, 0);
      ERL_NIF_TERM to_small[16];
      ERL_NIF_TERM* to = b - a <= 16 ? to_small : enif_alloc(sizeof(ERL_NIF_TERM) * (size_t)(b - a));
      if (!to) {
        answer(c, err_term(env, -ENOMEM));
        continue;
      }
      enif_rwlock_rlock(r->nodes.lk);
      enif_rwlock_rlock(r->groups.lk);
      for (uint64_t j = a; j < b; ++j) {
        to[j - a] = bytes_term(env, w->rfbytes + w->rfoff[j], (size_t)(w->rfoff[j + 1] - w->rfoff[j]));
        const uint32_t d = w->route_dest[j];
        const ERL_NIF_TERM dt = (d & EMQXGM_DEST_GROUP) ? tab_get(env, &r->groups, d & ~EMQXGM_DEST_GROUP)
                                                        : tab_get(env, &r->nodes, d);
        ents = enif_make_list_cell(env, enif_make_tuple2(env, to[j - a], dt), ents);
      }
      enif_rwlock_runlock(r->groups.lk);
      enif_rwlock_runlock(r->nodes.lk);
      enif_rwlock_rlock(r->subs.lk);
      for (uint64_t j = w->deliver_ptr[i]; j < w->deliver_ptr[i + 1]; ++j) {
        ERL_NIF_TERM t = A_UNDEFINED;
        for (uint64_t q = a; q < b; ++q)
          if (w->route_filter[q] == w->deliver_filter[j]) {
            t = to[q - a];
            break;
          }
        dels = enif_make_list_cell(env, enif_make_tuple2(env, t, tab_get(env, &r->subs, w->deliver_sub[j])), dels);
      }
      enif_rwlock_runlock(r->subs.lk);
      if (to != to_small) enif_free(to);
      res = enif_make_tuple3(env, A_ROUTES, ents, dels);
    }
    answer(c, res);
  }
}

static int opt_uint(ErlNifEnv* env, ERL_NIF_TERM map, ERL_NIF_TERM key, ErlNifSInt64 dflt, ErlNifSInt64* v) {
  ERL_NIF_TERM t;
  *v = dflt;
  return !enif_get_map_value(env, map, key, &t) || enif_get_int64(env, t, v);
}

/* open(Devices, WindowTopics, WindowBytes, WindowUs, MaxLevels, Opts) -> {ok, Res} | {error, R}
 * broker.perf.gpu_match.{devices, batch_max, batch_window_us, max_levels} (src/
 * emqx_trie_gpu_schema.erl): one engine per device, windows of WindowTopics topics.  Opts:
 * #{spin_us => N (0: a completer blocks at once instead of polling; the default),
 *   bg_build => N (emqxgm_tune "bg_build"), publish => boolean() (a publish_async layer too),
 *   report_threads => N (emqxgm_async_cfg.deliver_threads, default 8: a window's calls are
 *   answered -- terms built, enif_send -- by up to N threads, not by the completer alone),
 *   fail_threshold => N (emqxgm_async_cfg.fail_threshold, default 3: that many timed-out calls or
 *   failed windows in a row mark the engines stale, and every later call is refused with
 *   {error, estale} -- the caller's reference path -- until the mirror's repair),
 *   eager => boolean() (EMQXGM_ASYNC_EAGER: a window goes to the device as soon as a pipe is
 *   free, not WindowUs after its first call: an idle broker answers in one pass)} */
static ERL_NIF_TERM nif_open(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  unsigned ndev, wt, wb, wus, ml;
  ERL_NIF_TERM list = argv[0], head, pub, eag;
  ErlNifSInt64 spin, bg, rth, fth;
  (void)argc;
  if (!enif_get_list_length(env, list, &ndev) || ndev == 0 || ndev > GM_MAX_DEVICES ||
      !enif_get_uint(env, argv[1], &wt) || !enif_get_uint(env, argv[2], &wb) ||
      !enif_get_uint(env, argv[3], &wus) || !enif_get_uint(env, argv[4], &ml) ||
      !opt_uint(env, argv[5], A_SPIN_US, 0, &spin) || !opt_uint(env, argv[5], A_BG_BUILD, 16384, &bg) ||
      !opt_uint(env, argv[5], A_REPORT_THREADS, 8, &rth) || rth < 0 || rth > 64 ||
      !opt_uint(env, argv[5], A_FAIL_THRESHOLD, 3, &fth) || fth < 0 || fth > 1000000)
    return enif_make_badarg(env);
  const int publish = enif_get_map_value(env, argv[5], A_PUBLISH, &pub) && pub == A_TRUE;
  const uint32_t eager = enif_get_map_value(env, argv[5], A_EAGER, &eag) && eag == A_TRUE ? EMQXGM_ASYNC_EAGER : 0u;
  gm_res* r = enif_alloc_resource(RT, sizeof(gm_res));
  memset(r, 0, sizeof *r);
  if (!tab_init(&r->nodes, "emqx_trie_gpu.nodes") || !tab_init(&r->groups, "emqx_trie_gpu.groups") ||
      !tab_init(&r->subs, "emqx_trie_gpu.subs")) {
    enif_release_resource(r);
    return err_term(env, -ENOMEM);
  }
  r->next_tag = 1;
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
    if (!rc) {
      r->nh = k + 1;
      rc = emqxgm_tune(r->h[k], "spin_us", spin);
      if (!rc) rc = emqxgm_tune(r->h[k], "bg_build", bg);
    }
  }
  emqxgm_async_cfg ac;
  memset(&ac, 0, sizeof ac);
  ac.window_topics = wt;
  ac.window_bytes = wb;
  ac.window_us = wus;
  ac.max_levels = ml;
  ac.deliver_threads = (uint32_t)rth;
  ac.fail_threshold = (uint32_t)fth;
  ac.flags = eager;
  if (!rc) rc = emqxgm_async_create(r->h, r->nh, &ac, on_window, r, &r->a);
  if (!rc && publish) {
    ac.flags = EMQXGM_ASYNC_PUBLISH | eager;
    rc = emqxgm_async_create(r->h, r->nh, &ac, on_window, r, &r->ap);
  }
  if (!rc) {
    emqxgm_async_t* layers[2] = {r->a, r->ap};
    rc = emqxgm_handles_create(layers, r->ap ? 2 : 1, &r->hr);
  }
  if (rc) {
    enif_release_resource(r); /* the destructor frees what was made */
    return err_term(env, rc);
  }
  ERL_NIF_TERM t = enif_make_resource(env, r);
  enif_release_resource(r);
  return enif_make_tuple2(env, A_OK, t);
}

/* Packs a list of binaries (or of tuples whose first element is one) for a batch call:
 * bytes / offsets allocated with enif_alloc.  Filters longer than a topic can be
 * (emqx_topic.erl:47) are never routes: 0, or -E2BIG. */
typedef struct {
  unsigned n;
  uint8_t* bytes;
  uint64_t* off;
} packed;

static void packed_free(packed* p) {
  enif_free(p->bytes);
  enif_free(p->off);
  memset(p, 0, sizeof *p);
}

/* elem: the binary of each list item (item itself, or element 1 of a tuple when tuples) */
static int pack_list(ErlNifEnv* env, ERL_NIF_TERM list, int tuples, packed* p) {
  ERL_NIF_TERM head, l = list;
  size_t total = 0;
  memset(p, 0, sizeof *p);
  if (!enif_get_list_length(env, list, &p->n)) return -EINVAL;
  p->off = enif_alloc(sizeof(uint64_t) * ((size_t)p->n + 1));
  if (!p->off) return -ENOMEM;
  p->off[0] = 0;
  for (unsigned i = 0; i < p->n; ++i) { /* first pass: sizes */
    ErlNifBinary b;
    int ar;
    const ERL_NIF_TERM* el;
    if (!enif_get_list_cell(env, l, &head, &l)) return -EINVAL;
    if (tuples) {
      if (!enif_get_tuple(env, head, &ar, &el) || ar < 2) return -EINVAL;
      head = el[0];
    }
    if (!enif_inspect_binary(env, head, &b)) return -EINVAL;
    if (b.size > GM_MAX_TOPIC) return -E2BIG;
    total += b.size;
    p->off[i + 1] = total;
  }
  p->bytes = enif_alloc(total ? total : 1);
  if (!p->bytes) return -ENOMEM;
  l = list;
  for (unsigned i = 0; i < p->n; ++i) {
    ErlNifBinary b;
    int ar;
    const ERL_NIF_TERM* el;
    enif_get_list_cell(env, l, &head, &l);
    if (tuples) {
      enif_get_tuple(env, head, &ar, &el);
      head = el[0];
    }
    enif_inspect_binary(env, head, &b);
    if (b.size) memcpy(p->bytes + p->off[i], b.data, b.size);
  }
  return 0;
}

/* One call on every engine of the resource.  A bulk call (a resync chunk) on several engines runs
 * one thread per engine: each engine holds its own registry and model, so the call costs one
 * engine's time instead of nh of them (8 GPUs: 11 s -> ~1.4 s per 10M-route resync). */
#define GM_PAR_MIN 1024
typedef struct {
  emqxgm_t* h;
  int (*fn)(void* a, emqxgm_t* h, uint64_t* epoch);
  void* a;
  int rc;
  uint64_t epoch;
} eng_job;

static void* eng_job_run(void* p) {
  eng_job* j = p;
  j->rc = j->fn(j->a, j->h, &j->epoch);
  return NULL;
}

static int on_engines(gm_res* r, size_t n, int (*fn)(void*, emqxgm_t*, uint64_t*), void* a,
                      uint64_t* epoch) {
  eng_job job[GM_MAX_DEVICES];
  ErlNifTid tid[GM_MAX_DEVICES];
  int started[GM_MAX_DEVICES] = {0};
  const int par = r->nh > 1 && n >= GM_PAR_MIN;
  int rc = 0;
  for (unsigned k = 0; k < r->nh; ++k) {
    job[k].h = r->h[k];
    job[k].fn = fn;
    job[k].a = a;
    job[k].rc = 0;
    job[k].epoch = 0;
    if (par && k > 0 && enif_thread_create("emqx_trie_gpu_set", &tid[k], eng_job_run, &job[k], NULL) == 0)
      started[k] = 1;
  }
  /* engine 0 on this (dirty) scheduler thread; the others in theirs, or here when a thread could
   * not start.  Every engine runs the call even after one refused it: the refusing engine marked
   * itself stale (it answers no match until a repair), the others must not miss the change. */
  for (unsigned k = 0; k < r->nh; ++k) {
    if (started[k]) continue;
    eng_job_run(&job[k]);
    if (!rc) rc = job[k].rc;
  }
  for (unsigned k = 0; k < r->nh; ++k) {
    if (!started[k]) continue;
    enif_thread_join(tid[k], NULL);
    if (!rc) rc = job[k].rc;
  }
  if (epoch) *epoch = job[0].epoch;
  return rc;
}

typedef struct {
  const packed* p;
  const uint8_t* present;
  const uint32_t *ptr, *v0, *v1;
  uint32_t flags;
  int pr;
} set_args;

static int fn_route_set_batch(void* a, emqxgm_t* h, uint64_t* epoch) {
  const set_args* s = a;
  return emqxgm_route_set_batch(h, s->p->bytes, s->p->off, s->present, s->p->n, s->flags, epoch);
}
static int fn_route_set_many(void* a, emqxgm_t* h, uint64_t* epoch) {
  const set_args* s = a;
  (void)epoch;
  return emqxgm_route_set_many(h, s->p->bytes, s->p->off, s->p->n, s->pr);
}
static int fn_route_dests(void* a, emqxgm_t* h, uint64_t* epoch) {
  const set_args* s = a;
  return emqxgm_route_dests_batch(h, s->p->bytes, s->p->off, s->p->n, s->ptr, s->v0, s->v1, s->flags, epoch);
}
static int fn_subscribers(void* a, emqxgm_t* h, uint64_t* epoch) {
  const set_args* s = a;
  return emqxgm_subscribers_batch(h, s->p->bytes, s->p->off, s->p->n, s->ptr, s->v0, s->flags, epoch);
}

/* route_sync(Res, [{Filter, Present :: boolean()}]) -> {ok, Epoch} | {error, R}: the writing node's
 * hook after emqx_router:do_add_route/2, do_delete_route/2 (emqx_router.erl:124-138, 171-179) and
 * the mirror's batched table events: membership set AND committed before the return
 * (emqxgm_route_set_batch with EMQXGM_SET_COMMIT).  It waits for a background full build only
 * when the call's delta does not fit the current tables while that build runs: the dirty CPU
 * scheduler is then held until the build's install (stats/1 bg_waits counts these). */
static ERL_NIF_TERM nif_route_sync(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  packed p;
  (void)argc;
  if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
  int rc = pack_list(env, argv[1], 1, &p);
  uint8_t* pr = rc ? NULL : enif_alloc(p.n ? p.n : 1);
  if (!rc && !pr) rc = -ENOMEM;
  if (!rc) {
    ERL_NIF_TERM head, l = argv[1];
    for (unsigned i = 0; i < p.n && !rc; ++i) {
      int ar;
      const ERL_NIF_TERM* el;
      enif_get_list_cell(env, l, &head, &l);
      enif_get_tuple(env, head, &ar, &el);
      if (el[1] != A_TRUE && el[1] != A_FALSE) rc = -EINVAL;
      pr[i] = el[1] == A_TRUE;
    }
  }
  uint64_t epoch = 0;
  if (!rc) {
    set_args sa = {&p, pr, NULL, NULL, NULL, EMQXGM_SET_COMMIT, 0};
    rc = on_engines(r, p.n, fn_route_set_batch, &sa, &epoch);
  }
  enif_free(pr);
  packed_free(&p);
  if (rc == -EINVAL) return enif_make_badarg(env);
  return rc ? err_term(env, rc) : enif_make_tuple2(env, A_OK, enif_make_uint64(env, epoch));
}

/* route_set_many(Res, [Filter], Present) -> ok | {error, R}: a resync chunk (emqxgm_route_set_many
 * on every engine; committed by commit/1 after sync_end/2). */
static ERL_NIF_TERM nif_route_set_many(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  packed p;
  (void)argc;
  if (!get_res(env, argv[0], &r) || (argv[2] != A_TRUE && argv[2] != A_FALSE)) return enif_make_badarg(env);
  int rc = pack_list(env, argv[1], 0, &p);
  if (!rc) {
    set_args sa = {&p, NULL, NULL, NULL, NULL, 0, argv[2] == A_TRUE};
    rc = on_engines(r, p.n, fn_route_set_many, &sa, NULL);
  }
  packed_free(&p);
  if (rc == -EINVAL) return enif_make_badarg(env);
  return rc ? err_term(env, rc) : A_OK;
}

static int get_commit(ERL_NIF_TERM t, uint32_t* flags) {
  if (t != A_TRUE && t != A_FALSE) return 0;
  *flags = t == A_TRUE ? EMQXGM_SET_COMMIT : 0;
  return 1;
}

/* route_dests(Res, [{Filter, [{NodeH, GroupH | none}]}], Commit) -> {ok, Epoch} | {error, R}: each
 * filter's rows of the emqx_route bag (emqx_router.erl:72-92) as dest handles (register/3 maps
 * them to the dest terms): emqxgm_route_dests_batch. */
static ERL_NIF_TERM nif_route_dests(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  packed p;
  uint32_t flags;
  (void)argc;
  if (!get_res(env, argv[0], &r) || !get_commit(argv[2], &flags)) return enif_make_badarg(env);
  int rc = pack_list(env, argv[1], 1, &p);
  uint32_t *dptr = NULL, *node = NULL, *group = NULL;
  unsigned nd = 0;
  if (!rc) {
    ERL_NIF_TERM head, l = argv[1];
    dptr = enif_alloc(sizeof(uint32_t) * ((size_t)p.n + 1));
    if (!dptr) rc = -ENOMEM;
    for (unsigned i = 0; i < p.n && !rc; ++i) { /* count */
      int ar;
      const ERL_NIF_TERM* el;
      unsigned k;
      enif_get_list_cell(env, l, &head, &l);
      enif_get_tuple(env, head, &ar, &el);
      if (!enif_get_list_length(env, el[1], &k)) rc = -EINVAL;
      nd += k;
    }
    if (!rc) {
      node = enif_alloc(sizeof(uint32_t) * (nd ? nd : 1));
      group = enif_alloc(sizeof(uint32_t) * (nd ? nd : 1));
      if (!node || !group) rc = -ENOMEM;
    }
    l = argv[1];
    unsigned j = 0;
    for (unsigned i = 0; i < p.n && !rc; ++i) {
      int ar, dar;
      const ERL_NIF_TERM *el, *de;
      ERL_NIF_TERM dh, dl;
      enif_get_list_cell(env, l, &head, &l);
      enif_get_tuple(env, head, &ar, &el);
      dptr[i] = j;
      for (dl = el[1]; !rc && enif_get_list_cell(env, dl, &dh, &dl); ++j) {
        unsigned nv = 0, gv = EMQXGM_NONE;
        if (!enif_get_tuple(env, dh, &dar, &de) || dar != 2 || !enif_get_uint(env, de[0], &nv) ||
            (de[1] != A_NONE && !enif_get_uint(env, de[1], &gv)))
          rc = -EINVAL;
        node[j] = nv;
        group[j] = gv;
      }
    }
    if (!rc) dptr[p.n] = j;
  }
  uint64_t epoch = 0;
  if (!rc) {
    set_args sa = {&p, NULL, dptr, node, group, flags, 0};
    rc = on_engines(r, p.n, fn_route_dests, &sa, &epoch);
  }
  enif_free(dptr);
  enif_free(node);
  enif_free(group);
  packed_free(&p);
  if (rc == -EINVAL) return enif_make_badarg(env);
  return rc ? err_term(env, rc) : enif_make_tuple2(env, A_OK, enif_make_uint64(env, epoch));
}

/* subscribers(Res, [{Filter, [SubH]}], Commit) -> {ok, Epoch} | {error, R}: each filter's local
 * subscribers (the emqx_subscriber bag, emqx_broker.erl:546-552; shard rows flattened) as
 * handles: emqxgm_subscribers_batch. */
static ERL_NIF_TERM nif_subscribers(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  packed p;
  uint32_t flags;
  (void)argc;
  if (!get_res(env, argv[0], &r) || !get_commit(argv[2], &flags)) return enif_make_badarg(env);
  int rc = pack_list(env, argv[1], 1, &p);
  uint32_t *sptr = NULL, *subs = NULL;
  unsigned ns = 0;
  if (!rc) {
    ERL_NIF_TERM head, l = argv[1];
    sptr = enif_alloc(sizeof(uint32_t) * ((size_t)p.n + 1));
    if (!sptr) rc = -ENOMEM;
    for (unsigned i = 0; i < p.n && !rc; ++i) {
      int ar;
      const ERL_NIF_TERM* el;
      unsigned k;
      enif_get_list_cell(env, l, &head, &l);
      enif_get_tuple(env, head, &ar, &el);
      if (!enif_get_list_length(env, el[1], &k)) rc = -EINVAL;
      ns += k;
    }
    if (!rc && !(subs = enif_alloc(sizeof(uint32_t) * (ns ? ns : 1)))) rc = -ENOMEM;
    l = argv[1];
    unsigned j = 0;
    for (unsigned i = 0; i < p.n && !rc; ++i) {
      int ar;
      const ERL_NIF_TERM* el;
      ERL_NIF_TERM sh, sl;
      enif_get_list_cell(env, l, &head, &l);
      enif_get_tuple(env, head, &ar, &el);
      sptr[i] = j;
      for (sl = el[1]; !rc && enif_get_list_cell(env, sl, &sh, &sl); ++j) {
        unsigned v;
        if (!enif_get_uint(env, sh, &v)) rc = -EINVAL;
        subs[j] = v;
      }
    }
    if (!rc) sptr[p.n] = j;
  }
  uint64_t epoch = 0;
  if (!rc) {
    set_args sa = {&p, NULL, sptr, subs, NULL, flags, 0};
    rc = on_engines(r, p.n, fn_subscribers, &sa, &epoch);
  }
  enif_free(sptr);
  enif_free(subs);
  packed_free(&p);
  if (rc == -EINVAL) return enif_make_badarg(env);
  return rc ? err_term(env, rc) : enif_make_tuple2(env, A_OK, enif_make_uint64(env, epoch));
}

/* register(Res, node | group | sub, [{Handle, Term}]) -> ok: the terms publish_async answers with */
static ERL_NIF_TERM nif_register(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  ERL_NIF_TERM head, l = argv[2];
  (void)argc;
  if (!get_res(env, argv[0], &r) || !enif_is_list(env, argv[2])) return enif_make_badarg(env);
  term_tab* t = argv[1] == A_NODE ? &r->nodes : argv[1] == A_GROUP ? &r->groups : argv[1] == A_SUB ? &r->subs : NULL;
  if (!t) return enif_make_badarg(env);
  int bad = 0;
  enif_rwlock_rwlock(t->lk);
  while (!bad && enif_get_list_cell(env, l, &head, &l)) {
    int ar;
    const ERL_NIF_TERM* el;
    unsigned hv;
    if (!enif_get_tuple(env, head, &ar, &el) || ar != 2 || !enif_get_uint(env, el[0], &hv) ||
        hv >= 0x7FFFFFFFu) {
      bad = 1;
      break;
    }
    if (hv >= t->n) {
      unsigned n2 = t->n ? t->n : 64;
      while (n2 <= hv) n2 *= 2;
      term_slot* v = enif_realloc(t->v, sizeof(term_slot) * n2);
      if (!v) {
        bad = 2;
        break;
      }
      memset(v + t->n, 0, sizeof(term_slot) * (n2 - t->n));
      t->v = v;
      t->n = n2;
    }
    term_slot* sl = &t->v[hv];
    if (sl->env) {
      enif_clear_env(sl->env);
    } else if (!(sl->env = enif_alloc_env())) {
      bad = 2;
      break;
    }
    sl->t = enif_make_copy(sl->env, el[1]);
  }
  enif_rwlock_rwunlock(t->lk);
  if (bad == 1) return enif_make_badarg(env);
  return bad ? err_term(env, -ENOMEM) : A_OK;
}

static term_tab* kind_tab(gm_res* r, ERL_NIF_TERM k, uint32_t* kind) {
  if (k == A_NODE) return *kind = 0, &r->nodes;
  if (k == A_GROUP) return *kind = 1, &r->groups;
  if (k == A_SUB) return *kind = 2, &r->subs;
  return NULL;
}

/* alloc_handle(Res, node | group | sub) -> {ok, N} | {error, e2big}: a handle number for a new
 * term (emqxgm_handles_alloc: a released one once every window submitted before its release was
 * answered, else a never-used one); register/3 then gives it its term */
static ERL_NIF_TERM nif_alloc_handle(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  uint32_t kind, h;
  (void)argc;
  if (!get_res(env, argv[0], &r) || !r->hr || !kind_tab(r, argv[1], &kind)) return enif_make_badarg(env);
  const int rc = emqxgm_handles_alloc(r->hr, kind, &h);
  return rc ? err_term(env, rc) : enif_make_tuple2(env, A_OK, enif_make_uint(env, h));
}

/* release_handle(Res, node | group | sub, N) -> ok | {error, enoent}: N's term is gone from
 * every list on the device (the hooks that removed it committed): its term copy is freed now
 * (a window still in flight answers `undefined` for it, which dispatch skips) and the number is
 * reused once the windows submitted before now are answered (emqx_broker.erl:361-380) */
static ERL_NIF_TERM nif_release_handle(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  uint32_t kind;
  unsigned hv;
  (void)argc;
  term_tab* t;
  if (!get_res(env, argv[0], &r) || !r->hr || !(t = kind_tab(r, argv[1], &kind)) ||
      !enif_get_uint(env, argv[2], &hv))
    return enif_make_badarg(env);
  enif_rwlock_rwlock(t->lk);
  if (hv < t->n && t->v[hv].env) {
    enif_free_env(t->v[hv].env);
    t->v[hv].env = NULL;
    t->v[hv].t = 0;
  }
  enif_rwlock_rwunlock(t->lk);
  const int rc = emqxgm_handles_release(r->hr, kind, hv);
  return rc ? err_term(env, rc) : A_OK;
}

/* reset_handles(Res) -> ok: every allocated handle of every kind released and its term copy
 * freed (a restarted mirror, whose handles table died with the old process) */
static ERL_NIF_TERM nif_reset_handles(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  (void)argc;
  if (!get_res(env, argv[0], &r) || !r->hr) return enif_make_badarg(env);
  term_tab* tabs[3] = {&r->nodes, &r->groups, &r->subs};
  for (int k = 0; k < 3; ++k) {
    term_tab* t = tabs[k];
    enif_rwlock_rwlock(t->lk);
    for (unsigned i = 0; i < t->n; ++i)
      if (t->v[i].env) {
        enif_free_env(t->v[i].env);
        t->v[i].env = NULL;
      }
    enif_rwlock_rwunlock(t->lk);
  }
  const int rc = emqxgm_handles_reset(r->hr);
  return rc ? err_term(env, rc) : A_OK;
}

/* set_local_node(Res, NodeH) -> ok: node()'s dest handle (emqxgm_set_local_node) */
static ERL_NIF_TERM nif_set_local_node(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  unsigned v;
  (void)argc;
  if (!get_res(env, argv[0], &r) || !enif_get_uint(env, argv[1], &v)) return enif_make_badarg(env);
  int rc = 0;
  for (unsigned k = 0; k < r->nh; ++k) { /* every engine, as on_engines */
    const int e = emqxgm_set_local_node(r->h[k], v);
    if (!rc) rc = e;
  }
  return rc ? err_term(env, rc) : A_OK;
}

/* route_set(Res, Filter, Present) -> ok | {error, Reason}: one filter's membership in every engine
 * (no commit: the resync's and the mirror's unbatched form) */
static ERL_NIF_TERM nif_route_set(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  ErlNifBinary bin;
  (void)argc;
  if (!get_res(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &bin) ||
      (argv[2] != A_TRUE && argv[2] != A_FALSE))
    return enif_make_badarg(env);
  if (bin.size > GM_MAX_TOPIC) return err_term(env, -E2BIG);
  int rc = 0;
  for (unsigned k = 0; k < r->nh; ++k) { /* every engine, as on_engines */
    const int e = emqxgm_route_set(r->h[k], bin.data, (uint32_t)bin.size, argv[2] == A_TRUE);
    if (!rc) rc = e;
  }
  return rc ? err_term(env, rc) : A_OK;
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

/* commit(Res) -> {ok, Epoch} | {error, R}: everything pending visible on every engine (a delta
 * patch, or a full build -- in the background for a large registry, this call waiting for its
 * install; dirty CPU).  Every engine commits even after one failed; {error, estale}: committed,
 * but an engine is still stale (no resync since its last failure, include "Health"). */
static ERL_NIF_TERM nif_commit(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  uint64_t epoch = 0;
  int rc = 0;
  (void)argc;
  if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
  for (unsigned k = 0; k < r->nh; ++k) {
    uint64_t e = 0;
    const int c = emqxgm_commit(r->h[k], &e);
    if (!rc) rc = c;
    if (k == 0) epoch = e;
  }
  return rc ? err_term(env, rc) : enif_make_tuple2(env, A_OK, enif_make_uint64(env, epoch));
}

/* snapshot_save(Res, Path :: binary()) -> ok | {error, R}: the committed index of engine 0 (every
 * engine holds the same one) -- emqxgm_snapshot_save.  snapshot_load(Res, Path) -> ok | {error, R}:
 * into every engine of a fresh resource, before its first resync (emqxgm_snapshot_load: no full
 * build; the resync then commits only what changed since, as a delta).  The reference rebuilds its
 * ram_copies route tables from its peers at start (emqx_router.erl:78-92). */
static int get_path(ErlNifEnv* env, ERL_NIF_TERM t, char* buf, size_t cap) {
  ErlNifBinary b;
  if (!enif_inspect_binary(env, t, &b) || b.size == 0 || b.size >= cap || memchr(b.data, 0, b.size)) return 0;
  memcpy(buf, b.data, b.size);
  buf[b.size] = 0;
  return 1;
}

static ERL_NIF_TERM nif_snapshot_save(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  char path[4096];
  (void)argc;
  if (!get_res(env, argv[0], &r) || !get_path(env, argv[1], path, sizeof path)) return enif_make_badarg(env);
  const int rc = emqxgm_snapshot_save(r->h[0], path);
  return rc ? err_term(env, rc) : A_OK;
}

static ERL_NIF_TERM nif_snapshot_load(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  char path[4096];
  (void)argc;
  if (!get_res(env, argv[0], &r) || !get_path(env, argv[1], path, sizeof path)) return enif_make_badarg(env);
  for (unsigned k = 0; k < r->nh; ++k) {
    const int rc = emqxgm_snapshot_load(r->h[k], path);
    if (rc) return err_term(env, rc);
  }
  return A_OK;
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
  if (!get_res(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &bin)) return enif_make_badarg(env);
  if (bin.size > GM_MAX_TOPIC) return A_FALSE; /* never a filter (emqx_topic.erl:47) */
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

/* match_async(Res, Topic, Ref) / publish_async(Res, Topic, Ref) -> {ok, Call} | {error, R}: Topic
 * joins the open window of the layer on the caller's own scheduler (a copy into pinned memory);
 * the caller (self()) later receives {emqx_trie_gpu, Ref, ...}.  e2big: deeper than max_levels or
 * longer than a topic can be (the caller takes emqx_trie:match/1 then); ebusy: every window full;
 * einval: no publish layer. */
static ERL_NIF_TERM do_async(ErlNifEnv* env, const ERL_NIF_TERM argv[], int publish) {
  gm_res* r;
  ErlNifBinary bin;
  ErlNifPid self;
  if (!get_res(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &bin) ||
      !enif_is_ref(env, argv[2]) || !enif_self(env, &self))
    return enif_make_badarg(env);
  emqxgm_async_t* a = publish ? r->ap : r->a;
  if (!a) return err_term(env, -EINVAL);
  if (bin.size > GM_MAX_TOPIC) return err_term(env, -E2BIG);
  gm_call* c = enif_alloc_resource(CALL_RT, sizeof(gm_call));
  if (!c) return err_term(env, -ENOMEM);
  memset(c, 0, sizeof *c);
  ERL_NIF_TERM t = enif_make_resource(env, c); /* the caller's handle (cancel/2) */
  enif_release_resource(c);                    /* ... owns the allocation now */
  if (!(c->env = enif_alloc_env())) return err_term(env, -ENOMEM);
  c->ref = enif_make_copy(c->env, argv[2]);
  c->pid = self;
  c->publish = publish;
  c->tag = __atomic_fetch_add(&r->next_tag, 1, __ATOMIC_RELAXED);
  enif_keep_resource(c); /* the in-flight reference: released by its answer or its cancel */
  const int rc = emqxgm_async_match(a, bin.data, (uint32_t)bin.size, c->tag, (uint64_t)(uintptr_t)c);
  if (rc) {
    enif_release_resource(c);
    return err_term(env, rc);
  }
  return enif_make_tuple2(env, A_OK, t);
}

static ERL_NIF_TERM nif_match_async(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  return do_async(env, argv, 0);
}

static ERL_NIF_TERM nif_publish_async(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  return do_async(env, argv, 1);
}

/* cancel(Res, Call) -> true | false: true = the call will never be answered; false = its answer
 * is already in the caller's mailbox.  Dirty IO: may wait while the call's window is reported. */
static ERL_NIF_TERM nif_cancel(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  gm_call* c;
  (void)argc;
  if (!get_res(env, argv[0], &r) || !enif_get_resource(env, argv[1], CALL_RT, (void**)&c))
    return enif_make_badarg(env);
  emqxgm_async_t* a = c->publish ? r->ap : r->a;
  if (!a || c->tag == 0) return A_FALSE;
  const int rc = emqxgm_async_cancel(a, c->tag, (uint64_t)(uintptr_t)c);
  if (rc < 0) return err_term(env, rc);
  if (rc == 0) return A_FALSE;
  enif_release_resource(c); /* never answered: the in-flight reference goes here */
  return A_TRUE;
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

/* stats(Res) -> #{calls, windows, reported, busy, cancelled, too_deep, failed, outstanding,
 * bg_builds, bg_waits, last_build_ms, stale_engines, timeouts, refused, marks, repairs} */
static ERL_NIF_TERM nif_stats(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  static const char* keys[8] = {"calls", "windows", "reported", "busy",
                                "cancelled", "too_deep", "failed", "outstanding"};
  gm_res* r;
  uint64_t v[8];
  emqxgm_stats st;
  (void)argc;
  if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
  int rc = emqxgm_async_stats(r->a, v);
  if (!rc) rc = emqxgm_get_stats(r->h[0], &st);
  if (rc) return err_term(env, rc);
  ERL_NIF_TERM m = enif_make_new_map(env);
  for (int i = 0; i < 8; ++i)
    enif_make_map_put(env, m, enif_make_atom(env, keys[i]), enif_make_uint64(env, v[i]), &m);
  enif_make_map_put(env, m, enif_make_atom(env, "bg_builds"), enif_make_uint64(env, st.bg_builds), &m);
  enif_make_map_put(env, m, enif_make_atom(env, "bg_waits"), enif_make_uint64(env, st.bg_waits), &m);
  enif_make_map_put(env, m, enif_make_atom(env, "last_build_ms"), enif_make_double(env, st.last_build_ms), &m);
  /* health (include "Health"): engines stale now, timed-out calls, calls refused; engine marks
   * and repairs summed */
  uint64_t hv[4];
  if (emqxgm_async_health(r->a, hv) >= 0) {
    enif_make_map_put(env, m, enif_make_atom(env, "stale_engines"), enif_make_uint64(env, hv[0]), &m);
    enif_make_map_put(env, m, enif_make_atom(env, "timeouts"), enif_make_uint64(env, hv[1]), &m);
    enif_make_map_put(env, m, enif_make_atom(env, "refused"), enif_make_uint64(env, hv[3]), &m);
  }
  uint64_t marks = 0, repairs = 0;
  for (unsigned k = 0; k < r->nh; ++k) {
    emqxgm_health_t h;
    if (emqxgm_get_health(r->h[k], &h) >= 0) {
      marks += h.marks;
      repairs += h.repairs;
    }
  }
  enif_make_map_put(env, m, enif_make_atom(env, "marks"), enif_make_uint64(env, marks), &m);
  enif_make_map_put(env, m, enif_make_atom(env, "repairs"), enif_make_uint64(env, repairs), &m);
  return m;
}

/* ---- the retainer's reverse match and the ordered topic rules ------------
 * emqx_retainer_mnesia keeps its messages; its topics (with their expiry) are mirrored into an
 * emqxgm_retain_t store, and match_messages/3 (emqx_retainer_mnesia.erl:185-195) asks the device
 * for the stored topics a batch of filters selects (search_table/3's set, :300-330); the caller
 * reads the messages of those topics from its own table.  emqx_authz_rule:match_topics/3 and
 * emqx_rewrite:match_and_rewrite/3 keep their rule lists; match_rules/3 returns per name the
 * index of the first matching rule (emqxgm_match_rules). */
typedef struct {
  emqxgm_retain_t* r;
  ErlNifMutex* mu; /* the store is single-writer; matches read its committed state */
} gm_retain;

static void gm_retain_dtor(ErlNifEnv* env, void* obj) {
  gm_retain* g = (gm_retain*)obj;
  (void)env;
  if (g->r) emqxgm_retain_destroy(g->r);
  if (g->mu) enif_mutex_destroy(g->mu);
}

static int get_retain(ErlNifEnv* env, ERL_NIF_TERM t, gm_retain** g) {
  return enif_get_resource(env, t, RETAIN_RT, (void**)g) && (*g)->r;
}

/* retain_open(Device, IndexSpecs :: [[Pos]]) -> {ok, R} | {error, Reason}
 * (retainer.backend.index_specs, emqx_retainer_schema.erl:24-29; [] = the full scan only) */
static ERL_NIF_TERM nif_retain_open(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  int dev;
  unsigned ns;
  (void)argc;
  if (!enif_get_int(env, argv[0], &dev) || !enif_get_list_length(env, argv[1], &ns) || ns > 64)
    return enif_make_badarg(env);
  uint32_t pos[64 * 16], off[65];
  ERL_NIF_TERM l = argv[1], spec;
  unsigned np = 0;
  off[0] = 0;
  for (unsigned i = 0; i < ns; ++i) {
    ERL_NIF_TERM sl, ph;
    if (!enif_get_list_cell(env, l, &spec, &l)) return enif_make_badarg(env);
    for (sl = spec; enif_get_list_cell(env, sl, &ph, &sl);) {
      unsigned v;
      if (np >= 64 * 16 || !enif_get_uint(env, ph, &v)) return enif_make_badarg(env);
      pos[np++] = v;
    }
    off[i + 1] = np;
  }
  gm_retain* g = enif_alloc_resource(RETAIN_RT, sizeof(gm_retain));
  memset(g, 0, sizeof *g);
  g->mu = enif_mutex_create("emqx_trie_gpu.retain");
  int rc = g->mu ? emqxgm_retain_create(dev, &g->r) : -ENOMEM;
  if (!rc) rc = emqxgm_retain_set_indices(g->r, pos, off, ns);
  if (rc) {
    enif_release_resource(g);
    return rc == -EINVAL ? enif_make_badarg(env) : err_term(env, rc);
  }
  ERL_NIF_TERM t = enif_make_resource(env, g);
  enif_release_resource(g);
  return enif_make_tuple2(env, A_OK, t);
}

/* retain_store(R, Topic, ExpiryMs) -> ok (store_retained/2, :138-152; 0 = never expires),
 * retain_delete(R, Topic) -> ok (delete_message/2, :166-170), retain_clean(R) -> ok (clean/1),
 * retain_commit(R) -> ok: the mutations visible to retain_match/3 */
static ERL_NIF_TERM nif_retain_store(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_retain* g;
  ErlNifBinary b;
  ErlNifUInt64 exp;
  uint32_t id;
  (void)argc;
  if (!get_retain(env, argv[0], &g) || !enif_inspect_binary(env, argv[1], &b) ||
      !enif_get_uint64(env, argv[2], &exp))
    return enif_make_badarg(env);
  if (b.size > GM_MAX_TOPIC) return err_term(env, -E2BIG);
  enif_mutex_lock(g->mu);
  const int rc = emqxgm_retain_store(g->r, b.data, (uint32_t)b.size, exp, &id);
  enif_mutex_unlock(g->mu);
  return rc ? err_term(env, rc) : A_OK;
}

static ERL_NIF_TERM nif_retain_delete(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_retain* g;
  ErlNifBinary b;
  (void)argc;
  if (!get_retain(env, argv[0], &g) || !enif_inspect_binary(env, argv[1], &b)) return enif_make_badarg(env);
  if (b.size > GM_MAX_TOPIC) return A_OK; /* never stored */
  enif_mutex_lock(g->mu);
  const int rc = emqxgm_retain_delete(g->r, b.data, (uint32_t)b.size);
  enif_mutex_unlock(g->mu);
  return rc ? err_term(env, rc) : A_OK;
}

static ERL_NIF_TERM nif_retain_clean(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_retain* g;
  (void)argc;
  if (!get_retain(env, argv[0], &g)) return enif_make_badarg(env);
  enif_mutex_lock(g->mu);
  const int rc = emqxgm_retain_clean(g->r);
  enif_mutex_unlock(g->mu);
  return rc ? err_term(env, rc) : A_OK;
}

static ERL_NIF_TERM nif_retain_commit(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_retain* g;
  (void)argc;
  if (!get_retain(env, argv[0], &g)) return enif_make_badarg(env);
  enif_mutex_lock(g->mu);
  const int rc = emqxgm_retain_commit(g->r);
  enif_mutex_unlock(g->mu);
  return rc ? err_term(env, rc) : A_OK;
}

/* the packed list with 32-bit offsets (the retainer and rules entry points take those) */
static uint32_t* off32(const packed* p) {
  uint32_t* o = enif_alloc(sizeof(uint32_t) * ((size_t)p->n + 1));
  if (o)
    for (unsigned i = 0; i <= p->n; ++i) o[i] = (uint32_t)p->off[i];
  return o;
}

/* retain_match(R, [Filter], NowMs) -> [[Topic]] | {error, Reason}: match_messages/3 for a batch
 * of filters -- per filter the stored, live topics it selects (its messages are the caller's) */
static ERL_NIF_TERM nif_retain_match(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_retain* g;
  packed p;
  ErlNifUInt64 now;
  (void)argc;
  if (!get_retain(env, argv[0], &g) || !enif_get_uint64(env, argv[2], &now)) return enif_make_badarg(env);
  int rc = pack_list(env, argv[1], 0, &p);
  uint32_t* o = rc ? NULL : off32(&p);
  if (!rc && !o) rc = -ENOMEM;
  if (!rc && p.off[p.n] > 0xFFFFFFFFull) rc = -E2BIG;
  emqxgm_retain_out out;
  memset(&out, 0, sizeof out);
  ERL_NIF_TERM res = 0;
  if (!rc) {
    enif_mutex_lock(g->mu); /* the result lives in the store's buffers until its next call */
    rc = emqxgm_retain_match(g->r, p.bytes, o, p.n, now, &out);
    if (!rc) {
      res = enif_make_list(env, 0);
      for (uint32_t i = out.n; i-- > 0;) {
        ERL_NIF_TERM tl = enif_make_list(env, 0);
        for (uint64_t j = out.ptr[i + 1]; j-- > out.ptr[i];) {
          const uint8_t* tp;
          uint32_t tlen;
          if (emqxgm_retain_topic(g->r, out.id[j], &tp, &tlen) == 0)
            tl = enif_make_list_cell(env, bytes_term(env, tp, tlen), tl);
        }
        res = enif_make_list_cell(env, tl, res);
      }
    }
    enif_mutex_unlock(g->mu);
  }
  enif_free(o);
  packed_free(&p);
  if (rc == -EINVAL) return enif_make_badarg(env);
  return rc ? err_term(env, rc) : res;
}

/* match_rules(Res, [Name], [{Filter, eq | words | binary}]) -> [Index | none]: the first rule
 * each name matches (emqx_authz_rule:match_topics/3 with eq / words, emqx_rewrite's binary
 * match/2; placeholders substituted by the caller), on engine 0's device */
static ERL_NIF_TERM nif_match_rules(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  gm_res* r;
  packed nm, ru;
  (void)argc;
  if (!get_res(env, argv[0], &r)) return enif_make_badarg(env);
  int rc = pack_list(env, argv[1], 0, &nm);
  if (!rc) rc = pack_list(env, argv[2], 1, &ru);
  else memset(&ru, 0, sizeof ru);
  uint32_t *no = NULL, *ro = NULL, *fl = NULL, *out = NULL;
  if (!rc) {
    no = off32(&nm);
    ro = off32(&ru);
    fl = enif_alloc(sizeof(uint32_t) * (ru.n ? ru.n : 1));
    out = enif_alloc(sizeof(uint32_t) * (nm.n ? nm.n : 1));
    if (!no || !ro || !fl || !out) rc = -ENOMEM;
  }
  if (!rc && (nm.off[nm.n] > 0xFFFFFFFFull || ru.off[ru.n] > 0xFFFFFFFFull)) rc = -E2BIG;
  ERL_NIF_TERM head, l = argv[2];
  for (unsigned i = 0; !rc && i < ru.n; ++i) {
    int ar;
    const ERL_NIF_TERM* el;
    enif_get_list_cell(env, l, &head, &l);
    enif_get_tuple(env, head, &ar, &el);
    if (ar != 2) rc = -EINVAL;
    else if (el[1] == A_EQ) fl[i] = EMQXGM_RULE_EQ;
    else if (el[1] == A_WORDS) fl[i] = EMQXGM_RULE_WORDS;
    else if (el[1] == A_BINARY) fl[i] = 0;
    else rc = -EINVAL;
  }
  if (!rc) rc = emqxgm_match_rules(r->h[0], nm.bytes, no, nm.n, ru.bytes, ro, fl, ru.n, out);
  ERL_NIF_TERM res = enif_make_list(env, 0);
  for (uint32_t i = nm.n; !rc && i-- > 0;)
    res = enif_make_list_cell(env, out[i] == EMQXGM_NONE ? A_NONE : enif_make_uint(env, out[i]), res);
  enif_free(no);
  enif_free(ro);
  enif_free(fl);
  enif_free(out);
  packed_free(&nm);
  packed_free(&ru);
  if (rc == -EINVAL) return enif_make_badarg(env);
  return rc ? err_term(env, rc) : res;
}

static int load(ErlNifEnv* env, void** priv, ERL_NIF_TERM info) {
  (void)priv;
  (void)info;
  RT = enif_open_resource_type(env, NULL, "emqx_trie_gpu", gm_res_dtor, ERL_NIF_RT_CREATE, NULL);
  CALL_RT = enif_open_resource_type(env, NULL, "emqx_trie_gpu_call", gm_call_dtor, ERL_NIF_RT_CREATE, NULL);
  RETAIN_RT = enif_open_resource_type(env, NULL, "emqx_trie_gpu_retain", gm_retain_dtor, ERL_NIF_RT_CREATE, NULL);
  if (!RT || !CALL_RT || !RETAIN_RT || emqxgm_abi_version() != EMQXGM_ABI_VERSION) return -1;
  A_OK = enif_make_atom(env, "ok");
  A_ERROR = enif_make_atom(env, "error");
  A_TRUE = enif_make_atom(env, "true");
  A_FALSE = enif_make_atom(env, "false");
  A_MOD = enif_make_atom(env, "emqx_trie_gpu");
  A_ROUTES = enif_make_atom(env, "routes");
  A_NONE = enif_make_atom(env, "none");
  A_NODE = enif_make_atom(env, "node");
  A_GROUP = enif_make_atom(env, "group");
  A_SUB = enif_make_atom(env, "sub");
  A_SPIN_US = enif_make_atom(env, "spin_us");
  A_BG_BUILD = enif_make_atom(env, "bg_build");
  A_REPORT_THREADS = enif_make_atom(env, "report_threads");
  A_FAIL_THRESHOLD = enif_make_atom(env, "fail_threshold");
  A_EAGER = enif_make_atom(env, "eager");
  A_EQ = enif_make_atom(env, "eq");
  A_WORDS = enif_make_atom(env, "words");
  A_BINARY = enif_make_atom(env, "binary");
  A_PUBLISH = enif_make_atom(env, "publish");
  A_UNDEFINED = enif_make_atom(env, "undefined");
  return 0;
}

static ErlNifFunc funcs[] = {
    {"open", 6, nif_open, ERL_NIF_DIRTY_JOB_IO_BOUND},
    /* the writer lock: a commit that must wait for a background build holds a dirty scheduler */
    {"route_sync", 2, nif_route_sync, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"route_set", 3, nif_route_set, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"route_set_many", 3, nif_route_set_many, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"route_dests", 3, nif_route_dests, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"subscribers", 3, nif_subscribers, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"register", 3, nif_register, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"alloc_handle", 2, nif_alloc_handle, 0},
    {"release_handle", 3, nif_release_handle, 0},
    {"reset_handles", 1, nif_reset_handles, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"set_local_node", 2, nif_set_local_node, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"sync_begin", 1, nif_sync_begin, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"sync_end", 2, nif_sync_end, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"commit", 1, nif_commit, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"snapshot_save", 2, nif_snapshot_save, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"snapshot_load", 2, nif_snapshot_load, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"empty", 1, nif_empty, 0},
    {"trie_member", 2, nif_trie_member, 0},
    {"route_member", 2, nif_route_member, 0},
    {"match_async", 3, nif_match_async, 0},
    {"publish_async", 3, nif_publish_async, 0},
    {"cancel", 2, nif_cancel, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"tune", 3, nif_tune, ERL_NIF_DIRTY_JOB_IO_BOUND}, /* some keys drain the passes in flight */
    {"stats", 1, nif_stats, 0},
    {"retain_open", 2, nif_retain_open, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"retain_store", 3, nif_retain_store, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"retain_delete", 2, nif_retain_delete, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"retain_clean", 1, nif_retain_clean, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"retain_commit", 1, nif_retain_commit, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"retain_match", 3, nif_retain_match, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"match_rules", 3, nif_match_rules, ERL_NIF_DIRTY_JOB_IO_BOUND},
};

ERL_NIF_INIT(emqx_trie_gpu_nif, funcs, load, NULL, NULL, NULL)
