/* Test infrastructure only: the declarations of the erl_nif calls c_src/emqx_trie_gpu_nif.c
 * uses, with OTP's signatures, so tests/test_nif_syntax.py can compile-check the NIF where no
 * Erlang runtime (and so no erl_nif.h) exists.  Never linked, never run. */
#include <stddef.h>
typedef unsigned long ERL_NIF_TERM;
typedef struct enif_environment_t ErlNifEnv;
typedef struct { size_t size; unsigned char* data; } ErlNifBinary;
typedef struct { ERL_NIF_TERM pid; } ErlNifPid;
typedef struct enif_resource_type_t ErlNifResourceType;
typedef long ErlNifSInt; typedef unsigned long ErlNifUInt;
typedef enum { ERL_NIF_LATIN1 = 1 } ErlNifCharEncoding;
#define ERL_NIF_LATIN1 ERL_NIF_LATIN1
typedef enum { ERL_NIF_RT_CREATE = 1 } ErlNifResourceFlags;
#define ERL_NIF_DIRTY_JOB_CPU_BOUND 1
#define ERL_NIF_DIRTY_JOB_IO_BOUND 2
typedef struct { const char* name; unsigned arity; ERL_NIF_TERM (*fptr)(ErlNifEnv*, int, const ERL_NIF_TERM[]); unsigned flags; } ErlNifFunc;
typedef void ErlNifResourceDtor(ErlNifEnv*, void*);
ErlNifEnv* enif_alloc_env(void); void enif_free_env(ErlNifEnv*); void enif_clear_env(ErlNifEnv*);
void* enif_alloc_resource(ErlNifResourceType*, size_t); void enif_release_resource(void*);
int enif_get_atom(ErlNifEnv*, ERL_NIF_TERM, char*, unsigned, ErlNifCharEncoding);
int enif_get_int(ErlNifEnv*, ERL_NIF_TERM, int*); int enif_get_uint(ErlNifEnv*, ERL_NIF_TERM, unsigned*);
int enif_get_list_cell(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM*, ERL_NIF_TERM*);
int enif_get_list_length(ErlNifEnv*, ERL_NIF_TERM, unsigned*);
int enif_get_resource(ErlNifEnv*, ERL_NIF_TERM, ErlNifResourceType*, void**);
int enif_inspect_binary(ErlNifEnv*, ERL_NIF_TERM, ErlNifBinary*);
ERL_NIF_TERM enif_make_atom(ErlNifEnv*, const char*); ERL_NIF_TERM enif_make_badarg(ErlNifEnv*);
ERL_NIF_TERM enif_make_list(ErlNifEnv*, unsigned, ...); ERL_NIF_TERM enif_make_list_cell(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM);
int enif_make_map_put(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM*);
unsigned char* enif_make_new_binary(ErlNifEnv*, size_t, ERL_NIF_TERM*); ERL_NIF_TERM enif_make_new_map(ErlNifEnv*);
ERL_NIF_TERM enif_make_resource(ErlNifEnv*, void*); ERL_NIF_TERM enif_make_tuple(ErlNifEnv*, unsigned, ...);
ERL_NIF_TERM enif_make_uint(ErlNifEnv*, unsigned);
ErlNifResourceType* enif_open_resource_type(ErlNifEnv*, const char*, const char*, ErlNifResourceDtor*, ErlNifResourceFlags, ErlNifResourceFlags*);
ErlNifPid* enif_self(ErlNifEnv*, ErlNifPid*); int enif_send(ErlNifEnv*, const ErlNifPid*, ErlNifEnv*, ERL_NIF_TERM);
#define ERL_NIF_INIT(name, funcs, load, reload, upgrade, unload) void* nif_init_##name(void) { (void)funcs; (void)load; (void)upgrade; (void)unload; return 0; }
typedef unsigned long ErlNifUInt64; typedef long ErlNifSInt64;
ERL_NIF_TERM enif_make_tuple2(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_tuple3(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_tuple4(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_uint64(ErlNifEnv*, ErlNifUInt64); ERL_NIF_TERM enif_make_int(ErlNifEnv*, int);
ERL_NIF_TERM enif_make_int64(ErlNifEnv*, ErlNifSInt64);
int enif_get_uint64(ErlNifEnv*, ERL_NIF_TERM, ErlNifUInt64*); int enif_get_int64(ErlNifEnv*, ERL_NIF_TERM, ErlNifSInt64*);
int enif_is_list(ErlNifEnv*, ERL_NIF_TERM); ERL_NIF_TERM enif_make_list_from_array(ErlNifEnv*, const ERL_NIF_TERM*, unsigned);
ERL_NIF_TERM enif_make_double(ErlNifEnv*, double);
void* enif_alloc(size_t); void enif_free(void*);
int enif_keep_resource(void*); ERL_NIF_TERM enif_make_copy(ErlNifEnv*, ERL_NIF_TERM);
int enif_is_ref(ErlNifEnv*, ERL_NIF_TERM); int enif_is_atom(ErlNifEnv*, ERL_NIF_TERM);
int enif_is_identical(ERL_NIF_TERM, ERL_NIF_TERM);
int enif_get_tuple(ErlNifEnv*, ERL_NIF_TERM, int*, const ERL_NIF_TERM**);
int enif_get_map_value(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM*);
typedef struct ErlNifRWLock ErlNifRWLock;
ErlNifRWLock* enif_rwlock_create(char*); void enif_rwlock_destroy(ErlNifRWLock*);
void enif_rwlock_rlock(ErlNifRWLock*); void enif_rwlock_runlock(ErlNifRWLock*);
void enif_rwlock_rwlock(ErlNifRWLock*); void enif_rwlock_rwunlock(ErlNifRWLock*);
void* enif_realloc(void*, size_t);
typedef unsigned long ErlNifTid; typedef struct ErlNifThreadOpts ErlNifThreadOpts;
int enif_thread_create(char*, ErlNifTid*, void* (*)(void*), void*, ErlNifThreadOpts*);
int enif_thread_join(ErlNifTid, void**);
typedef struct ErlNifMutex ErlNifMutex;
ErlNifMutex* enif_mutex_create(char*); void enif_mutex_destroy(ErlNifMutex*);
void enif_mutex_lock(ErlNifMutex*); void enif_mutex_unlock(ErlNifMutex*);
