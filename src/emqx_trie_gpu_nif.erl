%%--------------------------------------------------------------------
%% emqx_trie_gpu_nif -- the NIF stubs of c_src/emqx_trie_gpu_nif.c (libemqx_gpumatch.so,
%% include/emqx_gpumatch.h).  Replaced at load time; every stub raises nif_not_loaded.
%%--------------------------------------------------------------------
-module(emqx_trie_gpu_nif).

-export([
    open/6,
    route_sync/2,
    route_set/3,
    route_set_many/3,
    route_dests/3,
    subscribers/3,
    register/3,
    alloc_handle/2,
    release_handle/3,
    reset_handles/1,
    set_local_node/2,
    sync_begin/1,
    sync_end/2,
    commit/1,
    snapshot_save/2,
    snapshot_load/2,
    empty/1,
    trie_member/2,
    route_member/2,
    match_async/3,
    publish_async/3,
    cancel/2,
    tune/3,
    stats/1,
    retain_open/2,
    retain_store/3,
    retain_delete/2,
    retain_clean/1,
    retain_commit/1,
    retain_match/3,
    match_rules/3
]).

-on_load(init/0).

init() ->
    PrivDir =
        case code:priv_dir(emqx) of
            {error, _} -> "priv";
            Dir -> Dir
        end,
    erlang:load_nif(filename:join(PrivDir, "emqx_trie_gpu_nif"), 0).

-define(NOT_LOADED, erlang:nif_error(nif_not_loaded)).

%% open(Devices, WindowTopics, WindowBytes, WindowUs, MaxLevels,
%%      #{spin_us => N, bg_build => N, publish => boolean()}) -> {ok, Res} | {error, Reason}
open(_Devices, _WindowTopics, _WindowBytes, _WindowUs, _MaxLevels, _Opts) -> ?NOT_LOADED.
%% route_sync(Res, [{Filter, Present :: boolean()}]) -> {ok, Epoch}: set and committed (visible to
%% every later publish) before it returns; never waits for a background full build
route_sync(_Res, _Items) -> ?NOT_LOADED.
%% route_set(Res, Filter, Present :: boolean()) -> ok | {error, Reason} (pending until commit/1)
route_set(_Res, _Filter, _Present) -> ?NOT_LOADED.
%% route_set_many(Res, [Filter], Present) -> ok | {error, Reason} (a resync chunk, pending)
route_set_many(_Res, _Filters, _Present) -> ?NOT_LOADED.
%% route_dests(Res, [{Filter, [{NodeH, GroupH | none}]}], Commit :: boolean()) -> {ok, Epoch}
route_dests(_Res, _Items, _Commit) -> ?NOT_LOADED.
%% subscribers(Res, [{Filter, [SubH]}], Commit :: boolean()) -> {ok, Epoch}
subscribers(_Res, _Items, _Commit) -> ?NOT_LOADED.
%% register(Res, node | group | sub, [{Handle, Term}]) -> ok
register(_Res, _Kind, _Items) -> ?NOT_LOADED.

%% alloc_handle(Res, node | group | sub) -> {ok, N} | {error, e2big}
alloc_handle(_Res, _Kind) -> ?NOT_LOADED.

%% release_handle(Res, node | group | sub, N) -> ok | {error, enoent}
release_handle(_Res, _Kind, _N) -> ?NOT_LOADED.

%% reset_handles(Res) -> ok: every handle released (a restarted mirror's, whose table died)
reset_handles(_Res) -> ?NOT_LOADED.
%% set_local_node(Res, NodeH) -> ok
set_local_node(_Res, _NodeH) -> ?NOT_LOADED.
%% sync_begin(Res) -> {ok, Gen}
sync_begin(_Res) -> ?NOT_LOADED.
%% ---- the retainer's reverse match (emqx_retainer_mnesia.erl:138-195, 241-247) ----
%% retain_open(Device, IndexSpecs :: [[pos_integer()]]) -> {ok, R} | {error, Reason}
retain_open(_Device, _IndexSpecs) -> ?NOT_LOADED.
%% retain_store(R, Topic, ExpiryMs) -> ok (store_retained/2; 0: never expires)
retain_store(_R, _Topic, _ExpiryMs) -> ?NOT_LOADED.
%% retain_delete(R, Topic) -> ok (delete_message/2 of one topic)
retain_delete(_R, _Topic) -> ?NOT_LOADED.
%% retain_clean(R) -> ok (clean/1)
retain_clean(_R) -> ?NOT_LOADED.
%% retain_commit(R) -> ok: the mutations visible to retain_match/3
retain_commit(_R) -> ?NOT_LOADED.
%% retain_match(R, [Filter], NowMs) -> [[Topic]]: match_messages/3 for a batch of filters
retain_match(_R, _Filters, _NowMs) -> ?NOT_LOADED.
%% match_rules(Res, [Name], [{Filter, eq | words | binary}]) -> [Index | none]: the first rule
%% each name matches (emqx_authz_rule:match_topics/3, emqx_rewrite:match_and_rewrite/3)
match_rules(_Res, _Names, _Rules) -> ?NOT_LOADED.
%% snapshot_save(Res, Path :: binary()) -> ok | {error, Reason}: the committed index to a file
snapshot_save(_Res, _Path) -> ?NOT_LOADED.
%% snapshot_load(Res, Path :: binary()) -> ok | {error, Reason}: into a fresh resource, no build
snapshot_load(_Res, _Path) -> ?NOT_LOADED.
%% sync_end(Res, Gen) -> {ok, Removed}
sync_end(_Res, _Gen) -> ?NOT_LOADED.
%% commit(Res) -> {ok, Epoch}
commit(_Res) -> ?NOT_LOADED.
empty(_Res) -> ?NOT_LOADED.
trie_member(_Res, _Filter) -> ?NOT_LOADED.
route_member(_Res, _Filter) -> ?NOT_LOADED.
%% match_async(Res, Topic, Ref) -> {ok, Call} | {error, e2big | ebusy | eshutdown}; later the
%% caller gets {emqx_trie_gpu, Ref, [Filter], ExactHit :: boolean()} | {emqx_trie_gpu, Ref, {error, R}}
match_async(_Res, _Topic, _Ref) -> ?NOT_LOADED.
%% publish_async(Res, Topic, Ref) -> {ok, Call} | {error, R}; later
%% {emqx_trie_gpu, Ref, {routes, [{To, Node | Group}], [{To, SubPid}]}} | {emqx_trie_gpu, Ref, {error, R}}
publish_async(_Res, _Topic, _Ref) -> ?NOT_LOADED.
%% cancel(Res, Call) -> true (never answered) | false (the answer is in the mailbox)
cancel(_Res, _Call) -> ?NOT_LOADED.
tune(_Res, _Key, _Value) -> ?NOT_LOADED.
stats(_Res) -> ?NOT_LOADED.
