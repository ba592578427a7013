%%--------------------------------------------------------------------
%% emqx_trie_gpu_nif -- the NIF stubs of c_src/emqx_trie_gpu_nif.c (libemqx_gpumatch.so,
%% include/emqx_gpumatch.h).  Replaced at load time; every stub raises nif_not_loaded.
%%--------------------------------------------------------------------
-module(emqx_trie_gpu_nif).

-export([
    open/5,
    route_set/3,
    sync_begin/1,
    sync_end/2,
    commit/1,
    empty/1,
    trie_member/2,
    route_member/2,
    match_async/3,
    cancel/2,
    tune/3,
    stats/1
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

%% open(Devices, WindowTopics, WindowBytes, WindowUs, MaxLevels) -> {ok, Res} | {error, Reason}
open(_Devices, _WindowTopics, _WindowBytes, _WindowUs, _MaxLevels) -> ?NOT_LOADED.
%% route_set(Res, Filter, Present :: boolean()) -> ok | {error, Reason}
route_set(_Res, _Filter, _Present) -> ?NOT_LOADED.
%% sync_begin(Res) -> {ok, Gen}
sync_begin(_Res) -> ?NOT_LOADED.
%% sync_end(Res, Gen) -> {ok, Removed}
sync_end(_Res, _Gen) -> ?NOT_LOADED.
%% commit(Res) -> {ok, Epoch}
commit(_Res) -> ?NOT_LOADED.
empty(_Res) -> ?NOT_LOADED.
trie_member(_Res, _Filter) -> ?NOT_LOADED.
route_member(_Res, _Filter) -> ?NOT_LOADED.
%% match_async(Res, Topic, Id) -> ok | {error, e2big | ebusy | eshutdown}; later the caller gets
%% {emqx_trie_gpu, Id, [Filter] | {error, Reason}}
match_async(_Res, _Topic, _Id) -> ?NOT_LOADED.
%% cancel(Res, Id) -> true (never answered) | false (the answer is in the mailbox)
cancel(_Res, _Id) -> ?NOT_LOADED.
tune(_Res, _Key, _Value) -> ?NOT_LOADED.
stats(_Res) -> ?NOT_LOADED.
