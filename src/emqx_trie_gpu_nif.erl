%%--------------------------------------------------------------------
%% emqx_trie_gpu_nif -- the NIF stubs of c_src/emqx_trie_gpu_nif.c (libemqx_gpumatch.so,
%% include/emqx_gpumatch.h).  Replaced at load time; every stub raises nif_not_loaded.
%%--------------------------------------------------------------------
-module(emqx_trie_gpu_nif).

-export([
    open/4,
    trie_insert/2,
    trie_delete/2,
    route_ref/2,
    route_unref/2,
    commit/1,
    empty/1,
    add/3,
    due/1,
    flush/1,
    collect/2,
    tune/3
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

%% open(Device, WindowTopics, WindowBytes, WindowUs) -> {ok, Handle} | {error, Reason}
open(_Device, _WindowTopics, _WindowBytes, _WindowUs) -> ?NOT_LOADED.
trie_insert(_H, _Filter) -> ?NOT_LOADED.
trie_delete(_H, _Filter) -> ?NOT_LOADED.
route_ref(_H, _Filter) -> ?NOT_LOADED.
route_unref(_H, _Filter) -> ?NOT_LOADED.
%% commit(H) -> {ok, Epoch}
commit(_H) -> ?NOT_LOADED.
empty(_H) -> ?NOT_LOADED.
%% add(H, Topic, Tag) -> ok | full | {error, enospc | e2big}
add(_H, _Topic, _Tag) -> ?NOT_LOADED.
due(_H) -> ?NOT_LOADED.
%% flush(H) -> {ok, WindowId} | empty | {error, ebusy}
flush(_H) -> ?NOT_LOADED.
%% collect(H, WindowId) -> {ok, [{Tag, [Filter], ExactHit}]}
collect(_H, _WindowId) -> ?NOT_LOADED.
tune(_H, _Key, _Value) -> ?NOT_LOADED.
