%%--------------------------------------------------------------------
%% emqx_trie_gpu -- emqx_trie:match/1, match_session/1 and emqx_router:match_routes/1 on the
%% MI355X engine.
%%
%%   emqx_trie:match/1, match_session/1        apps/emqx/src/emqx_trie.erl:147-169
%%   emqx_trie:empty/0, empty_session/0                                  :172-178
%%   emqx_router:match_trie/1, match_routes/1  apps/emqx/src/emqx_router.erl:141-153
%%
%% Every publisher process calls in itself, concurrently, as it calls emqx_trie:match/1 in the
%% reference (emqx_broker.erl:218-232): match_async/3 hands the topic to the engine's open window
%% on the caller's own scheduler and the caller waits for {emqx_trie_gpu, Id, Result}, which an
%% engine completer thread sends once the window's device pass is done.  No process sits between
%% the publishers and the device.
%%
%% The route tables (emqx_route; the session router's when persistent sessions are enabled) stay
%% the source of truth: emqx_trie_gpu_sync mirrors their committed state into the device indexes
%% and publishes an index only once its first full sync has been committed.  With enable = false,
%% before that, and whenever the device cannot answer (a topic deeper than max_levels, every
%% window busy, a device error, a timeout) the call is the reference's own.
%%--------------------------------------------------------------------
-module(emqx_trie_gpu).

-include_lib("emqx/include/emqx.hrl").

-export([child_specs/0, enabled/0, handle/1, publish/2]).
-export([match/1, match_session/1, match_trie/1, match_routes/1, empty/0, empty_session/0]).

-define(KEY(Index), {?MODULE, Index}).
-define(CONF(K, D), emqx_config:get([broker, perf, gpu_match, K], D)).

%% the supervisor's children (a maintainer adds them to emqx_broker_sup, INTEGRATION.md 4): one
%% mirror per index; each opens its engines in init/1
-spec child_specs() -> [supervisor:child_spec()].
child_specs() ->
    Indexes =
        case emqx_persistent_session:is_store_enabled() of
            true -> [route, session];
            false -> [route]
        end,
    [
        #{
            id => {emqx_trie_gpu_sync, I},
            start => {emqx_trie_gpu_sync, start_link, [I]},
            restart => permanent
        }
     || I <- Indexes
    ].

%% the published engines of index route | session, or undefined (not synced yet)
handle(Index) ->
    persistent_term:get(?KEY(Index), undefined).

%% called by emqx_trie_gpu_sync once the index's first full sync is committed
publish(Index, H) ->
    persistent_term:put(?KEY(Index), H).

enabled() ->
    device(route) =/= undefined.

device(Index) ->
    case ?CONF(enable, false) of
        true -> handle(Index);
        false -> undefined
    end.

%% emqx_trie:match/1: the wildcard filters of the trie matching Topic (a set; [] for a wildcard
%% topic name, emqx_trie.erl:157-166 -- the device applies that rule itself)
-spec match(emqx_types:topic()) -> [emqx_types:topic()].
match(Topic) when is_binary(Topic) ->
    match(route, Topic).

%% emqx_trie:match_session/1 (emqx_session_router:match_trie/1, emqx_session_router.erl:154-159)
-spec match_session(emqx_types:topic()) -> [emqx_types:topic()].
match_session(Topic) when is_binary(Topic) ->
    match(session, Topic).

match(Index, Topic) ->
    case device(Index) of
        undefined -> ref_match(Index, Topic);
        H -> device_match(Index, H, Topic)
    end.

ref_match(route, Topic) -> emqx_trie:match(Topic);
ref_match(session, Topic) -> emqx_trie:match_session(Topic).

device_match(Index, H, Topic) ->
    Id = erlang:unique_integer([positive]),
    case emqx_trie_gpu_nif:match_async(H, Topic, Id) of
        ok ->
            receive
                {emqx_trie_gpu, Id, Filters} when is_list(Filters) -> Filters;
                {emqx_trie_gpu, Id, {error, _}} -> ref_match(Index, Topic)
            after ?CONF(timeout_ms, 5000) ->
                case emqx_trie_gpu_nif:cancel(H, Id) of
                    true ->
                        ref_match(Index, Topic);
                    false ->
                        %% reported while we gave up: the answer is in the mailbox already
                        receive
                            {emqx_trie_gpu, Id, Filters} when is_list(Filters) -> Filters;
                            {emqx_trie_gpu, Id, _} -> ref_match(Index, Topic)
                        after 0 -> ref_match(Index, Topic)
                        end
                end
            end;
        {error, _} ->
            %% deeper than max_levels, every window busy, or shutting down
            ref_match(Index, Topic)
    end.

%% emqx_router:match_trie/1
match_trie(Topic) ->
    case empty() of
        true -> [];
        false -> match(Topic)
    end.

%% emqx_router:match_routes/1: the routes of the topic itself (even a wildcard string), then
%% those of every matched filter
-spec match_routes(emqx_types:topic()) -> [emqx_types:route()].
match_routes(Topic) when is_binary(Topic) ->
    case match_trie(Topic) of
        [] -> emqx_router:lookup_routes(Topic);
        Matched -> lists:append([emqx_router:lookup_routes(To) || To <- [Topic | Matched]])
    end.

%% emqx_trie:empty/0, empty_session/0 of the committed device index
empty() ->
    case device(route) of
        undefined -> emqx_trie:empty();
        H -> emqx_trie_gpu_nif:empty(H)
    end.

empty_session() ->
    case device(session) of
        undefined -> emqx_trie:empty_session();
        H -> emqx_trie_gpu_nif:empty(H)
    end.
