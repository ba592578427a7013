%%--------------------------------------------------------------------
%% emqx_trie_gpu -- emqx_trie:match/1 and emqx_router:match_routes/1 on the MI355X engine.
%%
%%   emqx_trie:match/1        apps/emqx/src/emqx_trie.erl:147-169
%%   emqx_router:match_trie/1 apps/emqx/src/emqx_router.erl:149-153
%%   emqx_router:match_routes/1                      :141-146
%%
%% The route bag (emqx_route) and the mnesia trie stay the source of truth; the device index
%% mirrors their committed state (emqx_trie_gpu_sync) and answers the match through the
%% batcher (emqx_trie_gpu_batcher).  Configuration: broker.perf.gpu_match
%% (emqx_trie_gpu_schema); with enable = false every call is the reference's own.
%%--------------------------------------------------------------------
-module(emqx_trie_gpu).

-include_lib("emqx/include/emqx.hrl").

-export([start_link/0, child_specs/0, enabled/0, handle/0]).
-export([match/1, match_trie/1, match_routes/1, empty/0]).

-define(HANDLE_KEY, {?MODULE, handle}).

enabled() ->
    emqx_config:get([broker, perf, gpu_match, enable], false) andalso
        persistent_term:get(?HANDLE_KEY, undefined) =/= undefined.

handle() ->
    persistent_term:get(?HANDLE_KEY).

%% opens the device index (broker.perf.gpu_match) and publishes its handle
start_link() ->
    Conf = emqx_config:get([broker, perf, gpu_match]),
    #{devices := [Device | _], batch_max := Max, batch_window_us := Us} = Conf,
    case emqx_trie_gpu_nif:open(Device, Max, 64 * Max, Us) of
        {ok, H} ->
            persistent_term:put(?HANDLE_KEY, H),
            ignore;
        {error, Reason} ->
            {error, {gpu_match_open, Reason}}
    end.

child_specs() ->
    [
        #{id => emqx_trie_gpu, start => {?MODULE, start_link, []}, restart => transient},
        #{
            id => emqx_trie_gpu_batcher,
            start => {emqx_trie_gpu_batcher, start_link, [handle()]},
            restart => permanent
        },
        #{id => emqx_trie_gpu_sync, start => {emqx_trie_gpu_sync, start_link, [handle()]}}
    ].

%% emqx_trie:match/1: the wildcard filters of the trie matching Topic (a set; [] for a
%% wildcard topic name, emqx_trie.erl:157-166).  Topics deeper than max_levels (the zone's
%% mqtt.max_topic_levels, emqx_mqtt_caps.erl:94-97, bypassed by internal publishes) take the
%% reference's path.
-spec match(emqx_types:topic()) -> [emqx_types:topic()].
match(Topic) when is_binary(Topic) ->
    case enabled() of
        false ->
            emqx_trie:match(Topic);
        true ->
            Words = emqx_topic:words(Topic),
            case emqx_topic:wildcard(Words) of
                true ->
                    [];
                false ->
                    case length(Words) > emqx_config:get([broker, perf, gpu_match, max_levels]) of
                        true -> emqx_trie:match(Topic);
                        false -> emqx_trie_gpu_batcher:match(Topic)
                    end
            end
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

%% emqx_trie:empty/0 of the committed device index
empty() ->
    case enabled() of
        false -> emqx_trie:empty();
        true -> emqx_trie_gpu_nif:empty(handle())
    end.
