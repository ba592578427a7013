%%--------------------------------------------------------------------
%% emqx_trie_gpu_sync -- mirrors the committed route table into the device index.
%%
%% emqx_trie:insert/delete run inside mria transactions that may abort and retry
%% (emqx_router_utils.erl:74-135), so the device only ever follows committed state: this process
%% subscribes to the route table's events, as emqx_router_helper does for its own table
%% (emqx_router_helper.erl:107), and applies the membership rule of emqx_router_utils.erl:34-39,
%% 57-71 -- a route key exists while its filter has a route, a wildcard filter is in the trie
%% while it has one.  Changes are committed (one atomic epoch swap) on a short tick; matches
%% never wait for it.
%%--------------------------------------------------------------------
-module(emqx_trie_gpu_sync).

-behaviour(gen_server).

-include_lib("emqx/include/emqx.hrl").

-export([start_link/1]).
-export([init/1, handle_call/3, handle_cast/2, handle_info/2]).

-define(ROUTE_TAB, emqx_route).
-define(TICK_MS, 2).

start_link(Handle) ->
    gen_server:start_link({local, ?MODULE}, ?MODULE, Handle, []).

init(H) ->
    {ok, _} = mnesia:subscribe({table, ?ROUTE_TAB, simple}),
    %% the routes that exist already: one full build
    lists:foreach(
        fun(Topic) -> first_route(H, Topic) end,
        lists:usort([T || #route{topic = T} <- ets:tab2list(?ROUTE_TAB)])
    ),
    {ok, _Epoch} = emqx_trie_gpu_nif:commit(H),
    {ok, #{h => H, dirty => false}}.

handle_call(_Req, _From, S) ->
    {reply, ignored, S}.

handle_cast(_Msg, S) ->
    {noreply, S}.

handle_info({mnesia_table_event, {write, #route{topic = T}, _}}, S = #{h := H}) ->
    case emqx_router:lookup_routes(T) of
        [_] -> first_route(H, T);
        _ -> ok
    end,
    {noreply, tick(S)};
handle_info({mnesia_table_event, {delete_object, #route{topic = T}, _}}, S = #{h := H}) ->
    case emqx_router:lookup_routes(T) of
        [] -> last_route(H, T);
        _ -> ok
    end,
    {noreply, tick(S)};
handle_info({mnesia_table_event, {delete, {?ROUTE_TAB, T}, _}}, S = #{h := H}) ->
    last_route(H, T),
    {noreply, tick(S)};
handle_info(commit, S = #{h := H}) ->
    {ok, _Epoch} = emqx_trie_gpu_nif:commit(H),
    {noreply, S#{dirty := false}};
handle_info(_Info, S) ->
    {noreply, S}.

first_route(H, Topic) ->
    ok = emqx_trie_gpu_nif:route_ref(H, Topic),
    emqx_topic:wildcard(Topic) andalso (ok = emqx_trie_gpu_nif:trie_insert(H, Topic)),
    ok.

last_route(H, Topic) ->
    ok = emqx_trie_gpu_nif:route_unref(H, Topic),
    emqx_topic:wildcard(Topic) andalso (ok = emqx_trie_gpu_nif:trie_delete(H, Topic)),
    ok.

tick(S = #{dirty := true}) ->
    S;
tick(S) ->
    erlang:send_after(?TICK_MS, self(), commit),
    S#{dirty := true}.
