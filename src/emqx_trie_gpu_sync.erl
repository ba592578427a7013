%%--------------------------------------------------------------------
%% emqx_trie_gpu_sync -- mirrors one committed route table into its device index.
%%
%% Index route   : the route table emqx_route (emqx_router.erl:72-92) -> emqx_trie's trie;
%% Index session : the session router's table (emqx_session_router.erl:64-65, 312-316) -> the
%%                 session trie (emqx_trie.erl:117-119, 135-137, 151-153).
%%
%% emqx_trie:insert/delete run inside mria transactions that may abort and retry
%% (emqx_router_utils.erl:74-135), so the device follows committed state only.  The mirror is
%% LEVEL-triggered: whatever event arrives for a topic T, it reads the table as it is now and
%% sets T's membership to match it (emqxgm_route_set: a route key while T has a route, a trie
%% member while a wildcard T has one -- the rule of emqx_router_utils.erl:34-39, 57-71).  The
%% number and order of events therefore never matter: two dests added before the first event is
%% handled, paired deletes, events queued while init/1 scans the table, a restart -- each ends in
%% the table's state.  Changes are committed (one atomic epoch swap) on a short tick; matches
%% never wait for it.
%%
%% Full resyncs (init/1, then every resync_interval_ms): sync_begin, every topic of the table set
%% present, sync_end -- which removes every route key the scan did not see.  Events that arrive
%% during a scan are handled after it, against the table as it is then, so they win.  The
%% periodic resync is what keeps a node that never sees the table's mnesia events in step: on a
%% mria replicant the route shard is replayed from the core nodes' rlog (emqx_router.erl:78-92)
%% and mnesia table events may not fire there, so such a node lags by at most one interval.
%%--------------------------------------------------------------------
-module(emqx_trie_gpu_sync).

-behaviour(gen_server).

-export([start_link/1]).
-export([init/1, handle_call/3, handle_cast/2, handle_info/2]).

-define(TICK_MS, 2).
-define(CONF(K, D), emqx_config:get([broker, perf, gpu_match, K], D)).

start_link(Index) ->
    gen_server:start_link({local, name(Index)}, ?MODULE, Index, []).

name(route) -> emqx_trie_gpu_sync_route;
name(session) -> emqx_trie_gpu_sync_session.

%% emqx_session_router:route_tab/0 (emqx_session_router.erl:312-316)
table(route) ->
    emqx_route;
table(session) ->
    case emqx_persistent_session:storage_type() of
        disc -> emqx_session_route_disc;
        ram -> emqx_session_route_ram
    end.

init(Index) ->
    Tab = table(Index),
    case open(Index) of
        {ok, H} ->
            {ok, _} = mnesia:subscribe({table, Tab, simple}),
            ok = tune(H),
            S = #{index => Index, h => H, tab => Tab, dirty => false},
            ok = resync(S),
            {ok, _Epoch} = emqx_trie_gpu_nif:commit(H),
            %% only now may publishers use it (before, they take the reference's path)
            emqx_trie_gpu:publish(Index, H),
            schedule_resync(),
            {ok, S};
        {error, Reason} ->
            {stop, {gpu_match_open, Reason}}
    end.

%% a restart keeps the engines (and their index) it published: the resync repairs whatever
%% changed meanwhile
open(Index) ->
    case emqx_trie_gpu:handle(Index) of
        undefined ->
            emqx_trie_gpu_nif:open(
                ?CONF(devices, [0]),
                ?CONF(batch_max, 65536),
                64 * ?CONF(batch_max, 65536),
                ?CONF(batch_window_us, 50),
                ?CONF(max_levels, 128)
            );
        H ->
            {ok, H}
    end.

tune(H) ->
    Delta =
        case ?CONF(delta_commit, small) of
            never -> 0;
            small -> 1;
            always -> 2
        end,
    emqx_trie_gpu_nif:tune(H, delta_commit, Delta).

handle_call(_Req, _From, S) ->
    {reply, ignored, S}.

handle_cast(_Msg, S) ->
    {noreply, S}.

%% simple table events: the record's first field is the topic, whatever its tag
handle_info({mnesia_table_event, {write, Route, _}}, S) ->
    {noreply, set(element(2, Route), S)};
handle_info({mnesia_table_event, {delete_object, Route, _}}, S) ->
    {noreply, set(element(2, Route), S)};
handle_info({mnesia_table_event, {delete, {_Tab, Topic}, _}}, S) ->
    {noreply, set(Topic, S)};
handle_info(commit, S = #{h := H}) ->
    {ok, _Epoch} = emqx_trie_gpu_nif:commit(H),
    {noreply, S#{dirty := false}};
handle_info(resync, S) ->
    ok = resync(S),
    schedule_resync(),
    {noreply, tick(S)};
handle_info(_Info, S) ->
    {noreply, S}.

%% T's membership := whether the table holds a route for T now
set(Topic, S = #{h := H, tab := Tab}) ->
    case emqx_trie_gpu_nif:route_set(H, Topic, ets:member(Tab, Topic)) of
        ok ->
            tick(S);
        {error, _} ->
            %% the engine refused (out of memory): a full resync retries every key
            self() ! resync,
            S
    end.

resync(#{h := H, tab := Tab}) ->
    {ok, Gen} = emqx_trie_gpu_nif:sync_begin(H),
    ets:foldl(
        fun(Route, ok) -> emqx_trie_gpu_nif:route_set(H, element(2, Route), true) end,
        ok,
        Tab
    ),
    {ok, _Removed} = emqx_trie_gpu_nif:sync_end(H, Gen),
    ok.

schedule_resync() ->
    erlang:send_after(?CONF(resync_interval_ms, 30000), self(), resync).

tick(S = #{dirty := true}) ->
    S;
tick(S) ->
    erlang:send_after(?TICK_MS, self(), commit),
    S#{dirty := true}.
