%%--------------------------------------------------------------------
%% emqx_trie_gpu_sync -- mirrors one committed table set into its device index.
%%
%% Index route   : the route table emqx_route (emqx_router.erl:72-92) -> emqx_trie's trie, the
%%                 route keys and every route's dests; the local subscriber bag emqx_subscriber
%%                 (emqx_broker.erl:546-579) -> the fan-out's local dispatch lists;
%% Index session : the session router's table (emqx_session_router.erl:64-65, 312-316) -> the
%%                 session trie (emqx_trie.erl:117-119, 135-137, 151-153).
%%
%% emqx_trie:insert/delete run inside mria transactions that may abort and retry
%% (emqx_router_utils.erl:74-135), so the device follows committed state only.  The mirror is
%% LEVEL-triggered: whatever event arrives for a topic T, it reads the table as it is now and
%% sets T's state on the device to it (its dests -- and with them the route key and, for a
%% wildcard T, the trie membership: the rule of emqx_router_utils.erl:34-39, 57-71 as a state).
%% The number and order of events therefore never matter.
%%
%% Table events are handled in batches: every event queued when the process gets to them becomes
%% one device call that is committed before it returns (emqxgm_route_dests_batch with
%% EMQXGM_SET_COMMIT), with no tick.  It never waits for a full build: a build (the first one, or
%% one the tables' load starts) runs in the background while these commits patch the index the
%% publishers read.  The writing node's own changes do not wait for this process at all: its hooks
%% (emqx_trie_gpu:route_changed/1, subscribers_changed/1) commit them before SUBACK.
%%
%% Full resyncs: at start (handle_continue, so the supervisor is not held) and, where table events
%% may be missed -- a mria replicant, whose route shard is replayed from the core nodes' rlog
%% (emqx_router.erl:78-92) -- every resync_interval_ms.  sync_begin, every topic of the table in
%% chunks of ?CHUNK distinct topics per dirty NIF call, the local subscriber lists, sync_end
%% (removes every route key and subscriber list the scan did not give), commit.  Events that arrive during a scan are handled after it, against the
%% table as it is then, so they win.
%%
%% Failing closed (r06).  No NIF result is matched with `ok =`: an engine that refuses a call has
%% marked itself stale (it answers no publisher until a repair, include/emqx_gpumatch.h "Health"),
%% and this process repairs it -- a full resync and a commit, retried with a doubling backoff
%% (?BACKOFF_MIN .. ?BACKOFF_MAX ms) until the engines are healthy -- instead of crashing and taking
%% emqx_broker_sup down with it after the restart intensity.  repair/1 casts (a hook's refused
%% commit, a publisher's timeout or failed window) queued while one runs are folded into it.  The
%% index is published after the first successful repair only.
%%--------------------------------------------------------------------
-module(emqx_trie_gpu_sync).

-behaviour(gen_server).

-include_lib("emqx/include/emqx.hrl").
-include_lib("emqx/include/logger.hrl").

-export([start_link/1, table/1, repair/1]).
-export([init/1, handle_continue/2, handle_call/3, handle_cast/2, handle_info/2, terminate/2]).

-define(CHUNK, 65536).       %% distinct topics per resync call
-define(BATCH, 65536).       %% table events per device call
-define(CONF(K, D), emqx_config:get([broker, perf, gpu_match, K], D)).
-define(BACKOFF_MIN, 100).
-define(SAMPLE_MS, 100).     %% the load-adaptive choice's rate sample (emqx_trie_gpu:sample_load/2)
-define(BACKOFF_MAX, 30000).

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

%% a device call was refused, a window failed or a publisher timed out: resync and commit
repair(Index) ->
    gen_server:cast(name(Index), resync).

init(Index) ->
    %% a restarted mirror: publishers take the reference's path until its resync is committed
    %% (the handles table died with the old process)
    process_flag(trap_exit, true),
    ok = emqx_trie_gpu:publish(Index, undefined),
    {ok,
        #{
            index => Index,
            h => undefined,
            tab => table(Index),
            published => false,
            backoff => 0,
            retry => undefined,
            load => undefined
        },
        {continue, open}}.

handle_continue(open, S = #{index := Index, tab := Tab}) ->
    case open(Index) of
        {ok, H, Fresh} ->
            %% fresh engines start from the last snapshot, when there is one: no full build,
            %% the resync below commits what changed since as a delta
            _ = Fresh andalso load_snapshot(Index, H),
            {ok, _} = mnesia:subscribe({table, Tab, simple}),
            S1 = S#{h := H},
            %% (a refused step leaves the engines unpublished until a repair succeeds)
            _ = (catch prepare(Index, H)),
            S2 = repair_now(S1),
            schedule_resync(),
            _ = Index =:= route andalso erlang:send_after(?SAMPLE_MS, self(), sample_load),
            {noreply, S2};
        {error, Reason} ->
            {stop, {gpu_match_open, Reason}, S}
    end.

%% A full resync and a commit.  Success: the engines are healthy again (and the index is published,
%% the first time: before, publishers take the reference's path).  Failure: retried after the
%% backoff, which doubles up to ?BACKOFF_MAX.
repair_now(S = #{index := Index, h := H, published := Pub, backoff := B}) ->
    drop_queued_repairs(),
    S1 = cancel_retry(S),
    Result =
        case resync(S1) of
            ok -> emqx_trie_gpu_nif:commit(H);
            {error, _} = E -> E
        end,
    case Result of
        {ok, _Epoch} ->
            _ = Pub orelse emqx_trie_gpu:publish(Index, H),
            S1#{published := true, backoff := 0};
        {error, Reason} ->
            B1 = min(?BACKOFF_MAX, max(?BACKOFF_MIN, 2 * B)),
            ?SLOG(warning, #{msg => "gpu_match_repair_failed", index => Index, reason => Reason,
                             retry_ms => B1}),
            S1#{backoff := B1, retry := erlang:send_after(B1, self(), repair)}
    end.

cancel_retry(S = #{retry := undefined}) ->
    S;
cancel_retry(S = #{retry := T}) ->
    _ = erlang:cancel_timer(T),
    receive
        repair -> ok
    after 0 -> ok
    end,
    S#{retry := undefined}.

%% repair/1 casts queued behind this one: this repair covers them
drop_queued_repairs() ->
    receive
        {'$gen_cast', resync} -> drop_queued_repairs()
    after 0 -> ok
    end.

%% a restart keeps the engines (and their index) it published: the resync repairs whatever
%% changed meanwhile
open(Index) ->
    case persistent_term:get({emqx_trie_gpu, {engines, Index}}, undefined) of
        undefined ->
            Opts = #{
                spin_us => ?CONF(spin_us, 0),
                bg_build => ?CONF(bg_build, 16384),
                report_threads => ?CONF(report_threads, 8),
                fail_threshold => ?CONF(fail_threshold, 3),
                eager => ?CONF(eager_windows, true),
                publish => Index =:= route andalso ?CONF(publish, true)
            },
            case
                emqx_trie_gpu_nif:open(
                    ?CONF(devices, [0]),
                    ?CONF(batch_max, 65536),
                    64 * ?CONF(batch_max, 65536),
                    ?CONF(batch_window_us, 50),
                    ?CONF(max_levels, 128),
                    Opts
                )
            of
                {ok, H} ->
                    persistent_term:put({emqx_trie_gpu, {engines, Index}}, H),
                    {ok, H, true};
                Error ->
                    Error
            end;
        H ->
            {ok, H, false}
    end.

%% broker.perf.gpu_match.snapshot_dir: the index of each table saved there at shutdown and loaded
%% at the next start (emqxgm_snapshot_save / _load)
snapshot_path(Index) ->
    case ?CONF(snapshot_dir, undefined) of
        undefined -> undefined;
        Dir -> iolist_to_binary(filename:join(Dir, ["emqx_trie_gpu.", atom_to_list(Index), ".snap"]))
    end.

load_snapshot(Index, H) ->
    case snapshot_path(Index) of
        undefined ->
            ok;
        Path ->
            case filelib:is_regular(Path) andalso emqx_trie_gpu_nif:snapshot_load(H, Path) of
                ok -> ok;
                false -> ok;
                %% a snapshot of another configuration: the resync's full build instead
                {error, _} -> ok
            end
    end.

terminate(_Reason, #{index := Index, h := H}) when H =/= undefined ->
    case snapshot_path(Index) of
        undefined -> ok;
        Path -> _ = emqx_trie_gpu_nif:snapshot_save(H, Path), ok
    end;
terminate(_Reason, _S) ->
    ok.

%% the engines' knobs; for the route index the handle registry (node(), the dest and subscriber
%% handles made so far) -- from here on every new handle is registered as it is made
prepare(Index, H) ->
    Delta =
        case ?CONF(delta_commit, small) of
            never -> 0;
            small -> 1;
            always -> 2
        end,
    ok = emqx_trie_gpu_nif:tune(H, delta_commit, Delta),
    case Index of
        session ->
            ok;
        route ->
            Tab = emqx_trie_gpu:handles_table(),
            _ = ets:info(Tab, name) =:= undefined andalso
                ets:new(Tab, [named_table, public, set, {read_concurrency, true}]),
            %% a restarted mirror's handles table died with the old process: every number the
            %% engines' registry still holds goes back (reused once the windows in flight are
            %% answered; the resync rewrites every list with the new numbers)
            ok = emqx_trie_gpu_nif:reset_handles(H),
            ok = emqx_trie_gpu:publish(registry, H),
            {NodeH, none} = hd(emqx_trie_gpu:dest_handles([node()])),
            lists:foreach(
                fun(Kind) ->
                    Hs = ets:select(Tab, [{{{Kind, '$1'}, '$2'}, [], [{{'$2', '$1'}}]}]),
                    ok = emqx_trie_gpu_nif:register(H, Kind, Hs)
                end,
                [node, group, sub]
            ),
            emqx_trie_gpu_nif:set_local_node(H, NodeH)
    end.

handle_call(_Req, _From, S) ->
    {reply, ignored, S}.

handle_cast(resync, S = #{h := H}) when H =/= undefined ->
    {noreply, repair_now(S)};
handle_cast(_Msg, S) ->
    {noreply, S}.

%% simple table events: the record's first field is the topic, whatever its tag.  Every event
%% queued now joins one batch.
handle_info({mnesia_table_event, _} = E, S) ->
    Topics = collect([event_topic(E)], ?BATCH),
    {noreply, sync(Topics, S)};
handle_info(resync, S) ->
    S1 = repair_now(S),
    schedule_resync(),
    {noreply, S1};
handle_info(repair, S) ->
    {noreply, repair_now(S#{retry := undefined})};
handle_info(sample_load, S = #{load := L}) ->
    L1 = emqx_trie_gpu:sample_load(L, ?CONF(adaptive_below_rate, 0)),
    erlang:send_after(?SAMPLE_MS, self(), sample_load),
    {noreply, S#{load := L1}};
handle_info(_Info, S) ->
    {noreply, S}.

event_topic({mnesia_table_event, {write, Route, _}}) -> element(2, Route);
event_topic({mnesia_table_event, {delete_object, Route, _}}) -> element(2, Route);
event_topic({mnesia_table_event, {delete, {_Tab, Topic}, _}}) -> Topic.

collect(Acc, 0) ->
    lists:usort(Acc);
collect(Acc, N) ->
    receive
        {mnesia_table_event, _} = E -> collect([event_topic(E) | Acc], N - 1)
    after 0 -> lists:usort(Acc)
    end.

%% the topics' state := the table's now, committed before the call returns
sync(Topics, S = #{index := route, h := H, tab := Tab}) ->
    check(emqx_trie_gpu_nif:route_dests(H, emqx_trie_gpu:route_items(Tab, Topics), true), S);
sync(Topics, S = #{index := session, h := H, tab := Tab}) ->
    check(emqx_trie_gpu_nif:route_sync(H, [{T, ets:member(Tab, T)} || T <- Topics]), S).

check({ok, _Epoch}, S) ->
    S;
check({error, _}, S) ->
    %% the engine refused (it is stale now and answers no publisher): a full resync and a commit
    %% retry every key
    repair_now(S).

%% every topic of the table (and for the route index every local subscriber list), in chunks of
%% ?CHUNK distinct topics per dirty NIF call; then every route key the scan did not see goes.
%% A bag's rows of one key come together in the scan: the key is read once, with all its rows.
%% ok | {error, Reason}: the first refused step ends it (the caller retries the whole resync)
resync(#{index := Index, h := H, tab := Tab}) ->
    try
        {ok, Gen} = emqx_trie_gpu_nif:sync_begin(H),
        Flush = fun(Topics) -> ok = flush(Index, H, Tab, Topics) end,
        {_, Last, _} = ets:foldl(
            fun(Row, {Prev, Acc, N}) ->
                case element(2, Row) of
                    Prev ->
                        {Prev, Acc, N};
                    T when N + 1 >= ?CHUNK ->
                        Flush([T | Acc]),
                        {T, [], 0};
                    T ->
                        {T, [T | Acc], N + 1}
                end
            end,
            {undefined, [], 0},
            Tab
        ),
        Flush(Last),
        %% the subscriber lists before sync_end: it clears every list the resync did not give
        %% (a topic whose subscribers all left is not in the table any more)
        ok =
            case Index of
                route -> resync_subscribers(H);
                session -> ok
            end,
        {ok, _Removed} = emqx_trie_gpu_nif:sync_end(H, Gen),
        ok
    catch
        error:{badmatch, {error, Reason}} -> {error, Reason}
    end.

flush(_Index, _H, _Tab, []) ->
    ok;
flush(route, H, Tab, Topics) ->
    case emqx_trie_gpu_nif:route_dests(H, emqx_trie_gpu:route_items(Tab, Topics), false) of
        {ok, _} -> ok;
        E -> E
    end;
flush(session, H, _Tab, Topics) ->
    emqx_trie_gpu_nif:route_set_many(H, Topics, true).

%% the local subscriber bag: every topic's list (its shard rows expanded)
resync_subscribers(H) ->
    Topics = lists:usort([T || {T, _} <- ets:tab2list(emqx_subscriber), is_binary(T)]),
    lists:foreach(
        fun(Chunk) ->
            {ok, _} = emqx_trie_gpu_nif:subscribers(H, emqx_trie_gpu:subscriber_items(Chunk), false)
        end,
        chunks(Topics, ?CHUNK)
    ).

chunks([], _N) -> [];
chunks(L, N) when length(L) =< N -> [L];
chunks(L, N) ->
    {A, B} = lists:split(N, L),
    [A | chunks(B, N)].

%% periodic resyncs only where table events may be missed (a replicant), unless configured
schedule_resync() ->
    Default =
        case mria_rlog:role() of
            replicant -> 30000;
            core -> 0
        end,
    case ?CONF(resync_interval_ms, Default) of
        0 -> ok;
        Ms -> _ = erlang:send_after(Ms, self(), resync), ok
    end.
