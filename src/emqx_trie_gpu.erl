%%--------------------------------------------------------------------
%% emqx_trie_gpu -- emqx_trie:match/1, match_session/1, emqx_router:match_routes/1 and the
%% routing of emqx_broker:publish/1 on the MI355X engine.
%%
%%   emqx_trie:match/1, match_session/1        apps/emqx/src/emqx_trie.erl:147-169
%%   emqx_trie:empty/0, empty_session/0                                  :172-178
%%   emqx_router:match_trie/1, match_routes/1  apps/emqx/src/emqx_router.erl:141-157
%%   emqx_broker:publish/1's route(aggre(match_routes(Topic)), Delivery)
%%                                             apps/emqx/src/emqx_broker.erl:231, 262-355, 546-579
%%
%% Every publisher process calls in itself, concurrently, as it calls emqx_router:match_routes/1
%% in the reference (emqx_broker.erl:218-232): match_async/3 or publish_async/3 hands the topic to
%% the engine's open window on the caller's own scheduler with a fresh reference, and the caller
%% waits for {emqx_trie_gpu, Ref, ...} (a receive on a new reference: OTP skips the mailbox), which
%% an engine completer thread sends once the window's device pass is done.  No process sits
%% between the publishers and the device.
%%
%% The tables (emqx_route, the local emqx_subscriber bag; the session router's route table when
%% persistent sessions are enabled) stay the source of truth.  Their committed state reaches the
%% device two ways: the writing node's own changes through the hooks below, called right after
%% the reference's write and committed before they return (so the node's next publish sees them,
%% as the reference's does: emqx_broker.erl:163-168, 484-486 -> emqx_router.erl:124-138), and every
%% node's changes through emqx_trie_gpu_sync's table events.  Both are level-triggered: they read
%% the table and set the device to it.  With enable = false, before the first sync, and whenever the
%% device cannot answer (a topic deeper than max_levels, every window busy, a device error, a
%% timeout) the call is the reference's own.
%%
%% Failing closed (r06, SURVEY 5 "Failure detection").  The reference's route write fails in its
%% caller (an aborted mria transaction, emqx_router_utils.erl:114-118); here the table already holds
%% the change when the device refuses it.  The engine then marks itself stale and refuses every call
%% ({error, estale}) until the mirror's repair (a full resync and a commit) -- so no publish is ever
%% answered from an index that lacks a committed change -- and the hooks still return ok.  A
%% publisher that times out cancels its call; fail_threshold such timeouts (or failed windows) in a
%% row mark the engines stale too, so a hung GPU costs the calls in flight one timeout_ms each and
%% every later call is refused at once.  Timeouts and failed windows ask the mirror to repair.  (The
%% persistent_term handle stays: erasing it would make OTP scan every process's heap; the engine's
%% refusal is one atomic load.)
%%--------------------------------------------------------------------
-module(emqx_trie_gpu).

-include_lib("emqx/include/emqx.hrl").
-include_lib("emqx/include/logger.hrl").

-export([child_specs/0, enabled/0, handle/1, publish/2]).
-export([match/1, match_session/1, match_trie/1, match_routes/1, empty/0, empty_session/0]).
-export([route/2]).
%% the writing node's hooks (INTEGRATION.md 4) and the mirror's helpers
-export([route_changed/1, session_route_changed/1, subscribers_changed/1, subscriber_down/1]).
-export([route_items/2, subscriber_items/1, dest_handles/1, handles_table/0]).
%% the load-adaptive choice (the mirror samples the rate)
-export([load_counter/0, sample_load/2]).

-define(KEY(Index), {?MODULE, Index}).
-define(CONF(K, D), emqx_config:get([broker, perf, gpu_match, K], D)).
-define(HANDLES, emqx_trie_gpu_handles).

%% the supervisor's children (a maintainer adds them to emqx_broker_sup, INTEGRATION.md 4): one
%% mirror per index; each opens its engines in handle_continue/2
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

%% called by emqx_trie_gpu_sync: registry -- the route index's engines take handle
%% registrations from now on; route | session -- the index's first full sync is committed and
%% publishers may use it (undefined: not any more, a restarted mirror resyncs first)
publish(Key, undefined) ->
    _ = persistent_term:erase(?KEY(Key)),
    ok;
publish(Key, H) ->
    persistent_term:put(?KEY(Key), H).

enabled() ->
    device(route) =/= undefined.

device(Index) ->
    case ?CONF(enable, false) of
        true -> handle(Index);
        false -> undefined
    end.

%%--------------------------------------------------------------------
%% Match
%%--------------------------------------------------------------------

%% emqx_trie:match/1: the wildcard filters of the trie matching Topic (a set; [] for a wildcard
%% topic name, emqx_trie.erl:157-166 -- the device applies that rule itself)
-spec match(emqx_types:topic()) -> [emqx_types:topic()].
match(Topic) when is_binary(Topic) ->
    element(1, match(route, Topic)).

%% emqx_trie:match_session/1 (emqx_session_router:match_trie/1, emqx_session_router.erl:154-159)
-spec match_session(emqx_types:topic()) -> [emqx_types:topic()].
match_session(Topic) when is_binary(Topic) ->
    element(1, match(session, Topic)).

%% {Filters, Exact}: Exact = whether Topic itself is a committed route key (false: no route of
%% the topic's own name exists in the epoch that answered; unknown: the reference answered)
match(Index, Topic) ->
    case device(Index) of
        undefined -> {ref_match(Index, Topic), unknown};
        H ->
            case low_load() of
                true -> {ref_match(Index, Topic), unknown};
                false -> device_match(Index, H, Topic)
            end
    end.

ref_match(route, Topic) -> emqx_trie:match(Topic);
ref_match(session, Topic) -> emqx_trie:match_session(Topic).

device_match(Index, H, Topic) ->
    Ref = make_ref(),
    case emqx_trie_gpu_nif:match_async(H, Topic, Ref) of
        {ok, Call} ->
            receive
                {emqx_trie_gpu, Ref, Filters, Exact} -> {Filters, Exact};
                {emqx_trie_gpu, Ref, {error, E}} -> failed(Index, E), {ref_match(Index, Topic), unknown}
            after ?CONF(timeout_ms, 500) ->
                case emqx_trie_gpu_nif:cancel(H, Call) of
                    true ->
                        failed(Index, timeout),
                        {ref_match(Index, Topic), unknown};
                    false ->
                        %% answered while we gave up: the answer is in the mailbox already
                        receive
                            {emqx_trie_gpu, Ref, Filters, Exact} -> {Filters, Exact};
                            {emqx_trie_gpu, Ref, _} -> {ref_match(Index, Topic), unknown}
                        after 0 -> {ref_match(Index, Topic), unknown}
                        end
                end
            end;
        {error, _} ->
            %% deeper than max_levels, longer than a topic can be, every window busy, the index
            %% stale (estale: a repair is under way), or shutting down: the reference's own path
            {ref_match(Index, Topic), unknown}
    end.

%% a window that failed or a call that timed out: the mirror repairs the index (a cast it dedups;
%% a stale engine's refusals, estale, need none -- whoever marked it asked already)
failed(_Index, estale) -> ok;
failed(Index, _) -> emqx_trie_gpu_sync:repair(Index).

%% emqx_router:match_trie/1
match_trie(Topic) ->
    case empty() of
        true -> [];
        false -> match(Topic)
    end.

%% emqx_router:match_routes/1: the routes of the topic itself (even a wildcard string), then
%% those of every matched filter.  The device says whether the topic is a route key: when it is
%% not, its own lookup is skipped (an empty bag lookup in the reference).
-spec match_routes(emqx_types:topic()) -> [emqx_types:route()].
match_routes(Topic) when is_binary(Topic) ->
    case match(route, Topic) of
        {[], false} -> [];
        {[], _} -> emqx_router:lookup_routes(Topic);
        {Matched, false} -> lists:append([emqx_router:lookup_routes(To) || To <- Matched]);
        {Matched, _} -> lists:append([emqx_router:lookup_routes(To) || To <- [Topic | Matched]])
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

%%--------------------------------------------------------------------
%% Load-adaptive choice (r06, VERDICT r05 item 4).  At idle a publish answered by the device
%% waits for its window's timer and one pass (the bench's nif_concurrent idle p50: ~94 us at
%% cfg3), while the reference's trie walk on the publisher's own core takes ~22 us (the CPU
%% baseline: 0.71 M topics/s on 16 cores).  Below broker.perf.gpu_match.adaptive_below_rate
%% publishes per second the reference path answers (it costs less than a core there); above it,
%% the device (the reference's cost grows with the rate, the device's does not).  Every publish
%% counts itself (one atomics add); the mirror samples the count every ?SAMPLE_MS and sets the
%% flag publishers read (one atomics get).  0 (the default) = always the device.
%%--------------------------------------------------------------------

-define(LOAD, {?MODULE, load}).  %% atomics: 1 = publishes so far, 2 = 1 when under the rate

load_counter() ->
    case persistent_term:get(?LOAD, undefined) of
        undefined ->
            A = atomics:new(2, [{signed, false}]),
            persistent_term:put(?LOAD, A),
            A;
        A ->
            A
    end.

low_load() ->
    case persistent_term:get(?LOAD, undefined) of
        undefined ->
            false;
        A ->
            atomics:add(A, 1, 1),
            atomics:get(A, 2) =:= 1
    end.

%% the mirror's sample: Prev = {Count, Ms} of the last one; returns the new {Count, Ms}
sample_load(undefined, Threshold) ->
    sample_load({atomics:get(load_counter(), 1), erlang:monotonic_time(millisecond)}, Threshold);
sample_load({C0, T0}, Threshold) ->
    A = load_counter(),
    C1 = atomics:get(A, 1),
    T1 = erlang:monotonic_time(millisecond),
    Rate = (C1 - C0) * 1000 div max(1, T1 - T0),
    atomics:put(A, 2, case Threshold > 0 andalso Rate < Threshold of true -> 1; false -> 0 end),
    {C1, T1}.

%%--------------------------------------------------------------------
%% Publish: route(aggre(match_routes(Topic)), Delivery) with the device's fan-out
%%--------------------------------------------------------------------

%% emqx_broker:publish/1 calls this instead of route(aggre(emqx_router:match_routes(Topic)),
%% Delivery) (emqx_broker.erl:231).  The aggre/1 entries (:284-300) and, for each {To, node()}
%% entry, the local subscribers of To (subscribers/1, :546-552) come from the device in one
%% answer: no ets:lookup per matched filter, no subscriber bag lookup.  The rest is route/2's
%% (:262-282): local dispatch, forward to other nodes, shared-group dispatch.
-spec route(emqx_types:topic(), emqx_types:delivery()) -> emqx_types:publish_result().
route(Topic, Delivery = #delivery{message = Msg}) ->
    {Entries, Local} =
        case publish_match(Topic) of
            {ok, Es, Subs} -> {Es, {subs, Subs}};
            reference -> {aggre(emqx_router:match_routes(Topic)), broker}
        end,
    case Entries of
        [] ->
            ok = emqx_hooks:run('message.dropped', [Msg, #{node => node()}, no_subscribers]),
            ok = inc_dropped_cnt(Msg),
            [];
        _ ->
            lists:foldl(fun(E, Acc) -> [do_route(E, Local, Delivery) | Acc] end, [], Entries)
    end.

publish_match(Topic) ->
    case device(route) of
        undefined ->
            reference;
        H ->
            case low_load() of
                true -> reference;
                false -> publish_device(H, Topic)
            end
    end.

publish_device(H, Topic) ->
    Ref = make_ref(),
    case emqx_trie_gpu_nif:publish_async(H, Topic, Ref) of
        {ok, Call} ->
            receive
                {emqx_trie_gpu, Ref, {routes, Es, Subs}} -> {ok, Es, Subs};
                {emqx_trie_gpu, Ref, {error, E}} -> failed(route, E), reference
            after ?CONF(timeout_ms, 500) ->
                case emqx_trie_gpu_nif:cancel(H, Call) of
                    true ->
                        failed(route, timeout),
                        reference;
                    false ->
                        receive
                            {emqx_trie_gpu, Ref, {routes, Es, Subs}} -> {ok, Es, Subs};
                            {emqx_trie_gpu, Ref, _} -> reference
                        after 0 -> reference
                        end
                end
            end;
        {error, _} ->
            reference
    end.

%% emqx_broker:do_route/2 (emqx_broker.erl:270-275)
do_route({To, Node}, Local, Delivery) when Node =:= node() ->
    {Node, To, dispatch(To, Local, Delivery)};
do_route({To, Node}, _Local, Delivery) when is_atom(Node) ->
    {Node, To, forward(Node, To, Delivery, emqx:get_config([rpc, mode]))};
do_route({To, Group}, _Local, Delivery) when is_tuple(Group); is_binary(Group) ->
    {share, To, emqx_shared_sub:dispatch(Group, To, Delivery)}.

%% emqx_broker:aggre/1 (emqx_broker.erl:284-300), for the reference's path
aggre([]) ->
    [];
aggre([#route{topic = To, dest = Node}]) when is_atom(Node) ->
    [{To, Node}];
aggre([#route{topic = To, dest = {Group, _Node}}]) ->
    [{To, Group}];
aggre(Routes) ->
    lists:foldl(
        fun
            (#route{topic = To, dest = Node}, Acc) when is_atom(Node) ->
                [{To, Node} | Acc];
            (#route{topic = To, dest = {Group, _Node}}, Acc) ->
                lists:usort([{To, Group} | Acc])
        end,
        [],
        Routes
    ).

%% emqx_broker:forward/4 (emqx_broker.erl:302-324)
forward(Node, To, Delivery, async) ->
    true = emqx_broker_proto_v1:forward_async(Node, To, Delivery),
    emqx_metrics:inc('messages.forward');
forward(Node, To, Delivery, sync) ->
    case emqx_broker_proto_v1:forward(Node, To, Delivery) of
        {Err, Reason} when Err =:= badrpc; Err =:= badtcp ->
            ?SLOG(
                error,
                #{
                    msg => "sync_forward_msg_to_node_failed",
                    node => Node,
                    Err => Reason
                },
                #{topic => To}
            ),
            {error, badrpc};
        Result ->
            emqx_metrics:inc('messages.forward'),
            Result
    end.

%% emqx_broker:dispatch/2 + do_dispatch/2,3 (emqx_broker.erl:326-340, 546-579) over the device's
%% subscribers of To (shard rows flattened by the mirror)
dispatch(To, broker, Delivery) ->
    emqx_broker:dispatch(To, Delivery);
dispatch(To, {subs, Subs}, #delivery{message = Msg}) ->
    case emqx:is_running() of
        false ->
            {error, not_running};
        true ->
            N = lists:foldl(
                fun
                    ({T, Pid}, Acc) when T =:= To, is_pid(Pid) -> Acc + send(Pid, To, Msg);
                    (_, Acc) -> Acc
                end,
                0,
                Subs
            ),
            case N of
                0 ->
                    ok = emqx_hooks:run('message.dropped', [Msg, #{node => node()}, no_subscribers]),
                    ok = inc_dropped_cnt(Msg),
                    {error, no_subscribers};
                _ ->
                    {ok, N}
            end
    end.

send(SubPid, Topic, Msg) ->
    case erlang:is_process_alive(SubPid) of
        true ->
            SubPid ! {deliver, Topic, Msg},
            1;
        false ->
            0
    end.

inc_dropped_cnt(Msg) ->
    case emqx_message:is_sys(Msg) of
        true ->
            ok;
        false ->
            ok = emqx_metrics:inc('messages.dropped'),
            emqx_metrics:inc('messages.dropped.no_subscribers')
    end.

%%--------------------------------------------------------------------
%% The writing node's hooks: committed before they return
%%--------------------------------------------------------------------

%% after emqx_router:do_add_route/2 and do_delete_route/2 returned ok (emqx_router.erl:124-138,
%% 171-179: the post-maybe_trans hook of SURVEY 8b).  Topic's rows of emqx_route, read now, go to
%% the device and are committed before this returns: the node's next publish matches them.  Always
%% ok: an engine that refuses the commit marks itself stale and answers nothing until the mirror's
%% repair (publishers take the reference's path meanwhile).  When the delta does not fit the
%% current tables while a background full build runs, the commit waits for that build's install
%% (emqxgm_route_dests_batch, EMQXGM_SET_COMMIT; a dirty CPU scheduler is held meanwhile).
route_changed(Topic) ->
    case handle(route) of
        undefined -> ok;
        H -> sync_result(emqx_trie_gpu_nif:route_dests(H, route_items(emqx_route, [Topic]), true))
    end.

%% the same for the session router's table (emqx_session_router.erl:126-176)
session_route_changed(Topic) ->
    case handle(session) of
        undefined ->
            ok;
        H ->
            Tab = emqx_trie_gpu_sync:table(session),
            case emqx_trie_gpu_nif:route_sync(H, [{Topic, ets:member(Tab, Topic)}]) of
                {ok, _} -> ok;
                {error, _} -> emqx_trie_gpu_sync:repair(session)
            end
    end.

%% after emqx_broker's do_subscribe/4, do_unsubscribe/4 and subscriber_down/1 changed Topic's
%% rows of the emqx_subscriber bag (emqx_broker.erl:160-212, 361-380)
subscribers_changed(Topic) ->
    case handle(route) of
        undefined -> ok;
        H -> sync_result(emqx_trie_gpu_nif:subscribers(H, subscriber_items([Topic]), true))
    end.

%% a refused change: the engine is stale now (it refuses every publisher until the repair, so no
%% answer comes from an index without this change); the mirror repairs it.  The hook's caller
%% (the broker pool's subscribe) goes on as the reference's would.
sync_result({ok, _Epoch}) -> ok;
sync_result({error, _}) -> emqx_trie_gpu_sync:repair(route).

%%--------------------------------------------------------------------
%% Handles: the engine's 32-bit names of dests and subscribers
%%--------------------------------------------------------------------

handles_table() -> ?HANDLES.

%% [{Topic, [{NodeH, GroupH | none}]}] of Topics' rows of the route table Tab (dests() of
%% #route{}, emqx.hrl:97-100): a node, or a shared-subscription {Group, Node}
route_items(Tab, Topics) ->
    [{T, dest_handles([R#route.dest || R <- ets:lookup(Tab, T)])} || T <- Topics].

dest_handles(Dests) ->
    [dest_handle(D) || D <- Dests].

dest_handle({Group, Node}) -> {term_handle(node, Node), term_handle(group, Group)};
dest_handle(Node) -> {term_handle(node, Node), none}.

%% [{Topic, [SubH]}]: Topic's local subscribers, its {shard, I} rows expanded
%% (emqx_broker.erl:546-579)
subscriber_items(Topics) ->
    [{T, [term_handle(sub, P) || P <- subscribers(T)]} || T <- Topics].

subscribers(Topic) ->
    lists:flatmap(
        fun
            ({shard, I}) -> [P || {_, P} <- ets:lookup(emqx_subscriber, {shard, Topic, I})];
            (Pid) -> [Pid]
        end,
        [S || {_, S} <- ets:lookup(emqx_subscriber, Topic)]
    ).

%% the handle of Term: allocated by the NIF's handle registry (a released number once every
%% window submitted before its release was answered, else a new one) and registered on first use.
%% Only called once the route index's engines are open (emqx_trie_gpu_sync:prepare/2 publishes the
%% registry before it makes the first handle; the hooks run once the index is published).
term_handle(Kind, Term) ->
    case ets:lookup(?HANDLES, {Kind, Term}) of
        [{_, H}] ->
            H;
        [] ->
            N = new_handle(Kind),
            case ets:insert_new(?HANDLES, {{Kind, Term}, N}) of
                true ->
                    ok = register_term(Kind, N, Term),
                    N;
                false ->
                    %% another process made Term's handle first: N was never in a list
                    ok = release_number(Kind, N),
                    term_handle(Kind, Term)
            end
    end.

new_handle(Kind) ->
    {ok, N} = emqx_trie_gpu_nif:alloc_handle(persistent_term:get(?KEY(registry)), Kind),
    N.

release_number(Kind, N) ->
    case persistent_term:get(?KEY(registry), undefined) of
        undefined -> ok;
        H -> _ = emqx_trie_gpu_nif:release_handle(H, Kind, N), ok
    end.

%% after emqx_broker:subscriber_down/1 (emqx_broker.erl:361-380) removed SubPid's rows and the
%% subscribers_changed/1 hook of each of its topics committed the lists without it: SubPid's handle
%% goes back to the registry and its term copy is freed, so a broker whose clients reconnect (a new
%% pid per connection) keeps handle and term tables as large as its live subscribers
%% (emqx_broker_helper.erl:133-165 removes every trace of the pid likewise).
subscriber_down(SubPid) ->
    case ets:take(?HANDLES, {sub, SubPid}) of
        [{_, N}] -> release_number(sub, N);
        [] -> ok
    end.

%% (registered as soon as the route index's engines are open: emqx_trie_gpu_sync sweeps the
%% handles made before that into the NIF, then publishes the index)
register_term(Kind, N, Term) ->
    case persistent_term:get(?KEY(registry), undefined) of
        undefined -> ok;
        H -> emqx_trie_gpu_nif:register(H, Kind, [{N, Term}])
    end.
