%%--------------------------------------------------------------------
%% emqx_trie_gpu_batcher -- the one process that batches the publish-time trie matches of all
%% publishers into device windows (SURVEY 8b "NIF shim": a per-node batcher in front of
%% emqx_trie:match/1, apps/emqx/src/emqx_trie.erl:147-169).
%%
%% Each {match, Topic} call joins the open window of the NIF batcher core
%% (emqxgm_batcher_add, include/emqx_gpumatch.h); the window is submitted when it is full or when
%% the mailbox runs empty (so an idle broker answers one publish at once and a busy one fills
%% windows), the oldest window is collected whenever EMQXGM_HOST_PIPES are in flight, and every
%% caller of a collected window is replied to with its filter list.  A topic longer than a
%% window, or a window the device fails, is answered by the reference's own emqx_trie:match/1:
%% the mnesia/ETS trie stays intact and authoritative (INTEGRATION.md 4).
%%--------------------------------------------------------------------
-module(emqx_trie_gpu_batcher).

-behaviour(gen_server).

-export([start_link/1, match/1, match/2]).

-export([init/1, handle_call/3, handle_cast/2, handle_info/2, terminate/2]).

%% EMQXGM_HOST_PIPES (include/emqx_gpumatch.h): windows in flight
-define(PIPES, 3).

start_link(Handle) ->
    gen_server:start_link({local, ?MODULE}, ?MODULE, Handle, []).

-spec match(emqx_types:topic()) -> [emqx_types:topic()].
match(Topic) ->
    match(Topic, 5000).

match(Topic, Timeout) ->
    gen_server:call(?MODULE, {match, Topic}, Timeout).

init(Handle) ->
    {ok, #{
        h => Handle,
        tag => 0,
        %% Tag => {From, Topic} of every caller not yet answered
        waiting => #{},
        %% windows in flight, oldest first: {WindowId, FirstTag, LastTag}
        inflight => queue:new(),
        %% first tag of the open window
        open_first => 0
    }}.

handle_call({match, Topic}, From, S = #{h := H, tag := Tag, waiting := W}) ->
    S1 = S#{tag := Tag + 1, waiting := W#{Tag => {From, Topic}}},
    case emqx_trie_gpu_nif:add(H, Topic, Tag) of
        ok ->
            {noreply, S1, 0};
        full ->
            {noreply, flush(S1#{tag := Tag + 1}), 0};
        {error, enospc} ->
            %% the open window cannot take it: submit that window, the topic opens the next
            S2 = flush(S1#{tag := Tag}),
            case emqx_trie_gpu_nif:add(H, Topic, Tag) of
                ok -> {noreply, S2#{tag := Tag + 1}, 0};
                full -> {noreply, flush(S2#{tag := Tag + 1}), 0}
            end;
        {error, _} ->
            {reply, emqx_trie:match(Topic), S#{tag := Tag + 1}, 0}
    end;
handle_call(_Req, _From, S) ->
    {reply, ignored, S, 0}.

handle_cast(_Msg, S) ->
    {noreply, S, 0}.

%% the mailbox is empty: submit the open window and complete every window in flight
handle_info(timeout, S) ->
    {noreply, drain(flush(S))};
handle_info(_Info, S) ->
    {noreply, S, 0}.

terminate(_Reason, S) ->
    _ = drain(S),
    ok.

%% submit the open window (windows up to the tag counter), first making room for it
flush(S = #{h := H, tag := Tag, open_first := First}) ->
    S1 =
        case queue:len(maps:get(inflight, S)) >= ?PIPES of
            true -> collect_oldest(S);
            false -> S
        end,
    case emqx_trie_gpu_nif:flush(H) of
        {ok, Id} ->
            Q = maps:get(inflight, S1),
            S1#{inflight := queue:in({Id, First, Tag - 1}, Q), open_first := Tag};
        empty ->
            S1
    end.

collect_oldest(S = #{h := H, inflight := Q, waiting := W}) ->
    {{value, {Id, First, Last}}, Q1} = queue:out(Q),
    W1 =
        case emqx_trie_gpu_nif:collect(H, Id) of
            {ok, Rows} ->
                lists:foldl(
                    fun({Tag, Filters, _ExactHit}, Acc) ->
                        {{From, _Topic}, Acc1} = maps:take(Tag, Acc),
                        gen_server:reply(From, Filters),
                        Acc1
                    end,
                    W,
                    Rows
                );
            {error, _Reason} ->
                %% the device failed this window: the reference's own match for its callers
                lists:foldl(
                    fun(Tag, Acc) ->
                        case maps:take(Tag, Acc) of
                            {{From, Topic}, Acc1} ->
                                gen_server:reply(From, emqx_trie:match(Topic)),
                                Acc1;
                            error ->
                                Acc
                        end
                    end,
                    W,
                    lists:seq(First, Last)
                )
        end,
    S#{inflight := Q1, waiting := W1}.

drain(S = #{inflight := Q}) ->
    case queue:is_empty(Q) of
        true -> S;
        false -> drain(collect_oldest(S))
    end.
