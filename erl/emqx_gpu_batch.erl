%%--------------------------------------------------------------------
%% emqx_gpu_batch — the batching process in front of emqx_gpu_match for the
%% publish path.
%%
%% The reference looks routes up one message at a time in the publisher's
%% process (emqx_broker:publish/1 -> emqx_router:match_routes/1,
%% apps/emqx/src/emqx_broker.erl:200-209).  A GPU batch pays off only for many
%% topics at once, so publishers call match_routes/1 here: the topic joins the
%% pending batch (committed at batch_size topics or linger_ms after the first,
%% the policy of apps/emqx/src/emqx_batch.erl:50-81, with an item counter
%% instead of emqx_batch's length/1 per push), a commit submits the whole batch
%% to the GPU pipeline (emqx_gpu_match:submit/3 stages it in pinned memory and
%% returns a ticket at once), and one monitored waiter process per ticket blocks
%% in emqx_gpu_match:wait/2 (dirty I/O scheduler) and answers the batch's
%% callers.  Up to `depth` tickets are in flight, so batch k's copy back
%% overlaps batch k+1's match; further commits queue here.
%%
%% Result = emqx_router:match_routes/1 exactly (emqx_router.erl:129-134):
%% the GPU table mirrors emqx_trie (the wildcard filters that have routes,
%% kept by emqx_gpu_routes after each route transaction commits), the batch is
%% matched in TRIE mode (emqx_trie:match/1), and the caller expands
%% [Topic | Matched] with lookup_routes/1, so the topic's own exact routes are
%% included just as the reference includes them.
%%
%% Subscribe -> publish ordering: a wildcard route whose add started before
%% a caller's match_routes/1 call may not be in the table epoch yet.  Before
%% each submit the batch takes emqx_gpu_routes:overlay/0 (the filters whose
%% add started — emqx_gpu_routes:with_pending/2, run before the route
%% transaction — and that no published epoch holds yet); the waiter gives each
%% caller those F with emqx_topic:match(Topic, F), merged into Matched without
%% duplicates (the protocol: erl/emqx_gpu_routes.erl, steps 1-3).
%%
%% Semantics never change on failure: a NIF error, a dead or absent server, a
%% killed waiter or a timeout all end in emqx_router:match_routes/1.  Late
%% replies are dropped (gen_server:call uses a process alias, OTP >= 24).
%% A ticket is a NIF resource: if its waiter dies before wait/2, the resource's
%% destructor cancels it (egm_match_cancel) and the slot is reclaimed.
%%
%% Not compiled in this repository's CI (no ERTS in the build image);
%% emqx_amd/gpu_batch.py mirrors this logic and is tested, and
%% tests/test_erl_lint.py checks this module against the reference's erl_opts.
%%--------------------------------------------------------------------
-module(emqx_gpu_batch).
-behaviour(gen_server).

-export([start_link/1, match_routes/1, match_routes/2]).
-export([init/1, handle_call/3, handle_cast/2, handle_info/2, terminate/2]).

-define(MODE_TRIE, 0).

-record(st, {ctx,
             size,                    %% commit at this many topics
             linger,                  %% ... or this many ms after the first
             depth,                   %% tickets in flight
             items = [],              %% pending [{From, Topic}], newest first
             n = 0,                   %% length(items), kept instead of recounted
             timer,                   %% linger timer of the pending batch
             waiters = #{},           %% MonitorRef -> Items of that ticket
             queue = queue:new()}).   %% committed batches waiting for a ticket

start_link(Opts) when is_map(Opts) ->
    gen_server:start_link({local, ?MODULE}, ?MODULE, Opts, []).

%% emqx_router:match_routes/1, batched on the GPU.
match_routes(Topic) -> match_routes(Topic, 5000).

match_routes(Topic, Timeout) when is_binary(Topic) ->
    Res = try gen_server:call(?MODULE, {match, Topic}, Timeout)
          catch exit:_ -> {error, unavailable}   %% noproc, timeout, server down
          end,
    case Res of
        {ok, Ids, Extra} ->
            Matched0 = emqx_gpu_match:filters_of(Ids),
            Matched = Matched0 ++ [F || F <- Extra, not lists:member(F, Matched0)],
            lists:append([emqx_router:lookup_routes(To) || To <- [Topic | Matched]]);
        {error, _} ->
            emqx_router:match_routes(Topic)
    end.

init(Opts) ->
    {ok, #st{ctx = emqx_gpu_match:ctx(),
             size = maps:get(batch_size, Opts, 4096),
             linger = maps:get(linger_ms, Opts, 1),
             depth = maps:get(depth, Opts, 2)}}.

handle_call({match, Topic}, From, St = #st{items = Items, n = N, size = Size, linger = Ms}) ->
    St1 = St#st{items = [{From, Topic} | Items], n = N + 1},
    St2 = case N of
              0 -> St1#st{timer = erlang:send_after(Ms, self(), linger)};
              _ -> St1
          end,
    case N + 1 >= Size of
        true -> {noreply, commit(St2)};
        false -> {noreply, St2}
    end;
handle_call(_Req, _From, St) ->
    {reply, ignored, St}.

handle_cast(_Msg, St) ->
    {noreply, St}.

handle_info(linger, St = #st{n = 0}) ->
    {noreply, St#st{timer = undefined}};
handle_info(linger, St) ->
    {noreply, commit(St#st{timer = undefined})};
handle_info({'DOWN', Ref, process, _Pid, Reason}, St = #st{waiters = W}) ->
    case maps:take(Ref, W) of
        {Items, W1} ->
            %% a waiter answers before it exits normally; any other exit leaves
            %% its callers unanswered: they fall back to the reference
            Reason =:= normal orelse answer(Items, [], {error, {waiter_down, Reason}}),
            {noreply, next(St#st{waiters = W1})};
        error ->
            {noreply, St}
    end;
handle_info(_Info, St) ->
    {noreply, St}.

terminate(_Reason, _St) ->
    ok.

%% The pending batch is committed: submitted now, or queued behind `depth`
%% tickets in flight.
commit(St = #st{items = Items, timer = T, queue = Q}) ->
    _ = T =:= undefined orelse erlang:cancel_timer(T),
    next(St#st{items = [], n = 0, timer = undefined, queue = queue:in(lists:reverse(Items), Q)}).

next(St = #st{waiters = W, depth = D, queue = Q}) ->
    case map_size(W) < D andalso queue:out(Q) of
        {{value, Items}, Q1} -> next(submit(Items, St#st{queue = Q1}));
        _ -> St
    end.

%% Submit one committed batch and start its (monitored) waiter.  The overlay
%% is read before the submit (emqx_gpu_routes, step 2).
submit(Items, St) ->
    Topics = [T || {_From, T} <- Items],
    case emqx_gpu_routes:overlay() of
        {ok, Ov} -> submit(Items, Topics, Ov, St);
        unavailable ->   %% no route sync: the GPU table is not kept in step
            answer(Items, [], {error, no_route_sync}),
            St
    end.

submit(Items, Topics, Ov, St = #st{ctx = Ctx, waiters = W}) ->
    case emqx_gpu_match:submit(Ctx, Topics, ?MODE_TRIE) of
        {ok, Ticket} ->
            {_Pid, Ref} = spawn_monitor(fun() -> answer(Items, Ov, emqx_gpu_match:wait(Ctx, Ticket)) end),
            St#st{waiters = W#{Ref => Items}};
        {error, _} = Err ->
            answer(Items, [], Err),
            St
    end.

answer(Items, Ov, {ok, Rows}) ->
    lists:foreach(fun({{From, Topic}, Ids}) ->
                          Extra = case Ov =/= [] andalso not emqx_topic:wildcard(Topic) of
                                      true -> [F || F <- Ov, emqx_topic:match(Topic, F)];
                                      false -> []
                                  end,
                          gen_server:reply(From, {ok, Ids, Extra})
                  end, lists:zip(Items, Rows));
answer(Items, _Ov, Err) ->
    lists:foreach(fun({From, _}) -> gen_server:reply(From, Err) end, Items).
