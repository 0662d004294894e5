%%--------------------------------------------------------------------
%% emqx_gpu_batch — the batching process in front of emqx_gpu_match for the
%% publish path.
%%
%% The reference looks routes up one message at a time in the publisher's
%% process (emqx_broker:publish/1 -> emqx_router:match_routes/1,
%% apps/emqx/src/emqx_broker.erl:200-209).  A GPU batch pays off only for many
%% topics at once, so publishers call match_routes/1 here: the topic is pushed
%% into an emqx_batch (apps/emqx/src/emqx_batch.erl: commit on batch_size
%% items or linger_ms after the first), a commit submits the whole batch to the
%% GPU pipeline (emqx_gpu_match:submit/3 stages it in pinned memory and
%% returns a ticket at once), and one waiter process per ticket blocks in
%% emqx_gpu_match:wait/2 (dirty I/O scheduler) and answers the batch's callers.
%% Up to `depth` tickets are in flight, so batch k's copy back overlaps batch
%% k+1's match; further commits queue here.  Any NIF error is handed to the
%% callers, which fall back to emqx_router:match_routes/1: semantics never
%% change.
%%
%% Not compiled in this repository's CI (no ERTS in the build image).
%%--------------------------------------------------------------------
-module(emqx_gpu_batch).
-behaviour(gen_server).

-export([start_link/1, match_routes/1, match_routes/2]).
-export([init/1, handle_call/3, handle_cast/2, handle_info/2, terminate/2]).

-define(MODE_ROUTES, 1).

-record(st, {ctx, batch, depth, inflight = 0, queue = queue:new()}).

start_link(Opts) when is_map(Opts) ->
    gen_server:start_link({local, ?MODULE}, ?MODULE, Opts, []).

%% emqx_router:match_routes/1, batched on the GPU.
match_routes(Topic) -> match_routes(Topic, 5000).

match_routes(Topic, Timeout) when is_binary(Topic) ->
    case gen_server:call(?MODULE, {match, Topic}, Timeout) of
        {ok, Ids} ->
            lists:append([emqx_router:lookup_routes(emqx_gpu_match:filter_of(Id)) || Id <- Ids]);
        {error, _} ->
            emqx_router:match_routes(Topic)
    end.

init(Opts) ->
    process_flag(trap_exit, true),
    Server = self(),
    Batch = emqx_batch:init(#{batch_size => maps:get(batch_size, Opts, 65536),
                              linger_ms => maps:get(linger_ms, Opts, 1),
                              commit_fun => fun(Items) -> Server ! {commit, Items} end}),
    {ok, #st{ctx = emqx_gpu_match:ctx(), batch = Batch, depth = maps:get(depth, Opts, 2)}}.

handle_call({match, Topic}, From, St = #st{batch = B}) ->
    {noreply, St#st{batch = emqx_batch:push({From, Topic}, B)}};
handle_call(_Req, _From, St) ->
    {reply, ignored, St}.

handle_cast(_Msg, St) ->
    {noreply, St}.

handle_info(batch_linger_expired, St = #st{batch = B}) ->
    {noreply, St#st{batch = emqx_batch:commit(B)}};
handle_info({commit, Items}, St = #st{inflight = N, depth = D}) when N < D ->
    {noreply, submit(Items, St)};
handle_info({commit, Items}, St = #st{queue = Q}) ->
    {noreply, St#st{queue = queue:in(Items, Q)}};
handle_info({'EXIT', _Waiter, _Reason}, St = #st{inflight = N, queue = Q}) ->
    St1 = St#st{inflight = N - 1},
    case queue:out(Q) of
        {{value, Items}, Q1} -> {noreply, submit(Items, St1#st{queue = Q1})};
        {empty, _} -> {noreply, St1}
    end;
handle_info(_Info, St) ->
    {noreply, St}.

terminate(_Reason, _St) ->
    ok.

%% Submit one committed batch and start its waiter.
submit(Items, St = #st{ctx = Ctx, inflight = N}) ->
    Topics = [T || {_From, T} <- Items],
    case emqx_gpu_match:submit(Ctx, Topics, ?MODE_ROUTES) of
        {ok, Ticket} ->
            _ = spawn_link(fun() -> answer(Items, emqx_gpu_match:wait(Ctx, Ticket)) end),
            St#st{inflight = N + 1};
        {error, _} = Err ->
            answer(Items, Err),
            St
    end.

answer(Items, {ok, Rows}) ->
    lists:foreach(fun({{From, _}, Ids}) -> gen_server:reply(From, {ok, Ids}) end, lists:zip(Items, Rows));
answer(Items, Err) ->
    lists:foreach(fun({From, _}) -> gen_server:reply(From, Err) end, Items).
