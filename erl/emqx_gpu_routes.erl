%%--------------------------------------------------------------------
%% emqx_gpu_routes — keeps the GPU filter table equal to emqx_trie's content
%% (the wildcard filters that have at least one route) without touching the
%% route transactions.
%%
%% The reference inserts a wildcard filter into emqx_trie with its first route
%% and deletes it with its last, inside the route's mnesia transaction
%% (apps/emqx/src/emqx_router.erl:114-125,164-170,230-248, maybe_trans
%% :252-269).  A GPU epoch commit has no place inside that transaction (an
%% aborted transaction would leave the filter in the GPU table, and one commit
%% per filter caps the subscribe rate).  Instead this process subscribes to
%% the table events of emqx_route, which mnesia delivers after a commit on
%% every node holding the table (remote routes arrive by replication, the
%% trie's own path), collects the wildcard topics the events touch, and every
%% linger_ms (or at batch_size topics) publishes them in ONE apply_delta +
%% commit: a touched topic is in the GPU table iff it has routes at flush time
%% (emqx_router:has_routes/1, :148-150) — the same rule as insert_trie_route /
%% delete_trie_route, evaluated after the commit, so the final state never
%% depends on event interleaving.  Route changes of one topic are serialised
%% by the router pool (pick/1, :186-187), and in-flight GPU batches keep the
%% epoch they started with.
%%
%% Not compiled in this repository's CI (no ERTS in the build image);
%% emqx_amd/gpu_batch.py (RouteSync) mirrors this logic and is tested.
%%--------------------------------------------------------------------
-module(emqx_gpu_routes).
-behaviour(gen_server).

-include("emqx.hrl").   %% #route{} (apps/emqx/include/emqx.hrl:90-93)

-export([start_link/1, flush/0]).
-export([init/1, handle_call/3, handle_cast/2, handle_info/2, terminate/2]).

-record(st, {touched = #{}, n = 0, size, linger, timer}).

start_link(Opts) when is_map(Opts) ->
    gen_server:start_link({local, ?MODULE}, ?MODULE, Opts, []).

%% Publish the touched topics now (tests, shutdown).
flush() -> gen_server:call(?MODULE, flush, infinity).

init(Opts) ->
    {ok, _} = mnesia:subscribe({table, ?ROUTE_TAB, simple}),
    %% initial image: every wildcard filter with a route (emqx_trie's content)
    ok = emqx_gpu_match:build([T || T <- emqx_router:topics(), emqx_topic:wildcard(T)]),
    {ok, #st{size = maps:get(batch_size, Opts, 65536), linger = maps:get(linger_ms, Opts, 5)}}.

handle_call(flush, _From, St) ->
    {reply, ok, publish(St)};
handle_call(_Req, _From, St) ->
    {reply, ignored, St}.

handle_cast(_Msg, St) ->
    {noreply, St}.

handle_info({mnesia_table_event, {write, #route{topic = T}, _}}, St) -> {noreply, touch(T, St)};
handle_info({mnesia_table_event, {delete_object, #route{topic = T}, _}}, St) -> {noreply, touch(T, St)};
handle_info({mnesia_table_event, {delete, {?ROUTE_TAB, T}, _}}, St) -> {noreply, touch(T, St)};
handle_info(linger, St) ->
    {noreply, publish(St#st{timer = undefined})};
handle_info(_Info, St) ->
    {noreply, St}.

terminate(_Reason, St) ->
    _ = publish(St),
    ok.

touch(T, St = #st{touched = M, n = N, size = Size, linger = Ms, timer = Tm}) ->
    case emqx_topic:wildcard(T) andalso not maps:is_key(T, M) of
        false -> St;   %% exact filters never enter the trie (emqx_router.erl:120-124)
        true ->
            St1 = St#st{touched = M#{T => true}, n = N + 1,
                        timer = case Tm of undefined -> erlang:send_after(Ms, self(), linger); _ -> Tm end},
            case N + 1 >= Size of
                true -> publish(St1);
                false -> St1
            end
    end.

publish(St = #st{n = 0}) ->
    St;
publish(St = #st{touched = M, timer = Tm}) ->
    _ = Tm =:= undefined orelse erlang:cancel_timer(Tm),
    {Ins, Del} = lists:partition(fun emqx_router:has_routes/1, maps:keys(M)),
    ok = emqx_gpu_match:sync(Ins, Del),
    St#st{touched = #{}, n = 0, timer = undefined}.
