%%--------------------------------------------------------------------
%% emqx_gpu_routes — keeps the GPU filter table equal to emqx_trie's content
%% (the wildcard filters that have at least one route) without touching the
%% route transactions, and gives the GPU publish path the reference's
%% subscribe -> publish ordering.
%%
%% Table sync.  The reference inserts a wildcard filter into emqx_trie with
%% its first route and deletes it with its last, inside the route's mnesia
%% transaction (apps/emqx/src/emqx_router.erl:114-125,164-170,230-248,
%% maybe_trans :252-269).  A GPU epoch commit has no place inside that
%% transaction (an aborted transaction would leave the filter in the GPU
%% table, and one commit per filter caps the subscribe rate).  Instead this
%% process subscribes to the table events of emqx_route, which mnesia delivers
%% after a commit on every node holding the table (remote routes arrive by
%% replication, the trie's own path), collects the wildcard topics the events
%% touch, and every linger_ms (or at batch_size topics) publishes them in ONE
%% apply_delta + commit: a touched topic is in the GPU table iff it has routes
%% at flush time (emqx_router:has_routes/1, :148-150) — the rule of
%% insert_trie_route / delete_trie_route, evaluated after the commit, so the
%% final state never depends on event interleaving.
%%
%% Simple table events carry the record tagged with the TABLE name
%% ({write, {emqx_route, Topic, Dest}, ActivityId}), not with its record name
%% `route` (emqx_router.erl:78-81 creates emqx_route with {record_name, route};
%% emqx_router_helper.erl:120 matches its own table's events the same way).
%%
%% Ordering (read-your-writes).  In the reference a PUBLISH issued after
%% emqx_broker:subscribe/3 returns sees the new route: the broker pool call
%% (emqx_broker.erl:153) runs emqx_router:do_add_route/1 (:438-440), whose
%% transaction puts the filter in emqx_trie.  Here the filter reaches the GPU
%% at the next flush, so a public ETS set bridges the gap:
%%   ?PENDING  {Topic, Ref, pending | done}
%% 1. with_pending/2 wraps the wildcard branch of emqx_router:do_add_route/2
%%    (the one line the integration adds there, INTEGRATION.md §2): it inserts
%%    {Topic, Ref, pending} BEFORE the route transaction, in the caller, so
%%    before subscribe returns; marks it done after a commit; deletes it after
%%    an abort or a crash.
%% 2. emqx_gpu_batch reads overlay/0 (every ?PENDING topic) BEFORE it submits
%%    a batch; the waiter adds to each topic's matches the overlay filters F
%%    with emqx_topic:match(Topic, F) (deduplicated), and lookup_routes/1 drops
%%    a filter whose route is not (or no longer) there.
%% 3. A flush deletes a topic's ?PENDING object (compare-and-delete of the
%%    object it read before has_routes/1) only AFTER the epoch that holds the
%%    topic is published; a `pending` entry whose route is not committed yet
%%    is kept (its commit's event flushes it later); a `done` entry without
%%    routes (deleted since) is dropped.
%% So for a filter whose add started before a publish call: at the batch's
%% submit it is either still in ?PENDING (added by step 2), or its entry was
%% removed after an epoch holding it was published — and the batch, submitted
%% later, is matched against that epoch or a newer one.
%%
%% Not compiled in this repository's CI (no ERTS in the build image);
%% emqx_amd/gpu_batch.py (Overlay, RouteSync) mirrors this logic and is tested.
%%--------------------------------------------------------------------
-module(emqx_gpu_routes).
-behaviour(gen_server).

%% The route table's name.  emqx_router defines it privately
%% (apps/emqx/src/emqx_router.erl:70), not in apps/emqx/include/emqx.hrl.
-define(ROUTE_TAB, emqx_route).

-export([start_link/1, flush/0, with_pending/2, overlay/0]).
-export([init/1, handle_call/3, handle_cast/2, handle_info/2, terminate/2]).

-define(PENDING, emqx_gpu_pending).

-record(st, {touched = #{}, n = 0, size, linger, timer}).

start_link(Opts) when is_map(Opts) ->
    gen_server:start_link({local, ?MODULE}, ?MODULE, Opts, []).

%% Publish the touched topics now (tests, shutdown).
flush() -> gen_server:call(?MODULE, flush, infinity).

%% Around the wildcard branch of emqx_router:do_add_route/2:
%%   true -> emqx_gpu_routes:with_pending(Topic, fun() -> maybe_trans(fun insert_trie_route/1, [Route]) end);
%% Runs in the caller (a broker pool worker inside subscribe's call).
with_pending(Topic, Trans) ->
    Ref = make_ref(),
    Pending = {Topic, Ref, pending},
    Tracked = try ets:insert(?PENDING, Pending)
              catch error:badarg -> false     %% the GPU path is not running
              end,
    try Trans() of
        ok when Tracked ->
            %% compare-and-set: only if no newer add replaced the entry and no flush took it
            _ = ets:select_replace(?PENDING, [{Pending, [], [{const, {Topic, Ref, done}}]}]),
            ok;
        Res ->
            _ = Tracked andalso ets:delete_object(?PENDING, Pending),
            Res
    catch
        C:E:St ->
            _ = Tracked andalso ets:delete_object(?PENDING, Pending),
            erlang:raise(C, E, St)
    end.

%% The wildcard filters whose add started but is not yet in a published
%% epoch (step 2; read before a submit).  `unavailable` when this process (the
%% table's owner) is down: the GPU table is then not kept in step either, and
%% callers fall back to the reference.
overlay() ->
    try {ok, ets:select(?PENDING, [{{'$1', '_', '_'}, [], ['$1']}])}
    catch error:badarg -> unavailable
    end.

init(Opts) ->
    _ = ets:new(?PENDING, [named_table, public, set, {read_concurrency, true}, {write_concurrency, true}]),
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

handle_info({mnesia_table_event, {write, {?ROUTE_TAB, T, _Dest}, _}}, St) -> {noreply, touch(T, St)};
handle_info({mnesia_table_event, {delete_object, {?ROUTE_TAB, T, _Dest}, _}}, St) -> {noreply, touch(T, St)};
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
    Touched = maps:keys(M),
    Snap = [{T, ets:lookup(?PENDING, T)} || T <- Touched],   %% before has_routes/1
    {Ins, Del} = lists:partition(fun emqx_router:has_routes/1, Touched),
    ok = emqx_gpu_match:sync(Ins, Del),   %% returns after the epoch holding Ins is published
    InsSet = maps:from_list([{T, true} || T <- Ins]),
    lists:foreach(
      fun({T, Objs}) ->
              case maps:is_key(T, InsSet) of
                  true -> [ets:delete_object(?PENDING, O) || O <- Objs];
                  false -> [ets:delete_object(?PENDING, O) || O = {_, _, done} <- Objs]
              end
      end, Snap),
    St#st{touched = #{}, n = 0, timer = undefined}.
