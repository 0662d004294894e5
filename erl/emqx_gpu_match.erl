%%--------------------------------------------------------------------
%% emqx_gpu_match — Erlang side of the MI355X route lookup (NIF wrapper).
%%
%% A drop-in behind emqx_router:match_routes/1 and emqx_trie:match/1
%% (EMQ X 5.0-alpha.3: apps/emqx/src/emqx_router.erl:129-141,
%% apps/emqx/src/emqx_trie.erl:100-114).  Filters are identified by dense
%% integer ids assigned here in insertion order; the id -> filter binary map
%% lives in an ETS set so match results translate back to the [binary()] the
%% reference returns.  Every NIF failure returns {error, _} and the callers
%% below fall back to the reference implementation, so semantics never change.
%%
%% Not compiled in this repository's CI (no ERTS in the build image); see
%% INTEGRATION.md for the build line.  emqx_gpu_batch is the batching process
%% that turns per-message publish calls into pipelined GPU batches;
%% emqx_gpu_routes keeps the table equal to emqx_trie after each route
%% transaction commits (never inside it).
%%--------------------------------------------------------------------
-module(emqx_gpu_match).

-export([open/1, build/2, apply_delta/3, match_batch/3, submit/3, wait/2, cancel/2, subs_build/2,
         subs_delta/3, publish_batch/2]).
-export([init/0, ctx/0, filter_of/1, filters_of/1, build/1, sync/2, match/1, match_routes/1]).

-on_load(load_nif/0).

-define(TAB, emqx_gpu_match_ids).        %% Id -> Filter and {filter, Filter} -> Id
-define(MODE_TRIE, 0).
-define(MODE_ROUTES, 1).

load_nif() ->
    Dir = case code:priv_dir(emqx) of
              {error, _} -> "priv";
              P -> P
          end,
    erlang:load_nif(filename:join(Dir, "emqx_gpu_match_nif"), 0).

%% NIF stubs (replaced on load)
open(_Device) -> erlang:nif_error(nif_not_loaded).
build(_Ctx, _Filters) -> erlang:nif_error(nif_not_loaded).
apply_delta(_Ctx, _Inserts, _Deletes) -> erlang:nif_error(nif_not_loaded).
match_batch(_Ctx, _Topics, _Mode) -> erlang:nif_error(nif_not_loaded).
submit(_Ctx, _Topics, _Mode) -> erlang:nif_error(nif_not_loaded).
wait(_Ctx, _Ticket) -> erlang:nif_error(nif_not_loaded).
cancel(_Ctx, _Ticket) -> erlang:nif_error(nif_not_loaded).
subs_build(_Ctx, _SubsByFilterId) -> erlang:nif_error(nif_not_loaded).
subs_delta(_Ctx, _Adds, _Dels) -> erlang:nif_error(nif_not_loaded).
publish_batch(_Ctx, _Topics) -> erlang:nif_error(nif_not_loaded).

%% ---------------------------------------------------------------------
%% emqx_trie-shaped API
%% ---------------------------------------------------------------------

init() ->
    _ = ets:new(?TAB, [named_table, public, set, {read_concurrency, true}]),
    {ok, Ctx} = open(0),
    persistent_term:put(?MODULE, Ctx),
    ets:insert(?TAB, {next_id, 0}),
    ok.

ctx() -> persistent_term:get(?MODULE).

%% Filter binary of a filter id (ids are assigned by build/1 and sync/2).
filter_of(Id) -> ets:lookup_element(?TAB, Id, 2).

%% Filter binaries of matched ids; an id deleted since its batch was matched
%% is skipped (its filter has no routes left; ids are never reused).
filters_of(Ids) -> [F || Id <- Ids, {_, F} <- ets:lookup(?TAB, Id)].

%% The whole table: the wildcard filters that have routes (emqx_trie's
%% content, emqx_trie.erl:82-87 applied to each).  Called by emqx_gpu_routes.
build(Filters) when is_list(Filters) ->
    ets:match_delete(?TAB, {'_', '_'}),
    ets:insert(?TAB, {next_id, length(Filters)}),
    {_, Rows} = lists:foldl(fun(F, {I, Acc}) -> {I + 1, [{I, F}, {{filter, F}, I} | Acc]} end,
                            {0, []}, Filters),
    ets:insert(?TAB, Rows),
    ok = build(ctx(), Filters).

%% One epoch for a batch of trie changes, applied after their route
%% transactions committed (emqx_gpu_routes): inserts are idempotent
%% (emqx_trie.erl:84-85), deletes of absent filters are no-ops (:93-95).
sync(Inserts, Deletes) ->
    New = [F || F <- Inserts, ets:lookup(?TAB, {filter, F}) =:= []],
    Gone = [{F, Id} || F <- Deletes, {_, Id} <- ets:lookup(?TAB, {filter, F})],
    case New =:= [] andalso Gone =:= [] of
        true -> ok;
        false ->
            Ins = [{F, ets:update_counter(?TAB, next_id, 1) - 1} || F <- New],
            ets:insert(?TAB, lists:append([[{Id, F}, {{filter, F}, Id}] || {F, Id} <- Ins])),
            {ok, _Epoch} = apply_delta(ctx(), Ins, [F || {F, _} <- Gone]),
            %% ids leave the map only after the epoch without them is published
            lists:foreach(fun({F, Id}) -> ets:delete(?TAB, Id), ets:delete(?TAB, {filter, F}) end, Gone),
            ok
    end.

%% emqx_trie:match/1 — one topic; production callers go through the batcher.
%% The overlay of filters not yet in a published epoch is read before the
%% match (erl/emqx_gpu_routes.erl, steps 1-3).
match(Topic) when is_binary(Topic) ->
    case with_overlay(fun() -> match_batch(ctx(), [Topic], ?MODE_TRIE) end) of
        {ok, [Ids], Ov} ->   %% a pending filter is in emqx_trie once its route committed
            merge_overlay(Topic, filters_of(Ids), [F || F <- Ov, emqx_router:has_routes(F)]);
        {error, _} -> emqx_trie:match(Topic)
    end.

%% emqx_router:match_routes/1 (emqx_router.erl:129-134) for one topic: the
%% topic's own routes, then the routes of every trie match.
match_routes(Topic) when is_binary(Topic) ->
    case with_overlay(fun() -> match_batch(ctx(), [Topic], ?MODE_TRIE) end) of
        {ok, [Ids], Ov} ->
            Matched = merge_overlay(Topic, filters_of(Ids), Ov),
            lists:append([emqx_router:lookup_routes(To) || To <- [Topic | Matched]]);
        {error, _} -> emqx_router:match_routes(Topic)
    end.

%% The overlay is read before the match (emqx_gpu_routes, step 2).
with_overlay(Match) ->
    case emqx_gpu_routes:overlay() of
        {ok, Ov} ->
            case Match() of
                {ok, Rows} -> {ok, Rows, Ov};
                {error, _} = E -> E
            end;
        unavailable -> {error, no_route_sync}
    end.

merge_overlay(Topic, Matched, Ov) ->
    case emqx_topic:wildcard(Topic) of
        true -> Matched;   %% match_trie/1 of a wildcard topic is [] (emqx_trie.erl:102-111)
        false -> Matched ++ [F || F <- Ov, emqx_topic:match(Topic, F), not lists:member(F, Matched)]
    end.
