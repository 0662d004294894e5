/*
 * emqx_gpu_match_nif.c — Erlang NIF shim over libemqx_gpu_match.so.
 *
 * Binds the C-ABI in include/emqx_gpu_match.h to the Erlang module
 * erl/emqx_gpu_match.erl.  Written against the documented erl_nif API; it
 * compiles only where an ERTS include directory exists (there is none in the
 * build container: see INTEGRATION.md for the command line).
 *
 * Mapping to the reference (EMQ X 5.0-alpha.3):
 *   open/1          -> egm_open            (one context per node, device ordinal)
 *   build/2         -> egm_table_build     (bulk load of the route filters)
 *   apply_delta/3   -> egm_table_apply_delta + egm_table_commit
 *                      (emqx_trie:insert/1, delete/1 — apps/emqx/src/emqx_trie.erl:82-96)
 *   match_batch/3   -> egm_match_batch     (emqx_trie:match/1 and the filter set of
 *                      emqx_router:match_routes/1 — emqx_router.erl:129-141 — for a
 *                      list of publish topics; returns [[FilterId]])
 *   submit/3, wait/2 -> egm_match_submit / egm_match_wait (the batcher's pipeline:
 *                      submit returns a ticket at once, wait blocks for its rows).
 *                      The ticket is a resource: collected unwaited (its waiter
 *                      died), its destructor calls egm_match_cancel, so a dead
 *                      waiter never keeps a pipeline slot busy.
 *   cancel/2        -> egm_match_cancel
 *   subs_delta/3    -> egm_subs_apply_delta + egm_subs_commit (subscriber changes)
 *   subs_build/2    -> egm_subs_build      (filter id -> subscriber ids: the
 *                      emqx_subscriber bag flattened, emqx_broker.erl:116-162)
 *   publish_batch/2 -> egm_match_batch (routes mode) + egm_fanout_batch: the
 *                      match_routes/1 + dispatch/2 expansion of emqx_broker:publish/1
 *                      (emqx_broker.erl:200-209, 283-308) for a list of topics;
 *                      returns [{[FilterId], [{FilterId, Sub}]}]
 *
 * Threading: match_batch and apply_delta run on dirty CPU schedulers
 * (ERL_NIF_DIRTY_JOB_CPU_BOUND) — a batch takes well over 1 ms.  The library
 * serialises calls per context.  Inputs (Erlang binaries) are borrowed only
 * for the duration of the call: they are packed into one contiguous buffer
 * here and the library copies them to device memory before returning.
 * Errors: bad arguments -> enif_make_badarg (the reference's function_clause);
 * library / device failures -> {error, Reason} so the caller can fall back to
 * emqx_trie:match/1.
 */
#include <erl_nif.h>
#include <stdlib.h>
#include <string.h>

#include "../include/emqx_gpu_match.h"

typedef struct {
  egm_ctx* ctx;
} egm_res_t;

static ErlNifResourceType* EGM_RES;
static ErlNifResourceType* EGM_TICKET;

/* A submitted batch: keeps its context alive until it is waited or cancelled. */
typedef struct {
  egm_res_t* owner;   /* enif_keep_resource'd */
  uint64_t ticket;
  int live;           /* not yet waited or cancelled */
} egm_ticket_t;
static ERL_NIF_TERM ATOM_OK, ATOM_ERROR;

static void egm_res_dtor(ErlNifEnv* env, void* obj) {
  (void)env;
  egm_res_t* r = (egm_res_t*)obj;
  if (r->ctx) egm_close(r->ctx);
  r->ctx = NULL;
}

static void egm_ticket_dtor(ErlNifEnv* env, void* obj) {
  (void)env;
  egm_ticket_t* t = (egm_ticket_t*)obj;
  if (t->live && t->owner && t->owner->ctx) egm_match_cancel(t->owner->ctx, t->ticket);
  t->live = 0;
  if (t->owner) enif_release_resource(t->owner);
  t->owner = NULL;
}

static int load(ErlNifEnv* env, void** priv, ERL_NIF_TERM info) {
  (void)priv;
  (void)info;
  EGM_RES = enif_open_resource_type(env, NULL, "emqx_gpu_match_ctx", egm_res_dtor,
                                    ERL_NIF_RT_CREATE | ERL_NIF_RT_TAKEOVER, NULL);
  EGM_TICKET = enif_open_resource_type(env, NULL, "emqx_gpu_match_ticket", egm_ticket_dtor,
                                       ERL_NIF_RT_CREATE | ERL_NIF_RT_TAKEOVER, NULL);
  ATOM_OK = enif_make_atom(env, "ok");
  ATOM_ERROR = enif_make_atom(env, "error");
  return (EGM_RES && EGM_TICKET) ? 0 : -1;
}

static ERL_NIF_TERM error_tuple(ErlNifEnv* env, egm_ctx* ctx, int rc) {
  const char* msg = ctx ? egm_last_error(ctx) : "egm error";
  return enif_make_tuple2(env, ATOM_ERROR,
                          enif_make_tuple2(env, enif_make_int(env, rc), enif_make_string(env, msg, ERL_NIF_LATIN1)));
}

/* Pack a proper list of binaries into blob + offsets (caller frees). */
static int pack_list(ErlNifEnv* env, ERL_NIF_TERM list, uint8_t** blob, uint32_t** off, uint32_t* n) {
  unsigned len;
  if (!enif_get_list_length(env, list, &len)) return 0;
  uint32_t* o = (uint32_t*)malloc(((size_t)len + 1) * sizeof(uint32_t));
  if (!o) return 0;
  size_t total = 0;
  ERL_NIF_TERM head, tail = list;
  ErlNifBinary bin;
  o[0] = 0;
  for (unsigned i = 0; i < len; ++i) {
    if (!enif_get_list_cell(env, tail, &head, &tail) || !enif_inspect_binary(env, head, &bin) ||
        total + bin.size > 0xFFFFFFFFu) {
      free(o);
      return 0;
    }
    total += bin.size;
    o[i + 1] = (uint32_t)total;
  }
  uint8_t* b = (uint8_t*)malloc(total + 16);
  if (!b) {
    free(o);
    return 0;
  }
  tail = list;
  for (unsigned i = 0; i < len; ++i) {
    enif_get_list_cell(env, tail, &head, &tail);
    enif_inspect_binary(env, head, &bin);
    memcpy(b + o[i], bin.data, bin.size);
  }
  *blob = b;
  *off = o;
  *n = len;
  return 1;
}

static int get_ctx(ErlNifEnv* env, ERL_NIF_TERM t, egm_res_t** r) {
  return enif_get_resource(env, t, EGM_RES, (void**)r) && (*r)->ctx;
}

/* open(Device :: non_neg_integer()) -> {ok, Ctx} | {error, _} */
static ERL_NIF_TERM nif_open(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  int dev;
  if (argc != 1 || !enif_get_int(env, argv[0], &dev) || dev < 0) return enif_make_badarg(env);
  egm_config cfg = {dev, 1, 0, 1000};
  egm_ctx* ctx = NULL;
  int rc = egm_open(&cfg, &ctx);
  if (rc) return error_tuple(env, NULL, rc);
  egm_res_t* r = (egm_res_t*)enif_alloc_resource(EGM_RES, sizeof(egm_res_t));
  r->ctx = ctx;
  ERL_NIF_TERM term = enif_make_resource(env, r);
  enif_release_resource(r);
  return enif_make_tuple2(env, ATOM_OK, term);
}

/* build(Ctx, [Filter :: binary()]) -> ok | {error, _}   (ids = list positions) */
static ERL_NIF_TERM nif_build(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  egm_res_t* r;
  uint8_t* blob;
  uint32_t *off, n;
  if (argc != 2 || !get_ctx(env, argv[0], &r) || !pack_list(env, argv[1], &blob, &off, &n))
    return enif_make_badarg(env);
  int rc = egm_table_build(r->ctx, blob, off, n, NULL);
  free(blob);
  free(off);
  return rc ? error_tuple(env, r->ctx, rc) : ATOM_OK;
}

/* apply_delta(Ctx, [{Filter, Id}] inserts, [Filter] deletes) -> {ok, Epoch} | {error, _} */
static ERL_NIF_TERM nif_apply_delta(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  egm_res_t* r;
  if (argc != 3 || !get_ctx(env, argv[0], &r)) return enif_make_badarg(env);
  unsigned ni;
  if (!enif_get_list_length(env, argv[1], &ni)) return enif_make_badarg(env);
  ERL_NIF_TERM filters = enif_make_list(env, 0), head, tail = argv[1];
  uint32_t* ids = (uint32_t*)malloc(((size_t)ni + 1) * sizeof(uint32_t));
  for (unsigned i = 0; i < ni; ++i) {
    const ERL_NIF_TERM* tup;
    int arity;
    unsigned id;
    if (!enif_get_list_cell(env, tail, &head, &tail) || !enif_get_tuple(env, head, &arity, &tup) || arity != 2 ||
        !enif_get_uint(env, tup[1], &id)) {
      free(ids);
      return enif_make_badarg(env);
    }
    ids[i] = id;
    filters = enif_make_list_cell(env, tup[0], filters);
  }
  ERL_NIF_TERM rev;
  enif_make_reverse_list(env, filters, &rev);
  uint8_t *ib = NULL, *db = NULL;
  uint32_t *io = NULL, *dof = NULL, nin = 0, nd = 0;
  if (!pack_list(env, rev, &ib, &io, &nin) || !pack_list(env, argv[2], &db, &dof, &nd)) {
    free(ids);
    free(ib);
    free(io);
    return enif_make_badarg(env);
  }
  egm_delta ins = {ib, io, nin, ids}, del = {db, dof, nd, NULL};
  uint64_t epoch = 0;
  int rc = egm_table_apply_delta(r->ctx, &ins, &del);
  if (!rc) rc = egm_table_commit(r->ctx, &epoch);
  free(ids);
  free(ib);
  free(io);
  free(db);
  free(dof);
  if (rc) return error_tuple(env, r->ctx, rc);
  return enif_make_tuple2(env, ATOM_OK, enif_make_uint64(env, epoch));
}

/* Rows of a CSR as [[Id]] (shared by match_batch and wait); either result
   form — wait/2's batches are submitted packed (EGM_RESULT_PACKED). */
static ERL_NIF_TERM rows_term(ErlNifEnv* env, const egm_result* res) {
  ERL_NIF_TERM rows = enif_make_list(env, 0);
  for (uint32_t i = res->n_topics; i-- > 0;) {
    ERL_NIF_TERM row = enif_make_list(env, 0);
    for (uint64_t k = egm_result_row(res, i + 1); k-- > egm_result_row(res, i);)
      row = enif_make_list_cell(env, enif_make_uint(env, egm_result_id(res, k)), row);
    rows = enif_make_list_cell(env, row, rows);
  }
  return rows;
}

/* match_batch(Ctx, [Topic :: binary()], Mode :: 0 | 1) -> {ok, [[Id]]} | {error, _} */
static ERL_NIF_TERM nif_match_batch(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  egm_res_t* r;
  int mode;
  uint8_t* blob;
  uint32_t *off, n;
  if (argc != 3 || !get_ctx(env, argv[0], &r) || !enif_get_int(env, argv[2], &mode) ||
      (mode != EGM_MODE_TRIE && mode != EGM_MODE_ROUTES) || !pack_list(env, argv[1], &blob, &off, &n))
    return enif_make_badarg(env);
  egm_result* res = NULL;
  int rc = egm_match_batch(r->ctx, blob, off, n, mode, &res);
  free(blob);
  free(off);
  if (rc && !res) return error_tuple(env, r->ctx, rc);
  if (rc) {
    egm_result_free(res);
    return error_tuple(env, r->ctx, rc);
  }
  ERL_NIF_TERM rows = rows_term(env, res);
  egm_result_free(res);
  return enif_make_tuple2(env, ATOM_OK, rows);
}

/* submit(Ctx, [Topic], Mode) -> {ok, Ticket} | {error, _}: the topics are
   staged in pinned memory before it returns; Ticket is a resource. */
static ERL_NIF_TERM nif_submit(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  egm_res_t* r;
  int mode;
  uint8_t* blob;
  uint32_t *off, n;
  if (argc != 3 || !get_ctx(env, argv[0], &r) || !enif_get_int(env, argv[2], &mode) ||
      (mode != EGM_MODE_TRIE && mode != EGM_MODE_ROUTES) || !pack_list(env, argv[1], &blob, &off, &n))
    return enif_make_badarg(env);
  uint64_t ticket = 0;
  int rc = egm_match_submit(r->ctx, blob, off, n, mode | EGM_RESULT_PACKED, &ticket);
  free(blob);
  free(off);
  if (rc) return error_tuple(env, r->ctx, rc);
  egm_ticket_t* t = (egm_ticket_t*)enif_alloc_resource(EGM_TICKET, sizeof(egm_ticket_t));
  enif_keep_resource(r);
  t->owner = r;
  t->ticket = ticket;
  t->live = 1;
  ERL_NIF_TERM term = enif_make_resource(env, t);
  enif_release_resource(t);
  return enif_make_tuple2(env, ATOM_OK, term);
}

static int get_ticket(ErlNifEnv* env, ERL_NIF_TERM term, egm_res_t* r, egm_ticket_t** t) {
  return enif_get_resource(env, term, EGM_TICKET, (void**)t) && (*t)->live && (*t)->owner == r;
}

/* wait(Ctx, Ticket) -> {ok, [[Id]]} | {error, _} (a ticket is waited once) */
static ERL_NIF_TERM nif_wait(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  egm_res_t* r;
  egm_ticket_t* t;
  if (argc != 2 || !get_ctx(env, argv[0], &r) || !get_ticket(env, argv[1], r, &t)) return enif_make_badarg(env);
  t->live = 0;   /* from here the library owns the outcome: no cancel in the destructor */
  egm_result* res = NULL;
  int rc = egm_match_wait(r->ctx, t->ticket, &res);
  if (rc) {
    if (res) egm_result_free(res);
    return error_tuple(env, r->ctx, rc);
  }
  ERL_NIF_TERM rows = rows_term(env, res);
  egm_result_free(res);
  return enif_make_tuple2(env, ATOM_OK, rows);
}

/* cancel(Ctx, Ticket) -> ok | {error, _}: give the batch up without its rows.
   A normal (not dirty) NIF: egm_match_cancel never blocks — while a build or
   commit holds the context it queues the cancel — so this call and the ticket
   destructor (run on whatever scheduler collects the ticket) return at once.
   Always ok for a ticket of this context: egm_match_cancel answers EGM_OK for
   a queued (unvalidated) cancel and EGM_E_STATE for a stale ticket only when
   the context happened to be free, so that difference is lock contention,
   not a result (include/emqx_gpu_match.h). */
static ERL_NIF_TERM nif_cancel(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  egm_res_t* r;
  egm_ticket_t* t;
  if (argc != 2 || !get_ctx(env, argv[0], &r) || !get_ticket(env, argv[1], r, &t)) return enif_make_badarg(env);
  t->live = 0;
  int rc = egm_match_cancel(r->ctx, t->ticket);
  return (rc == EGM_OK || rc == EGM_E_STATE) ? ATOM_OK : error_tuple(env, r->ctx, rc);
}

/* subs_build(Ctx, [[Sub]]) -> ok | {error, _}: list position = filter id; a
   shared group is the integer GroupId bor 16#80000000. */
static ERL_NIF_TERM nif_subs_build(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  egm_res_t* r;
  unsigned nf;
  if (argc != 2 || !get_ctx(env, argv[0], &r) || !enif_get_list_length(env, argv[1], &nf))
    return enif_make_badarg(env);
  uint64_t* row = (uint64_t*)malloc(((size_t)nf + 1) * sizeof(uint64_t));
  if (!row) return enif_make_badarg(env);
  ERL_NIF_TERM head, tail = argv[1];
  row[0] = 0;
  for (unsigned i = 0; i < nf; ++i) {
    unsigned len;
    if (!enif_get_list_cell(env, tail, &head, &tail) || !enif_get_list_length(env, head, &len)) {
      free(row);
      return enif_make_badarg(env);
    }
    row[i + 1] = row[i] + len;
  }
  uint32_t* subs = (uint32_t*)malloc((size_t)(row[nf] ? row[nf] : 1) * sizeof(uint32_t));
  if (!subs) {
    free(row);
    return enif_make_badarg(env);
  }
  tail = argv[1];
  for (unsigned i = 0; i < nf; ++i) {
    ERL_NIF_TERM h2, t2;
    enif_get_list_cell(env, tail, &head, &tail);
    t2 = head;
    for (uint64_t k = row[i]; k < row[i + 1]; ++k) {
      unsigned v;
      if (!enif_get_list_cell(env, t2, &h2, &t2) || !enif_get_uint(env, h2, &v)) {
        free(row);
        free(subs);
        return enif_make_badarg(env);
      }
      subs[k] = v;
    }
  }
  int rc = egm_subs_build(r->ctx, row, nf, subs);
  free(row);
  free(subs);
  return rc ? error_tuple(env, r->ctx, rc) : ATOM_OK;
}

/* [{FilterId, Sub}] -> egm_sub_pair[] (malloc'd; *n pairs); 0 on a bad term */
static int get_pairs(ErlNifEnv* env, ERL_NIF_TERM list, egm_sub_pair** out, unsigned* n) {
  ERL_NIF_TERM head, tail = list;
  if (!enif_get_list_length(env, list, n)) return 0;
  *out = (egm_sub_pair*)malloc(sizeof(egm_sub_pair) * (*n ? *n : 1));
  if (!*out) return 0;
  for (unsigned i = 0; i < *n; ++i) {
    const ERL_NIF_TERM* el;
    int arity;
    unsigned f, sub;
    if (!enif_get_list_cell(env, tail, &head, &tail) || !enif_get_tuple(env, head, &arity, &el) || arity != 2 ||
        !enif_get_uint(env, el[0], &f) || !enif_get_uint(env, el[1], &sub)) {
      free(*out);
      *out = NULL;
      return 0;
    }
    (*out)[i].fid = f;
    (*out)[i].sub = sub;
  }
  return 1;
}

/* subs_delta(Ctx, Adds, Dels) -> {ok, Epoch} | {error, _}: the subscriber
   changes since the last call ({FilterId, Sub} pairs; a $share group as
   GroupId bor 16#80000000) in one epoch of the fan-out's table —
   emqx_broker:subscribe/3, unsubscribe/1 and subscriber_down/1
   (emqx_broker.erl:144-197, 331-345).  Adds and Dels are NET effects: a pair
   in both lists is refused ({error, einval}, nothing applied); an
   unsubscribe-then-resubscribe since the last call is the add alone. */
static ERL_NIF_TERM nif_subs_delta(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  egm_res_t* r;
  egm_sub_pair *add = NULL, *del = NULL;
  unsigned na = 0, nd = 0;
  if (argc != 3 || !get_ctx(env, argv[0], &r)) return enif_make_badarg(env);
  if (!get_pairs(env, argv[1], &add, &na)) return enif_make_badarg(env);
  if (!get_pairs(env, argv[2], &del, &nd)) {
    free(add);
    return enif_make_badarg(env);
  }
  uint64_t epoch = 0;
  int rc = egm_subs_apply_delta(r->ctx, add, na, del, nd);
  if (!rc) rc = egm_subs_commit(r->ctx, &epoch);
  free(add);
  free(del);
  return rc ? error_tuple(env, r->ctx, rc) : enif_make_tuple2(env, ATOM_OK, enif_make_uint64(env, epoch));
}

/* publish_batch(Ctx, [Topic]) -> {ok, [{[FilterId], [{FilterId, Sub}]}]} | {error, _} */
static ERL_NIF_TERM nif_publish_batch(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  egm_res_t* r;
  uint8_t* blob;
  uint32_t *off, n;
  if (argc != 2 || !get_ctx(env, argv[0], &r) || !pack_list(env, argv[1], &blob, &off, &n))
    return enif_make_badarg(env);
  egm_result* res = NULL;
  egm_delivery* dl = NULL;
  int rc = egm_match_batch(r->ctx, blob, off, n, EGM_MODE_ROUTES, &res);
  free(blob);
  free(off);
  if (!rc) rc = egm_fanout_batch(r->ctx, res, &dl);
  if (rc) {
    if (res) egm_result_free(res);
    if (dl) egm_result_free(dl);
    return error_tuple(env, r->ctx, rc);
  }
  ERL_NIF_TERM out = enif_make_list(env, 0);
  for (uint32_t i = n; i-- > 0;) {
    ERL_NIF_TERM ids = enif_make_list(env, 0), dv = enif_make_list(env, 0);
    for (uint64_t k = res->row_ptr[i + 1]; k-- > res->row_ptr[i];)
      ids = enif_make_list_cell(env, enif_make_uint(env, res->ids[k]), ids);
    for (uint64_t k = dl->row_ptr[i + 1]; k-- > dl->row_ptr[i];)
      dv = enif_make_list_cell(
          env, enif_make_tuple2(env, enif_make_uint(env, dl->fid[k]), enif_make_uint(env, dl->sub[k])), dv);
    out = enif_make_list_cell(env, enif_make_tuple2(env, ids, dv), out);
  }
  egm_result_free(res);
  egm_result_free(dl);
  return enif_make_tuple2(env, ATOM_OK, out);
}

static ErlNifFunc nif_funcs[] = {
    {"open", 1, nif_open, 0},
    {"build", 2, nif_build, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"apply_delta", 3, nif_apply_delta, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"match_batch", 3, nif_match_batch, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"submit", 3, nif_submit, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"wait", 2, nif_wait, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"cancel", 2, nif_cancel, 0},
    {"subs_build", 2, nif_subs_build, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"subs_delta", 3, nif_subs_delta, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"publish_batch", 2, nif_publish_batch, ERL_NIF_DIRTY_JOB_CPU_BOUND},
};

ERL_NIF_INIT(emqx_gpu_match, nif_funcs, load, NULL, NULL, NULL)
