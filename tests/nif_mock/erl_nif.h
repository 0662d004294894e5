/* Declarations-only stand-in for ERTS's erl_nif.h, used by
 * tests/test_nif_compile.py to type-check c_src/emqx_gpu_match_nif.c with
 * gcc -fsyntax-only (there is no Erlang installation in the build image).
 * Only the erl_nif API the shim uses is declared; nothing here is linked. */
#pragma once
#include <stddef.h>
#include <stdint.h>
typedef uint64_t ERL_NIF_TERM;
typedef struct enif_environment_t ErlNifEnv;
typedef struct enif_resource_type_t ErlNifResourceType;
typedef uint64_t ErlNifUInt64;
typedef struct {
  size_t size;
  unsigned char* data;
} ErlNifBinary;
typedef void ErlNifResourceDtor(ErlNifEnv*, void*);
typedef enum { ERL_NIF_RT_CREATE = 1, ERL_NIF_RT_TAKEOVER = 2 } ErlNifResourceFlags;
typedef enum { ERL_NIF_LATIN1 = 1 } ErlNifCharEncoding;
#define ERL_NIF_DIRTY_JOB_CPU_BOUND 1
#define ERL_NIF_DIRTY_JOB_IO_BOUND 2
typedef struct {
  const char* name;
  unsigned arity;
  ERL_NIF_TERM (*fptr)(ErlNifEnv*, int, const ERL_NIF_TERM[]);
  unsigned flags;
} ErlNifFunc;
ErlNifResourceType* enif_open_resource_type(ErlNifEnv*, const char*, const char*, ErlNifResourceDtor*,
                                            ErlNifResourceFlags, ErlNifResourceFlags*);
ERL_NIF_TERM enif_make_atom(ErlNifEnv*, const char*);
ERL_NIF_TERM enif_make_tuple2(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_int(ErlNifEnv*, int);
ERL_NIF_TERM enif_make_uint(ErlNifEnv*, unsigned);
ERL_NIF_TERM enif_make_uint64(ErlNifEnv*, ErlNifUInt64);
ERL_NIF_TERM enif_make_string(ErlNifEnv*, const char*, ErlNifCharEncoding);
ERL_NIF_TERM enif_make_list(ErlNifEnv*, unsigned, ...);
ERL_NIF_TERM enif_make_list_cell(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM);
int enif_make_reverse_list(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM*);
ERL_NIF_TERM enif_make_badarg(ErlNifEnv*);
ERL_NIF_TERM enif_make_resource(ErlNifEnv*, void*);
int enif_get_list_length(ErlNifEnv*, ERL_NIF_TERM, unsigned*);
int enif_get_list_cell(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM*, ERL_NIF_TERM*);
int enif_inspect_binary(ErlNifEnv*, ERL_NIF_TERM, ErlNifBinary*);
int enif_get_int(ErlNifEnv*, ERL_NIF_TERM, int*);
int enif_get_uint(ErlNifEnv*, ERL_NIF_TERM, unsigned*);
int enif_get_uint64(ErlNifEnv*, ERL_NIF_TERM, ErlNifUInt64*);
int enif_get_tuple(ErlNifEnv*, ERL_NIF_TERM, int*, const ERL_NIF_TERM**);
int enif_get_resource(ErlNifEnv*, ERL_NIF_TERM, ErlNifResourceType*, void**);
void* enif_alloc_resource(ErlNifResourceType*, size_t);
void enif_release_resource(void*);
int enif_keep_resource(void*);
#define ERL_NIF_INIT(name, funcs, load, reload, upgrade, unload) \
  const ErlNifFunc* name##_nif_table(void) { return funcs; } \
  int (*name##_nif_load)(ErlNifEnv*, void**, ERL_NIF_TERM) = load;
