"""The drop-in Erlang modules (erl/) must compile under the reference's
production options: erl_opts warn_unused_vars + warn_shadow_vars
(rebar.config:11-13) with warnings_as_errors (rebar.config.erl:141-145).
No ERTS in the image, so tests/erl_lint.py stands in for erlc; each
mutation below re-introduces a defect of the kind erlc stops on and must be
reported."""
import glob
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import erl_lint  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ERL = sorted(glob.glob(os.path.join(ROOT, "erl", "*.erl")))


def test_erl_modules_are_clean():
    assert len(ERL) == 3
    assert erl_lint.lint_files(ERL) == []


def _lint_mutated(tmp_path, name, old, new):
    paths = []
    for p in ERL:
        src = open(p).read()
        if os.path.basename(p) == name:
            assert old in src, (name, old)
            src = src.replace(old, new, 1)
        q = tmp_path / os.path.basename(p)
        q.write_text(src)
        paths.append(str(q))
    return erl_lint.lint_files(paths)


MUTATIONS = [
    # round 4's two defects (What's missing 1)
    ("emqx_gpu_routes.erl", "-define(ROUTE_TAB, emqx_route).", '-include("emqx.hrl").',
     "undefined macro 'ROUTE_TAB'"),
    ("emqx_gpu_batch.erl", "submit(Items, St) ->",
     "submit(Items, St = #st{ctx = Ctx, waiters = W}) ->", "variable 'Ctx' is unused"),
    # other erlc stops
    ("emqx_gpu_batch.erl", "answer(Items, [], {error, no_route_sync}),",
     "answer(Items, [], {error, no_route_sync}, x),", "function answer/4 undefined"),
    ("emqx_gpu_match.erl", "merge_overlay(Topic, Matched, Ov) ->",
     "merge_overlay(Topic, Matched, Ov) -> _ = [Ov || Ov <- Matched],",
     "variable 'Ov' shadowed in 'generate'"),
    ("emqx_gpu_batch.erl", "lists:foreach(fun({From, _}) -> gen_server:reply(From, Err) end, Items).",
     "lists:foreach(fun({From, Items}) -> gen_server:reply(From, Err) end, Items).",
     "variable 'Items' shadowed in 'fun'"),
    ("emqx_gpu_routes.erl", "fun emqx_router:has_routes/1", "fun emqx_router:has_route/1",
     "emqx_router:has_route/1 is not exported"),
    ("emqx_gpu_match.erl", "emqx_router:lookup_routes(To)", "emqx_router:lookup_route(To)",
     "emqx_router:lookup_route/1 is not exported"),
    ("emqx_gpu_batch.erl", "#st{ctx = emqx_gpu_match:ctx(),", "#state{ctx = emqx_gpu_match:ctx(),",
     "record state undefined"),
    ("emqx_gpu_match.erl", "-export([init/0, ctx/0, filter_of/1,", "-export([init/0, ctx/0,",
     "function filter_of/1 is unused"),
    ("emqx_gpu_routes.erl", "    Snap = [{T, ets:lookup(?PENDING, T)} || T <- Touched],",
     "    Snap = [{T, ets:lookup(?PENDING, T)} || T <- Touched, X <- Touched],",
     "variable 'X' is unused"),
]


@pytest.mark.parametrize("name,old,new,expect", MUTATIONS,
                         ids=[f"{m[0]}:{i}" for i, m in enumerate(MUTATIONS)])
def test_lint_reports_reintroduced_defect(tmp_path, name, old, new, expect):
    errs = _lint_mutated(tmp_path, name, old, new)
    assert errs, f"mutation {new!r} not reported"
    if expect is not None:
        assert any(expect in e for e in errs), errs


def test_route_tab_is_the_reference_table_name():
    """?ROUTE_TAB must name emqx_router's table (emqx_router.erl:70), which
    the route events are tagged with (emqx_router.erl:78-81)."""
    src = open(os.path.join(ROOT, "erl", "emqx_gpu_routes.erl")).read()
    assert "-define(ROUTE_TAB, emqx_route)." in src
    assert "ROUTE_TAB" not in " ".join(
        v for h in erl_lint.json.load(open(erl_lint.REF_API))["headers"].values()
        for v in h["macros"])


def test_integration_installs_every_module():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    for p in ERL:
        assert f"erl/{os.path.basename(p)}" in doc and "apps/emqx/src" in doc
