"""The Erlang NIF shim (c_src/emqx_gpu_match_nif.c) type-checks against the
C-ABI header: gcc -fsyntax-only with a declarations-only erl_nif.h
(tests/nif_mock/), since the build image has no Erlang installation.  Every
NIF entry's C-ABI call is checked against include/emqx_gpu_match.h this way."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc missing")
def test_nif_shim_type_checks():
    src = os.path.join(ROOT, "c_src", "emqx_gpu_match_nif.c")
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-fsyntax-only",
                        "-I", os.path.join(ROOT, "tests", "nif_mock"), src], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_nif_table_matches_erlang_exports():
    """Every NIF in the table has its stub in erl/emqx_gpu_match.erl, same arity."""
    c = open(os.path.join(ROOT, "c_src", "emqx_gpu_match_nif.c")).read()
    erl = open(os.path.join(ROOT, "erl", "emqx_gpu_match.erl")).read()
    table = re.findall(r'\{"(\w+)", (\d), nif_\w+', c)
    assert len(table) >= 8
    for name, arity in table:
        assert re.search(r"^%s\(%s\) -> erlang:nif_error" % (name, ", ".join(["_\\w*"] * int(arity))), erl, re.M), \
            (name, arity)
