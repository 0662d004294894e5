"""Generate tests/golden/erl_ref_api.json: the parts of the reference's
Erlang sources that the drop-in modules under erl/ compile against.

* the macro and record names each header of apps/emqx/include defines
  (apps/emqx/include/{emqx,logger,types,emqx_mqtt,emqx_release}.hrl);
* the export lists of the reference modules erl/ calls
  (apps/emqx/src/emqx_{router,topic,trie,broker,batch,shared_sub,broker_helper}.erl);
* the compile options the modules must pass: rebar.config:11-13 (erl_opts)
  and rebar.config.erl:141-145 (prod_compile_opts adds warnings_as_errors).

Data only (names and arities), no source text.  Run from the repo root in a
container that has /root/reference:

    python tests/golden/make_erl_ref_api.py
"""
import json
import os
import re
import sys

REF = "/root/reference"
HEADERS = ["emqx.hrl", "logger.hrl", "types.hrl", "emqx_mqtt.hrl", "emqx_release.hrl"]
MODULES = ["emqx_router", "emqx_topic", "emqx_trie", "emqx_broker", "emqx_batch",
           "emqx_shared_sub", "emqx_broker_helper"]


def strip_comments(text):
    out = []
    for line in text.splitlines():
        # a '%' outside a string starts a comment (headers and export lists
        # here carry no '%' inside strings on the lines we parse)
        q = False
        cut = len(line)
        for i, ch in enumerate(line):
            if ch == '"':
                q = not q
            elif ch == '%' and not q and (i == 0 or line[i - 1] != '$'):
                cut = i
                break
        out.append(line[:cut])
    return "\n".join(out)


def header_names(path):
    text = strip_comments(open(path, encoding="utf-8").read())
    macros = sorted(set(re.findall(r"-define\(\s*([A-Za-z_][A-Za-z0-9_@]*)", text)))
    records = sorted(set(re.findall(r"-record\(\s*([a-z][A-Za-z0-9_@]*)", text)))
    includes = sorted(set(re.findall(r'-include(?:_lib)?\(\s*"([^"]+)"', text)))
    return {"macros": macros, "records": records, "includes": includes}


def exports(path):
    text = strip_comments(open(path, encoding="utf-8").read())
    out = set()
    for body in re.findall(r"-export\(\s*\[(.*?)\]\s*\)\s*\.", text, re.S):
        for name, arity in re.findall(r"([a-z][A-Za-z0-9_@]*)\s*/\s*(\d+)", body):
            out.add(f"{name}/{arity}")
    return sorted(out)


def main():
    if not os.path.isdir(REF):
        sys.exit("needs /root/reference (run in the build container)")
    inc = os.path.join(REF, "apps/emqx/include")
    src = os.path.join(REF, "apps/emqx/src")
    data = {
        "source": "tyt0223/emqx (EMQ X 5.0-alpha.3) under /root/reference",
        "erl_opts": ["warn_unused_vars", "warn_shadow_vars", "warn_unused_import",
                     "warn_obsolete_guard", "warnings_as_errors"],
        "erl_opts_cite": "rebar.config:11-13; rebar.config.erl:141-145",
        "headers": {h: header_names(os.path.join(inc, h)) for h in HEADERS},
        "exports": {m: exports(os.path.join(src, m + ".erl")) for m in MODULES},
    }
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "erl_ref_api.json")
    with open(dst, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
        f.write("\n")
    print("wrote", dst)


if __name__ == "__main__":
    main()
