"""A static checker for the drop-in Erlang modules under erl/ (test
infrastructure; the image has no ERTS, so erlc cannot run here).

It reports what `erlc` would stop on under the reference's production
options (rebar.config:11-13 erl_opts warn_unused_vars, warn_shadow_vars;
rebar.config.erl:141-145 adds warnings_as_errors):

* an undefined macro (``?NAME`` not defined in the module before its use, not
  predefined, and not defined by a header the module includes — the
  reference headers' names are data, tests/golden/erl_ref_api.json);
* an undefined record;
* an unused variable (bound in a function clause, fun clause or
  comprehension scope and never used there) and a variable shadowed by a fun
  head or a comprehension generator;
* a local call with no definition of that arity (and not an auto-imported
  BIF), an exported function that is not defined, a defined function that is
  never used nor exported, and missing gen_server callbacks;
* a remote call to a reference module whose export list lacks that
  function/arity, or to an OTP function outside the list below (the list
  names what these modules call; extend it deliberately).

It is a conservative approximation of erl_lint: anything it reports is an
error erlc would report, but it does not find every error erlc would.
"""
import json
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
REF_API = os.path.join(HERE, "golden", "erl_ref_api.json")

KEYWORDS = {"after", "and", "andalso", "band", "begin", "bnot", "bor", "bsl", "bsr",
            "bxor", "case", "catch", "cond", "div", "end", "fun", "if", "let", "not",
            "of", "or", "orelse", "receive", "rem", "try", "when", "xor", "maybe", "else"}
BLOCK_OPEN = {"case", "if", "receive", "try", "begin", "maybe"}
PREDEFINED_MACROS = {"MODULE", "MODULE_STRING", "FILE", "LINE", "MACHINE",
                     "FUNCTION_NAME", "FUNCTION_ARITY", "OTP_RELEASE"}
# auto-imported BIFs these modules may call without a module prefix
AUTO_BIFS = {
    "abs/1", "apply/2", "apply/3", "atom_to_binary/2", "atom_to_list/1", "binary_to_atom/2",
    "binary_to_list/1", "binary_to_term/1", "bit_size/1", "byte_size/1", "demonitor/1",
    "demonitor/2", "element/2", "erase/1", "error/1", "error/2", "exit/1", "exit/2",
    "float/1", "get/1", "hd/1", "integer_to_binary/1", "integer_to_list/1", "is_atom/1",
    "is_binary/1", "is_function/1", "is_function/2", "is_integer/1", "is_list/1",
    "is_map/1", "is_pid/1", "is_process_alive/1", "is_reference/1", "is_tuple/1",
    "length/1", "link/1", "list_to_atom/1", "list_to_binary/1", "make_ref/0",
    "map_size/1", "max/2", "min/2", "monitor/2", "node/0", "put/2", "register/2",
    "round/1", "self/0", "setelement/3", "size/1", "spawn/1", "spawn_link/1",
    "spawn_monitor/1", "term_to_binary/1", "throw/1", "tl/1", "trunc/1", "tuple_size/1",
    "unlink/1", "whereis/1"}
# OTP functions the modules call (stdlib / kernel / erts / mnesia), by arity
OTP_FUNCS = {
    "erlang": {"load_nif/2", "nif_error/1", "raise/3", "send_after/3", "cancel_timer/1",
               "system_info/1", "phash2/2", "monotonic_time/0", "monotonic_time/1"},
    "ets": {"new/2", "insert/2", "lookup/2", "lookup_element/3", "delete/2",
            "delete_object/2", "select/2", "select_replace/2", "match_delete/2",
            "update_counter/3", "member/2", "info/2"},
    "gen_server": {"start_link/4", "call/2", "call/3", "cast/2", "reply/2"},
    "lists": {"append/1", "foldl/3", "foreach/2", "member/2", "partition/2", "reverse/1",
              "zip/2", "map/2", "filter/2", "usort/1", "sort/1", "keyfind/3", "flatten/1"},
    "maps": {"get/3", "get/2", "take/2", "keys/1", "is_key/2", "from_list/1", "put/3",
             "remove/2", "size/1"},
    "queue": {"new/0", "in/2", "out/1", "len/1", "is_empty/1"},
    "persistent_term": {"get/1", "put/2", "get/2"},
    "code": {"priv_dir/1"},
    "filename": {"join/2", "join/1"},
    "mnesia": {"subscribe/1", "unsubscribe/1"},
}
GEN_SERVER_REQUIRED = {"init/1", "handle_call/3", "handle_cast/2"}


class Tok:
    __slots__ = ("kind", "text", "line")

    def __init__(self, kind, text, line):
        self.kind, self.text, self.line = kind, text, line

    def __repr__(self):
        return f"{self.kind}:{self.text}@{self.line}"


_PUNCT = ["=:=", "=/=", "...", "<<", ">>", "||", "->", "<-", "<=", "=>", ":=", "::", "==",
          "/=", "=<", ">=", "++", "--", "??"]


def tokenize(src):
    toks, i, line, n = [], 0, 1, len(src)
    while i < n:
        c = src[i]
        if c == "\n":
            line += 1
            i += 1
        elif c.isspace():
            i += 1
        elif c == "%":
            while i < n and src[i] != "\n":
                i += 1
        elif c == '"' or c == "'":
            j = i + 1
            while j < n and src[j] != c:
                if src[j] == "\\":
                    j += 1
                if j < n and src[j] == "\n":
                    line += 1
                j += 1
            toks.append(Tok("str" if c == '"' else "atom", src[i + 1:j], line))
            i = j + 1
        elif c == "$":                       # character literal
            j = i + 1
            if j < n and src[j] == "\\":
                j += 1
            toks.append(Tok("char", src[i:j + 1], line))
            i = j + 1
        elif c.isdigit():
            m = re.match(r"\d+#[0-9A-Za-z_]+|\d[\d_]*(\.\d+([eE][+-]?\d+)?)?", src[i:])
            toks.append(Tok("num", m.group(0), line))
            i += len(m.group(0))
        elif c.isalpha() or c == "_":
            m = re.match(r"[A-Za-z_][A-Za-z0-9_@]*", src[i:])
            w = m.group(0)
            if w[0].isupper() or w[0] == "_":
                toks.append(Tok("var", w, line))
            else:
                toks.append(Tok("kw" if w in KEYWORDS else "atom", w, line))
            i += len(w)
        elif c == "?":
            m = re.match(r"\?\??([A-Za-z_][A-Za-z0-9_@]*)", src[i:])
            if not m:
                raise SyntaxError(f"line {line}: bad macro")
            toks.append(Tok("macro", m.group(1), line))
            i += len(m.group(0))
        elif c == "." and (i + 1 >= n or src[i + 1].isspace() or src[i + 1] == "%"):
            toks.append(Tok("dot", ".", line))
            i += 1
        else:
            for p in _PUNCT:
                if src.startswith(p, i):
                    toks.append(Tok("p", p, line))
                    i += len(p)
                    break
            else:
                toks.append(Tok("p", c, line))
                i += 1
    return toks


def split_forms(toks):
    forms, cur = [], []
    for t in toks:
        if t.kind == "dot":
            if cur:
                forms.append(cur)
            cur = []
        else:
            cur.append(t)
    if cur:
        raise SyntaxError(f"line {cur[0].line}: form without a terminating '.'")
    return forms


_OPEN = {"(": ")", "[": "]", "{": "}", "<<": ">>"}
_CLOSE = {v: k for k, v in _OPEN.items()}


def _is_fun_opener(toks, i):
    t = toks[i]
    if not (t.kind == "kw" and t.text == "fun"):
        return False
    nxt = toks[i + 1] if i + 1 < len(toks) else None
    return nxt is not None and (nxt.text == "(" or (nxt.kind == "var" and i + 2 < len(toks)
                                                     and toks[i + 2].text == "("))


def match_index(toks, start):
    """Index of the token closing the bracket or block that opens at start."""
    stack = []
    for i in range(start, len(toks)):
        t = toks[i]
        if t.kind == "p" and t.text in _OPEN:
            stack.append(_OPEN[t.text])
        elif t.kind == "kw" and (t.text in BLOCK_OPEN or _is_fun_opener(toks, i)):
            stack.append("end")
        elif (t.kind == "p" and t.text in _CLOSE) or (t.kind == "kw" and t.text == "end"):
            if not stack or stack[-1] != t.text:
                raise SyntaxError(f"line {t.line}: unbalanced '{t.text}'")
            stack.pop()
            if not stack:
                return i
    raise SyntaxError(f"line {toks[start].line}: '{toks[start].text}' never closed")


def split_top(toks, seps):
    """Split toks at separator tokens (texts in seps) at bracket/block depth 0."""
    parts, cur, i = [], [], 0
    while i < len(toks):
        t = toks[i]
        opens = (t.kind == "p" and t.text in _OPEN) or (
            t.kind == "kw" and (t.text in BLOCK_OPEN or _is_fun_opener(toks, i)))
        if opens:
            j = match_index(toks, i)
            cur.extend(toks[i:j + 1])
            i = j + 1
            continue
        if t.kind in ("p", "kw") and t.text in seps:
            parts.append(cur)
            cur = []
        else:
            cur.append(t)
        i += 1
    parts.append(cur)
    return parts


class Scope:
    def __init__(self, parent, kind):
        self.parent, self.kind = parent, kind
        self.count = {}      # var -> occurrences in this scope (incl. nested scopes)
        self.first = {}      # var -> line of its binding

    def lookup(self, v):
        s = self
        while s is not None:
            if v in s.count:
                return s
            s = s.parent
        return None


class Linter:
    def __init__(self, path, ref_api=None, own_exports=None):
        self.path = path
        self.name = os.path.basename(path)
        self.api = ref_api if ref_api is not None else json.load(open(REF_API))
        self.own_exports = own_exports or {}
        self.errors = []
        self.macros = set(PREDEFINED_MACROS)
        self.records = set()
        self.exports = set()
        self.defined = {}         # "f/N" -> line
        self.local_refs = set()   # f/N referenced locally (calls, fun f/N, on_load)
        self.behaviours = set()
        self.module = None

    def err(self, line, msg):
        self.errors.append(f"{self.name}:{line}: {msg}")

    # -- attributes -------------------------------------------------------
    def include(self, hdr, line):
        h = self.api["headers"].get(os.path.basename(hdr))
        if h is None:
            self.err(line, f"include of unknown header {hdr!r}")
            return
        self.macros.update(h["macros"])
        self.records.update(h["records"])
        for sub in h["includes"]:
            self.include(sub, line)

    def attribute(self, form):
        name = form[1].text
        args = form[3:-1] if len(form) > 3 and form[2].text == "(" else []
        line = form[0].line
        if name == "module":
            self.module = args[0].text
        elif name in ("include", "include_lib"):
            self.include(args[0].text, line)
        elif name == "define":
            self.check_macros(form, line, skip_define_name=True)
            self.macros.add(args[0].text)
        elif name == "record":
            self.records.add(args[0].text)
        elif name == "export":
            for f, a in re.findall(r"([a-z][A-Za-z0-9_@]*)/(\d+)",
                                   "".join(t.text for t in args)):
                self.exports.add(f"{f}/{a}")
        elif name == "on_load":
            self.local_refs.add("".join(t.text for t in args))
        elif name in ("behaviour", "behavior"):
            self.behaviours.add(args[0].text)
        else:
            self.check_macros(form, line)

    def check_macros(self, toks, line, skip_define_name=False):
        for k, t in enumerate(toks):
            if t.kind == "macro" and t.text not in self.macros:
                self.err(t.line, f"undefined macro '{t.text}'")

    # -- functions --------------------------------------------------------
    def function(self, form):
        fname = form[0].text
        clauses = split_top(form, {";"})
        arity = None
        for cl in clauses:
            if not cl or cl[0].text != fname or len(cl) < 2 or cl[1].text != "(":
                self.err(form[0].line, f"malformed clause of {fname}")
                return
            close = match_index(cl, 1)
            a = len([p for p in split_top(cl[2:close], {","}) if p])
            if arity is None:
                arity = a
            elif a != arity:
                self.err(cl[0].line, f"clause of {fname} has arity {a}, not {arity}")
            self.check_macros(cl, cl[0].line)
            self.check_records(cl)
            top = Scope(None, "clause")
            self.clause(cl[1:], top)
            self.report_unused(top)
        key = f"{fname}/{arity}"
        if key in self.defined:
            self.err(form[0].line, f"function {key} already defined")
        self.defined[key] = form[0].line

    def check_records(self, toks):
        for k in range(len(toks) - 1):
            if toks[k].text == "#" and toks[k].kind == "p" and toks[k + 1].kind == "atom":
                if toks[k + 1].text not in self.records:
                    self.err(toks[k + 1].line, f"record {toks[k + 1].text} undefined")

    def clause(self, toks, scope):
        """toks = '(' head ')' [when guard] '->' body.  Head vars bind in scope;
        a head var already bound in an enclosing scope is shadowed."""
        close = match_index(toks, 0)
        self.bind_pattern(toks[1:close], scope, shadow_what="fun" if scope.parent else None)
        rest = toks[close + 1:]
        arrow = next(i for i, t in enumerate(rest) if t.text == "->")
        self.exprs(rest[:arrow], scope)      # guard
        self.exprs(rest[arrow + 1:], scope)  # body

    def bind_pattern(self, toks, scope, shadow_what=None):
        """A pattern that starts a new scope (fun head, generator): every var in it
        binds in scope; one already bound outside is shadowed (warn_shadow_vars)."""
        i = 0
        while i < len(toks):
            t = toks[i]
            if t.kind == "var" and t.text != "_":
                outer = scope.parent.lookup(t.text) if scope.parent else None
                if outer is not None and shadow_what:
                    self.err(t.line, f"variable '{t.text}' shadowed in '{shadow_what}'")
                if t.text in scope.count:
                    scope.count[t.text] += 1
                else:
                    scope.count[t.text] = 1
                    scope.first[t.text] = t.line
                i += 1
            else:
                i += 1

    def use(self, t, scope):
        s = scope.lookup(t.text)
        if s is None:   # first occurrence: binds in the innermost scope
            scope.count[t.text] = 1
            scope.first[t.text] = t.line
        else:
            s.count[t.text] += 1

    def exprs(self, toks, scope):
        i = 0
        while i < len(toks):
            t = toks[i]
            if _is_fun_opener(toks, i):
                j = match_index(toks, i)
                body = toks[i + 1:j]
                if body[0].kind == "var":          # named fun: Name(...) -> ...
                    body = body[1:]
                for cl in split_top(body, {";"}):
                    if cl and cl[0].kind == "var":
                        cl = cl[1:]
                    fs = Scope(scope, "fun")
                    self.clause(cl, fs)
                    self.report_unused(fs)
                i = j + 1
                continue
            if t.kind == "kw" and t.text == "fun":
                # fun f/N or fun m:f/N: a reference, not a scope
                nx = toks[i + 1:i + 6]
                if len(nx) >= 3 and nx[1].text == "/" and nx[2].kind == "num":
                    self.local_refs.add(f"{nx[0].text}/{nx[2].text}")
                elif (len(nx) >= 5 and nx[1].text == ":" and nx[3].text == "/"
                      and nx[0].kind == "atom" and nx[4].kind == "num"):
                    self.remote_calls.append((nx[0].text, nx[2].text, int(nx[4].text), t.line))
                i += 1
                continue
            if t.kind == "p" and t.text in ("[", "<<"):
                j = match_index(toks, i)
                parts = split_top(toks[i + 1:j], {"||"})
                if len(parts) > 1:
                    self.comprehension(parts[0], parts[1], scope)
                    i = j + 1
                    continue
            if t.kind == "var" and t.text != "_":
                self.use(t, scope)
            elif t.kind == "atom" and i + 1 < len(toks) and toks[i + 1].text == "(":
                prev = toks[i - 1] if i > 0 else None
                if not (prev is not None and prev.text in (":", "#", "?")):
                    close = match_index(toks, i + 1)
                    a = len([p for p in split_top(toks[i + 2:close], {","}) if p])
                    self.local_refs.add(f"{t.text}/{a}")
                    self.local_calls.append((t.text, a, t.line))
                elif prev is not None and prev.text == ":" and i >= 2 and toks[i - 2].kind == "atom":
                    close = match_index(toks, i + 1)
                    a = len([p for p in split_top(toks[i + 2:close], {","}) if p])
                    self.remote_calls.append((toks[i - 2].text, t.text, a, t.line))
            i += 1

    def comprehension(self, template, quals, scope):
        lc = Scope(scope, "lc")
        for q in split_top(quals, {","}):
            parts = split_top(q, {"<-", "<="})
            if len(parts) > 1:
                k = len(parts[0])
                self.exprs(q[k + 1:], lc)             # the generator's list
                self.bind_pattern(q[:k], lc, shadow_what="generate")
            else:
                self.exprs(q, lc)                      # a filter
        self.exprs(template, lc)
        self.report_unused(lc)

    def report_unused(self, scope):
        for v, c in scope.count.items():
            if c == 1 and not v.startswith("_"):
                self.err(scope.first[v], f"variable '{v}' is unused")

    # -- module -----------------------------------------------------------
    def run(self):
        src = open(self.path, encoding="utf-8").read()
        self.local_calls, self.remote_calls = [], []
        try:
            forms = split_forms(tokenize(src))
            for form in forms:
                if form[0].text == "-":
                    self.attribute(form)
                elif form[0].kind == "atom":
                    self.function(form)
                else:
                    self.err(form[0].line, "unexpected form")
        except (SyntaxError, StopIteration, IndexError) as e:
            self.err(0, f"parse error: {e}")
            return self.errors
        for f, a, line in self.local_calls:
            key = f"{f}/{a}"
            if key not in self.defined and key not in AUTO_BIFS:
                self.err(line, f"function {key} undefined")
        for key in sorted(self.exports - set(self.defined)):
            self.err(0, f"function {key} exported but undefined")
        for key, line in sorted(self.defined.items()):
            if key not in self.exports and key not in self.local_refs:
                self.err(line, f"function {key} is unused")
        if "gen_server" in self.behaviours:
            for cb in sorted(GEN_SERVER_REQUIRED - self.exports):
                self.err(0, f"undefined callback function {cb} (behaviour 'gen_server')")
        for m, f, a, line in self.remote_calls:
            key = f"{f}/{a}"
            if m in self.api["exports"]:
                ok = key in self.api["exports"][m]
            elif m in OTP_FUNCS:
                ok = key in OTP_FUNCS[m]
            elif m in self.own_exports:
                ok = key in self.own_exports[m]
            else:
                self.err(line, f"call to unknown module {m}:{key}")
                continue
            if not ok:
                self.err(line, f"{m}:{key} is not exported")
        return self.errors


def module_exports(path):
    lt = Linter(path)
    lt.run()
    return lt.module, set(lt.exports)


def lint_files(paths):
    own = {}
    for p in paths:
        m, ex = module_exports(p)
        own[m] = ex
    errors = []
    for p in paths:
        errors += Linter(p, own_exports=own).run()
    return errors
