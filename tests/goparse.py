"""A small reader of Go source files' top-level declarations (test helper).

There is no Go toolchain in this image, so the drop-in checks of
tests/test_cgo_shim_cpu.py need the part of `go/parser` they use: the build
constraint, the package clause, and every top-level declaration -- funcs and
methods (receiver type, name, parameter types, result types), types, vars and
consts (grouped or not).  Comments, strings, raw strings and runes are
tokenised so that braces and parentheses inside them do not count.
"""
import re

_TOKEN = re.compile(r"""
    (?P<comment>//[^\n]*|/\*.*?\*/)
  | (?P<raw>`[^`]*`)
  | (?P<str>"(?:\\.|[^"\\\n])*")
  | (?P<rune>'(?:\\.|[^'\\\n])+')
  | (?P<ident>[A-Za-z_][A-Za-z0-9_]*)
  | (?P<num>[0-9][0-9A-Za-z_.]*)
  | (?P<nl>\n)
  | (?P<op>\.\.\.|:=|<-|&&|\|\||[-+*/%&|^<>=!]=?|[{}()\[\],;.:~])
  | (?P<ws>[ \t\r]+)
""", re.S | re.X)


def tokens(src):
    """(kind, text) pairs, comments and blanks dropped, newlines kept."""
    out, pos = [], 0
    while pos < len(src):
        m = _TOKEN.match(src, pos)
        if not m:
            raise ValueError(f"go tokenizer: cannot read {src[pos:pos + 20]!r}")
        pos = m.end()
        kind = m.lastgroup
        if kind in ("ws", "comment"):
            if kind == "comment" and "\n" in m.group():
                out.append(("nl", "\n"))
            continue
        out.append((kind, m.group()))
    return out


def build_constraint(src):
    m = re.match(r"\s*//go:build ([^\n]+)\n", src)
    return m.group(1).strip() if m else None


def build_ok(expr, tags):
    """Evaluates a //go:build expression (identifiers, !, &&, ||, parens)
    for the set of satisfied tags."""
    if expr is None:
        return True
    py = re.sub(r"[A-Za-z_][A-Za-z0-9_.]*", lambda m: "T" if m.group() in tags else "F", expr)
    py = py.replace("&&", " and ").replace("||", " or ").replace("!", " not ")
    return bool(eval(py, {"T": True, "F": False}))  # noqa: S307 (our own token set only)


def _split_top(toks, sep=","):
    """Split a token list at depth-0 separators."""
    parts, cur, depth = [], [], 0
    for t in toks:
        if t[1] in "([{":
            depth += 1
        elif t[1] in ")]}":
            depth -= 1
        if depth == 0 and t[1] == sep:
            parts.append(cur)
            cur = []
            continue
        cur.append(t)
    if cur:
        parts.append(cur)
    return parts


def _text(toks):
    s = " ".join(t[1] for t in toks)
    s = re.sub(r"\s*([\[\]().,*])\s*", r"\1", s)
    s = s.replace(",", ", ")
    return re.sub(r"(func|map|chan|struct|interface)\(", r"\1 (", s).strip()


def param_types(toks):
    """Types of a parameter (or result) list given without its parentheses:
    `a, b int, c string` -> [int, int, string]; `int, error` -> [int, error]."""
    groups = [[t for t in g if t[0] != "nl"] for g in _split_top(toks)]
    groups = [g for g in groups if g]
    named = any(len(g) >= 2 and g[0][0] == "ident" and g[1][1] not in (".",) for g in groups)
    if not named:
        return [_text(g) for g in groups]
    out, pending = [], 0
    for g in groups:
        if len(g) == 1:
            pending += 1
            continue
        ty = _text(g[1:])
        out += [ty] * (pending + 1)
        pending = 0
    return out


def _match(toks, i):
    """Index just past the bracket that closes the one at toks[i]."""
    pairs = {"(": ")", "[": "]", "{": "}"}
    want, depth = pairs[toks[i][1]], 0
    for j in range(i, len(toks)):
        if toks[j][1] == toks[i][1]:
            depth += 1
        elif toks[j][1] == want:
            depth -= 1
            if depth == 0:
                return j + 1
    raise ValueError("unbalanced bracket")


def declarations(src):
    """Top-level declarations of one Go file:
    {"package": name, "build": expr, "funcs": [...], "types": [...], "values": [...]}
    funcs: dicts with recv (type name or None), name, params, results, body
    (the body's tokens as text, or None)."""
    toks = tokens(src)
    out = {"package": None, "build": build_constraint(src), "funcs": [], "types": [], "values": []}
    i, n = 0, len(toks)
    while i < n:
        kind, tx = toks[i]
        if kind == "nl" or tx == ";":
            i += 1
            continue
        if tx == "package":
            out["package"] = toks[i + 1][1]
            i += 2
        elif tx == "import":
            i += 1
            while toks[i][0] == "nl":
                i += 1
            i = _match(toks, i) if toks[i][1] == "(" else i + 2 if toks[i][0] == "ident" else i + 1
        elif tx == "func":
            i += 1
            recv = None
            if toks[i][1] == "(":
                j = _match(toks, i)
                rt = [t[1] for t in toks[i + 1:j - 1] if t[0] == "ident"]
                recv = rt[-1]
                i = j
            name = toks[i][1]
            i += 1
            j = _match(toks, i)
            params = param_types(toks[i + 1:j - 1])
            i = j
            res = []
            if toks[i][1] == "(":
                j = _match(toks, i)
                res = param_types(toks[i + 1:j - 1])
                i = j
            else:
                k = i
                while toks[k][1] != "{" and toks[k][0] != "nl":
                    k += 1
                if k > i:
                    res = [_text(toks[i:k])]
                i = k
            body = None
            if toks[i][1] == "{":
                j = _match(toks, i)
                body = " ".join(t[1] for t in toks[i:j] if t[0] != "nl")
                i = j
            out["funcs"].append({"recv": recv, "name": name, "params": params, "results": res, "body": body})
        elif tx in ("type", "var", "const"):
            what = "types" if tx == "type" else "values"
            i += 1
            if toks[i][1] == "(":
                j = _match(toks, i)
                k, line_start = i + 1, True
                depth = 0
                while k < j - 1:
                    t = toks[k]
                    if t[1] in "([{":
                        depth += 1
                    elif t[1] in ")]}":
                        depth -= 1
                    if t[0] == "nl" or t[1] == ";":
                        line_start = depth == 0
                    elif line_start and depth == 0 and t[0] == "ident":
                        # one spec: its names (a, b = ...)
                        out[what].append(t[1])
                        m = k + 1
                        while m < j - 1 and toks[m][1] == ",":
                            out[what].append(toks[m + 1][1])
                            m += 2
                        line_start = False
                    else:
                        line_start = False
                    k += 1
                i = j
            else:
                out[what].append(toks[i][1])
                m = i + 1
                while toks[m][1] == ",":
                    out[what].append(toks[m + 1][1])
                    m += 2
                # skip to the end of the spec (depth-0 newline)
                depth = 0
                while m < n:
                    t = toks[m]
                    if t[1] in "([{":
                        depth += 1
                    elif t[1] in ")]}":
                        depth -= 1
                    elif t[0] == "nl" and depth == 0:
                        break
                    m += 1
                i = m
        else:
            raise ValueError(f"go reader: unexpected top-level token {tx!r}")
    return out


def package_scope(files, tags):
    """name -> [file] of every package-scope identifier (funcs without a
    receiver, types, vars, consts) of the files a build with `tags` compiles,
    plus (recv, method) -> [file]."""
    scope, methods = {}, {}
    for f, src in files.items():
        d = declarations(src)
        if not build_ok(d["build"], tags):
            continue
        for fn in d["funcs"]:
            if fn["recv"] is None:
                if fn["name"] not in ("init", "_"):
                    scope.setdefault(fn["name"], []).append(f)
            else:
                methods.setdefault((fn["recv"], fn["name"]), []).append(f)
        for nm in d["types"] + d["values"]:
            if nm != "_":
                scope.setdefault(nm, []).append(f)
    return scope, methods
