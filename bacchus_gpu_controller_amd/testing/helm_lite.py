"""A small Helm-compatible template renderer for chart tests (there is no `helm` binary
in the build image).

It implements the Go text/template subset our chart uses, with Helm's semantics:
  * actions {{ }}, trim markers {{- -}}, comments {{/* */}};
  * if / else if / else, with / else, range (with $v / $k, $v declarations), define,
    template, variable declaration and assignment, pipelines, parenthesised sub-pipelines;
  * the Sprig/Helm functions: include, default, quote, squote, toYaml, nindent, indent,
    trunc, trimSuffix, trimPrefix, replace, contains, printf, join, list, dict, index,
    eq/ne/lt/le/gt/ge, and/or/not, int/int64/float64/toString, lower/upper, b64enc,
    required, empty, hasKey, ternary;
  * numbers from values.yaml are float64 (Helm reads values through JSON), so they print
    the way Helm prints them (1073741824 -> "1.073741824e+09" unless piped to int64);
  * a missing map key is nil and renders as "" (Helm's missingkey=zero), while field access
    through nil is an error, like Go's "nil pointer evaluating interface {}.x".

render_chart(chart_dir, values_overrides, release) returns the rendered manifests keyed by
template file, in the form `helm template` would print them.
"""
import base64
import copy
import json
import math
import os
import re
from decimal import Decimal

import yaml


class TemplateError(Exception):
    pass


# ----------------------------------------------------------------------------- values

def _floatify(v):
    """Helm parses values through JSON: every number becomes float64."""
    if isinstance(v, bool) or v is None:
        return v
    if isinstance(v, (int, float)):
        return float(v)
    if isinstance(v, dict):
        return {k: _floatify(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_floatify(x) for x in v]
    return v


def _merge(base, over):
    out = copy.deepcopy(base)
    for k, v in (over or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = _merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


# ----------------------------------------------------------------------------- printing

def _go_float(f):
    """fmt.Sprint(float64) == strconv.FormatFloat(f, 'g', -1, 64): shortest round-trip
    digits, exponent form when the decimal exponent is < -4 or >= 6 (1e6 -> "1e+06")."""
    if math.isinf(f):
        return "+Inf" if f > 0 else "-Inf"
    if math.isnan(f):
        return "NaN"
    if f == 0:
        return "0"
    sign, digs, e = Decimal(repr(abs(f))).normalize().as_tuple()
    digits = "".join(map(str, digs))
    nd = len(digits)
    dp = nd + e  # decimal point position relative to the first digit
    exp = dp - 1
    neg = "-" if f < 0 else ""
    if exp < -4 or exp >= 6:
        m = digits[0] + ("." + digits[1:] if nd > 1 else "")
        return f"{neg}{m}e{'+' if exp >= 0 else '-'}{abs(exp):02d}"
    if dp <= 0:
        return neg + "0." + "0" * (-dp) + digits
    if dp >= nd:
        return neg + digits + "0" * (dp - nd)
    return neg + digits[:dp] + "." + digits[dp:]


def _go_str(v):
    if v is None:
        return ""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        return _go_float(v)
    if isinstance(v, int):
        return str(v)
    if isinstance(v, list):
        return "[" + " ".join(_go_str(x) for x in v) + "]"
    if isinstance(v, dict):
        return "map[" + " ".join(f"{k}:{_go_str(v[k])}" for k in sorted(v)) + "]"
    return str(v)


def _truthy(v):
    if v is None or v is False:
        return False
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return v != 0
    if isinstance(v, (str, list, dict, tuple)):
        return len(v) > 0
    return True


def _to_yaml(v):
    def ints(x):  # sigs.k8s.io/yaml round-trips JSON; integral numbers come back as ints
        if isinstance(x, float) and x.is_integer():
            return int(x)
        if isinstance(x, dict):
            return {k: ints(y) for k, y in x.items()}
        if isinstance(x, list):
            return [ints(y) for y in x]
        return x

    if v is None:
        return "null"
    out = yaml.safe_dump(ints(v), default_flow_style=False, sort_keys=True, allow_unicode=True, width=1 << 20)
    if out.endswith("...\n"):
        out = out[:-4]
    return out.rstrip("\n")


def _go_sprintf(fmt, args):
    out, i, ai = [], 0, 0
    while i < len(fmt):
        c = fmt[i]
        if c != "%":
            out.append(c)
            i += 1
            continue
        i += 1
        if i < len(fmt) and fmt[i] == "%":
            out.append("%")
            i += 1
            continue
        j = i
        while j < len(fmt) and fmt[j] in "0123456789.-+# ":
            j += 1
        verb = fmt[j]
        a = args[ai] if ai < len(args) else None
        ai += 1
        if verb in "sv":
            out.append(_go_str(a))
        elif verb == "d":
            out.append(str(int(a)))
        elif verb == "q":
            out.append(json.dumps(_go_str(a), ensure_ascii=False))
        else:
            raise TemplateError(f"printf verb %{verb} not supported")
        i = j + 1
    return "".join(out)


# ----------------------------------------------------------------------------- lexing

def _actions(src):
    """(start, end, left_trim, body, right_trim) of every {{ ... }} action, as Go's lexer
    finds them: a "}}" inside a quoted or raw (backquoted) string does not end the action
    (e.g. {{`{{ $labels.gpu }}`}}, how a chart emits Prometheus template text)."""
    pos = 0
    while True:
        start = src.find("{{", pos)
        if start < 0:
            return
        i = start + 2
        left = src.startswith("-", i) and i + 1 < len(src) and src[i + 1] in " \t\r\n"
        if left:
            i += 1
        body_start = i
        while True:
            if i >= len(src):
                raise TemplateError("unclosed action")
            c = src[i]
            if src.startswith("/*", i):
                j = src.find("*/", i + 2)
                if j < 0:
                    raise TemplateError("unclosed comment")
                i = j + 2
            elif c == '"':
                i += 1
                while i < len(src) and src[i] != '"':
                    i += 2 if src[i] == "\\" else 1
                i += 1
            elif c == "`":
                j = src.find("`", i + 1)
                if j < 0:
                    raise TemplateError("unclosed raw string")
                i = j + 1
            elif src.startswith("}}", i):
                break
            else:
                i += 1
        body, right = src[body_start:i], False
        if len(body) >= 2 and body[-1] == "-" and body[-2] in " \t\r\n":
            body, right = body[:-1], True
        yield start, i + 2, left, body, right
        pos = i + 2


def _lex(src):
    """-> list of ("text", s) / ("action", s) with trim markers applied."""
    items, pos = [], 0
    for start, end, left, body, right in _actions(src):
        text = src[pos:start]
        if left:
            text = text.rstrip(" \t\r\n")
        items.append(["text", text])
        items.append(["action", body.strip(), right])
        pos = end
    items.append(["text", src[pos:]])
    # right-trim markers eat leading whitespace of the following text
    out = []
    trim_next = False
    for it in items:
        if it[0] == "text":
            s = it[1].lstrip(" \t\r\n") if trim_next else it[1]
            trim_next = False
            if s:
                out.append(("text", s))
        else:
            trim_next = it[2]
            if not (it[1].startswith("/*") and it[1].endswith("*/")):
                out.append(("action", it[1]))
    return out


_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<str>"(?:[^"\\]|\\.)*")
  | (?P<raw>`[^`]*`)
  | (?P<num>-?\d+(?:\.\d+)?(?:[eE][-+]?\d+)?)
  | (?P<decl>:=)
  | (?P<assign>=)
  | (?P<pipe>\|)
  | (?P<lp>\()
  | (?P<rp>\))
  | (?P<comma>,)
  | (?P<var>\$[A-Za-z0-9_]*(?:\.[A-Za-z0-9_]+)*)
  | (?P<field>(?:\.[A-Za-z0-9_]+)+|\.)
  | (?P<ident>[A-Za-z_][A-Za-z0-9_]*)
  | (?P<chain>(?:\.[A-Za-z0-9_]+)+)
""", re.X)


def _tokens(s):
    out, pos = [], 0
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m:
            raise TemplateError(f"cannot tokenize action: {s!r} at {pos}")
        pos = m.end()
        kind = m.lastgroup
        if kind == "ws":
            continue
        out.append((kind, m.group(kind)))
    return out


# ----------------------------------------------------------------------------- parsing

class _P:
    def __init__(self, toks):
        self.t = toks
        self.i = 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else (None, None)

    def take(self):
        tok = self.peek()
        self.i += 1
        return tok


def _parse_pipeline(toks):
    """-> {"decl": [names] | None, "assign": bool, "cmds": [[operand, ...], ...]}"""
    p = _P(toks)
    decl, assign = None, False
    # "$a := ..." / "$k, $v := ..." / "$a = ..."
    j = 0
    names = []
    while p.peek(j)[0] == "var":
        names.append(p.peek(j)[1])
        if p.peek(j + 1)[0] == "comma":
            j += 2
            continue
        if p.peek(j + 1)[0] in ("decl", "assign"):
            assign = p.peek(j + 1)[0] == "assign"
            decl = names
            p.i = j + 2
        break
    cmds = [[]]
    while p.peek()[0] is not None:
        kind, val = p.take()
        if kind == "pipe":
            cmds.append([])
        elif kind == "lp":
            # collect the balanced sub-pipeline
            depth, sub = 1, []
            while depth:
                k2, v2 = p.take()
                if k2 is None:
                    raise TemplateError("unbalanced parenthesis")
                if k2 == "lp":
                    depth += 1
                elif k2 == "rp":
                    depth -= 1
                    if depth == 0:
                        break
                sub.append((k2, v2))
            chain = None
            if p.peek()[0] in ("chain", "field") and p.peek()[1] != ".":
                chain = p.take()[1]
            cmds[-1].append(("sub", _parse_pipeline(sub), chain))
        else:
            cmds[-1].append((kind, val))
    return {"decl": decl, "assign": assign, "cmds": cmds}


def _parse(items, i=0, stop=("end",)):
    """-> (nodes, index_after, terminator_action)"""
    nodes = []
    while i < len(items):
        kind, s = items[i]
        if kind == "text":
            nodes.append(("text", s))
            i += 1
            continue
        word = s.split(None, 1)[0] if s else ""
        rest = s[len(word):].strip()
        if word in ("end", "else"):
            if word not in stop and not (word == "else" and "else" in stop):
                raise TemplateError(f"unexpected {{{{{s}}}}}")
            return nodes, i + 1, s
        if word in ("if", "with", "range"):
            body, i, term = _parse(items, i + 1, stop=("end", "else"))
            node = {"kind": word, "pipe": _parse_pipeline(_tokens(rest)), "body": body, "else": None}
            nodes.append(("block", node))
            while term.startswith("else"):
                tail = term[4:].strip()
                if tail.startswith("if ") or tail.startswith("with "):
                    # "else if X" == else { if X ... } sharing the same end
                    w2 = tail.split(None, 1)[0]
                    body2, i, term = _parse(items, i, stop=("end", "else"))
                    sub = {"kind": w2, "pipe": _parse_pipeline(_tokens(tail[len(w2):].strip())), "body": body2,
                           "else": None}
                    node["else"] = [("block", sub)]
                    node = sub
                else:
                    body2, i, term = _parse(items, i, stop=("end",))
                    node["else"] = body2
            continue
        if word == "define":
            name = json.loads(rest)
            body, i, _ = _parse(items, i + 1, stop=("end",))
            nodes.append(("define", name, body))
            continue
        if word == "template":
            toks = _tokens(rest)
            name = json.loads(toks[0][1])
            nodes.append(("template", name, _parse_pipeline(toks[1:]) if len(toks) > 1 else None))
            i += 1
            continue
        nodes.append(("action", _parse_pipeline(_tokens(s))))
        i += 1
    if stop:
        raise TemplateError(f"missing {{{{end}}}} (expected one of {stop})")
    return nodes, i, None


# ----------------------------------------------------------------------------- evaluation

class _Scope:
    def __init__(self, root):
        self.frames = [{"$": root}]

    def push(self):
        self.frames.append({})

    def pop(self):
        self.frames.pop()

    def get(self, name):
        for f in reversed(self.frames):
            if name in f:
                return f[name]
        raise TemplateError(f"undefined variable {name}")

    def declare(self, name, v):
        self.frames[-1][name] = v

    def assign(self, name, v):
        for f in reversed(self.frames):
            if name in f:
                f[name] = v
                return
        raise TemplateError(f"assignment to undeclared variable {name}")


def _field(v, names, what):
    for n in names:
        if v is None:
            raise TemplateError(f"nil pointer evaluating interface {{}}.{n} in {what}")
        if isinstance(v, dict):
            v = v.get(n)
        else:
            raise TemplateError(f"can't evaluate field {n} in type {type(v).__name__} ({what})")
    return v


class Renderer:
    def __init__(self):
        self.defines = {}
        self.funcs = self._funcs()

    # -- templates
    def load(self, name, src):
        nodes, _, _ = _parse(_lex(src), 0, stop=())
        self._collect(nodes)
        return nodes

    def _collect(self, nodes):
        for n in nodes:
            if n[0] == "define":
                self.defines[n[1]] = n[2]

    def execute(self, nodes, dot):
        scope = _Scope(dot)
        out = []
        self._exec(nodes, dot, scope, out)
        return "".join(out)

    def include(self, name, dot):
        if name not in self.defines:
            raise TemplateError(f"template {name!r} not defined")
        return self.execute(self.defines[name], dot)

    def _exec(self, nodes, dot, scope, out):
        for n in nodes:
            k = n[0]
            if k == "text":
                out.append(n[1])
            elif k == "define":
                continue
            elif k == "template":
                arg = self._pipeline(n[2], dot, scope) if n[2] else None
                out.append(self.include(n[1], arg))
            elif k == "action":
                v = self._pipeline(n[1], dot, scope)
                if n[1]["decl"] is None:
                    out.append(_go_str(v))
            elif k == "block":
                self._block(n[1], dot, scope, out)

    def _block(self, b, dot, scope, out):
        kind = b["kind"]
        scope.push()
        try:
            if kind == "range":
                self._range(b, dot, scope, out)
                return
            v = self._pipeline(b["pipe"], dot, scope)
            if _truthy(v):
                self._exec(b["body"], v if kind == "with" else dot, scope, out)
            elif b["else"] is not None:
                self._exec(b["else"], dot, scope, out)
        finally:
            scope.pop()

    def _range(self, b, dot, scope, out):
        pipe = dict(b["pipe"])
        names = pipe.get("decl")
        pipe["decl"] = None
        coll = self._pipeline(pipe, dot, scope)
        if isinstance(coll, dict):
            pairs = [(k, coll[k]) for k in sorted(coll)]
        elif isinstance(coll, (list, tuple)):
            pairs = list(enumerate(coll))
        elif coll is None:
            pairs = []
        elif isinstance(coll, (int, float)):
            pairs = [(i, i) for i in range(int(coll))]
        else:
            raise TemplateError(f"range can't iterate over {coll!r}")
        if not pairs:
            if b["else"] is not None:
                self._exec(b["else"], dot, scope, out)
            return
        for k, v in pairs:
            if names:
                if len(names) == 1:
                    scope.declare(names[0], v)
                else:
                    scope.declare(names[0], k)
                    scope.declare(names[1], v)
            self._exec(b["body"], v, scope, out)

    # -- pipelines
    def _pipeline(self, pipe, dot, scope):
        val, have = None, False
        for cmd in pipe["cmds"]:
            val = self._command(cmd, dot, scope, val if have else _NOARG)
            have = True
        if pipe["decl"]:
            if pipe["assign"]:
                scope.assign(pipe["decl"][0], val)
            else:
                scope.declare(pipe["decl"][-1], val)
        return val

    def _operand(self, op, dot, scope):
        kind = op[0]
        if kind == "str":
            return json.loads(op[1])
        if kind == "raw":
            return op[1][1:-1]
        if kind == "num":
            return float(op[1]) if any(c in op[1] for c in ".eE") else int(op[1])
        if kind == "field":
            if op[1] == ".":
                return dot
            return _field(dot, op[1][1:].split("."), op[1])
        if kind == "var":
            name, *rest = op[1].split(".")
            return _field(scope.get(name), rest, op[1])
        if kind == "sub":
            v = self._pipeline(op[1], dot, scope)
            return _field(v, op[2][1:].split("."), op[2]) if op[2] else v
        if kind == "ident":
            if op[1] in ("true", "false"):
                return op[1] == "true"
            if op[1] == "nil":
                return None
            return self._call(op[1], [], dot, scope)
        raise TemplateError(f"unexpected operand {op}")

    def _command(self, cmd, dot, scope, piped):
        if not cmd:
            raise TemplateError("empty command")
        head = cmd[0]
        if head[0] == "ident" and head[1] not in ("true", "false", "nil"):
            args = [self._operand(a, dot, scope) for a in cmd[1:]]
            if piped is not _NOARG:
                args.append(piped)
            return self._call(head[1], args, dot, scope)
        if len(cmd) > 1 or piped is not _NOARG:
            # a method on an object, as .Files.Get "path"
            fn = self._operand(head, dot, scope) if head[0] in ("field", "chain", "var") else None
            if callable(fn):
                args = [self._operand(a, dot, scope) for a in cmd[1:]]
                if piped is not _NOARG:
                    args.append(piped)
                return fn(*args)
            raise TemplateError(f"can't give argument to non-function {head[1]}")
        return self._operand(head, dot, scope)

    def _call(self, name, args, dot, scope):
        if name == "include":
            return self.include(args[0], args[1] if len(args) > 1 else None)
        f = self.funcs.get(name)
        if f is None:
            raise TemplateError(f"function {name!r} not defined")
        return f(*args)

    # -- function table
    def _funcs(self):
        def default(d, v=None):
            return v if _truthy(v) else d

        def quote(*a):
            return " ".join(json.dumps(_go_str(x), ensure_ascii=False) for x in a if x is not None)

        def squote(*a):
            return " ".join("'" + _go_str(x) + "'" for x in a if x is not None)

        def indent(n, s):
            pad = " " * int(n)
            return "\n".join(pad + line for line in _go_str(s).split("\n"))

        def nindent(n, s):
            return "\n" + indent(n, s)

        def trunc(n, s):
            s = _go_str(s)
            n = int(n)
            return s[:n] if n >= 0 else s[n:]

        def index(coll, *keys):
            for k in keys:
                if coll is None:
                    return None
                coll = coll.get(k) if isinstance(coll, dict) else coll[int(k)]
            return coll

        def dict_(*kv):
            if len(kv) % 2:
                raise TemplateError("dict needs an even number of arguments")
            return {_go_str(kv[i]): kv[i + 1] for i in range(0, len(kv), 2)}

        def required(msg, v=None):
            if v is None or v == "":
                raise TemplateError(msg)
            return v

        def eq(a, *bs):
            return any(a == b for b in bs)

        def and_(*a):
            for x in a:
                if not _truthy(x):
                    return x
            return a[-1]

        def or_(*a):
            for x in a:
                if _truthy(x):
                    return x
            return a[-1]

        def to_int(v):
            if isinstance(v, str):
                try:
                    return int(float(v))
                except ValueError:
                    return 0
            return int(v or 0)

        return {
            "default": default, "quote": quote, "squote": squote, "indent": indent, "nindent": nindent,
            "toYaml": _to_yaml, "toJson": lambda v: json.dumps(v, separators=(",", ":"), sort_keys=True),
            "trunc": trunc, "trimSuffix": lambda suf, s: _go_str(s)[:-len(suf)] if suf and _go_str(s).endswith(suf) else _go_str(s),
            "trimPrefix": lambda pre, s: _go_str(s)[len(pre):] if _go_str(s).startswith(pre) else _go_str(s),
            "trim": lambda s: _go_str(s).strip(),
            "replace": lambda old, new, s: _go_str(s).replace(old, new),
            "contains": lambda sub, s: sub in _go_str(s),
            "hasPrefix": lambda pre, s: _go_str(s).startswith(pre),
            "printf": lambda fmt, *a: _go_sprintf(fmt, a),
            "print": lambda *a: "".join(_go_str(x) for x in a),
            "join": lambda sep, lst: sep.join(_go_str(x) for x in (lst or [])),
            "list": lambda *a: list(a), "dict": dict_, "index": index,
            "kindIs": lambda kind, v: {"float64": isinstance(v, float), "int64": isinstance(v, int) and not isinstance(v, bool),
                                       "int": isinstance(v, int) and not isinstance(v, bool), "string": isinstance(v, str),
                                       "bool": isinstance(v, bool), "map": isinstance(v, dict),
                                       "slice": isinstance(v, list), "invalid": v is None}.get(kind, False),
            # sprig get: a missing key is "" (not nil)
            "get": lambda d, k: d.get(_go_str(k), "") if isinstance(d, dict) else "",
            "eq": eq, "ne": lambda a, b: a != b, "lt": lambda a, b: a < b, "le": lambda a, b: a <= b,
            "gt": lambda a, b: a > b, "ge": lambda a, b: a >= b,
            "and": and_, "or": or_, "not": lambda a: not _truthy(a),
            "int": to_int, "int64": to_int, "float64": lambda v: float(v), "toString": _go_str,
            "lower": lambda s: _go_str(s).lower(), "upper": lambda s: _go_str(s).upper(),
            "b64enc": lambda s: base64.b64encode(_go_str(s).encode()).decode(),
            "required": required, "empty": lambda v: not _truthy(v),
            "hasKey": lambda d, k: isinstance(d, dict) and k in d,
            "ternary": lambda a, b, c: a if _truthy(c) else b,
            "len": lambda v: len(v or []),
        }


class _NoArg:
    pass


_NOARG = _NoArg()


# ----------------------------------------------------------------------------- charts

def render_chart(chart_dir, values=None, release=None):
    """Render every template of `chart_dir` -> {template_path: rendered_text}."""
    with open(os.path.join(chart_dir, "Chart.yaml")) as f:
        chart = yaml.safe_load(f)
    with open(os.path.join(chart_dir, "values.yaml")) as f:
        base = yaml.safe_load(f) or {}
    vals = _floatify(_merge(base, values or {}))
    rel = {"Name": "bgc", "Namespace": "bgc-system", "Service": "Helm", "IsInstall": True, "IsUpgrade": False,
           "Revision": 1}
    rel.update(release or {})
    chart_obj = {"Name": chart["name"], "Version": chart["version"], "AppVersion": chart.get("appVersion", ""),
                 "Description": chart.get("description", "")}
    r = Renderer()
    tdir = os.path.join(chart_dir, "templates")
    parsed = {}
    for fn in sorted(os.listdir(tdir)):
        with open(os.path.join(tdir, fn)) as f:
            parsed[fn] = r.load(fn, f.read())
    def files_get(path):
        """Helm's .Files.Get: a chart file's text ("" when missing), never from templates/."""
        full = os.path.normpath(os.path.join(chart_dir, path))
        if not full.startswith(os.path.normpath(chart_dir) + os.sep) or not os.path.isfile(full):
            return ""
        with open(full) as f:
            return f.read()

    root = {"Values": vals, "Release": rel, "Chart": chart_obj, "Capabilities": {"KubeVersion": {"Version": "v1.30.0"}},
            "Template": {"BasePath": f"{chart['name']}/templates"}, "Files": {"Get": files_get}}
    out = {}
    for fn, nodes in parsed.items():
        if fn.startswith("_") or not fn.endswith((".yaml", ".yml", ".tpl")) or fn.endswith(".tpl"):
            continue
        root_fn = dict(root, Template={"Name": f"{chart['name']}/templates/{fn}", "BasePath": root["Template"]["BasePath"]})
        out[fn] = r.execute(nodes, root_fn)
    return out


def manifests(rendered):
    """Parse rendered templates into a list of Kubernetes objects (empty documents dropped)."""
    objs = []
    for fn, text in rendered.items():
        for doc in yaml.safe_load_all(text):
            if doc:
                doc.setdefault("__source__", fn)
                objs.append(doc)
    return objs
