"""Minimal Helm template renderer (the subset this chart uses), for render tests.

No ``helm`` binary exists offline, so the chart in ``deploy/helm`` is rendered by
this engine in tests (``tests/test_deploy.py``): Go ``text/template`` actions
``{{ }}`` with ``{{-``/``-}}`` trimming, ``if/else if/else``, ``range`` (lists and
maps, with ``$k, $v :=``), ``with``, ``define``/``include``/``template``,
variables (``$``, ``$x := …``), pipelines, and the Sprig functions the chart
calls: ``default quote toYaml nindent indent trunc trimSuffix printf eq ne not
and or required b64enc lower upper replace hasKey toString int``.

``python deploy/render.py deploy/helm/nexus-supervisor-amd [-f values.yaml] [--set a.b=c]``
"""
from __future__ import annotations

import base64
import os
import re
import sys
from typing import Any, Dict, List, Optional, Tuple

import yaml

_TOKEN = re.compile(r"{{(-?)\s*(.*?)\s*(-?)}}", re.S)


class TemplateError(Exception):
    pass


# ------------------------------------------------------------------ parsing
class Node:
    pass


class Text(Node):
    def __init__(self, s):
        self.s = s


class Action(Node):
    def __init__(self, expr):
        self.expr = expr


class If(Node):
    def __init__(self):
        self.branches: List[Tuple[Optional[str], List[Node]]] = []


class Range(Node):
    def __init__(self, vars_, expr):
        self.vars = vars_
        self.expr = expr
        self.body: List[Node] = []
        self.else_body: List[Node] = []


class With(Node):
    def __init__(self, expr):
        self.expr = expr
        self.body: List[Node] = []
        self.else_body: List[Node] = []


class Define(Node):
    def __init__(self, name):
        self.name = name
        self.body: List[Node] = []


def _lex(src: str) -> List[Tuple[str, str]]:
    out: List[Tuple[str, str]] = []
    pos = 0
    for m in _TOKEN.finditer(src):
        text = src[pos:m.start()]
        if m.group(1):
            text = text.rstrip()
        if out and out[-1][0] == "trim_next":
            out.pop()
            text = text.lstrip()
        out.append(("text", text))
        body = m.group(2)
        if body.startswith("/*"):
            pass
        else:
            out.append(("action", body))
        if m.group(3):
            out.append(("trim_next", ""))
        pos = m.end()
    text = src[pos:]
    if out and out[-1][0] == "trim_next":
        out.pop()
        text = text.lstrip()
    out.append(("text", text))
    return out


def parse(src: str) -> Tuple[List[Node], Dict[str, List[Node]]]:
    toks = _lex(src)
    defines: Dict[str, List[Node]] = {}
    root: List[Node] = []
    stack: List[Tuple[Node, List[Node]]] = []
    cur = root
    for kind, val in toks:
        if kind == "text":
            if val:
                cur.append(Text(val))
            continue
        word = val.split(None, 1)
        head = word[0] if word else ""
        rest = word[1] if len(word) > 1 else ""
        if head == "if":
            n = If()
            n.branches.append((rest, []))
            cur.append(n)
            stack.append((n, cur))
            cur = n.branches[-1][1]
        elif head == "else":
            n, parent = stack[-1]
            if isinstance(n, If):
                cond = rest[3:].strip() if rest.startswith("if ") else None
                n.branches.append((cond, []))
                cur = n.branches[-1][1]
            elif isinstance(n, (Range, With)):
                cur = n.else_body
            else:
                raise TemplateError("else outside if/range/with")
        elif head == "range":
            m = re.match(r"(\$\w+)\s*(?:,\s*(\$\w+))?\s*:=\s*(.*)", rest)
            if m:
                n = Range([v for v in (m.group(1), m.group(2)) if v], m.group(3))
            else:
                n = Range([], rest)
            cur.append(n)
            stack.append((n, cur))
            cur = n.body
        elif head == "with":
            n = With(rest)
            cur.append(n)
            stack.append((n, cur))
            cur = n.body
        elif head == "define":
            name = rest.strip().strip('"')
            n = Define(name)
            stack.append((n, cur))
            cur = n.body
        elif head == "end":
            n, parent = stack.pop()
            if isinstance(n, Define):
                defines[n.name] = n.body
            cur = parent
        else:
            cur.append(Action(val))
    if stack:
        raise TemplateError("unclosed block")
    return root, defines


# ------------------------------------------------------------------ evaluation
def _to_yaml(v) -> str:
    if v is None or v == {} or v == []:
        return "{}" if isinstance(v, dict) else ("[]" if isinstance(v, list) else "")
    return yaml.safe_dump(v, default_flow_style=False, sort_keys=True).rstrip("\n")


def _truthy(v) -> bool:
    return bool(v) and v != 0


def _indent(n, s):
    pad = " " * int(n)
    return "\n".join(pad + line if line else line for line in str(s).split("\n"))


FUNCS = {
    "default": lambda d, v=None: v if _truthy(v) else d,
    "quote": lambda v="": '"' + str("" if v is None else v).replace('"', '\\"') + '"',
    "squote": lambda v="": "'" + str(v) + "'",
    "toYaml": _to_yaml,
    "nindent": lambda n, s: "\n" + _indent(n, s),
    "indent": _indent,
    "trunc": lambda n, s: str(s)[: int(n)],
    "trimSuffix": lambda suf, s: str(s)[: -len(suf)] if suf and str(s).endswith(suf) else str(s),
    "printf": lambda fmt, *a: re.sub(r"%[vsd]", "{}", fmt).format(*a),
    "eq": lambda a, b: a == b,
    "ne": lambda a, b: a != b,
    "gt": lambda a, b: a > b,
    "lt": lambda a, b: a < b,
    "not": lambda a: not _truthy(a),
    "and": lambda *a: all(_truthy(x) for x in a),
    "or": lambda *a: next((x for x in a if _truthy(x)), a[-1] if a else None),
    "b64enc": lambda s: base64.b64encode(str(s).encode()).decode(),
    "lower": lambda s: str(s).lower(),
    "upper": lambda s: str(s).upper(),
    "replace": lambda old, new, s: str(s).replace(old, new),
    "hasKey": lambda d, k: isinstance(d, dict) and k in d,
    "toString": lambda v: str(v),
    "int": lambda v: int(v),
    "join": lambda sep, lst: sep.join(str(x) for x in (lst or [])),
}


class Renderer:
    def __init__(self, defines: Dict[str, List[Node]]):
        self.defines = defines

    def _split_pipeline(self, expr: str) -> List[str]:
        parts, depth, cur, q = [], 0, "", None
        for ch in expr:
            if q:
                cur += ch
                if ch == q:
                    q = None
                continue
            if ch in "\"`":
                q = ch
                cur += ch
            elif ch == "(":
                depth += 1
                cur += ch
            elif ch == ")":
                depth -= 1
                cur += ch
            elif ch == "|" and depth == 0:
                parts.append(cur.strip())
                cur = ""
            else:
                cur += ch
        parts.append(cur.strip())
        return parts

    def _args(self, s: str) -> List[str]:
        out, cur, depth, q = [], "", 0, None
        for ch in s:
            if q:
                cur += ch
                if ch == q:
                    q = None
                continue
            if ch in "\"`":
                q = ch
                cur += ch
            elif ch == "(":
                depth += 1
                cur += ch
            elif ch == ")":
                depth -= 1
                cur += ch
            elif ch.isspace() and depth == 0:
                if cur:
                    out.append(cur)
                cur = ""
            else:
                cur += ch
        if cur:
            out.append(cur)
        return out

    def _atom(self, a: str, dot, scope):
        if a.startswith("(") and a.endswith(")"):
            return self.eval(a[1:-1], dot, scope)
        if a[0] in "\"`":
            return a[1:-1].replace('\\"', '"') if a[0] == '"' else a[1:-1]
        if re.fullmatch(r"-?\d+", a):
            return int(a)
        if a in ("true", "false"):
            return a == "true"
        if a == "nil":
            return None
        if a == ".":
            return dot
        if a.startswith("$"):
            name, _, path = a.partition(".")
            base = scope[name] if name in scope else scope["$"] if name == "$" else None
            if name not in scope:
                raise TemplateError(f"undefined variable {name}")
            return self._path(base, path)
        if a.startswith("."):
            return self._path(dot, a[1:])
        raise TemplateError(f"cannot evaluate {a!r}")

    @staticmethod
    def _path(obj, path: str):
        for part in filter(None, path.split(".")):
            if isinstance(obj, dict):
                obj = obj.get(part)
            else:
                return None
        return obj

    def _call(self, cmd: str, dot, scope, piped=None, has_piped=False):
        args = self._args(cmd)
        if not args:
            return piped
        head = args[0]
        if head in ("include", "template"):
            name = self._atom(args[1], dot, scope)
            ctx = self._atom(args[2], dot, scope) if len(args) > 2 else dot
            if name not in self.defines:
                raise TemplateError(f"no template {name!r}")
            return self.render(self.defines[name], ctx, {"$": scope["$"]})
        if head == "required":
            msg = self._atom(args[1], dot, scope)
            v = piped if has_piped else self._atom(args[2], dot, scope)
            if v in (None, ""):
                raise TemplateError(msg)
            return v
        if head in FUNCS:
            vals = [self._atom(x, dot, scope) for x in args[1:]]
            if has_piped:
                vals.append(piped)
            return FUNCS[head](*vals)
        if len(args) == 1:
            return self._atom(head, dot, scope)
        raise TemplateError(f"unknown function {head!r}")

    def eval(self, expr: str, dot, scope):
        m = re.match(r"(\$\w+)\s*(?::=|=)\s*(.*)", expr, re.S)
        if m:
            scope[m.group(1)] = self.eval(m.group(2), dot, scope)
            return ""
        val = None
        has = False
        for i, cmd in enumerate(self._split_pipeline(expr)):
            val = self._call(cmd, dot, scope, val, has)
            has = True
        return val

    def render(self, nodes: List[Node], dot, scope) -> str:
        out = []
        for n in nodes:
            if isinstance(n, Text):
                out.append(n.s)
            elif isinstance(n, Action):
                v = self.eval(n.expr, dot, scope)
                out.append("" if v is None else (v if isinstance(v, str) else _go_str(v)))
            elif isinstance(n, If):
                for cond, body in n.branches:
                    if cond is None or _truthy(self.eval(cond, dot, scope)):
                        out.append(self.render(body, dot, scope))
                        break
            elif isinstance(n, Range):
                coll = self.eval(n.expr, dot, scope)
                items = list(coll.items()) if isinstance(coll, dict) else list(enumerate(coll or []))
                if isinstance(coll, dict):
                    items.sort(key=lambda kv: kv[0])
                if not items:
                    out.append(self.render(n.else_body, dot, scope))
                for k, v in items:
                    sc = dict(scope)
                    if len(n.vars) == 2:
                        sc[n.vars[0]], sc[n.vars[1]] = k, v
                    elif len(n.vars) == 1:
                        sc[n.vars[0]] = v
                    out.append(self.render(n.body, v, sc))
            elif isinstance(n, With):
                v = self.eval(n.expr, dot, scope)
                out.append(self.render(n.body, v, scope) if _truthy(v) else self.render(n.else_body, dot, scope))
        return "".join(out)


def _go_str(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (dict, list)):
        return _to_yaml(v)
    return str(v)


def _deep_merge(a: Dict[str, Any], b: Dict[str, Any]) -> Dict[str, Any]:
    out = dict(a)
    for k, v in b.items():
        out[k] = _deep_merge(out[k], v) if isinstance(v, dict) and isinstance(out.get(k), dict) else v
    return out


def _set(values: Dict[str, Any], expr: str) -> None:
    key, _, raw = expr.partition("=")
    val: Any = yaml.safe_load(raw) if raw else ""
    cur = values
    parts = key.split(".")
    for p in parts[:-1]:
        cur = cur.setdefault(p, {})
    cur[parts[-1]] = val


def render_chart(chart_dir: str, values: Optional[Dict[str, Any]] = None, sets: Optional[List[str]] = None,
                 release: str = "nexus-supervisor", namespace: str = "nexus") -> Dict[str, str]:
    """Render every template; returns ``{template path: text}`` (helpers omitted)."""
    with open(os.path.join(chart_dir, "Chart.yaml")) as f:
        chart = yaml.safe_load(f)
    with open(os.path.join(chart_dir, "values.yaml")) as f:
        vals = yaml.safe_load(f) or {}
    if values:
        vals = _deep_merge(vals, values)
    for s in sets or []:
        _set(vals, s)
    tdir = os.path.join(chart_dir, "templates")
    files = sorted(os.listdir(tdir))
    defines: Dict[str, List[Node]] = {}
    parsed = {}
    for fn in files:
        with open(os.path.join(tdir, fn)) as f:
            nodes, d = parse(f.read())
        defines.update(d)
        parsed[fn] = nodes
    root = {"Values": vals, "Release": {"Name": release, "Namespace": namespace, "Service": "Helm"},
            "Chart": {"Name": chart["name"], "Version": chart["version"], "AppVersion": chart.get("appVersion", "")}}
    r = Renderer(defines)
    out = {}
    for fn, nodes in parsed.items():
        if fn.startswith("_"):
            continue
        out[fn] = r.render(nodes, root, {"$": root})
    return out


def render_docs(chart_dir: str, **kw) -> List[Dict[str, Any]]:
    docs = []
    for text in render_chart(chart_dir, **kw).values():
        for d in yaml.safe_load_all(text):
            if d:
                docs.append(d)
    return docs


def main(argv=None) -> int:
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("chart")
    ap.add_argument("-f", "--values")
    ap.add_argument("--set", action="append", default=[])
    a = ap.parse_args(argv)
    vals = None
    if a.values:
        with open(a.values) as f:
            vals = yaml.safe_load(f)
    for name, text in render_chart(a.chart, vals, a.set).items():
        if text.strip():
            print(f"---\n# Source: {name}\n{text.strip()}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
