"""The part of kubectl's JSONPath templates that scripts use: ``{.a.b[0].c}``, wildcards
``[*]`` / ``.*``, quoted keys ``['gpupool.amd.com/x']``, filters ``[?(@.type=="Ready")]``,
``{range .items[*]}...{end}`` and literal text (``{"\\n"}`` or plain) between expressions.
Results are printed as kubectl prints them: strings bare, several values space-separated, maps and
lists as JSON."""
from __future__ import annotations

import json
import re
from typing import Any

_TOKEN = re.compile(r"""
    \.(?P<name>[A-Za-z0-9_\-/$]+|\*)        # .name, .*
  | \[(?P<idx>-?\d+|\*)\]                  # [0], [-1], [*]
  | \[(?P<q>'[^']*'|"[^"]*")\]             # ['a.b/c']
  | \[\?\(@(?P<fpath>[^=!<>)]*)\s*(?P<op>==|!=)\s*(?P<fval>'[^']*'|"[^"]*"|[^)]+)\)\]
""", re.X)


class JsonPathError(ValueError):
    pass


def _steps(expr: str) -> list[tuple]:
    expr = expr.strip()
    if expr in ("", "."):
        return []
    if not expr.startswith((".", "[")):
        expr = "." + expr
    out, pos = [], 0
    while pos < len(expr):
        m = _TOKEN.match(expr, pos)
        if not m:
            raise JsonPathError(f"unsupported JSONPath at {expr[pos:]!r}")
        if m.group("name") is not None:
            out.append(("key", m.group("name")))
        elif m.group("idx") is not None:
            out.append(("idx", m.group("idx")))
        elif m.group("q") is not None:
            out.append(("key", m.group("q")[1:-1]))
        else:
            val = m.group("fval").strip()
            if val[:1] in "'\"":
                val = val[1:-1]
            out.append(("filter", _steps(m.group("fpath") or ""), m.group("op"), val))
        pos = m.end()
    return out


def _apply(values: list, step: tuple) -> list:
    out = []
    for v in values:
        if step[0] == "key":
            if step[1] == "*":
                out += list(v.values()) if isinstance(v, dict) else (v if isinstance(v, list) else [])
            elif isinstance(v, dict) and step[1] in v:
                out.append(v[step[1]])
        elif step[0] == "idx":
            if not isinstance(v, list):
                continue
            if step[1] == "*":
                out += v
            else:
                i = int(step[1])
                if -len(v) <= i < len(v):
                    out.append(v[i])
        else:  # filter over a list's elements
            _, sub, op, want = step
            for e in (v if isinstance(v, list) else []):
                got = evaluate(e, sub)
                hit = any(_str(g) == want for g in got)
                if hit == (op == "=="):
                    out.append(e)
    return out


def evaluate(obj: Any, steps: list[tuple] | str) -> list:
    if isinstance(steps, str):
        steps = _steps(steps)
    vals = [obj]
    for st in steps:
        vals = _apply(vals, st)
    return vals


def _str(v: Any) -> str:
    if isinstance(v, str):
        return v
    if isinstance(v, bool):
        return "true" if v else "false"
    if v is None:
        return ""
    if isinstance(v, (dict, list)):
        return json.dumps(v, separators=(",", ":"))
    return str(v)


def _parse_template(tpl: str) -> list:
    """[("text", s) | ("expr", steps) | ("range", steps, body) ]"""
    parts: list = []
    stack: list[list] = [parts]
    pos = 0
    while pos < len(tpl):
        i = tpl.find("{", pos)
        if i < 0:
            stack[-1].append(("text", tpl[pos:]))
            break
        if i > pos:
            stack[-1].append(("text", tpl[pos:i]))
        j = tpl.find("}", i)
        if j < 0:
            raise JsonPathError(f"unclosed {{ in {tpl!r}")
        inner = tpl[i + 1:j].strip()
        if inner.startswith("range "):
            body: list = []
            stack[-1].append(("range", _steps(inner[6:]), body))
            stack.append(body)
        elif inner == "end":
            if len(stack) == 1:
                raise JsonPathError("{end} without {range}")
            stack.pop()
        elif inner[:1] in "'\"":
            stack[-1].append(("text", json.loads(inner) if inner[0] == '"' else inner[1:-1]))
        else:
            stack[-1].append(("expr", _steps(inner)))
        pos = j + 1
    if len(stack) != 1:
        raise JsonPathError("{range} without {end}")
    return parts


def render(obj: Any, template: str) -> str:
    """``kubectl get -o jsonpath=TEMPLATE``."""
    def run(parts: list, cur: Any) -> str:
        out = []
        for p in parts:
            if p[0] == "text":
                out.append(p[1])
            elif p[0] == "expr":
                out.append(" ".join(_str(v) for v in evaluate(cur, p[1])))
            else:
                for item in evaluate(cur, p[1]):
                    out.append(run(p[2], item))
        return "".join(out)
    return run(_parse_template(template), obj)
