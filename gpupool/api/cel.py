"""The subset of CEL that the CRDs' ``x-kubernetes-validations`` rules use, for apiserver-sim.

A real kube-apiserver compiles these rules (Common Expression Language) and rejects a write that
breaks one, with the rule's message; apiserver-sim evaluates them with this interpreter so the
tests see the same admission behaviour. Supported: ``self`` and member access, ``has(x.f)``,
``size(x)``, int / double / string / bool / null literals, ``! - * / % + - < <= > >= == != in &&
|| ?:`` and parentheses — with CEL's semantics where they differ from Python's: ``&&`` / ``||``
tolerate an error on one side when the other decides the result, integer division truncates
toward zero, and a missing field is an error (``no such key``) unless tested with ``has()``.
"""
from __future__ import annotations

import re
from typing import Any

_TOK = re.compile(r"""
    \s*(?:
      (?P<num>\d+\.\d+|\d+)
    | (?P<str>"(?:[^"\\]|\\.)*"|'(?:[^'\\]|\\.)*')
    | (?P<op>\|\||&&|==|!=|<=|>=|[-+*/%<>!?:().,\[\]])
    | (?P<id>[A-Za-z_][A-Za-z0-9_]*)
    )""", re.X)


class CelError(Exception):
    pass


def _lex(src: str) -> list[tuple[str, Any]]:
    out, pos = [], 0
    src = src.rstrip()
    while pos < len(src):
        m = _TOK.match(src, pos)
        if not m or m.end() == pos:
            raise CelError(f"unexpected character at {pos}: {src[pos:pos + 10]!r}")
        pos = m.end()
        if m.group("num"):
            t = m.group("num")
            out.append(("num", float(t) if "." in t else int(t)))
        elif m.group("str"):
            out.append(("str", bytes(m.group("str")[1:-1], "utf-8").decode("unicode_escape")))
        elif m.group("op"):
            out.append(("op", m.group("op")))
        else:
            out.append(("id", m.group("id")))
    out.append(("end", None))
    return out


_BIN = {"||": 1, "&&": 2, "==": 3, "!=": 3, "<": 3, "<=": 3, ">": 3, ">=": 3, "in": 3,
        "+": 4, "-": 4, "*": 5, "/": 5, "%": 5}


class _Parser:
    """Pratt parser to a small AST of tuples."""

    def __init__(self, src: str):
        self.t = _lex(src)
        self.i = 0

    def peek(self):
        return self.t[self.i]

    def take(self, kind=None, val=None):
        k, v = self.t[self.i]
        if (kind and k != kind) or (val is not None and v != val):
            raise CelError(f"expected {val or kind}, got {v!r}")
        self.i += 1
        return v

    def parse(self):
        e = self.expr()
        self.take("end")
        return e

    def expr(self):
        cond = self.binary(1)
        if self.peek() == ("op", "?"):
            self.take()
            a = self.expr()
            self.take("op", ":")
            b = self.expr()
            return ("?:", cond, a, b)
        return cond

    def binary(self, minp):
        left = self.unary()
        while True:
            k, v = self.peek()
            op = v if k in ("op", "id") else None
            p = _BIN.get(op) if op is not None else None
            if p is None or p < minp:
                return left
            self.take()
            right = self.binary(p + 1)
            left = ("bin", op, left, right)

    def unary(self):
        k, v = self.peek()
        if k == "op" and v in ("!", "-"):
            self.take()
            return ("un", v, self.unary())
        return self.postfix(self.primary())

    def primary(self):
        k, v = self.peek()
        self.take()
        if k in ("num", "str"):
            return ("lit", v)
        if k == "id":
            if v in ("true", "false"):
                return ("lit", v == "true")
            if v == "null":
                return ("lit", None)
            if self.peek() == ("op", "("):  # a call: has(x.f), size(x)
                self.take()
                arg = self.expr()
                self.take("op", ")")
                if v not in ("has", "size", "int", "double", "string"):
                    raise CelError(f"unsupported function {v}")
                if v == "has" and arg[0] != "sel":
                    raise CelError("has() needs a field selection")
                return ("call", v, arg)
            return ("id", v)
        if (k, v) == ("op", "("):
            e = self.expr()
            self.take("op", ")")
            return e
        raise CelError(f"unexpected {v!r}")

    def postfix(self, e):
        while True:
            if self.peek() == ("op", "."):
                self.take()
                e = ("sel", e, self.take("id"))
            elif self.peek() == ("op", "["):
                self.take()
                idx = self.expr()
                self.take("op", "]")
                e = ("idx", e, idx)
            else:
                return e


_cache: dict[str, tuple] = {}


def compile_rule(src: str) -> tuple:
    ast = _cache.get(src)
    if ast is None:
        ast = _cache[src] = _Parser(src).parse()
    return ast


def evaluate(src_or_ast: Any, self_value: Any) -> Any:
    ast = compile_rule(src_or_ast) if isinstance(src_or_ast, str) else src_or_ast
    return _eval(ast, {"self": self_value})


def _eval(n: tuple, env: dict) -> Any:
    kind = n[0]
    if kind == "lit":
        return n[1]
    if kind == "id":
        if n[1] not in env:
            raise CelError(f"undeclared reference to {n[1]!r}")
        return env[n[1]]
    if kind == "sel":
        base = _eval(n[1], env)
        if not isinstance(base, dict) or n[2] not in base:
            raise CelError(f"no such key: {n[2]}")
        return base[n[2]]
    if kind == "idx":
        base, i = _eval(n[1], env), _eval(n[2], env)
        try:
            return base[i]
        except (KeyError, IndexError, TypeError):
            raise CelError(f"no such key: {i!r}") from None
    if kind == "call":
        fn, arg = n[1], n[2]
        if fn == "has":
            base = _eval(arg[1], env)
            return isinstance(base, dict) and arg[2] in base
        v = _eval(arg, env)
        if fn == "size":
            if not isinstance(v, (str, list, dict)):
                raise CelError("size() of a non-collection")
            return len(v)
        return {"int": int, "double": float, "string": str}[fn](v)
    if kind == "un":
        v = _eval(n[2], env)
        if n[1] == "!":
            if not isinstance(v, bool):
                raise CelError("! of a non-bool")
            return not v
        return -v
    if kind == "?:":
        c = _eval(n[1], env)
        if not isinstance(c, bool):
            raise CelError("?: condition is not a bool")
        return _eval(n[2] if c else n[3], env)
    op, a_n, b_n = n[1], n[2], n[3]
    if op in ("&&", "||"):  # commutative short-circuit with error absorption (CEL)
        try:
            a = _eval(a_n, env)
            a_err = None
        except CelError as e:
            a, a_err = None, e
        if a_err is None:
            if not isinstance(a, bool):
                raise CelError(f"{op} of a non-bool")
            if (op == "&&" and not a) or (op == "||" and a):
                return a
        b = _eval(b_n, env)
        if not isinstance(b, bool):
            raise CelError(f"{op} of a non-bool")
        if (op == "&&" and not b) or (op == "||" and b):
            return b
        if a_err is not None:
            raise a_err
        return b
    a, b = _eval(a_n, env), _eval(b_n, env)
    if op == "==":
        return a == b
    if op == "!=":
        return a != b
    if op == "in":
        return a in b
    num = (int, float)
    if op in ("<", "<=", ">", ">="):
        if not (isinstance(a, num) and isinstance(b, num)) and not (isinstance(a, str) and
                                                                     isinstance(b, str)):
            raise CelError(f"no such overload: {type(a).__name__} {op} {type(b).__name__}")
        return {"<": a < b, "<=": a <= b, ">": a > b, ">=": a >= b}[op]
    if op == "+" and isinstance(a, (str, list)) and type(a) is type(b):
        return a + b
    if not (isinstance(a, num) and isinstance(b, num)) or isinstance(a, bool) or isinstance(b, bool):
        raise CelError(f"no such overload: {type(a).__name__} {op} {type(b).__name__}")
    if op == "+":
        return a + b
    if op == "-":
        return a - b
    if op == "*":
        return a * b
    if b == 0:
        raise CelError("division by zero")
    if op == "/":
        return int(a / b) if isinstance(a, int) and isinstance(b, int) else a / b
    return int(a - b * int(a / b)) if isinstance(a, int) and isinstance(b, int) else a % b
