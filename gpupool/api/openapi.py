"""Structural OpenAPI v3 subset: validation, defaulting and pruning of custom resources.

This is what kube-apiserver does for a CRD with a structural schema; the apiserver-sim applies it
on every create/update so that e.g. ``replicas: -1`` is rejected at admission exactly as the
reference's ``+kubebuilder:validation:Minimum=0`` marker would (README.md:94-95).

Supported keywords: type, properties, required, additionalProperties (schema form), items,
enum, minimum, maximum, minLength, maxLength, pattern, minItems, maxItems, default, nullable,
x-kubernetes-preserve-unknown-fields, x-kubernetes-list-type=map + list-map-keys (uniqueness),
x-kubernetes-validations (CEL rules, the subset gpupool/api/cel.py interprets).

A schema is compiled once into nested checker closures (cached per schema object), so a write
pays only the checks its schema has — no keyword lookups per node — and a field path is rendered
only for a field that fails (the pool status of an 8-GPU pool is a few hundred nodes, validated on
every status write).
"""
from __future__ import annotations

import copy
import re
from typing import Any, Callable

_TYPE_CHECK = {
    "string": lambda v: isinstance(v, str),
    "integer": lambda v: isinstance(v, int) and not isinstance(v, bool),
    "number": lambda v: isinstance(v, (int, float)) and not isinstance(v, bool),
    "boolean": lambda v: isinstance(v, bool),
    "object": lambda v: isinstance(v, dict),
    "array": lambda v: isinstance(v, list),
}

_RE_CACHE: dict[str, re.Pattern] = {}


def _re(p: str) -> re.Pattern:
    r = _RE_CACHE.get(p)
    if r is None:
        r = _RE_CACHE[p] = re.compile(p)
    return r


def apply_defaults(obj: Any, schema: dict) -> Any:
    """Fill ``default`` values top-down (defaults of a defaulted object are applied too)."""
    fn = _cached(_DEFAULTS, schema, _build_defaults)
    return obj if fn is None else fn(obj)


def prune(obj: Any, schema: dict) -> Any:
    """Drop fields not in the schema (structural-schema pruning), in place."""
    fn = _cached(_PRUNE, schema, _build_prune)
    return obj if fn is None else fn(obj)


# Both walks are compiled once per schema into closures over only the subtrees that can change
# something (``None`` = nothing below this schema is defaulted / can be pruned): a write's pool
# status, hundreds of nodes without defaults, is not walked at all.
_DEFAULTS: dict[int, tuple[Any, Any]] = {}
_PRUNE: dict[int, tuple[Any, Any]] = {}


def _cached(cache: dict, s: Any, build: Callable) -> Any:
    if not isinstance(s, dict):
        return None
    hit = cache.get(id(s))
    if hit is not None and hit[0] is s:
        return hit[1]
    fn = build(s)
    cache[id(s)] = (s, fn)  # keeps ``s`` alive: its id is never reused for another schema
    return fn


def _build_defaults(s: dict) -> Callable | None:
    if s.get("type") == "object":
        props = s.get("properties") or {}
        fill = [(k, sub["default"]) for k, sub in props.items()
                if isinstance(sub, dict) and "default" in sub]
        kids = [(k, f) for k, f in ((k, _cached(_DEFAULTS, sub, _build_defaults))
                                    for k, sub in props.items()) if f is not None]
        ap = s.get("additionalProperties")
        ap_f = _cached(_DEFAULTS, ap, _build_defaults) if isinstance(ap, dict) else None
        if not fill and not kids and ap_f is None:
            return None

        def f_obj(v):
            if not isinstance(v, dict):
                return v
            for k, d in fill:
                if k not in v:
                    v[k] = copy.deepcopy(d)
            for k, f in kids:
                if k in v:
                    v[k] = f(v[k])
            if ap_f is not None:
                for k in list(v):
                    if k not in props:
                        v[k] = ap_f(v[k])
            return v
        return f_obj
    items = s.get("items")
    if isinstance(items, dict):
        it_f = _cached(_DEFAULTS, items, _build_defaults)
        if it_f is None:
            return None

        def f_arr(v):
            return [it_f(x) for x in v] if isinstance(v, list) else v
        return f_arr
    return None


def _build_prune(s: dict) -> Callable | None:
    if s.get("x-kubernetes-preserve-unknown-fields"):
        return None
    if s.get("type") == "object":
        props = s.get("properties")
        ap = s.get("additionalProperties")
        if props is None and ap is None:
            return None  # free-form object (e.g. metadata)
        props = props or {}
        closed = not (ap is True or isinstance(ap, dict))  # unknown keys are dropped
        kids = [(k, f) for k, f in ((k, _cached(_PRUNE, sub, _build_prune))
                                    for k, sub in props.items()) if f is not None]
        ap_f = _cached(_PRUNE, ap, _build_prune) if isinstance(ap, dict) else None

        def p_obj(v):
            if not isinstance(v, dict):
                return v
            if closed:
                for k in [k for k in v if k not in props]:
                    del v[k]
            for k, f in kids:
                if k in v:
                    v[k] = f(v[k])
            if ap_f is not None:
                for k in list(v):
                    if k not in props:
                        v[k] = ap_f(v[k])
            return v
        return p_obj
    items = s.get("items")
    if isinstance(items, dict):
        it_f = _cached(_PRUNE, items, _build_prune)
        if it_f is None:
            return None

        def p_arr(v):
            return [it_f(x) for x in v] if isinstance(v, list) else v
        return p_arr
    return None


# ---------------------------------------------------------------- validation
# A field path is a linked chain (parent, key): key str -> ".key", int -> "[i]"; built as the
# checkers descend (one small tuple per node) and rendered only when a check fails.
Trail = tuple
Check = Callable[[Any, Trail, list], None]


def _render(trail: Trail) -> str:
    parts = []
    while len(trail) == 2:
        trail, key = trail
        parts.append(f"[{key}]" if isinstance(key, int) else f".{key}")
    return trail[0] + "".join(reversed(parts))


_COMPILED: dict[int, tuple[dict, Check]] = {}


def _noop(v: Any, trail: Trail, errs: list) -> None:
    return None


def _compile(s: Any) -> Check:
    if not isinstance(s, dict):
        return _noop
    hit = _COMPILED.get(id(s))
    if hit is not None and hit[0] is s:
        return hit[1]
    fn = _build(s)
    _COMPILED[id(s)] = (s, fn)  # keeps ``s`` alive: its id is never reused for another schema
    return fn


def _build(s: dict) -> Check:
    t = s.get("type")
    nullable = bool(s.get("nullable"))
    tcheck = _TYPE_CHECK[t] if t else None
    checks: list[Check] = []

    if "enum" in s:
        enum = s["enum"]
        allowed = ", ".join(f'"{e}"' for e in enum)

        def c_enum(v, trail, errs):
            if v not in enum:
                errs.append(f"{_render(trail)}: Unsupported value: {_short(v)}: supported values: "
                            f"{allowed}")
        checks.append(c_enum)
    if t in ("integer", "number"):
        if "minimum" in s:
            lo = s["minimum"]

            def c_min(v, trail, errs):
                if v < lo:
                    p = _render(trail)
                    errs.append(f"{p}: Invalid value: {v}: {p} in body should be greater than or "
                                f"equal to {lo}")
            checks.append(c_min)
        if "maximum" in s:
            hi = s["maximum"]

            def c_max(v, trail, errs):
                if v > hi:
                    p = _render(trail)
                    errs.append(f"{p}: Invalid value: {v}: {p} in body should be less than or "
                                f"equal to {hi}")
            checks.append(c_max)
    elif t == "string":
        if "minLength" in s:
            mn = s["minLength"]

            def c_minlen(v, trail, errs):
                if len(v) < mn:
                    errs.append(f"{_render(trail)}: Invalid value: {_short(v)}: should be at least "
                                f"{mn} chars long")
            checks.append(c_minlen)
        if "maxLength" in s:
            mx = s["maxLength"]

            def c_maxlen(v, trail, errs):
                if len(v) > mx:
                    errs.append(f"{_render(trail)}: Too long: may not be longer than {mx}")
            checks.append(c_maxlen)
        if "pattern" in s:
            pat = s["pattern"]
            rx = _re(pat)

            def c_pat(v, trail, errs):
                if not rx.search(v):
                    p = _render(trail)
                    errs.append(f"{p}: Invalid value: {_short(v)}: {p} in body should match "
                                f"'{pat}'")
            checks.append(c_pat)
    elif t == "object":
        required = list(s.get("required", []))
        props = {k: _compile(sub) for k, sub in (s.get("properties") or {}).items()}
        ap = s.get("additionalProperties")
        ap_c = _compile(ap) if isinstance(ap, dict) else None

        def c_obj(v, trail, errs):
            for r in required:
                if r not in v:
                    errs.append(f"{_render((trail, r))}: Required value")
            for k, sub in v.items():
                c = props.get(k)
                if c is not None:
                    c(sub, (trail, k), errs)
                elif ap_c is not None:
                    ap_c(sub, (trail, k), errs)
        checks.append(c_obj)
    elif t == "array":
        if "minItems" in s:
            mni = s["minItems"]

            def c_minitems(v, trail, errs):
                if len(v) < mni:
                    errs.append(f"{_render(trail)}: Invalid value: should have at least {mni} items")
            checks.append(c_minitems)
        if "maxItems" in s:
            mxi = s["maxItems"]

            def c_maxitems(v, trail, errs):
                if len(v) > mxi:
                    errs.append(f"{_render(trail)}: Too many: {len(v)}: must have at most {mxi} "
                                f"items")
            checks.append(c_maxitems)
        item_c = _compile(s.get("items"))
        if item_c is not _noop:
            def c_items(v, trail, errs):
                for i, x in enumerate(v):
                    item_c(x, (trail, i), errs)
            checks.append(c_items)
        if s.get("x-kubernetes-list-type") == "map":
            keys = list(s.get("x-kubernetes-list-map-keys", []))

            def c_listmap(v, trail, errs):
                seen = set()
                for i, x in enumerate(v):
                    if isinstance(x, dict):
                        key = tuple(x.get(k) for k in keys)
                        hk = repr(key)  # a mistyped key (a list) must not make this a 500
                        if hk in seen:
                            errs.append(f"{_render((trail, i))}: Duplicate value: "
                                        f"{dict(zip(keys, key))}")
                        seen.add(hk)
            checks.append(c_listmap)

    if s.get("x-kubernetes-validations"):
        # CEL rules (apiserver-side cross-field validation), run once the node's own schema
        # checks passed, with ``self`` bound to the node (gpupool/api/cel.py)
        from . import cel
        rules = [(r["rule"], cel.compile_rule(r["rule"]), r.get("message") or
                  f"failed rule: {r['rule']}") for r in s["x-kubernetes-validations"]]

        def c_cel(v, trail, errs):
            for src, ast, msg in rules:
                try:
                    ok = cel.evaluate(ast, v)
                except cel.CelError as e:
                    errs.append(f"{_render(trail)}: Invalid value: \"object\": {msg} "
                                f"(rule evaluation error: {e})")
                    continue
                if ok is not True:
                    errs.append(f"{_render(trail)}: Invalid value: \"object\": {msg}")
        checks.append(c_cel)

    def check(v, trail, errs):
        if v is None:
            if nullable:
                return
            if t:
                p = _render(trail)
                errs.append(f'{p}: Invalid value: "null": {p} in body must be of type {t}')
            return
        if tcheck is not None and not tcheck(v):
            p = _render(trail)
            errs.append(f"{p}: Invalid value: {_short(v)}: {p} in body must be of type {t}")
            return
        for c in checks:
            c(v, trail, errs)
    return check


def validate(obj: Any, schema: dict, path: str = "") -> list[str]:
    """Return a list of ``field: message`` errors (empty when valid)."""
    errs: list[str] = []
    _compile(schema)(obj, (path or "<root>",), errs)
    return errs


def _short(v: Any) -> str:
    s = repr(v) if not isinstance(v, str) else f'"{v}"'
    return s if len(s) < 80 else s[:77] + "..."
