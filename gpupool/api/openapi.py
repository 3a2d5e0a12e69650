"""Structural OpenAPI v3 subset: validation, defaulting and pruning of custom resources.

This is what kube-apiserver does for a CRD with a structural schema; the apiserver-sim applies it
on every create/update so that e.g. ``replicas: -1`` is rejected at admission exactly as the
reference's ``+kubebuilder:validation:Minimum=0`` marker would (README.md:94-95).

Supported keywords: type, properties, required, additionalProperties (schema form), items,
enum, minimum, maximum, minLength, maxLength, pattern, minItems, maxItems, default, nullable,
x-kubernetes-preserve-unknown-fields, x-kubernetes-list-type=map + list-map-keys (uniqueness).
"""
from __future__ import annotations

import copy
import re
from typing import Any

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
    if not isinstance(schema, dict):
        return obj
    if isinstance(obj, dict) and schema.get("type") == "object":
        props = schema.get("properties", {})
        for name, sub in props.items():
            if name not in obj and "default" in sub:
                obj[name] = copy.deepcopy(sub["default"])
            if name in obj:
                obj[name] = apply_defaults(obj[name], sub)
        ap = schema.get("additionalProperties")
        if isinstance(ap, dict):
            for k in list(obj):
                if k not in props:
                    obj[k] = apply_defaults(obj[k], ap)
    elif isinstance(obj, list) and isinstance(schema.get("items"), dict):
        return [apply_defaults(x, schema["items"]) for x in obj]
    return obj


def prune(obj: Any, schema: dict) -> Any:
    """Drop fields not in the schema (structural-schema pruning)."""
    if not isinstance(schema, dict) or schema.get("x-kubernetes-preserve-unknown-fields"):
        return obj
    if isinstance(obj, dict) and schema.get("type") == "object":
        props = schema.get("properties")
        ap = schema.get("additionalProperties")
        if props is None and ap is None:
            return obj  # free-form object (e.g. metadata)
        out = {}
        for k, v in obj.items():
            if props and k in props:
                out[k] = prune(v, props[k])
            elif isinstance(ap, dict):
                out[k] = prune(v, ap)
            elif ap is True:
                out[k] = v
        return out
    if isinstance(obj, list) and isinstance(schema.get("items"), dict):
        return [prune(x, schema["items"]) for x in obj]
    return obj


def validate(obj: Any, schema: dict, path: str = "") -> list[str]:
    """Return a list of ``field: message`` errors (empty when valid)."""
    errs: list[str] = []
    _validate(obj, schema, path or "<root>", errs)
    return errs


def _validate(v: Any, s: dict, path: str, errs: list[str]) -> None:
    if not isinstance(s, dict):
        return
    if v is None:
        if s.get("nullable"):
            return
        if "type" in s:
            errs.append(f"{path}: Invalid value: \"null\": {path} in body must be of type {s['type']}")
        return
    t = s.get("type")
    if t and not _TYPE_CHECK[t](v):
        errs.append(f"{path}: Invalid value: {_short(v)}: {path} in body must be of type {t}")
        return
    if "enum" in s and v not in s["enum"]:
        allowed = ", ".join(f'"{e}"' for e in s["enum"])
        errs.append(f"{path}: Unsupported value: {_short(v)}: supported values: {allowed}")
    if t in ("integer", "number"):
        if "minimum" in s and v < s["minimum"]:
            errs.append(f"{path}: Invalid value: {v}: {path} in body should be greater than or "
                        f"equal to {s['minimum']}")
        if "maximum" in s and v > s["maximum"]:
            errs.append(f"{path}: Invalid value: {v}: {path} in body should be less than or "
                        f"equal to {s['maximum']}")
    elif t == "string":
        if "minLength" in s and len(v) < s["minLength"]:
            errs.append(f"{path}: Invalid value: {_short(v)}: should be at least "
                        f"{s['minLength']} chars long")
        if "maxLength" in s and len(v) > s["maxLength"]:
            errs.append(f"{path}: Too long: may not be longer than {s['maxLength']}")
        if "pattern" in s and not _re(s["pattern"]).search(v):
            errs.append(f"{path}: Invalid value: {_short(v)}: {path} in body should match "
                        f"'{s['pattern']}'")
    elif t == "object":
        for r in s.get("required", []):
            if r not in v:
                errs.append(f"{path}.{r}: Required value")
        props = s.get("properties", {})
        ap = s.get("additionalProperties")
        for k, sub in v.items():
            if k in props:
                _validate(sub, props[k], f"{path}.{k}", errs)
            elif isinstance(ap, dict):
                _validate(sub, ap, f"{path}.{k}", errs)
    elif t == "array":
        if "minItems" in s and len(v) < s["minItems"]:
            errs.append(f"{path}: Invalid value: should have at least {s['minItems']} items")
        if "maxItems" in s and len(v) > s["maxItems"]:
            errs.append(f"{path}: Too many: {len(v)}: must have at most {s['maxItems']} items")
        items = s.get("items")
        for i, x in enumerate(v):
            _validate(x, items, f"{path}[{i}]", errs)
        if s.get("x-kubernetes-list-type") == "map":
            keys = s.get("x-kubernetes-list-map-keys", [])
            seen = set()
            for i, x in enumerate(v):
                if isinstance(x, dict):
                    key = tuple(x.get(k) for k in keys)
                    if key in seen:
                        errs.append(f"{path}[{i}]: Duplicate value: {dict(zip(keys, key))}")
                    seen.add(key)


def _short(v: Any) -> str:
    s = repr(v) if not isinstance(v, str) else f'"{v}"'
    return s if len(s) < 80 else s[:77] + "..."
