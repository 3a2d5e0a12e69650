"""The apiserver-sim's structural-schema validator (gpupool/api/openapi.py), compiled once per
schema into checker closures, against a plain recursive oracle that walks the schema keywords
per node (the validator's previous implementation): same error messages, same order, on the
generated Mi355xPool / AzureVmPool / Mi355xJob schemas and on randomly corrupted objects."""
from __future__ import annotations

import copy
import os
import re

import yaml
from hypothesis import given, settings
from hypothesis import strategies as st

from gpupool.api import cel, openapi

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
_TYPES = {
    "string": lambda v: isinstance(v, str),
    "integer": lambda v: isinstance(v, int) and not isinstance(v, bool),
    "number": lambda v: isinstance(v, (int, float)) and not isinstance(v, bool),
    "boolean": lambda v: isinstance(v, bool),
    "object": lambda v: isinstance(v, dict),
    "array": lambda v: isinstance(v, list),
}


def oracle(v, s, path, errs):
    if not isinstance(s, dict):
        return
    if v is None:
        if s.get("nullable"):
            return
        if "type" in s:
            errs.append(f"{path}: Invalid value: \"null\": {path} in body must be of type {s['type']}")
        return
    t = s.get("type")
    if t and not _TYPES[t](v):
        errs.append(f"{path}: Invalid value: {openapi._short(v)}: {path} in body must be of type {t}")
        return
    if "enum" in s and v not in s["enum"]:
        allowed = ", ".join(f'"{e}"' for e in s["enum"])
        errs.append(f"{path}: Unsupported value: {openapi._short(v)}: supported values: {allowed}")
    if t in ("integer", "number"):
        if "minimum" in s and v < s["minimum"]:
            errs.append(f"{path}: Invalid value: {v}: {path} in body should be greater than or "
                        f"equal to {s['minimum']}")
        if "maximum" in s and v > s["maximum"]:
            errs.append(f"{path}: Invalid value: {v}: {path} in body should be less than or "
                        f"equal to {s['maximum']}")
    elif t == "string":
        if "minLength" in s and len(v) < s["minLength"]:
            errs.append(f"{path}: Invalid value: {openapi._short(v)}: should be at least "
                        f"{s['minLength']} chars long")
        if "maxLength" in s and len(v) > s["maxLength"]:
            errs.append(f"{path}: Too long: may not be longer than {s['maxLength']}")
        if "pattern" in s and not re.search(s["pattern"], v):
            errs.append(f"{path}: Invalid value: {openapi._short(v)}: {path} in body should match "
                        f"'{s['pattern']}'")
    elif t == "object":
        for r in s.get("required", []):
            if r not in v:
                errs.append(f"{path}.{r}: Required value")
        props = s.get("properties", {})
        ap = s.get("additionalProperties")
        for k, sub in v.items():
            if k in props:
                oracle(sub, props[k], f"{path}.{k}", errs)
            elif isinstance(ap, dict):
                oracle(sub, ap, f"{path}.{k}", errs)
        for r in s.get("x-kubernetes-validations", []):  # CEL (the interpreter: test_cel.py)
            msg = r.get("message") or f"failed rule: {r['rule']}"
            try:
                ok = cel.evaluate(r["rule"], v)
            except cel.CelError as e:
                errs.append(f'{path}: Invalid value: "object": {msg} (rule evaluation error: {e})')
                continue
            if ok is not True:
                errs.append(f'{path}: Invalid value: "object": {msg}')
    elif t == "array":
        if "minItems" in s and len(v) < s["minItems"]:
            errs.append(f"{path}: Invalid value: should have at least {s['minItems']} items")
        if "maxItems" in s and len(v) > s["maxItems"]:
            errs.append(f"{path}: Too many: {len(v)}: must have at most {s['maxItems']} items")
        for i, x in enumerate(v):
            oracle(x, s.get("items"), f"{path}[{i}]", errs)
        if s.get("x-kubernetes-list-type") == "map":
            keys = s.get("x-kubernetes-list-map-keys", [])
            seen = set()
            for i, x in enumerate(v):
                if isinstance(x, dict):
                    key = tuple(x.get(k) for k in keys)
                    if repr(key) in seen:
                        errs.append(f"{path}[{i}]: Duplicate value: {dict(zip(keys, key))}")
                    seen.add(repr(key))


def schemas() -> dict[str, dict]:
    out = {}
    d = os.path.join(ROOT, "config", "crd")
    for f in sorted(os.listdir(d)):
        if f.endswith(".yaml"):
            doc = yaml.safe_load(open(os.path.join(d, f)))
            kind = doc["spec"]["names"]["kind"]
            out[kind] = doc["spec"]["versions"][0]["schema"]["openAPIV3Schema"]
    return out


SCHEMAS = schemas()
POOL = {"spec": {"replicas": 2, "resourceName": "amd.com/gpu", "topologyPolicy": "xgmi-packed",
                 "probe": {"enabled": True, "hbmBytes": 1 << 30, "minHbmGBps": 4000,
                           "xgmiPeerCheck": True},
                 "health": {"maxCorrectableECC": 10, "maxRetiredPages": 4},
                 "sharing": {"replicasPerGPU": 4, "hbmBytesPerSlot": 8 << 30, "cuPerSlot": 64},
                 "drain": {"gracePeriodSeconds": 30}},
        "status": {"replicas": 2, "readyReplicas": 2, "observedGeneration": 3,
                   "conditions": [{"type": "Ready", "status": "True", "reason": "AllReady",
                                   "message": "2/2", "lastTransitionTime": "2026-01-01T00:00:00Z"}],
                   "devices": [{"uuid": f"u{i}", "index": i, "node": "n0", "health": "Healthy",
                                "advertised": True, "reasons": [], "pods": []} for i in range(2)]}}


def _both(obj, schema):
    want: list[str] = []
    oracle(obj, schema, "<root>", want)
    return openapi.validate(obj, schema), want


def test_valid_objects_have_no_errors():
    got, want = _both(POOL, SCHEMAS["Mi355xPool"])
    assert got == want == []


def test_fixed_invalid_cases_match_the_oracle():
    s = SCHEMAS["Mi355xPool"]
    bad = copy.deepcopy(POOL)
    bad["spec"]["replicas"] = -1
    bad["spec"]["topologyPolicy"] = "ring"
    bad["spec"]["probe"]["hbmBytes"] = "big"
    bad["spec"]["resourceName"] = "Bad Name"
    bad["status"]["conditions"].append(dict(bad["status"]["conditions"][0]))  # duplicate map key
    bad["status"]["devices"][1]["index"] = None
    got, want = _both(bad, s)
    assert got == want and len(got) >= 4, (got, want)
    assert any("spec.replicas in body should be greater than or equal to 0" in e for e in got)


def _paths(o, prefix=()):
    yield prefix
    if isinstance(o, dict):
        for k, v in o.items():
            yield from _paths(v, prefix + (k,))
    elif isinstance(o, list):
        for i, v in enumerate(o):
            yield from _paths(v, prefix + (i,))


PATHS = list(_paths(POOL))[1:]
JUNK = st.one_of(st.none(), st.booleans(), st.integers(-5, 5), st.floats(allow_nan=False),
                 st.text(max_size=5), st.lists(st.integers(), max_size=2),
                 st.dictionaries(st.text(max_size=3), st.integers(), max_size=2))


@settings(max_examples=300, deadline=None)
@given(st.lists(st.tuples(st.sampled_from(PATHS), JUNK), min_size=1, max_size=4),
       st.sampled_from(sorted(SCHEMAS)))
def test_random_corruptions_match_the_oracle(edits, kind):
    obj = copy.deepcopy(POOL)
    for path, val in edits:
        cur = obj
        try:
            for k in path[:-1]:
                cur = cur[k]
            cur[path[-1]] = val
        except (KeyError, IndexError, TypeError):
            continue
    got, want = _both(obj, SCHEMAS[kind])
    assert got == want


def oracle_defaults(obj, schema):
    if not isinstance(schema, dict):
        return obj
    if isinstance(obj, dict) and schema.get("type") == "object":
        props = schema.get("properties", {})
        for name, sub in props.items():
            if name not in obj and "default" in sub:
                obj[name] = copy.deepcopy(sub["default"])
            if name in obj:
                obj[name] = oracle_defaults(obj[name], sub)
        ap = schema.get("additionalProperties")
        if isinstance(ap, dict):
            for k in list(obj):
                if k not in props:
                    obj[k] = oracle_defaults(obj[k], ap)
    elif isinstance(obj, list) and isinstance(schema.get("items"), dict):
        return [oracle_defaults(x, schema["items"]) for x in obj]
    return obj


def oracle_prune(obj, schema):
    if not isinstance(schema, dict) or schema.get("x-kubernetes-preserve-unknown-fields"):
        return obj
    if isinstance(obj, dict) and schema.get("type") == "object":
        props = schema.get("properties")
        ap = schema.get("additionalProperties")
        if props is None and ap is None:
            return obj
        out = {}
        for k, v in obj.items():
            if props and k in props:
                out[k] = oracle_prune(v, props[k])
            elif isinstance(ap, dict):
                out[k] = oracle_prune(v, ap)
            elif ap is True:
                out[k] = v
        return out
    if isinstance(obj, list) and isinstance(schema.get("items"), dict):
        return [oracle_prune(x, schema["items"]) for x in obj]
    return obj


@settings(max_examples=300, deadline=None)
@given(st.lists(st.tuples(st.sampled_from(PATHS + [("spec", "bogus"), ("status", "devices", 0, "x"),
                                                   ("spec", "probe"), ("spec", "health"), ("junk",)]),
                          JUNK), max_size=4),
       st.sampled_from(sorted(SCHEMAS)))
def test_prune_and_defaults_match_the_oracle(edits, kind):
    """Pruning drops exactly the unknown fields and defaulting fills exactly the declared
    defaults (compiled walks vs the plain recursive ones), on objects with unknown and
    missing fields."""
    obj = copy.deepcopy(POOL)
    for path, val in edits:
        cur = obj
        try:
            for k in path[:-1]:
                cur = cur[k]
            if isinstance(val, (dict, list)) or path[-1] not in ("spec", "status"):
                cur[path[-1]] = val
        except (KeyError, IndexError, TypeError):
            continue
    s = SCHEMAS[kind]
    want = oracle_defaults(oracle_prune(copy.deepcopy(obj), s), s)
    got = openapi.apply_defaults(openapi.prune(copy.deepcopy(obj), s), s)
    assert got == want
