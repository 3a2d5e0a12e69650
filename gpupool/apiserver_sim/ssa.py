"""Server-side apply (``application/apply-patch+yaml``) and field ownership (``managedFields``).

What the kube-apiserver does, as far as a client can observe it:

* An apply names its ``fieldManager`` and sends the fields that manager wants set — its whole
  intent, not a diff. The object becomes the current object with those fields set; a field this
  manager applied last time and no longer sends is removed, unless another manager also owns it.
* Each manager's fields are recorded in ``metadata.managedFields`` (``FieldsV1``: ``f:<field>``,
  ``k:{<list-map keys>}`` for an element of a keyed list, ``v:<value>`` for a member of a set,
  ``.`` for "this element itself"), one entry per (manager, operation, subresource).
* Applying a value that differs from the current one for a field another manager owns is a
  conflict: 409 naming each field and its owner. ``force=true`` takes ownership instead. Applying
  the same value makes the ownership shared.
* A non-apply write (PUT, merge / strategic / JSON patch) takes the fields it changed away from
  every other manager and records them under its own manager with ``operation: Update``. The
  manager is the ``fieldManager`` query parameter, else the request's User-Agent up to its first
  ``/`` (``kubectl``), else ``unknown``.

List semantics follow the schema: built-in kinds use their ``patchMergeKey`` table
(``smp.MERGE_KEYS``), custom resources their CRD's ``x-kubernetes-list-type: map`` /
``x-kubernetes-list-map-keys`` and ``set``; every other list is atomic (owned and replaced whole).

One documented difference: objects nobody has applied carry no ``managedFields`` here, and
non-apply writes to them record none (ownership bookkeeping costs a full-object field walk per
write; the operator's own status writes stay on the fast path). The first apply to such an object
records its existing fields under ``before-first-apply`` (operation Update), which is what the
apiserver does for an object whose managedFields were cleared.
"""
from __future__ import annotations

import copy
import json
from typing import Any

from ..api.smp import _META, MERGE_KEYS

# identity and server-owned fields: never owned, never applied
_SKIP_TOP = {"apiVersion", "kind"}
_SKIP_META = {"name", "namespace", "uid", "resourceVersion", "generation", "creationTimestamp",
              "deletionTimestamp", "deletionGracePeriodSeconds", "managedFields", "selfLink"}
_MISSING = object()
BEFORE_FIRST_APPLY = "before-first-apply"


class Conflict(Exception):
    """Apply conflicts: [(manager, dotted field path)]."""

    def __init__(self, conflicts: list[tuple[str, str]]):
        super().__init__(conflicts)
        self.conflicts = conflicts


def list_keys(kind: str, schema: dict | None) -> dict[tuple, str]:
    """List strategies of a kind: logical path -> merge key ("" = a set). Custom resources: from
    the CRD's structural schema; built-ins: the strategic merge table."""
    if schema is None:
        return MERGE_KEYS.get(kind, _META)
    out = dict(_META)

    def walk(s: dict, path: tuple) -> None:
        if not isinstance(s, dict):
            return
        if s.get("type") == "array":
            lt = s.get("x-kubernetes-list-type")
            mk = s.get("x-kubernetes-list-map-keys") or []
            if lt == "map" and len(mk) == 1:
                out[path] = mk[0]
            elif lt == "set":
                out[path] = ""
            walk(s.get("items") or {}, path)
            return
        for k, v in (s.get("properties") or {}).items():
            walk(v, path + (k,))
    walk(schema, ())
    return out


def _strip(obj: dict, status_sub: bool, subresource: str) -> dict:
    """The part of an object (or applied configuration) whose fields can be owned through this
    endpoint: identity and server fields dropped; ``status`` only through /status when the type
    has that subresource, and nothing but ``status`` there."""
    out = {k: v for k, v in obj.items() if k not in _SKIP_TOP}
    md = {k: v for k, v in (out.get("metadata") or {}).items() if k not in _SKIP_META}
    out.pop("metadata", None)
    if md:
        out["metadata"] = md
    if status_sub:
        if subresource == "status":
            out = {"status": out["status"]} if "status" in out else {}
        else:
            out.pop("status", None)
    return out


def _tok_key(mk: str, val: Any) -> str:
    return "k:" + json.dumps({mk: val}, separators=(",", ":"), sort_keys=True)


def field_set(obj: Any, keys: dict, path: tuple = (), lpath: tuple = (), out=None) -> set:
    """Every owned field path of ``obj``: leaf values, atomic lists, keyed-list elements (the
    element itself, ending in a ``k:`` token) and set members (``v:``)."""
    out = set() if out is None else out
    for k, v in obj.items():
        p, lp = path + ("f:" + k,), lpath + (k,)
        if isinstance(v, dict) and v:
            field_set(v, keys, p, lp, out)
        elif isinstance(v, list) and lp in keys:
            mk = keys[lp]
            for e in v:
                if mk == "":
                    out.add(p + ("v:" + json.dumps(e, separators=(",", ":"), sort_keys=True),))
                elif isinstance(e, dict) and mk in e:
                    ep = p + (_tok_key(mk, e[mk]),)
                    out.add(ep)
                    field_set(e, keys, ep, lp, out)
        else:
            out.add(p)
    return out


def _get(obj: Any, path: tuple) -> Any:
    cur = obj
    for t in path:
        if t.startswith("f:"):
            if not isinstance(cur, dict) or t[2:] not in cur:
                return _MISSING
            cur = cur[t[2:]]
        elif t.startswith("k:"):
            (mk, val), = json.loads(t[2:]).items()
            cur = next((e for e in cur if isinstance(e, dict) and e.get(mk) == val), _MISSING) \
                if isinstance(cur, list) else _MISSING
            if cur is _MISSING:
                return cur
        elif t.startswith("v:"):
            val = json.loads(t[2:])
            return True if isinstance(cur, list) and val in cur else _MISSING
    return cur


def _remove(obj: dict, path: tuple) -> None:
    parent = obj
    for t in path[:-1]:
        parent = _get(parent, (t,))
        if parent is _MISSING:
            return
    t = path[-1]
    if t.startswith("f:") and isinstance(parent, dict):
        parent.pop(t[2:], None)
    elif t.startswith("k:") and isinstance(parent, list):
        (mk, val), = json.loads(t[2:]).items()
        parent[:] = [e for e in parent if not (isinstance(e, dict) and e.get(mk) == val)]
    elif t.startswith("v:") and isinstance(parent, list):
        val = json.loads(t[2:])
        parent[:] = [e for e in parent if e != val]


def _merge(cur: dict, cfg: dict, keys: dict, lpath: tuple) -> dict:
    out = dict(cur)
    for k, v in cfg.items():
        lp = lpath + (k,)
        c = out.get(k)
        if isinstance(v, dict) and isinstance(c, dict):
            out[k] = _merge(c, v, keys, lp)
        elif isinstance(v, list) and isinstance(c, list) and lp in keys:
            mk = keys[lp]
            if mk == "":
                out[k] = list(c) + [e for e in v if e not in c]
                continue
            merged = [copy.deepcopy(e) for e in c]
            for e in v:
                if not isinstance(e, dict) or mk not in e:
                    continue
                i = next((j for j, x in enumerate(merged)
                          if isinstance(x, dict) and x.get(mk) == e[mk]), None)
                if i is None:
                    merged.append(copy.deepcopy(e))
                else:
                    merged[i] = _merge(merged[i], e, keys, lp)
            out[k] = merged
        else:
            out[k] = copy.deepcopy(v)
    return out


def dotted(path: tuple) -> str:
    return ".".join(t[2:] if t.startswith("f:") else t for t in path)


# ---------------------------------------------------------------- FieldsV1 <-> path sets
def to_fields_v1(paths: set) -> dict:
    root: dict = {}
    for p in sorted(paths):
        node = root
        for t in p:
            node = node.setdefault(t, {})
        if p and p[-1].startswith("k:"):
            node["."] = {}
    return root


def from_fields_v1(f: dict, prefix: tuple = (), out=None) -> set:
    out = set() if out is None else out
    for t, sub in (f or {}).items():
        if t == ".":
            out.add(prefix)
            continue
        p = prefix + (t,)
        if not sub:
            out.add(p)
        else:
            from_fields_v1(sub, p, out)
    return out


def _entries(md: dict) -> list[dict]:
    return [e for e in (md.get("managedFields") or []) if isinstance(e, dict)]


def _owned(entries: list[dict]) -> list[tuple[dict, set]]:
    return [(e, from_fields_v1(e.get("fieldsV1") or {})) for e in entries]


def _write_entries(owned: list[tuple[dict, set]], now: str, touched: set) -> list[dict]:
    out = []
    for e, fs in owned:
        if not fs:
            continue
        e = {k: v for k, v in e.items() if k != "fieldsV1"}
        if e.get("manager") in touched:
            e["time"] = now
        e["fieldsType"] = "FieldsV1"
        e["fieldsV1"] = to_fields_v1(fs)
        out.append(e)
    return out


def _same_entry(e: dict, manager: str, op: str, sub: str) -> bool:
    return e.get("manager") == manager and e.get("operation") == op and \
        (e.get("subresource") or "") == sub


def _is_key_of_kept(p: tuple, keys: dict) -> bool:
    """``p`` is the merge-key field of a list element (``...k:{"type":"X"}, f:type``): it goes
    with its element, never alone."""
    if len(p) < 2 or not p[-2].startswith("k:") or not p[-1].startswith("f:"):
        return False
    (mk, _), = json.loads(p[-2][2:]).items()
    return p[-1][2:] == mk


def apply(cur: dict | None, cfg: dict, manager: str, force: bool, keys: dict, status_sub: bool,
          subresource: str, api_version: str, now: str) -> dict:
    """The object after ``manager`` applies ``cfg`` to ``cur`` (None: the object is created).
    Raises ``Conflict``. The caller validates, admits and stores the result."""
    cfg_own = _strip(cfg, status_sub, subresource)
    want = field_set(cfg_own, keys)
    base = copy.deepcopy(cur) if cur is not None else \
        {"apiVersion": cfg.get("apiVersion"), "kind": cfg.get("kind"),
         "metadata": {k: v for k, v in (cfg.get("metadata") or {}).items()
                      if k in ("name", "namespace")}}
    md = base.setdefault("metadata", {})
    entries = _entries(md)
    if cur is not None and not entries:  # nobody applied before: existing fields have an owner
        existing = field_set(_strip(cur, status_sub, subresource), keys)
        if existing:
            entries = [{"manager": BEFORE_FIRST_APPLY, "operation": "Update",
                        "apiVersion": api_version, "time": now, "fieldsType": "FieldsV1",
                        "fieldsV1": to_fields_v1(existing)}]
    owned = _owned(entries)
    mine = next(((e, fs) for e, fs in owned if _same_entry(e, manager, "Apply", subresource)),
                None)
    me = mine[0] if mine else None
    conflicts: list[tuple[str, tuple]] = []
    for p in sorted(want):
        if p[-1].startswith(("k:", "v:")):
            continue  # presence only: nothing to disagree about
        new_v, cur_v = _get(cfg_own, p), _get(base, p)
        if cur_v is _MISSING or cur_v == new_v:
            continue
        conflicts += [(e.get("manager", ""), p) for e, fs in owned if e is not me and p in fs]
    if conflicts and not force:
        raise Conflict([(m, dotted(p)) for m, p in conflicts])
    stolen = {p for _, p in conflicts}
    for e, fs in owned:
        if e is not me:
            fs -= stolen
    merged = _merge(base, cfg_own, keys, ())
    # fields this manager applied before and no longer sends: gone unless someone else owns them
    if mine is not None:
        others = set().union(*(fs for e, fs in owned if e is not me))
        keep = others | want
        drop = [p for p in mine[1] - want if p not in others and
                not any(len(q) > len(p) and q[:len(p)] == p for q in keep)]
        gone = set()
        for p in sorted(drop, key=len):  # an element first: its own fields go with it
            if any(p[:i] in gone for i in range(1, len(p))) or _is_key_of_kept(p, keys):
                continue
            _remove(merged, p)
            gone.add(p)
        mine[1].clear()
        mine[1].update(want)
        entry = mine[0]
    else:
        entry = {"manager": manager, "operation": "Apply", "apiVersion": api_version}
        if subresource:
            entry["subresource"] = subresource
        owned.append((entry, set(want)))
    merged["metadata"]["managedFields"] = _write_entries(owned, now, {manager})
    return merged


def record_update(cur: dict, new: dict, manager: str, keys: dict, status_sub: bool,
                  subresource: str, api_version: str, now: str) -> None:
    """A non-apply write from ``cur`` to ``new``: ``manager`` takes the fields it set or changed,
    removed fields leave every set. Only for objects that carry managedFields already."""
    entries = _entries(cur.get("metadata") or {})
    if not entries:
        new.get("metadata", {}).pop("managedFields", None)
        return
    a = field_set(_strip(cur, status_sub, subresource), keys)
    b = field_set(_strip(new, status_sub, subresource), keys)
    changed = {p for p in b if p not in a or
               (not p[-1].startswith(("k:", "v:")) and _get(cur, p) != _get(new, p))}
    removed = a - b
    owned = _owned(entries)
    if not changed and not removed:
        new["metadata"]["managedFields"] = entries
        return
    for _, fs in owned:
        fs -= changed
        fs -= removed
    mine = next(((e, fs) for e, fs in owned if _same_entry(e, manager, "Update", subresource)),
                None)
    if mine is None:
        entry = {"manager": manager, "operation": "Update", "apiVersion": api_version}
        if subresource:
            entry["subresource"] = subresource
        owned.append((entry, set()))
        mine = owned[-1]
    mine[1].update(changed)
    new["metadata"]["managedFields"] = _write_entries(owned, now, {manager} if changed else set())
