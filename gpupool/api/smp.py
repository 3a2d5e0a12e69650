"""Strategic merge patch (``application/strategic-merge-patch+json``) for the built-in kinds.

A real kube-apiserver merges a list of maps element by element when the Go type declares a
``patchMergeKey`` (``status.conditions`` of a Node or Pod merge by ``type``; containers, env,
volumes by ``name``) and merges primitive lists marked ``patchStrategy: merge``
(``metadata.finalizers``). Every other list is replaced whole, as in a JSON merge patch. The
directives this implements are the ones kubelet and kubectl send: ``$patch: replace|delete|merge``
(on a map or as a list element), ``$deleteFromPrimitiveList/<f>``, ``$setElementOrder/<f>`` and
``$retainKeys``. Custom resources do not support strategic merge patch (the apiserver answers
415): the caller checks that before calling here.

Why the simulator needs it: a component that writes its own Node condition with a merge patch
over a GET of the whole ``status`` reverts whatever the kubelet wrote in between; one that sends
only its own condition as a strategic merge patch leaves the kubelet's conditions, capacity and
allocatable alone. With merge-patch-only semantics the simulator could not tell the two apart.
"""
from __future__ import annotations

import copy
from typing import Any

# merge strategy of a list field: a merge-key name (list of maps), "" (primitive list merged as a
# set), or absent (the list is atomic: replaced whole)
_META = {("metadata", "finalizers"): "", ("metadata", "ownerReferences"): "uid"}

_CONTAINER = {("ports",): "containerPort", ("env",): "name", ("volumeMounts",): "mountPath",
              ("volumeDevices",): "devicePath", ("resizePolicy",): "resourceName"}

_POD_SPEC = {("volumes",): "name", ("containers",): "name", ("initContainers",): "name",
             ("ephemeralContainers",): "name", ("imagePullSecrets",): "name",
             ("hostAliases",): "ip", ("topologySpreadConstraints",): "topologyKey",
             ("resourceClaims",): "name", ("schedulingGates",): "name"}
for _c in ("containers", "initContainers", "ephemeralContainers"):
    for _k, _v in _CONTAINER.items():
        _POD_SPEC[(_c,) + _k] = _v


def _under(prefix: tuple, table: dict) -> dict:
    return {prefix + k: v for k, v in table.items()}


_CONDITIONS = {("status", "conditions"): "type"}

MERGE_KEYS: dict[str, dict[tuple, str]] = {
    "Node": {**_META, **_CONDITIONS, ("status", "addresses"): "type",
             ("status", "volumesAttached"): "name", ("spec", "podCIDRs"): ""},
    "Pod": {**_META, **_CONDITIONS, **_under(("spec",), _POD_SPEC),
            ("status", "podIPs"): "ip", ("status", "hostIPs"): "ip",
            ("status", "resourceClaimStatuses"): "name"},
    "Deployment": {**_META, **_CONDITIONS, **_under(("spec", "template", "spec"), _POD_SPEC)},
    "DaemonSet": {**_META, **_CONDITIONS, **_under(("spec", "template", "spec"), _POD_SPEC)},
    "Service": {**_META, ("spec", "ports"): "port", **_CONDITIONS},
    "PodDisruptionBudget": {**_META, **_CONDITIONS},
    "PersistentVolumeClaim": {**_META, **_CONDITIONS},
    "Namespace": {**_META, ("spec", "finalizers"): "", **_CONDITIONS},
}


class PatchError(ValueError):
    """The patch is malformed for the target's schema (the apiserver's 422)."""


def strategic_merge(target: Any, patch: Any, kind: str) -> Any:
    """``patch`` applied to a copy of ``target`` with the list strategies of ``kind``."""
    if not isinstance(patch, dict):
        raise PatchError("a strategic merge patch must be a JSON object")
    keys = MERGE_KEYS.get(kind, _META)
    out = _map(copy.deepcopy(target) if isinstance(target, dict) else {}, patch, keys, ())
    return {} if out is None else out


def _plain(v: Any) -> Any:
    """A patch value with its directives removed (what a replaced subtree stores)."""
    if isinstance(v, dict):
        return {k: _plain(x) for k, x in v.items() if not k.startswith("$") and x is not None}
    if isinstance(v, list):
        return [_plain(x) for x in v if not (isinstance(x, dict) and "$patch" in x)]
    return v


def _map(out: dict, patch: dict, keys: dict, path: tuple) -> dict | None:
    directive = patch.get("$patch")
    if directive == "delete":
        return None
    if directive == "replace":
        return _plain(patch)
    if directive not in (None, "merge"):
        raise PatchError(f"unknown patch directive {directive!r} at {'.'.join(path) or '<root>'}")
    orders: dict[str, list] = {}
    retain = patch.get("$retainKeys")
    for k, v in patch.items():
        if k.startswith("$deleteFromPrimitiveList/"):
            f = k.split("/", 1)[1]
            if isinstance(out.get(f), list):
                out[f] = [x for x in out[f] if x not in (v or [])]
        elif k.startswith("$setElementOrder/"):
            orders[k.split("/", 1)[1]] = list(v or [])
    for k, v in patch.items():
        if k.startswith("$"):
            continue
        sub = path + (k,)
        if v is None:
            out.pop(k, None)
        elif isinstance(v, dict):
            cur = out.get(k)
            r = _map(cur if isinstance(cur, dict) else {}, v, keys, sub)
            if r is None:
                out.pop(k, None)
            else:
                out[k] = r
        elif isinstance(v, list):
            if sub in keys:
                cur = out.get(k)
                out[k] = _list(cur if isinstance(cur, list) else [], v, keys[sub], keys, sub)
            else:
                out[k] = _plain(v)
        else:
            out[k] = v
    for f, order in orders.items():
        if isinstance(out.get(f), list):
            out[f] = _ordered(out[f], order, keys.get(path + (f,)))
    if retain is not None:
        keep = set(retain)
        for k in [k for k in out if k not in keep]:
            del out[k]
    return out


def _list(cur: list, patch: list, key: str, keys: dict, path: tuple) -> list:
    if any(isinstance(e, dict) and e.get("$patch") == "replace" for e in patch):
        return _plain(patch)
    if key == "":  # primitive list, merged as a set in order of first appearance
        out = list(cur)
        for e in patch:
            if isinstance(e, dict):
                raise PatchError(f"{'.'.join(path)}: a map in a list of primitives")
            if e not in out:
                out.append(e)
        return out
    out = [copy.deepcopy(e) for e in cur]
    for e in patch:
        if not isinstance(e, dict):
            raise PatchError(f"{'.'.join(path)}: expected maps merged by {key!r}, got {e!r}")
        if key not in e:
            raise PatchError(f"map: {e} does not contain declared merge key: {key}")
        idx = next((i for i, x in enumerate(out) if isinstance(x, dict) and x.get(key) == e[key]),
                   None)
        if e.get("$patch") == "delete":
            if idx is not None:
                out.pop(idx)
            continue
        if idx is None:
            out.append(_plain(e))
        else:
            merged = _map(out[idx], e, keys, path)
            if merged is None:
                out.pop(idx)
            else:
                out[idx] = merged
    return out


def _ordered(items: list, order: list, key: str | None) -> list:
    """``$setElementOrder``: the named elements in the given order, then the rest as they were."""
    def ident(x: Any) -> Any:
        return x.get(key) if key and isinstance(x, dict) else x
    want = [ident(o) for o in order]
    rank = {w: i for i, w in enumerate(want) if isinstance(w, (str, int, float, bool))}
    named = sorted((x for x in items if ident(x) in rank), key=lambda x: rank[ident(x)])
    return named + [x for x in items if ident(x) not in rank]


def two_way(original: dict, modified: dict, kind: str) -> dict:
    """The strategic merge patch that turns ``original`` into ``modified`` for the keyed lists of
    ``kind`` (what kubectl and the kubelet compute client-side): maps recurse, keyed lists carry
    only changed or new elements plus ``$patch: delete`` for removed ones and a
    ``$setElementOrder``, other values are sent when they differ, removed keys as null."""
    keys = MERGE_KEYS.get(kind, _META)
    return _diff(original, modified, keys, ())


def _diff(a: dict, b: dict, keys: dict, path: tuple) -> dict:
    out: dict = {}
    for k in a:
        if k not in b:
            out[k] = None
    for k, v in b.items():
        sub = path + (k,)
        old = a.get(k)
        if old == v:
            continue
        if isinstance(v, dict) and isinstance(old, dict):
            d = _diff(old, v, keys, sub)
            if d:
                out[k] = d
        elif isinstance(v, list) and isinstance(old, list) and keys.get(sub):
            mk = keys[sub]
            olds = {x.get(mk): x for x in old if isinstance(x, dict)}
            news = {x.get(mk): x for x in v if isinstance(x, dict)}
            items = []
            for ident, x in news.items():
                if ident not in olds:
                    items.append(x)
                elif olds[ident] != x:
                    items.append({mk: ident, **_diff(olds[ident], x, keys, sub)})
            items += [{mk: ident, "$patch": "delete"} for ident in olds if ident not in news]
            if items:
                out[k] = items
                out[f"$setElementOrder/{k}"] = [{mk: x.get(mk)} for x in v if isinstance(x, dict)]
        else:
            out[k] = v
    return out


def three_way(original: dict | None, modified: dict, current: dict, kind: str | None) -> dict:
    """``kubectl apply``'s client-side patch: what changed from ``current`` to ``modified``
    (additions and changes), plus deletions of what the last apply set (``original``, the
    last-applied-configuration) and this one no longer does. Fields neither apply set — written by
    controllers, other users, defaulting — are left alone. ``kind=None``: a JSON merge patch (a
    custom resource: lists are atomic); else a strategic merge patch with ``kind``'s list keys."""
    keys = {} if kind is None else MERGE_KEYS.get(kind, _META)
    return _three(original or {}, modified, current or {}, keys, (), kind is not None)


def _three(orig: dict, mod: dict, cur: dict, keys: dict, path: tuple, strategic: bool) -> dict:
    out: dict = {}
    for k in orig:
        if k not in mod and k in cur:
            out[k] = None
    for k, v in mod.items():
        sub = path + (k,)
        c, o = cur.get(k), orig.get(k)
        if isinstance(v, dict) and isinstance(c, dict):
            d = _three(o if isinstance(o, dict) else {}, v, c, keys, sub, strategic)
            if d:
                out[k] = d
        elif strategic and isinstance(v, list) and isinstance(c, list) and sub in keys:
            mk = keys[sub]
            if mk == "":  # a set: add what is missing, delete what the last apply had
                add = [x for x in v if x not in c]
                gone = [x for x in (o if isinstance(o, list) else []) if x not in v and x in c]
                if add:
                    out[k] = add
                if gone:
                    out[f"$deleteFromPrimitiveList/{k}"] = gone
                continue
            curs = {x.get(mk): x for x in c if isinstance(x, dict)}
            origs = {x.get(mk): x for x in (o if isinstance(o, list) else []) if isinstance(x, dict)}
            items, ids = [], set()
            for x in v:
                if not isinstance(x, dict):
                    continue
                ident = x.get(mk)
                ids.add(ident)
                if ident not in curs:
                    items.append(x)
                else:
                    d = _three(origs.get(ident) or {}, x, curs[ident], keys, sub, strategic)
                    if d:
                        items.append({mk: ident, **d})
            items += [{mk: i, "$patch": "delete"} for i in origs if i not in ids and i in curs]
            if items:
                out[k] = items
                out[f"$setElementOrder/{k}"] = [{mk: x.get(mk)} for x in v if isinstance(x, dict)]
        elif c != v:
            out[k] = v
    return out
