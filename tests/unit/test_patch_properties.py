"""Hypothesis properties of the patch machinery every component writes through
(gpupool/api/smp.py, gpupool/apiserver_sim/ssa.py):

* a strategic two-way diff applied to its source gives its target, for Pod-shaped objects with
  keyed lists (containers by name, env by name, conditions by type) and atomic lists;
* ``kubectl apply`` (three-way): after an apply every field of the manifest has the manifest's
  value, a field another writer set that no apply ever set survives, and a field an earlier apply
  set that the manifest dropped is gone;
* server-side apply: a manager's applied fields end with the applied values and ownership, and a
  second manager's fields it never touched survive.
"""
from __future__ import annotations

import copy

from hypothesis import given, settings
from hypothesis import strategies as st

from gpupool.api.smp import strategic_merge, three_way, two_way
from gpupool.apiserver_sim import ssa

NAMES = st.sampled_from(["a", "b", "c", "d"])
VALS = st.one_of(st.integers(0, 3), st.sampled_from(["x", "y", "z"]))


@st.composite
def env(draw):
    names = draw(st.lists(NAMES, unique=True, max_size=3))
    return [{"name": n, "value": str(draw(VALS))} for n in names]


@st.composite
def pod(draw):
    cnames = draw(st.lists(NAMES, unique=True, min_size=1, max_size=3))
    containers = []
    for n in cnames:
        c = {"name": n, "image": draw(st.sampled_from(["i1", "i2"]))}
        if draw(st.booleans()):
            c["env"] = draw(env())
        if draw(st.booleans()):
            c["args"] = draw(st.lists(st.sampled_from(["-v", "-q", "--x"]), max_size=2))
        containers.append(c)
    obj = {"metadata": {"name": "p", "labels": draw(st.dictionaries(NAMES, VALS, max_size=3))},
           "spec": {"containers": containers}}
    if draw(st.booleans()):
        obj["spec"]["nodeName"] = draw(st.sampled_from(["n1", "n2"]))
    conds = draw(st.lists(st.sampled_from(["Ready", "Initialized", "Scheduled"]), unique=True,
                          max_size=3))
    if conds:
        obj["status"] = {"conditions": [{"type": t, "status": draw(st.sampled_from(
            ["True", "False"]))} for t in conds]}
    return obj


def _norm(o):
    """Order-insensitive view of keyed lists (strategic merge appends new elements)."""
    if isinstance(o, dict):
        return {k: _norm(v) for k, v in o.items()}
    if isinstance(o, list) and o and all(isinstance(x, dict) and ("name" in x or "type" in x)
                                         for x in o):
        return sorted((_norm(x) for x in o), key=lambda x: (x.get("name") or x.get("type")))
    if isinstance(o, list):
        return [_norm(x) for x in o]
    return o


@settings(max_examples=150, deadline=None)
@given(pod(), pod())
def test_two_way_diff_round_trips(a, b):
    assert _norm(strategic_merge(a, two_way(a, b, "Pod"), "Pod")) == _norm(b)


def _flat(o, prefix=()):
    """Leaf paths of maps only (lists are compared whole). An empty map is no leaf: a manifest's
    ``x: {}`` asks for nothing (merge semantics keep what others put under it)."""
    out = {}
    for k, v in o.items():
        if isinstance(v, dict):
            out.update(_flat(v, prefix + (k,)))
        else:
            out[prefix + (k,)] = v
    return out


def _apply_json(live, last, manifest):
    """What gpuctl's client-side apply does for a custom resource (JSON merge patch)."""
    from gpupool.apiserver_sim.store import merge_patch
    patch = three_way(last, manifest, live, None)
    return merge_patch(live, patch)


SPEC = st.dictionaries(NAMES, st.one_of(VALS, st.dictionaries(NAMES, VALS, max_size=2)),
                       max_size=4)


@settings(max_examples=200, deadline=None)
@given(SPEC, SPEC, SPEC)
def test_three_way_apply_keeps_others_and_drops_what_the_manifest_dropped(m1, others, m2):
    live = {"spec": copy.deepcopy(m1)}
    # another writer sets fields no apply set (only where the manifest has nothing)
    for k, v in others.items():
        if k not in m1:
            live["spec"][k] = v
    live = _apply_json(live, None, {"spec": m1})            # first apply (no last-applied)
    out = _apply_json(live, {"spec": m1}, {"spec": m2})       # the manifest changes
    got, want, first = _flat(out["spec"]), _flat(m2), _flat(m1)
    for p, v in want.items():
        assert got.get(p) == v, (p, out, m2)                   # the manifest wins
    for k, v in others.items():
        if k not in m1 and k not in m2:
            assert out["spec"].get(k) == v                     # others' fields survive
    for p in first:
        if p not in want and not any(p[:i] in want for i in range(1, len(p))) and \
                p[0] not in others:
            assert p not in got or p[:1] in [q[:1] for q in want], (p, out)  # dropped


@settings(max_examples=150, deadline=None)
@given(SPEC, SPEC, SPEC)
def test_server_side_apply_owns_what_it_applied(mine1, theirs, mine2):
    keys: dict = {}
    cur = None
    cur = ssa.apply(cur, {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "c"},
                          "data": mine1}, "me", False, keys, False, "", "v1", "t")
    # another manager force-applies its own fields (shared where equal, taken where different)
    cur = ssa.apply(cur, {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "c"},
                          "data": theirs}, "them", True, keys, False, "", "v1", "t")
    cur = ssa.apply(cur, {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "c"},
                          "data": mine2}, "me", True, keys, False, "", "v1", "t")
    data = _flat(cur.get("data") or {})
    for p, v in _flat(mine2).items():
        assert data.get(p) == v                                # applied values hold
    owners = {e["manager"]: ssa.from_fields_v1(e["fieldsV1"]) for e in
              cur["metadata"]["managedFields"]}
    for p in _flat(mine2):
        assert ("f:data",) + tuple("f:" + x for x in p) in owners.get("me", set())
    for p, v in _flat(theirs).items():
        if not _covered(p, mine2):
            assert data.get(p) == v, (p, cur)                  # the other manager's survive


def _covered(path: tuple, applied: dict) -> bool:
    """Does the applied configuration set ``path`` or a field above it (a scalar, or an empty
    map, which server-side apply owns as a value)?"""
    node = applied
    for k in path:
        if not isinstance(node, dict) or k not in node:
            return False
        node = node[k]
        if not isinstance(node, dict) or not node:
            return True
    return True
