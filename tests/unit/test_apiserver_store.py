"""apiserver-sim semantics (SURVEY.md §4.2 'Python unit' row; §7.3 hard part 1)."""
from __future__ import annotations

import copy
import glob
import os

import pytest
import yaml

from gpupool.apiserver_sim.store import ApiError, Store, json_patch, merge_patch, \
    parse_label_selector

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@pytest.fixture
def store():
    s = Store(window=100)
    crd_rt = s.types[("apiextensions.k8s.io", "customresourcedefinitions")]
    for p in sorted(glob.glob(os.path.join(ROOT, "config", "crd", "*.yaml"))):
        s.create(crd_rt, None, yaml.safe_load(open(p)))
    return s


def pool(name="p", replicas=1, **spec):
    return {"apiVersion": "compute.my.domain/v1alpha1", "kind": "Mi355xPool",
            "metadata": {"name": name}, "spec": {"replicas": replicas, **spec}}


def mi(s):
    return s.lookup("compute.my.domain", "mi355xpools")


def test_rv_strictly_increasing_and_generation(store):
    rt = mi(store)
    a = store.create(rt, "default", pool("a"))
    b = store.create(rt, "default", pool("b"))
    assert int(b["metadata"]["resourceVersion"]) > int(a["metadata"]["resourceVersion"])
    assert a["metadata"]["generation"] == 1
    a["spec"]["replicas"] = 3
    a2 = store.update(rt, "default", "a", a)
    assert a2["metadata"]["generation"] == 2
    # metadata-only change: no generation bump
    a2["metadata"]["labels"] = {"x": "y"}
    a3 = store.update(rt, "default", "a", a2)
    assert a3["metadata"]["generation"] == 2
    assert int(a3["metadata"]["resourceVersion"]) > int(a2["metadata"]["resourceVersion"])


def test_stale_update_conflicts(store):
    rt = mi(store)
    a = store.create(rt, "default", pool("a"))
    fresh = copy.deepcopy(a)
    fresh["spec"]["replicas"] = 2
    store.update(rt, "default", "a", fresh)
    a["spec"]["replicas"] = 5
    with pytest.raises(ApiError) as e:
        store.update(rt, "default", "a", a)
    assert e.value.code == 409


def test_noop_update_keeps_rv(store):
    rt = mi(store)
    a = store.create(rt, "default", pool("a"))
    b = store.update(rt, "default", "a", copy.deepcopy(a))
    assert b["metadata"]["resourceVersion"] == a["metadata"]["resourceVersion"]


def test_status_subresource_isolation(store):
    rt = mi(store)
    a = store.create(rt, "default", {**pool("a"), "status": {"readyReplicas": 9}})
    assert "status" not in a  # status not settable on create
    a["status"] = {"readyReplicas": 1}
    a["spec"]["replicas"] = 7
    b = store.update(rt, "default", "a", a, subresource="status")
    assert b["status"]["readyReplicas"] == 1
    assert b["spec"]["replicas"] == 1  # spec change via /status ignored
    assert b["metadata"]["generation"] == 1
    b["status"] = {"readyReplicas": 42}
    c = store.update(rt, "default", "a", b)  # status change via main resource ignored
    assert c["status"]["readyReplicas"] == 1


def test_validation_and_defaulting(store):
    rt = mi(store)
    with pytest.raises(ApiError) as e:
        store.create(rt, "default", pool("neg", replicas=-1))
    assert e.value.code == 422 and "spec.replicas" in e.value.message
    with pytest.raises(ApiError):
        store.create(rt, "default", pool("bad", resourceName="NOT VALID"))
    a = store.create(rt, "default", pool("d", unknownField=1))
    assert "unknownField" not in a["spec"]  # pruned
    assert a["spec"]["resourceName"] == "amd.com/gpu"
    assert a["spec"]["probe"]["hbmBytes"] == 1 << 30
    assert a["spec"]["health"]["maxUncorrectableECC"] == 0


def test_azure_required_fields(store):
    rt = store.lookup("compute.my.domain", "azurevmpools")
    doc = yaml.safe_load(open(os.path.join(ROOT, "config", "samples",
                                           "compute_v1alpha1_azurevmpool.yaml")))
    store.create(rt, "default", doc)
    del doc["spec"]["vmSize"]
    doc["metadata"]["name"] = "x"
    with pytest.raises(ApiError) as e:
        store.create(rt, "default", doc)
    assert "vmSize" in e.value.message


def test_finalizer_two_phase_delete(store):
    rt = mi(store)
    a = store.create(rt, "default", {**pool("a"), "metadata": {"name": "a",
                                                              "finalizers": ["x/y"]}})
    d = store.delete(rt, "default", "a")
    assert d["metadata"]["deletionTimestamp"]
    assert d["metadata"]["generation"] == 2
    cur = store.get(rt, "default", "a")
    cur["metadata"]["finalizers"] = ["x/y", "new/one"]
    with pytest.raises(ApiError):
        store.update(rt, "default", "a", cur)  # no new finalizers while deleting
    cur["metadata"]["finalizers"] = []
    store.update(rt, "default", "a", cur)
    with pytest.raises(ApiError) as e:
        store.get(rt, "default", "a")
    assert e.value.code == 404
    assert a["metadata"]["uid"]


def test_pod_graceful_delete_and_eviction(store):
    pods = store.types[("", "pods")]
    store.create(pods, "default", {"metadata": {"name": "p"}, "spec": {
        "nodeName": "n0", "containers": [{"name": "c"}]}})
    store.evict("default", "p", {"deleteOptions": {"gracePeriodSeconds": 5}})
    p = store.get(pods, "default", "p")
    assert p["metadata"]["deletionTimestamp"] and p["metadata"]["deletionGracePeriodSeconds"] == 5
    store.delete(pods, "default", "p", grace=0)
    with pytest.raises(ApiError):
        store.get(pods, "default", "p")
    # unbound pods go away immediately
    store.create(pods, "default", {"metadata": {"name": "q"}, "spec": {"containers": [{}]}})
    store.delete(pods, "default", "q")
    with pytest.raises(ApiError):
        store.get(pods, "default", "q")


def test_watch_window_compaction(store):
    rt = mi(store)
    store.create(rt, "default", pool("a"))
    first = store.rv
    for i in range(150):
        store.create(rt, "default", pool(f"x{i}"))
    with pytest.raises(ApiError) as e:
        store.events_since(rt, first - 1)
    assert e.value.code == 410
    evs = store.events_since(rt, store.rv - 3)
    assert len(evs) == 3


def test_scale_subresource(store):
    rt = mi(store)
    store.create(rt, "default", pool("a", replicas=1))
    sc = store.get_scale(rt, "default", "a")
    assert sc["spec"]["replicas"] == 1
    sc["spec"]["replicas"] = 4
    out = store.update_scale(rt, "default", "a", sc)
    assert out["spec"]["replicas"] == 4
    assert store.get(rt, "default", "a")["metadata"]["generation"] == 2


def test_owner_gc_and_namespace_cascade(store):
    rt = mi(store)
    ev = store.types[("", "events")]
    a = store.create(rt, "team", pool("a"))
    store.create(ev, "team", {"metadata": {"name": "e1", "ownerReferences": [
        {"uid": a["metadata"]["uid"], "kind": "Mi355xPool", "name": "a"}]}})
    store.delete(rt, "team", "a")
    with pytest.raises(ApiError):
        store.get(ev, "team", "e1")
    store.create(ev, "team", {"metadata": {"name": "e2"}})
    store.delete(store.types[("", "namespaces")], None, "team")
    assert store.list(ev, "team")["items"] == []


def test_secret_string_data_and_selectors(store):
    sec = store.types[("", "secrets")]
    s = store.create(sec, "default", {"metadata": {"name": "s", "labels": {"a": "1"}},
                                      "stringData": {"K": "v"}})
    assert s["data"]["K"] == "dg=="
    assert parse_label_selector("a=1,b!=2")({"a": "1"})
    assert not parse_label_selector("a in (2,3)")({"a": "1"})
    assert parse_label_selector("!c,a")({"a": "x"})
    assert len(store.list(sec, "default", label_selector="a=1")["items"]) == 1
    assert store.list(sec, "default", field_selector="metadata.name=zz")["items"] == []


def test_patches():
    assert merge_patch({"a": {"b": 1, "c": 2}}, {"a": {"b": None, "d": 3}}) == {"a": {"c": 2, "d": 3}}
    doc = {"a": [1, 2], "b": {"c": 1}}
    out = json_patch(doc, [{"op": "add", "path": "/a/-", "value": 3},
                           {"op": "replace", "path": "/b/c", "value": 5},
                           {"op": "test", "path": "/b/c", "value": 5},
                           {"op": "move", "from": "/b/c", "path": "/z"}])
    assert out == {"a": [1, 2, 3], "b": {}, "z": 5}
    with pytest.raises(ApiError):
        json_patch(doc, [{"op": "test", "path": "/a/0", "value": 9}])


def test_crd_deletion_removes_instances(store):
    rt = mi(store)
    store.create(rt, "default", pool("a"))
    crd_rt = store.types[("apiextensions.k8s.io", "customresourcedefinitions")]
    store.delete(crd_rt, None, "mi355xpools.compute.my.domain")
    with pytest.raises(ApiError):
        store.lookup("compute.my.domain", "mi355xpools")


def _gpu_pod(name, n=None, phase=None):
    c = {"name": "m", "image": "x"}
    if n is not None:
        c["resources"] = {"limits": {"amd.com/gpu": n}}
    p = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name}, "spec": {"containers": [c]}}
    if phase:
        p["status"] = {"phase": phase}
    return p


def test_limitrange_defaults_and_bounds_gpu_per_container(store):
    """LimitRange (GPU调度平台搭建.md:802): a container naming no GPU gets the default; one asking
    above max (or a pod summing above the Pod max) is refused with 403 Forbidden."""
    lr, pods = store.types[("", "limitranges")], store.types[("", "pods")]
    store.create(lr, "team", {"metadata": {"name": "gpu-limits"}, "spec": {"limits": [
        {"type": "Container", "default": {"amd.com/gpu": 1}, "max": {"amd.com/gpu": "4"}},
        {"type": "Pod", "max": {"amd.com/gpu": 6}}]}})
    p = store.create(pods, "team", _gpu_pod("d"))
    res = p["spec"]["containers"][0]["resources"]
    assert res["limits"]["amd.com/gpu"] == 1 and res["requests"]["amd.com/gpu"] == 1
    with pytest.raises(ApiError) as e:
        store.create(pods, "team", _gpu_pod("big", 8))
    assert e.value.code == 403 and "maximum amd.com/gpu usage per Container is 4" in str(e.value)
    two = _gpu_pod("two", 4)
    two["spec"]["containers"].append({"name": "n", "image": "x",
                                      "resources": {"limits": {"amd.com/gpu": 4}}})
    with pytest.raises(ApiError) as e:
        store.create(pods, "team", two)
    assert e.value.code == 403 and "per Pod is 6" in str(e.value)
    # other namespaces are unaffected
    assert "resources" not in store.create(pods, "default", _gpu_pod("free"))["spec"]["containers"][0]


def test_resourcequota_admission_and_status_used(store):
    q, pods = store.types[("", "resourcequotas")], store.types[("", "pods")]
    store.create(q, "team", {"metadata": {"name": "gpu-quota"},
                             "spec": {"hard": {"requests.amd.com/gpu": "3", "pods": "5"}}})
    store.create(pods, "team", _gpu_pod("a", 2))
    got = store.get(q, "team", "gpu-quota")["status"]
    assert got["used"] == {"requests.amd.com/gpu": "2", "pods": "1"}
    with pytest.raises(ApiError) as e:
        store.create(pods, "team", _gpu_pod("b", 2))
    assert e.value.code == 403 and "exceeded quota: gpu-quota" in str(e.value) and \
        "used: requests.amd.com/gpu=2" in str(e.value)
    store.create(pods, "team", _gpu_pod("c", 1))
    # a finished pod no longer counts; deleting one frees its share
    done = store.get(pods, "team", "a")
    done["status"] = {"phase": "Succeeded"}
    store.update(pods, "team", "a", done, subresource="status")
    assert store.get(q, "team", "gpu-quota")["status"]["used"]["requests.amd.com/gpu"] == "1"
    store.create(pods, "team", _gpu_pod("b", 2))
    store.delete(pods, "team", "b")
    assert store.get(q, "team", "gpu-quota")["status"]["used"]["requests.amd.com/gpu"] == "1"


def test_resourcequota_table_shows_used_over_hard():
    """`gpuctl get quota` (the Table the sim serves, kubectl's columns): per-resource used/hard,
    requests and limits apart — the team's GPU budget at a glance (GPU调度平台搭建.md:802)."""
    from gpupool.apiserver_sim.server import to_table
    st = Store()
    rt = st.types[("", "resourcequotas")]
    q = {"metadata": {"name": "gpu-quota", "creationTimestamp": "2026-01-01T00:00:00Z"},
         "spec": {"hard": {"requests.amd.com/gpu": "4", "limits.amd.com/gpu": "4", "pods": "10"}},
         "status": {"hard": {"requests.amd.com/gpu": "4", "limits.amd.com/gpu": "4", "pods": "10"},
                    "used": {"requests.amd.com/gpu": "3", "pods": "2"}}}
    tbl = to_table(rt, [q], "1")
    cols = [c["name"] for c in tbl["columnDefinitions"]]
    assert cols == ["Name", "Age", "Request", "Limit"]
    cells = tbl["rows"][0]["cells"]
    assert cells[2] == "pods: 2/10, requests.amd.com/gpu: 3/4"
    assert cells[3] == "limits.amd.com/gpu: 0/4"


def test_old_watch_events_are_compacted_but_still_served():
    """Events older than the newest LIVE_EVENTS keep only their encoded watch line (no object
    tree for the garbage collector); a watch resuming from far back still gets them decoded."""
    st = Store()
    rt = st.types[("", "configmaps")]
    n = Store.LIVE_EVENTS + 100
    for i in range(n):
        st.create(rt, "default", {"metadata": {"name": f"c{i}"}, "data": {"i": str(i)}})
    evs = st.events_since(rt, 0)
    assert len(evs) == n
    assert evs[0]._obj is None and evs[-1]._obj is not None
    assert [e.obj["data"]["i"] for e in evs] == [str(i) for i in range(n)]
    assert sum(1 for e in st.log if e._obj is not None) == Store.LIVE_EVENTS


def test_update_copy_semantics(store):
    """The store never shares its objects with a caller unless asked: default writes copy the
    body in and the result out; the HTTP front-end (owned body, copy_out=False) gets the stored
    object for serialisation, and the watch event keeps its own copy either way."""
    rt = mi(store)
    store.create(rt, "default", pool("a"))
    body = store.get(rt, "default", "a")
    body["status"] = {"readyReplicas": 0}
    out = store.update(rt, "default", "a", body, "status")
    body["status"]["readyReplicas"] = 5
    out["status"]["readyReplicas"] = 6
    assert store.get(rt, "default", "a")["status"]["readyReplicas"] == 0
    body = store.get(rt, "default", "a")
    body["status"] = {"readyReplicas": 1}
    out = store.update(rt, "default", "a", body, "status", owned=True, copy_out=False)
    assert out is store.objects[rt.key][("default", "a")] and out["status"] is body["status"]
    ev = store.log[-1]
    assert ev.obj is not out and ev.obj == out


def test_events_since_filters_by_type_and_resource_version(store):
    """A resuming watch gets exactly its own type's events newer than its resourceVersion, in
    order, with other types' events interleaved in the log."""
    mi_rt = mi(store)
    cm_rt = store.lookup("", "configmaps") if ("", "configmaps") in store.types else None
    other = cm_rt or store.types[("", "namespaces")]
    a = store.create(mi_rt, "default", pool("a"))
    rv_a = int(a["metadata"]["resourceVersion"])
    for i in range(5):
        store.patch(mi_rt, "default", "a", {"spec": {"replicas": i + 2}}, "merge")
        if other.kind == "Namespace":
            store.create(other, None, {"apiVersion": "v1", "kind": "Namespace",
                                       "metadata": {"name": f"ns{i}"}})
        else:
            store.create(other, "default", {"apiVersion": "v1", "kind": "ConfigMap",
                                            "metadata": {"name": f"c{i}"}})
    evs = store.events_since(mi_rt, rv_a)
    assert [e.rtype for e in evs] == [mi_rt.key] * 5
    assert [e.obj["spec"]["replicas"] for e in evs] == [2, 3, 4, 5, 6]
    assert all(e.rv > rv_a for e in evs) and [e.rv for e in evs] == sorted(e.rv for e in evs)
    assert store.events_since(mi_rt, store.rv) == []
    mid = evs[2].rv
    assert [e.obj["spec"]["replicas"] for e in store.events_since(mi_rt, mid)] == [5, 6]
