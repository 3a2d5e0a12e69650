"""Strategic merge patch in apiserver-sim (gpupool/api/smp.py): list merge by
patchMergeKey for the built-in kinds, the patch directives, and the apiserver's 415 answers
(strategic merge patch on a custom resource, unknown patch media types)."""
from __future__ import annotations

import threading
import time

import pytest

from gpupool.api.smp import PatchError, strategic_merge, two_way
from gpupool.apiserver_sim.store import ApiError, Store
from gpupool.kube import MI355XPOOLS, NODES, PODS, Client, KubeError
from tests.unit.test_apiserver_http import SimThread


def _node(conds):
    return {"metadata": {"name": "n"}, "status": {"capacity": {"amd.com/gpu": "8"},
                                                   "conditions": conds}}


def test_conditions_merge_by_type():
    cur = _node([{"type": "Ready", "status": "True", "lastHeartbeatTime": "T0"},
                 {"type": "ROCmReady", "status": "True", "lastTransitionTime": "A"}])
    out = strategic_merge(cur, {"status": {"conditions": [
        {"type": "ROCmReady", "status": "False", "lastTransitionTime": "B"},
        {"type": "GPUPoolAgentReady", "status": "True"}]}}, "Node")
    by = {c["type"]: c for c in out["status"]["conditions"]}
    assert by["Ready"] == {"type": "Ready", "status": "True", "lastHeartbeatTime": "T0"}
    assert by["ROCmReady"]["status"] == "False" and by["ROCmReady"]["lastTransitionTime"] == "B"
    assert by["GPUPoolAgentReady"]["status"] == "True"
    assert out["status"]["capacity"] == {"amd.com/gpu": "8"}
    assert cur["status"]["conditions"][1]["status"] == "True"  # the target is not modified


def test_merge_patch_would_have_replaced_the_list():
    """The contrast the simulator now draws: a JSON merge patch replaces lists whole."""
    from gpupool.apiserver_sim.store import merge_patch
    cur = _node([{"type": "Ready", "status": "True"}])
    out = merge_patch(cur, {"status": {"conditions": [{"type": "ROCmReady", "status": "True"}]}})
    assert [c["type"] for c in out["status"]["conditions"]] == ["ROCmReady"]


def test_directives():
    cur = {"metadata": {"finalizers": ["a", "b"], "labels": {"x": "1", "y": "2"}},
           "spec": {"containers": [{"name": "c1", "image": "i1",
                                    "env": [{"name": "A", "value": "1"}, {"name": "B", "value": "2"}]},
                                   {"name": "c2", "image": "i2"}]}}
    # primitive list with merge strategy: union
    out = strategic_merge(cur, {"metadata": {"finalizers": ["c", "a"]}}, "Pod")
    assert out["metadata"]["finalizers"] == ["a", "b", "c"]
    # $deleteFromPrimitiveList
    out = strategic_merge(cur, {"metadata": {"$deleteFromPrimitiveList/finalizers": ["a"]}}, "Pod")
    assert out["metadata"]["finalizers"] == ["b"]
    # nested keyed lists (containers by name, env by name) and $patch: delete on an element
    out = strategic_merge(cur, {"spec": {"containers": [
        {"name": "c1", "env": [{"name": "B", "$patch": "delete"}, {"name": "C", "value": "3"}]},
        {"name": "c2", "$patch": "delete"}]}}, "Pod")
    assert [c["name"] for c in out["spec"]["containers"]] == ["c1"]
    assert out["spec"]["containers"][0]["image"] == "i1"
    assert out["spec"]["containers"][0]["env"] == [{"name": "A", "value": "1"},
                                                   {"name": "C", "value": "3"}]
    # $patch: replace on a map and as a list element
    out = strategic_merge(cur, {"metadata": {"labels": {"$patch": "replace", "z": "3"}}}, "Pod")
    assert out["metadata"]["labels"] == {"z": "3"}
    out = strategic_merge(cur, {"spec": {"containers": [{"$patch": "replace"},
                                                         {"name": "only", "image": "i"}]}}, "Pod")
    assert out["spec"]["containers"] == [{"name": "only", "image": "i"}]
    # $retainKeys and null deletes
    out = strategic_merge(cur, {"metadata": {"labels": {"$retainKeys": ["x"], "x": "9"}}}, "Pod")
    assert out["metadata"]["labels"] == {"x": "9"}
    out = strategic_merge(cur, {"metadata": {"labels": {"y": None}}}, "Pod")
    assert out["metadata"]["labels"] == {"x": "1"}
    # $setElementOrder
    out = strategic_merge(cur, {"spec": {"$setElementOrder/containers": [{"name": "c2"},
                                                                         {"name": "c1"}]}}, "Pod")
    assert [c["name"] for c in out["spec"]["containers"]] == ["c2", "c1"]
    # a list without a strategy is atomic (Node taints)
    out = strategic_merge({"spec": {"taints": [{"key": "a"}]}},
                          {"spec": {"taints": [{"key": "b"}]}}, "Node")
    assert out["spec"]["taints"] == [{"key": "b"}]


def test_errors():
    with pytest.raises(PatchError, match="merge key"):
        strategic_merge(_node([]), {"status": {"conditions": [{"status": "True"}]}}, "Node")
    with pytest.raises(PatchError):
        strategic_merge(_node([]), {"status": {"$patch": "bogus"}}, "Node")


def test_two_way_round_trips():
    a = _node([{"type": "Ready", "status": "True"}, {"type": "X", "status": "False"}])
    b = _node([{"type": "Ready", "status": "False"}, {"type": "Y", "status": "True"}])
    b["status"]["capacity"] = {"amd.com/gpu": "7"}
    p = two_way(a, b, "Node")
    assert strategic_merge(a, p, "Node") == b


def test_store_and_http_media_types():
    st = Store()
    st.create(st.lookup("", "nodes"), None, {"apiVersion": "v1", "kind": "Node",
                                             "metadata": {"name": "n"}})
    rt = st.lookup("", "nodes")
    st.patch(rt, None, "n", {"status": {"conditions": [{"type": "Ready", "status": "True"}]}},
             "strategic", "status")
    out = st.patch(rt, None, "n", {"status": {"conditions": [{"type": "ROCmReady",
                                                               "status": "True"}]}},
                   "strategic", "status")
    assert {c["type"] for c in out["status"]["conditions"]} == {"Ready", "ROCmReady"}
    with pytest.raises(ApiError) as ei:
        st.patch(rt, None, "n", {"status": {"conditions": [{"status": "x"}]}}, "strategic",
                 "status")
    assert ei.value.code == 422

    sim = SimThread()
    c = Client(sim.url)
    c.create(NODES, {"apiVersion": "v1", "kind": "Node", "metadata": {"name": "n1"}})
    c.patch(NODES, "n1", {"status": {"conditions": [{"type": "Ready", "status": "True"}]}},
            sub="status", ptype="strategic")
    c.patch(NODES, "n1", {"status": {"conditions": [{"type": "Other", "status": "True"}]}},
            sub="status", ptype="strategic")
    assert {x["type"] for x in c.get(NODES, "n1")["status"]["conditions"]} == {"Ready", "Other"}
    # custom resources: 415 for strategic merge patch (as a real apiserver answers)
    c.create(MI355XPOOLS, {"apiVersion": "compute.my.domain/v1alpha1", "kind": "Mi355xPool",
                           "metadata": {"name": "p"}, "spec": {"replicas": 1}}, "default")
    with pytest.raises(KubeError) as ei:
        c.patch(MI355XPOOLS, "p", {"spec": {"replicas": 2}}, "default", ptype="strategic")
    assert ei.value.code == 415
    c.patch(MI355XPOOLS, "p", {"spec": {"replicas": 2}}, "default")  # merge patch is fine
    # an unknown patch media type: 415
    with pytest.raises(KubeError) as ei:
        c.request("PATCH", PODS.path("default", "x"), {}, ctype="application/yaml")
    assert ei.value.code == 415


def test_paged_list_and_filtered_watch_semantics():
    """LIST pages (continue tokens carry the first page's resourceVersion and the last key) and
    a label-selected watch turning a write that leaves / enters the selection into DELETED /
    ADDED, as the apiserver's watch cache does (the manager's filtered informers rely on both)."""
    sim = SimThread()
    c = Client(sim.url)
    for i in range(7):
        c.create(PODS, {"apiVersion": "v1", "kind": "Pod",
                        "metadata": {"name": f"p{i}", "labels": {"gpu": "yes" if i % 2 else "no"}},
                        "spec": {"containers": [{"name": "c"}]}}, "pg")
    seen, cont, rvs = [], None, set()
    while True:
        q = {"limit": 3, **({"continue": cont} if cont else {})}
        page = c.request("GET", PODS.path("pg"), query=q)
        seen += [o["metadata"]["name"] for o in page["items"]]
        rvs.add(page["metadata"]["resourceVersion"])
        c.create(PODS, {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": f"late{len(seen)}"},
                        "spec": {"containers": [{"name": "c"}]}}, "other")  # writes between pages
        cont = page["metadata"].get("continue")
        if not cont:
            break
    assert seen == sorted(f"p{i}" for i in range(7)) and len(rvs) == 1
    rv = c.list(PODS, "pg")["metadata"]["resourceVersion"]
    stop, evs = threading.Event(), []

    def watch():
        try:
            for ev in Client(sim.url).watch(PODS, "pg", resource_version=rv,
                                            label_selector="gpu=yes", stop=stop,
                                            timeout_seconds=10):
                if ev["type"] != "BOOKMARK":
                    evs.append((ev["type"], ev["object"]["metadata"]["name"]))
        except Exception:  # noqa: BLE001 — the stop shut the socket down mid-read
            pass
    t = threading.Thread(target=watch, daemon=True)
    t.start()
    time.sleep(0.3)
    c.patch(PODS, "p1", {"metadata": {"labels": {"gpu": "no"}}}, "pg")    # leaves
    c.patch(PODS, "p2", {"metadata": {"labels": {"gpu": "yes"}}}, "pg")   # enters
    c.patch(PODS, "p3", {"metadata": {"labels": {"x": "1"}}}, "pg")       # stays in
    c.patch(PODS, "p4", {"metadata": {"labels": {"x": "1"}}}, "pg")       # stays out
    deadline = time.monotonic() + 5
    while len(evs) < 3 and time.monotonic() < deadline:
        time.sleep(0.05)
    stop.set()
    assert evs == [("DELETED", "p1"), ("ADDED", "p2"), ("MODIFIED", "p3")], evs
