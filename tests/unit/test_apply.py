"""``kubectl apply`` semantics: gpuctl's client-side three-way apply (last-applied-configuration)
and server-side apply with field ownership in apiserver-sim (gpupool/apiserver_sim/ssa.py).

Parity: the reference's users apply their manifests with ``kubectl apply -f``
(README.md:288-290, GPU调度平台搭建.md:500-510); re-applying a manifest must not undo what the
operator, a ``scale`` or another user changed outside it. Server-side apply's conflict and
ownership rules follow the Kubernetes documentation of the feature (parity unpinned: no
kube-apiserver runs in this container)."""
from __future__ import annotations

import json

import pytest

from gpupool.api.smp import strategic_merge, three_way
from gpupool.apiserver_sim.store import ApiError, Store
from gpupool.cli import gpuctl
from gpupool.kube import CONFIGMAPS, MI355XPOOLS, NODES, Client, KubeError, Res
from tests.unit.test_apiserver_http import SimThread

DEPLOYMENTS = Res("apps", "v1", "deployments")
LAST = Client.LAST_APPLIED


def _pool(replicas=1, labels=None, **spec):
    return {"apiVersion": "compute.my.domain/v1alpha1", "kind": "Mi355xPool",
            "metadata": {"name": "p", "labels": labels or {"team": "a"}},
            "spec": {"replicas": replicas, **spec}}


def _deploy(env):
    return {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "d"},
            "spec": {"replicas": 1, "selector": {"matchLabels": {"app": "d"}},
                     "template": {"metadata": {"labels": {"app": "d"}},
                                  "spec": {"containers": [{"name": "c", "image": "i",
                                                           "env": env}]}}}}


# ---------------------------------------------------------------- three-way, as a function
def test_three_way_keeps_what_others_set_and_drops_what_the_manifest_dropped():
    orig = {"metadata": {"labels": {"a": "1", "b": "2"}}, "spec": {"x": 1, "y": 2}}
    mod = {"metadata": {"labels": {"a": "1"}}, "spec": {"x": 5}}
    cur = {"metadata": {"labels": {"a": "1", "b": "2", "other": "o"}},
           "spec": {"x": 1, "y": 2, "z": 3}}
    p = three_way(orig, mod, cur, None)
    assert p == {"metadata": {"labels": {"b": None}}, "spec": {"y": None, "x": 5}}
    # keyed lists (strategic): an element the last apply had is deleted, one others added stays
    orig = {"spec": {"containers": [{"name": "a", "image": "1"}, {"name": "b", "image": "1"}]}}
    mod = {"spec": {"containers": [{"name": "a", "image": "2"}]}}
    cur = {"spec": {"containers": [{"name": "a", "image": "1"}, {"name": "b", "image": "1"},
                                   {"name": "sidecar", "image": "s"}]}}
    p = three_way(orig, mod, cur, "Pod")
    out = strategic_merge(cur, p, "Pod")
    assert out["spec"]["containers"] == [{"name": "a", "image": "2"},
                                         {"name": "sidecar", "image": "s"}]
    # nothing to do: an empty patch
    assert three_way(mod, mod, strategic_merge(cur, p, "Pod"), "Pod") == {}


# ---------------------------------------------------------------- client-side apply over HTTP
def test_client_side_apply_is_a_three_way_merge():
    sim = SimThread()
    c = Client(sim.url)
    action, o = c.apply(_pool(1, {"team": "a", "tier": "gold"}), "default")
    assert action == "created"
    assert json.loads(o["metadata"]["annotations"][LAST])["spec"] == {"replicas": 1}
    # another user labels it and sets a field the manifest does not carry
    c.patch(MI355XPOOLS, "p", {"metadata": {"labels": {"owner": "ops"}},
                               "spec": {"maxNodes": 4}}, "default")
    rv = c.get(MI355XPOOLS, "p", "default")["metadata"]["resourceVersion"]
    action, o = c.apply(_pool(1, {"team": "a", "tier": "gold"}), "default")
    assert action == "unchanged" and o["metadata"]["resourceVersion"] == rv
    # the manifest drops a label it had set and changes replicas: only those move
    action, o = c.apply(_pool(2, {"team": "a"}), "default")
    assert action == "configured"
    assert o["metadata"]["labels"] == {"team": "a", "owner": "ops"}
    assert o["spec"]["replicas"] == 2 and o["spec"]["maxNodes"] == 4
    # the old replace semantics would have reset maxNodes to its default (1)


def test_client_side_apply_on_a_builtin_uses_strategic_merge():
    sim = SimThread()
    c = Client(sim.url)
    c.apply(_deploy([{"name": "A", "value": "1"}, {"name": "B", "value": "2"}]), "default")
    # an admission webhook / another tool adds an env var to the same container
    c.patch(DEPLOYMENTS, "d", {"spec": {"template": {"spec": {"containers": [
        {"name": "c", "env": [{"name": "INJECTED", "value": "x"}]}]}}}}, "default",
        ptype="strategic")
    action, o = c.apply(_deploy([{"name": "A", "value": "1"}]), "default")
    assert action == "configured"
    env = o["spec"]["template"]["spec"]["containers"][0]["env"]
    assert {e["name"] for e in env} == {"A", "INJECTED"}


def test_gpuctl_apply_twice_reports_unchanged(tmp_path, capsys):
    sim = SimThread()
    f = tmp_path / "cm.yaml"
    f.write_text("apiVersion: v1\nkind: ConfigMap\nmetadata:\n  name: cm\ndata:\n  a: '1'\n")
    assert gpuctl.main(["--server", sim.url, "apply", "-f", str(f)]) == 0
    assert gpuctl.main(["--server", sim.url, "apply", "-f", str(f)]) == 0
    out = capsys.readouterr().out.splitlines()
    assert out[-2].endswith("created") and out[-1].endswith("unchanged")


# ---------------------------------------------------------------- server-side apply
def _cm(data, name="c", labels=None):
    md = {"name": name}
    if labels:
        md["labels"] = labels
    return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": md, "data": data}


def _owners(o):
    return {e["manager"]: (e["operation"], e["fieldsV1"]) for e in o["metadata"]["managedFields"]}


def test_ssa_ownership_conflicts_force_and_removal():
    st = Store()
    cm = st.lookup("", "configmaps")
    o = st.apply(cm, "default", "c", _cm({"x": "1", "y": "2"}, labels={"a": "1"}), "alice")
    assert _owners(o) == {"alice": ("Apply", {"f:data": {"f:x": {}, "f:y": {}},
                                              "f:metadata": {"f:labels": {"f:a": {}}}})}
    # a plain write takes the fields it changes, silently (operation Update)
    o = st.patch(cm, "default", "c", {"data": {"y": "20", "z": "3"}}, "merge", manager="bob")
    assert _owners(o)["bob"] == ("Update", {"f:data": {"f:y": {}, "f:z": {}}})
    assert _owners(o)["alice"][1]["f:data"] == {"f:x": {}}
    # alice re-applies a different z: a conflict naming bob
    with pytest.raises(ApiError) as ei:
        st.apply(cm, "default", "c", _cm({"x": "1", "z": "9"}), "alice")
    assert ei.value.code == 409 and 'conflict with "bob": .data.z' in str(ei.value)
    # the same value is no conflict: shared ownership
    o = st.apply(cm, "default", "c", _cm({"x": "1", "z": "3"}), "alice")
    assert "f:z" in _owners(o)["alice"][1]["f:data"] and "f:z" in _owners(o)["bob"][1]["f:data"]
    # alice stops applying x and the label: removed (nobody else owns them); y stays (bob's)
    o = st.apply(cm, "default", "c", _cm({"z": "3"}), "alice")
    assert o["data"] == {"y": "20", "z": "3"} and not o["metadata"].get("labels")
    # force takes the field
    o = st.apply(cm, "default", "c", _cm({"z": "4", "y": "5"}), "alice", force=True)
    assert o["data"] == {"y": "5", "z": "4"}
    assert "bob" not in _owners(o)  # bob owned only y and z: that entry is gone


def test_ssa_keyed_lists_node_conditions_and_first_apply():
    """The agent could own its Node conditions by server-side apply: kubelet's Ready is another
    manager's element of the same list and survives every apply, and a condition the agent stops
    applying disappears."""
    st = Store()
    nodes = st.lookup("", "nodes")
    st.create(nodes, None, {"apiVersion": "v1", "kind": "Node", "metadata": {"name": "n"},
                            "status": {"conditions": [{"type": "Ready", "status": "True"}]}})
    cfg = {"apiVersion": "v1", "kind": "Node", "metadata": {"name": "n"}, "status": {
        "conditions": [{"type": "ROCmReady", "status": "True"},
                       {"type": "GPUPoolAgentReady", "status": "True"}]}}
    o = st.apply(nodes, None, "n", cfg, "gpupool-agent", subresource="status")
    owners = _owners(o)
    assert owners["before-first-apply"][0] == "Update"  # the existing Ready has an owner
    assert 'k:{"type":"ROCmReady"}' in owners["gpupool-agent"][1]["f:status"]["f:conditions"]
    st.patch(nodes, None, "n", {"status": {"conditions": [{"type": "Ready", "status": "False"}]}},
             "strategic", "status", manager="kubelet")
    cfg["status"]["conditions"] = [{"type": "GPUPoolAgentReady", "status": "False"}]
    o = st.apply(nodes, None, "n", cfg, "gpupool-agent", subresource="status")
    assert {c["type"]: c["status"] for c in o["status"]["conditions"]} == \
        {"Ready": "False", "GPUPoolAgentReady": "False"}
    # status through the main resource is not applied (the type has a status subresource)
    o2 = st.apply(nodes, None, "n", {"apiVersion": "v1", "kind": "Node", "metadata": {
        "name": "n", "labels": {"x": "1"}}, "status": {"conditions": []}}, "someone")
    assert o2["status"] == o["status"] and o2["metadata"]["labels"] == {"x": "1"}


def test_ssa_over_http_with_gpuctl(tmp_path, capsys):
    sim = SimThread()
    c = Client(sim.url)
    f = tmp_path / "p.yaml"
    f.write_text(json.dumps(_pool(1)))
    base = ["--server", sim.url, "-n", "default"]
    assert gpuctl.main(base + ["apply", "--server-side", "--field-manager", "team-a", "-f",
                               str(f)]) == 0
    o = c.get(MI355XPOOLS, "p", "default")
    assert _owners(o)["team-a"][0] == "Apply" and o["spec"]["replicas"] == 1
    # gpuctl scale writes replicas (manager "gpuctl", from its User-Agent)
    assert gpuctl.main(base + ["scale", "mi355xpool", "p", "--replicas", "3"]) == 0
    f.write_text(json.dumps(_pool(2)))
    assert gpuctl.main(base + ["apply", "--server-side", "--field-manager", "team-a", "-f",
                               str(f)]) == 1
    assert 'conflict with "gpuctl": .spec.replicas' in capsys.readouterr().err
    assert gpuctl.main(base + ["apply", "--server-side", "--field-manager", "team-a",
                               "--force-conflicts", "-f", str(f)]) == 0
    o = c.get(MI355XPOOLS, "p", "default")
    assert o["spec"]["replicas"] == 2 and "gpuctl" not in _owners(o)
    # apply creates; fieldManager is required
    with pytest.raises(KubeError) as ei:
        c.request("PATCH", CONFIGMAPS.path("default", "new"), _cm({"a": "1"}, "new"),
                  ctype="application/apply-patch+yaml")
    assert ei.value.code == 400
    out = c.request("PATCH", CONFIGMAPS.path("default", "new"), _cm({"a": "1"}, "new"),
                    ctype="application/apply-patch+yaml", query={"fieldManager": "m"})
    assert out["data"] == {"a": "1"} and _owners(out)["m"][0] == "Apply"
    # plain writes on objects nobody applied record nothing (the fast path)
    c.create(NODES, {"apiVersion": "v1", "kind": "Node", "metadata": {"name": "plain"}})
    c.patch(NODES, "plain", {"metadata": {"labels": {"a": "b"}}})
    assert "managedFields" not in c.get(NODES, "plain")["metadata"]


def test_gpuctl_diff_shows_what_apply_would_change(tmp_path, capsys):
    """``kubectl diff``: a server-side dry run of the apply, compared with the live object."""
    sim = SimThread()
    c = Client(sim.url)
    f = tmp_path / "p.yaml"
    f.write_text(json.dumps(_pool(1)))
    base = ["--server", sim.url, "-n", "default"]
    assert gpuctl.main(base + ["diff", "-f", str(f)]) == 1  # not there yet: all of it is new
    out = capsys.readouterr().out
    assert "+  replicas: 1" in out and "+  resourceName: amd.com/gpu" in out  # defaulted
    assert gpuctl.main(base + ["apply", "-f", str(f)]) == 0
    capsys.readouterr()
    assert gpuctl.main(base + ["diff", "-f", str(f)]) == 0
    assert capsys.readouterr().out == ""
    f.write_text(json.dumps(_pool(3)))
    assert gpuctl.main(base + ["diff", "-f", str(f)]) == 1
    out = capsys.readouterr().out
    assert "-  replicas: 1" in out and "+  replicas: 3" in out
    assert c.get(MI355XPOOLS, "p", "default")["spec"]["replicas"] == 1  # a dry run only
    # server-side: the fields the client-side apply set have an owner (before-first-apply),
    # so changing one conflicts, as it would on a cluster, unless forced
    assert gpuctl.main(base + ["diff", "--server-side", "-f", str(f)]) == 2
    assert 'conflict with "before-first-apply": .spec.replicas' in capsys.readouterr().err
    assert gpuctl.main(base + ["diff", "--server-side", "--force-conflicts", "-f", str(f)]) == 1
    assert "+  replicas: 3" in capsys.readouterr().out


def test_jsonpath_output_and_wait(capsys):
    """``kubectl get -o jsonpath=`` / ``-o name`` and ``wait --for=jsonpath=`` (the reference's
    scripts read readyReplicas this way)."""
    from gpupool.cli.jsonpath import JsonPathError, render
    o = {"items": [{"metadata": {"name": "a", "annotations": {"gpupool.amd.com/x": "1"}},
                    "status": {"readyReplicas": 2, "conditions": [
                        {"type": "Ready", "status": "True"}, {"type": "X", "status": "False"}]}},
                   {"metadata": {"name": "b"}, "status": {"readyReplicas": 0}}]}
    assert render(o, '{range .items[*]}{.metadata.name}{"\\t"}{.status.readyReplicas}{"\\n"}{end}') \
        == "a\t2\nb\t0\n"
    assert render(o, "{.items[*].metadata.name}") == "a b"
    assert render(o, '{.items[0].status.conditions[?(@.type=="Ready")].status}') == "True"
    assert render(o, "{.items[0].metadata.annotations['gpupool.amd.com/x']}") == "1"
    assert render(o, "{.items[-1].metadata}") == '{"name":"b"}'
    with pytest.raises(JsonPathError):
        render(o, "{range .items[*]}{.x}")
    sim = SimThread()
    c = Client(sim.url)
    c.create(CONFIGMAPS, _cm({"a": "1"}, "one"), "default")
    base = ["--server", sim.url, "-n", "default"]
    assert gpuctl.main(base + ["get", "configmaps", "-o", "name"]) == 0
    assert "configmap/one" in capsys.readouterr().out.split()
    assert gpuctl.main(base + ["get", "configmaps", "one", "-o", "jsonpath={.data.a}"]) == 0
    assert capsys.readouterr().out == "1"
    assert gpuctl.main(base + ["wait", "configmaps", "one", "--for",
                               "jsonpath={.data.a}=1", "--timeout", "5"]) == 0
