"""`make deploy` path: every shipped manifest (CRDs, manager Namespace/SA/binding/Deployment,
generated RBAC for manager and agent, agent DaemonSet) applies cleanly, in the Makefile's order,
to the apiserver simulator through gpuctl; and the RBAC grants cover every API call the manager
and agent make (audited against their sources)."""
from __future__ import annotations

import glob
import os
import re
import subprocess
import sys

from gpupool.api import schema
from gpupool.kube import BY_KIND

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _gpuctl(server: str, *args: str) -> subprocess.CompletedProcess:
    env = dict(os.environ, PYTHONPATH=ROOT, GPUPOOL_APISERVER=server)
    return subprocess.run([sys.executable, "-m", "gpupool.cli", *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=60)


def test_deploy_order_applies_cleanly(cluster_factory):
    c = cluster_factory(nodes=[], manager=False)
    applied = []
    for d in ("config/crd", "config/manager", "config/rbac", "config/agent"):
        r = _gpuctl(c.url, "apply", "-f", d)
        assert r.returncode == 0, (d, r.stdout, r.stderr)
        applied += [line.split()[0] for line in r.stdout.splitlines() if line.strip()]
    kinds = {a.split("/")[0].split(".")[0] for a in applied}
    for k in ("customresourcedefinition", "namespace", "serviceaccount", "clusterrole",
              "clusterrolebinding", "deployment", "daemonset"):
        assert k in kinds, (k, applied)
    dep = c.client.get(BY_KIND["Deployment"], "gpupool-manager", "gpupool-system")
    assert dep["spec"]["template"]["spec"]["serviceAccountName"] == "gpupool-manager"
    ds = c.client.get(BY_KIND["DaemonSet"], "gpupool-agent", "gpupool-system")
    assert ds["spec"]["template"]["spec"]["serviceAccountName"] == "gpupool-agent"


def _granted(rules: list[dict]) -> set[tuple[str, str]]:
    return {(res, verb) for r in rules for res in r["resources"] for verb in r["verbs"]}


def test_manager_rbac_covers_native_api_calls():
    """Every (resource, verb) the C++ manager issues is granted by the generated ClusterRole."""
    src = ""
    for dirpath, _, files in os.walk(os.path.join(ROOT, "native", "src")):
        for f in files:
            if f.endswith(".cc"):
                src += open(os.path.join(dirpath, f)).read()
    verb_of = {"get": "get", "list": "list", "create": "create", "update": "update",
               "patch_merge": "patch", "del": "delete", "evict": "create"}
    used = set()
    for m in re.finditer(r"client_?(?:->|\.)(get|list|create|update|patch_merge|del)\(res::(\w+)\(\)"
                         r"(?:[^;]*?\"status\")?", src):
        verb, res = verb_of[m.group(1)], m.group(2)
        used.add((res + ("/status" if m.group(0).endswith('"status"') else ""), verb))
    if "evict(" in src:
        used.add(("pods/eviction", "create"))
    # the reconcilers' own kind (res_): status writes, finalizer patches, conflict re-reads
    for plural in ("mi355xpools", "azurevmpools"):
        used |= {(plural + "/status", "update"), (plural, "patch"), (plural, "get")}
    # informers list+watch
    for m in re.finditer(r"Informer \w+\(client, res::(\w+)\(\)", src):
        used |= {(m.group(1), "list"), (m.group(1), "watch")}
    granted = _granted(schema.rbac_role()["rules"])
    missing = sorted(u for u in used if u not in granted)
    assert used and not missing, missing


def test_agent_rbac_covers_agent_api_calls():
    import glob
    src = "".join(open(p).read() for p in glob.glob(os.path.join(ROOT, "gpupool", "agent", "*.py")))
    used = set()
    for m in re.finditer(r"(?:\bc|self\.client)\.(get|create|patch|update|delete|list)\((\w+)"
                         r"[^)]*?(sub=\"status\")?\)", src):
        res = {"NODES": "nodes", "PODS": "pods"}.get(m.group(2), m.group(2).lower())
        used.add((res + ("/status" if m.group(3) else ""), m.group(1)))
    granted = set()
    for o in schema.agent_rbac():
        if o["kind"] == "ClusterRole":
            granted = _granted(o["rules"])
    missing = sorted(u for u in used if u not in granted)
    assert used and not missing, (used, missing)
    # the kubelet registers Nodes: the agent can neither create one nor edit its spec/status
    # beyond what the ValidatingAdmissionPolicy admits (schema.agent_node_policy)
    assert ("nodes", "create") not in granted and ("nodes", "create") not in used
    kinds = [o["kind"] for o in schema.agent_rbac()]
    assert "ValidatingAdmissionPolicy" in kinds and "ValidatingAdmissionPolicyBinding" in kinds


def test_kustomization_lists_every_deploy_manifest():
    import glob

    import yaml
    kz = yaml.safe_load(open(os.path.join(ROOT, "config", "default", "kustomization.yaml")))
    listed = {os.path.normpath(os.path.join(ROOT, "config", "default", r)) for r in kz["resources"]}
    shipped = {os.path.normpath(p) for d in ("crd", "manager", "rbac", "agent")
               for p in glob.glob(os.path.join(ROOT, "config", d, "*.yaml"))}
    assert listed == shipped
    mon = list(yaml.safe_load_all(open(os.path.join(ROOT, "config", "prometheus", "monitor.yaml"))))
    assert {m["kind"] for m in mon} == {"Service", "ServiceMonitor"}


def _json_patch_add(doc, path: str, value) -> None:
    parts = [p.replace("~1", "/").replace("~0", "~") for p in path.lstrip("/").split("/")]
    for p in parts[:-1]:
        doc = doc[int(p)] if isinstance(doc, list) else doc[p]
    last = parts[-1]
    if isinstance(doc, list):
        doc.append(value) if last == "-" else doc.insert(int(last), value)
    else:
        doc[last] = value


def test_azure_overlay_flags_are_manager_flags(native_built):
    """config/azure (kustomize overlay): the patched Deployment runs the ARM provider, and every
    argument it passes is a flag the manager binary accepts."""
    import yaml

    from gpupool.testing.cluster import native_bin
    kz = yaml.safe_load(open(os.path.join(ROOT, "config", "azure", "kustomization.yaml")))
    assert kz["resources"] == ["../default"]
    dep = next(d for d in yaml.safe_load_all(open(os.path.join(ROOT, "config", "manager",
                                                               "manager.yaml")))
               if d and d["kind"] == "Deployment")
    for p in kz["patches"]:
        assert p["target"]["name"] == dep["metadata"]["name"]
        for op in yaml.safe_load(p["patch"]):
            assert op["op"] == "add"
            _json_patch_add(dep, op["path"], op["value"])
    spec = dep["spec"]["template"]["spec"]
    args = spec["containers"][0]["args"]
    assert args[args.index("--cloud") + 1] == "azure-arm"
    mounts = {m["name"] for m in spec["containers"][0]["volumeMounts"]}
    assert mounts <= {v["name"] for v in spec["volumes"]}
    assert dep["spec"]["template"]["metadata"]["labels"]["azure.workload.identity/use"] == "true"
    r = subprocess.run([native_bin("gpupool-manager"), *args, "--help"], capture_output=True,
                       text=True, timeout=30)
    assert r.returncode == 0, r.stderr


def test_every_sample_applies(cluster_factory):
    """Every manifest under config/samples passes admission (CRD schemas, built-in kinds incl. the
    NFS workspace PersistentVolume/Claim) on the apiserver simulator."""
    import glob
    c = cluster_factory(nodes=[], manager=False)
    files = sorted(glob.glob(os.path.join(ROOT, "config", "samples", "*.yaml")))
    assert files
    for f in files:
        r = _gpuctl(c.url, "apply", "-f", f)
        assert r.returncode == 0, (f, r.stdout, r.stderr)
    pvc = c.client.get(BY_KIND["PersistentVolumeClaim"], "workspace", "default")
    assert pvc["spec"]["volumeName"] == "gpupool-workspace"
    job = c.client.get(BY_KIND["Mi355xJob"], "fmnist-ddp", "default")
    assert job["spec"]["checkpointDir"].startswith("/workspace/")


def test_alert_rules_use_exported_metrics():
    """Every metric an alert in config/prometheus/alerts.yaml queries is exported by the manager
    (C++ sources) or the node agent, with the label values the rules select on."""
    import yaml
    doc = yaml.safe_load(open(os.path.join(ROOT, "config", "prometheus", "alerts.yaml")))
    src = "".join(open(f).read() for f in glob.glob(os.path.join(ROOT, "gpupool", "agent", "*.py")))
    for dirpath, _, files in os.walk(os.path.join(ROOT, "native", "src")):
        for f in files:
            if f.endswith(".cc"):
                src += open(os.path.join(dirpath, f)).read()
    rules = [r for g in doc["spec"]["groups"] for r in g["rules"]]
    assert len(rules) >= 8
    for r in rules:
        for m in re.findall(r"(?:gpupool|process)_[a-z_]+", r["expr"]):
            assert m in src, (r["alert"], m)
    for label in ('"uncorrectable"', '"hotspot"', '"error"', '"terminal"', 'state="{t}"'):
        assert label in src, label
