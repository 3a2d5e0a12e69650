"""A manager + agent pair across two apiserver-token rotations (round-5 missing #3: Workload
Identity / projected ServiceAccount tokens rotate, README.md:59-60, 312): apiserver-sim expires
each old token after its successor is in place; no reconcile may fail and no heartbeat be lost."""
from __future__ import annotations

import json
import os
import re
import time

from gpupool.api import schema
from gpupool.kube import MI355XPOOLS, NODES, Client
from gpupool.testing.cluster import NodeSpec

from .helpers import mi_pool, wait_ready

MANAGER = "system:serviceaccount:gpupool-system:gpupool-manager"


def _write(path: str, text: str) -> None:
    """What the kubelet does to a projected token: a new file swapped in atomically."""
    with open(path + ".tmp", "w") as f:
        f.write(text + "\n")
    os.replace(path + ".tmp", path)


def _metric(text: str, name: str, labels: str = "") -> float:
    tot = 0.0
    for ln in text.splitlines():
        if ln.startswith(name + ("{" if labels else "")) and labels in ln or ln.startswith(name + " "):
            try:
                tot += float(ln.rsplit(" ", 1)[1])
            except ValueError:
                pass
    return tot


def run_rotation(cluster_factory, tmp_path, manager_bin: str | None = None) -> dict:
    users = tmp_path / "users.json"
    mtok, atok = str(tmp_path / "manager-token"), str(tmp_path / "agent-token")
    agent_extra = {"authentication.kubernetes.io/node-name": ["rot-node"]}
    ident = {"m1": {"username": MANAGER}, "a1": {"username": schema.AGENT_SA_USER,
                                                  "extra": agent_extra}}
    users.write_text(json.dumps(ident))
    _write(mtok, "m1")
    _write(atok, "a1")
    kw = dict(nodes=[NodeSpec("rot-node", count=4,
                              extra_args=["--token-file", atok, "--heartbeat-interval", "0.2"])],
              token="admin", apiserver_args=["--users-file", str(users)],
              manager_args=["--token-file", mtok, "--workers", "4"])
    if manager_bin:
        kw["manager_bin"] = manager_bin
    c = cluster_factory(**kw)
    k = c.client
    admin = Client(c.url, "admin")
    k.create(MI355XPOOLS, mi_pool("rot", 2), "default")
    wait_ready(k, "rot", 2, timeout=60)
    sizes = [3, 1]
    for gen, size in zip((2, 3), sizes):
        new = {f"m{gen}": {"username": MANAGER},
               f"a{gen}": {"username": schema.AGENT_SA_USER, "extra": agent_extra}}
        admin.request("POST", "/debug/tokens", {"tokens": new, "merge": True})
        _write(mtok, f"m{gen}")
        _write(atok, f"a{gen}")
        time.sleep(0.3)
        # the old tokens expire now: every component's next call with them gets a 401
        old = {f"m{gen - 1}": {"username": MANAGER, "expiresAt": time.time() - 1},
               f"a{gen - 1}": {"username": schema.AGENT_SA_USER, "extra": agent_extra,
                               "expiresAt": time.time() - 1}}
        admin.request("POST", "/debug/tokens", {"tokens": old, "merge": True})
        k.patch(MI355XPOOLS, "rot", {"spec": {"replicas": size}}, "default")
        wait_ready(k, "rot", size, timeout=60)
        time.sleep(1.0)  # a few agent heartbeats on the new token
    node = k.get(NODES, "rot-node")
    conds = {x["type"]: x for x in node["status"]["conditions"]}
    mm = c.manager_metrics()
    am = c.agent_request("rot-node", "GET", "/metrics")
    sim = admin.request("GET", "/metrics")
    errors = _metric(mm, "gpupool_reconcile_total", 'result="error"') + \
        _metric(mm, "gpupool_reconcile_total", 'result="transient"')
    return {"errors": errors,
            "reloads": _metric(mm, "gpupool_credential_reloads", 'credential="apiserver-token"'),
            "heartbeat_failures": _metric(am, "gpupool_agent_node_heartbeat_failures"),
            "heartbeats": _metric(am, "gpupool_agent_node_heartbeats"),
            "auth_401s": _metric(sim if isinstance(sim, str) else "",
                                 "apiserver_authentication_failures_total"),
            "agent_ready": conds["GPUPoolAgentReady"]["status"],
            "reconcile_lines": [ln for ln in mm.splitlines()
                                if ln.startswith("gpupool_reconcile_total")]}
