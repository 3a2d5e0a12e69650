"""Shared helpers for the integration suites (CPU, fake 8x MI355X backend)."""
from __future__ import annotations

import time

from gpupool.kube import EVENTS, MI355XPOOLS


def mi_pool(name: str, replicas: int, **spec) -> dict:
    return {"apiVersion": "compute.my.domain/v1alpha1", "kind": "Mi355xPool",
            "metadata": {"name": name}, "spec": {"replicas": replicas, **spec}}


def conds(o: dict | None) -> dict:
    return {x["type"]: x for x in ((o or {}).get("status") or {}).get("conditions", [])}


def ready_at(r: int):
    def pred(o):
        st = (o or {}).get("status") or {}
        return bool(o) and st.get("observedGeneration") == o["metadata"].get("generation") and \
            st.get("readyReplicas") == r and len(st.get("devices", [])) == r and \
            conds(o).get("Ready", {}).get("status") == "True"
    return pred


def cond_is(ctype: str, status: str, reason: str | None = None):
    def pred(o):
        c = conds(o).get(ctype, {})
        return c.get("status") == status and (reason is None or c.get("reason") == reason)
    return pred


def wait_ready(client, name: str, r: int, ns: str = "default", timeout: float = 30.0) -> dict:
    return client.wait_for(MI355XPOOLS, name, ns, ready_at(r), timeout=timeout)


def pause_pod(name: str, resource: str = "amd.com/gpu", n: int = 1, grace: int = 1) -> dict:
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name},
            "spec": {"terminationGracePeriodSeconds": grace,
                     "containers": [{"name": "main", "command": ["sleep", "600"],
                                     "resources": {"limits": {resource: n}}}]}}


def settled_events(client, ns: str = "default", quiet: float = 0.15, timeout: float = 5.0) -> list:
    """The namespace's Events once the manager's recorder has gone quiet (it posts them
    asynchronously, a few ms after the pass that recorded them)."""
    deadline = time.monotonic() + timeout
    last = None
    while True:
        items = client.list(EVENTS, ns)["items"]
        sig = [(e["metadata"]["name"], e.get("count")) for e in items]
        if sig == last or time.monotonic() > deadline:
            return items
        last = sig
        time.sleep(quiet)
