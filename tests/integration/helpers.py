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


def settled_pools(client, ns: str, finals: dict, agent_views, timeout: float = 30.0):
    """One consistent snapshot of several pools once they have settled: every pool Ready at its
    final size, no pool changed while the agents were read, and each agent claim sits with the
    pool whose status lists it. Returns ``(pools, claims)`` — name -> object, and name -> the
    uuids the agents hold for that pool — from the last snapshot taken (the caller asserts on it).

    A pool's status is an observation written after the agent acted: a GPU released by pool A
    and claimed by pool B can sit in both statuses for the moment between B's status write and
    A's, and a fault event the agent sampled just before the faults cleared may still replace a
    GPU after A reads Ready. Exclusivity itself is the agent's (one record per GPU); the statuses
    agree with it once nothing moves any more, which is what this waits for."""
    deadline = time.monotonic() + timeout
    while True:
        pools = {n: client.get(MI355XPOOLS, n, ns) for n in finals}
        uid_to_name = {o["metadata"]["uid"]: n for n, o in pools.items()}
        claims: dict = {n: set() for n in finals}
        for view in agent_views():
            for d in view["devices"]:
                if d.get("poolUID") in uid_to_name:
                    claims[uid_to_name[d["poolUID"]]].add(d["uuid"])
        again = {n: client.get(MI355XPOOLS, n, ns) for n in finals}
        stable = all(again[n]["metadata"]["resourceVersion"] == o["metadata"]["resourceVersion"]
                     for n, o in pools.items())
        if stable and all(ready_at(r)(pools[n]) for n, r in finals.items()) and \
                all(claims[n] == {d["uuid"] for d in pools[n]["status"]["devices"]}
                    for n in finals):
            return pools, claims
        if time.monotonic() > deadline:
            return pools, claims
        time.sleep(0.1)


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
