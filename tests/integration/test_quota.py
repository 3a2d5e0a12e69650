"""Namespace GPU quota under concurrency (reference GPU调度平台搭建.md:802
"ResourceQuota + LimitRange").

The manager's workers reconcile pools in parallel; admission must be a reservation, not a read of
other pools' (lagging) status. These tests create and edit pools concurrently and watch the agent's
claim ledger the whole time: the GPUs a namespace holds never exceed the quota's hard limit.
"""
from __future__ import annotations

import threading
import time

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from gpupool.agent.ledger import read_claims
from gpupool.kube import MI355XPOOLS, KubeError, Res

from .helpers import cond_is, mi_pool, ready_at

QUOTAS = Res("", "v1", "resourcequotas")
pytestmark = pytest.mark.slow


class LedgerWatch:
    """Samples the node agent's ledger file every few ms; ``peak`` = most GPUs ever held."""

    def __init__(self, state_dir: str):
        self.state_dir = state_dir
        self.peak = 0
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def _run(self):
        while not self._stop.is_set():
            self.peak = max(self.peak, len(read_claims(self.state_dir)))
            time.sleep(0.003)

    def stop(self) -> int:
        self._stop.set()
        self._t.join()
        self.peak = max(self.peak, len(read_claims(self.state_dir)))
        return self.peak


def _state_dir(c) -> str:
    import os
    return os.path.join(c.workdir, "state-mi355x-node-0")


def _settled(o) -> bool:
    return ready_at(2)(o) or cond_is("Progressing", "False", "QuotaExceeded")(o)


def test_concurrent_pools_cannot_exceed_the_quota(cluster_factory):
    """Three replicas=2 pools created at once under a quota of 3, ten times: exactly one pool
    becomes Ready, the others report QuotaExceeded, and at no instant does the ledger hold more
    than 3 GPUs of the namespace."""
    c = cluster_factory()
    k = c.client
    for rep in range(10):
        ns = f"team{rep}"
        k.create(QUOTAS, {"metadata": {"name": "gpu-quota"},
                          "spec": {"hard": {"requests.amd.com/gpu": "3"}}}, ns)
        watch = LedgerWatch(_state_dir(c))
        ts = [threading.Thread(target=k.create, args=(MI355XPOOLS, mi_pool(n, 2), ns))
              for n in ("a", "b", "c")]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        objs = [k.wait_for(MI355XPOOLS, n, ns, _settled, timeout=30) for n in ("a", "b", "c")]
        time.sleep(0.2)  # any late claim would show in the ledger now
        peak = watch.stop()
        ready = [o["metadata"]["name"] for o in objs if ready_at(2)(o)]
        assert len(ready) == 1, (rep, [o["status"]["conditions"] for o in objs])
        assert peak <= 3, (rep, peak)
        for n in ("a", "b", "c"):
            k.delete(MI355XPOOLS, n, ns)
        for n in ("a", "b", "c"):
            k.wait_for(MI355XPOOLS, n, ns, lambda o: o is None, timeout=30)


OPS = st.lists(st.tuples(st.sampled_from(["create", "scale", "delete"]),
                         st.sampled_from(["p0", "p1", "p2", "p3"]), st.integers(0, 3)),
               min_size=3, max_size=8)


@settings(max_examples=8, deadline=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(batches=st.lists(OPS, min_size=1, max_size=3))
def test_random_concurrent_creates_and_edits_never_exceed_hard(cluster_factory, batches):
    """Hypothesis: batches of creates / replica edits / deletes of up to four pools, each batch
    applied concurrently, under a quota of 4 GPUs; the namespace's claimed GPUs (ledger, sampled
    every 3 ms) never exceed 4 and the pools converge with sum(readyReplicas) <= 4."""
    if not hasattr(test_random_concurrent_creates_and_edits_never_exceed_hard, "_c"):
        test_random_concurrent_creates_and_edits_never_exceed_hard._c = cluster_factory()
    c = test_random_concurrent_creates_and_edits_never_exceed_hard._c
    k = c.client
    ns = f"hq{time.monotonic_ns() % 10**9}"
    k.create(QUOTAS, {"metadata": {"name": "q"}, "spec": {"hard": {"amd.com/gpu": "4"}}}, ns)
    watch = LedgerWatch(_state_dir(c))

    def apply(op, name, r):
        try:
            if op == "create":
                k.create(MI355XPOOLS, mi_pool(name, r), ns)
            elif op == "scale":
                k.patch(MI355XPOOLS, name, {"spec": {"replicas": r}}, ns)
            else:
                k.delete(MI355XPOOLS, name, ns)
        except KubeError as e:
            if e.code not in (404, 409):
                raise
    try:
        for batch in batches:
            ts = [threading.Thread(target=apply, args=op) for op in batch]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            time.sleep(0.3)
        deadline = time.monotonic() + 20
        while time.monotonic() < deadline:  # converge: every pool Ready or quota-blocked
            items = k.list(MI355XPOOLS, ns)["items"]
            if all(not o["metadata"].get("deletionTimestamp") and (
                    ready_at(o["spec"]["replicas"])(o) or
                    cond_is("Progressing", "False", "QuotaExceeded")(o)) for o in items):
                break
            time.sleep(0.05)
        items = k.list(MI355XPOOLS, ns)["items"]
        assert sum((o.get("status") or {}).get("readyReplicas", 0) for o in items) <= 4
    finally:
        peak = watch.stop()
        for o in k.list(MI355XPOOLS, ns)["items"]:
            apply("delete", o["metadata"]["name"], 0)
        for o in k.list(MI355XPOOLS, ns)["items"]:
            k.wait_for(MI355XPOOLS, o["metadata"]["name"], ns, lambda x: x is None, timeout=30)
    assert peak <= 4, peak


def test_quota_hold_of_a_force_removed_pool_is_released(cluster_factory):
    """A pool that leaves without a finalizer pass — deleted while its agent is down, then its
    finalizer force-removed (merge-patch metadata.finalizers: []) — must not keep consuming its
    namespace's quota in the manager: a new pool under the same quota is admitted right away
    (the old pool's GPUs are orphans the sweep releases; the node has spare ones meanwhile)."""
    c = cluster_factory()
    k = c.client
    ns = "leak"
    k.create(QUOTAS, {"metadata": {"name": "gpu-quota"},
                      "spec": {"hard": {"requests.amd.com/gpu": "2"}}}, ns)
    k.create(MI355XPOOLS, mi_pool("old", 2), ns)
    k.wait_for(MI355XPOOLS, "old", ns, ready_at(2), timeout=30)
    c._kill("agent-mi355x-node-0")
    k.delete(MI355XPOOLS, "old", ns)
    time.sleep(0.5)  # the finalizer stays: the agent holding its GPUs does not answer
    assert k.get(MI355XPOOLS, "old", ns)["metadata"].get("finalizers")
    k.patch(MI355XPOOLS, "old", {"metadata": {"finalizers": []}}, ns)
    k.wait_for(MI355XPOOLS, "old", ns, lambda o: o is None, timeout=10)
    c.start_agent(c.nodes[0])
    t0 = time.monotonic()
    k.create(MI355XPOOLS, mi_pool("new", 2), ns)
    o = k.wait_for(MI355XPOOLS, "new", ns, _settled, timeout=30)
    assert ready_at(2)(o), o["status"]["conditions"]
    print(f"new pool Ready {time.monotonic() - t0:.3f} s after create")


def _set_apiserver_faults(c, faults: dict) -> None:
    import json
    import urllib.request
    req = urllib.request.Request(c.url + "/debug/faults", data=json.dumps(faults).encode(),
                                 method="POST", headers={"Content-Type": "application/json"})
    urllib.request.urlopen(req, timeout=5).read()


def test_unreadable_quotas_block_scale_up_as_quota_unknown(cluster_factory):
    """the ResourceQuota LIST fails before the manager's quota informer has
    synced. Admission fails closed — the pool reports Progressing=False, QuotaUnknown and claims
    nothing — until the quotas can be read; then it scales up (no quota in the namespace)."""
    c = cluster_factory(apiserver_args=["--fail-list", "resourcequotas"])
    k = c.client
    k.create(MI355XPOOLS, mi_pool("p", 2), "default")
    o = k.wait_for(MI355XPOOLS, "p", "default", cond_is("Progressing", "False", "QuotaUnknown"),
                   timeout=20)
    assert o["status"].get("readyReplicas", 0) == 0
    assert not read_claims(_state_dir(c))  # nothing claimed while the quota is unknown
    msg = next(x["message"] for x in o["status"]["conditions"] if x["type"] == "Progressing")
    assert "cannot be read" in msg and "--quota-fail-open" in msg
    _set_apiserver_faults(c, {"failList": {}})
    k.wait_for(MI355XPOOLS, "p", "default", ready_at(2), timeout=30)


def test_quota_fail_open_flag_admits_when_quotas_are_unreadable(cluster_factory):
    c = cluster_factory(apiserver_args=["--fail-list", "resourcequotas"],
                        manager_args=["--quota-fail-open"])
    k = c.client
    k.create(MI355XPOOLS, mi_pool("p", 2), "default")
    k.wait_for(MI355XPOOLS, "p", "default", ready_at(2), timeout=20)
