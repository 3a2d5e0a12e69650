"""Probe helpers leave tenant GPUs alone (round-5 weak #5): with a pod on a pool's GPU the agent
parks that GPU's helper (no process, no context), and restarts it — warm before release hands
the GPU back — once the pod is gone (CPU: helper-sim kernels; the GPU tier checks the HIP
context and VRAM on a real MI355X)."""
from __future__ import annotations

import time

import pytest

from gpupool.kube import MI355XPOOLS, PODS
from gpupool.testing.cluster import NodeSpec

from .helpers import mi_pool, pause_pod, wait_ready

pytestmark = pytest.mark.slow


def _wait(pred, timeout=30.0):
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        v = pred()
        if v:
            return v
        time.sleep(0.05)
    return pred()


def _counter(text: str, name: str) -> float:
    for ln in text.splitlines():
        if ln.startswith(name + " "):
            return float(ln.rsplit(" ", 1)[1])
    return 0.0


def test_helper_parked_while_a_pod_holds_the_gpu(cluster_factory):
    c = cluster_factory(nodes=[NodeSpec("park-node", count=2, probe="helper-sim")])
    k = c.client
    k.create(MI355XPOOLS, mi_pool("pp", 1, drain={"gracePeriodSeconds": 1}), "default")
    o = wait_ready(k, "pp", 1, timeout=60)
    gpu = o["status"]["devices"][0]["uuid"]

    def helper(view):
        return (view.get("probeHelpers") or {}).get(gpu) or {}
    view = c.agent_request("park-node", "GET", "/v1/node")
    pid = helper(view).get("pid")
    assert helper(view).get("alive") and pid
    k.create(PODS, pause_pod("tenant"), "default")
    k.wait_for(PODS, "tenant", "default", lambda p: p and p["status"].get("phase") == "Running",
               30)
    view = _wait(lambda: (lambda v: v if helper(v).get("parked") else None)(
        c.agent_request("park-node", "GET", "/v1/node")))
    assert view, "the helper of the tenant's GPU was not parked"
    dev = next(d for d in view["devices"] if d["uuid"] == gpu)
    assert dev.get("probeHelper") == "Parked"
    assert _wait(lambda: _counter(c.agent_request("park-node", "GET", "/metrics"),
                                  "gpupool_agent_probe_helper_parks_total") == 1)
    # pod gone and the pool scaled to 0: the release waits for the restarted helper
    k.delete(PODS, "tenant", "default")
    k.wait_for(PODS, "tenant", "default", lambda p: p is None, 30)
    k.patch(MI355XPOOLS, "pp", {"spec": {"replicas": 0}}, "default")
    wait_ready(k, "pp", 0, timeout=60)
    view = c.agent_request("park-node", "GET", "/v1/node")
    assert helper(view).get("alive") and not helper(view).get("parked")
    assert helper(view).get("pid") != pid  # a fresh process
    m = c.agent_request("park-node", "GET", "/metrics")
    assert _counter(m, "gpupool_agent_probe_helper_unparks_total") == 1
    assert _counter(m, "gpupool_agent_release_helper_waits") >= 1
    # and the GPU is claimable again with a warm helper
    k.patch(MI355XPOOLS, "pp", {"spec": {"replicas": 2}}, "default")
    wait_ready(k, "pp", 2, timeout=60)
