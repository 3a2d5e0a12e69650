"""Probe helpers leave tenant GPUs alone (round-5 weak #5): with a pod on a pool's GPU the agent
parks that GPU's helper (no process, no context), and restarts it once the pod is gone; claims
take warm GPUs before one whose helper is still starting (CPU: helper-sim kernels; the GPU tier checks the HIP
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
    # pod gone and the pool scaled to 0: the helper restarts (release does not wait for it)
    k.delete(PODS, "tenant", "default")
    k.wait_for(PODS, "tenant", "default", lambda p: p is None, 30)
    k.patch(MI355XPOOLS, "pp", {"spec": {"replicas": 0}}, "default")
    wait_ready(k, "pp", 0, timeout=60)
    view = _wait(lambda: (lambda v: v if helper(v).get("alive") else None)(
        c.agent_request("park-node", "GET", "/v1/node")))
    assert view and not helper(view).get("parked")
    assert helper(view).get("pid") != pid  # a fresh process
    m = c.agent_request("park-node", "GET", "/metrics")
    assert _counter(m, "gpupool_agent_probe_helper_unparks_total") == 1
    # and the GPU is claimable again
    k.patch(MI355XPOOLS, "pp", {"spec": {"replicas": 2}}, "default")
    wait_ready(k, "pp", 2, timeout=60)


def test_claims_take_warm_gpus_before_one_whose_helper_restarts(cluster_factory):
    """Release hands a GPU back while its parked helper restarts (2 s of simulated HIP init
    here); a claim arriving meanwhile takes the other, warm GPU instead of waiting for it."""
    c = cluster_factory(nodes=[NodeSpec("warm-node", count=2, probe="helper-sim")],
                        env={"GPUPOOL_HELPER_SIM_INIT_S": "2.0"})
    k = c.client
    k.create(MI355XPOOLS, mi_pool("pw", 1, drain={"gracePeriodSeconds": 1}), "default")
    first = wait_ready(k, "pw", 1, timeout=60)["status"]["devices"][0]["uuid"]
    k.create(PODS, pause_pod("tenant"), "default")
    k.wait_for(PODS, "tenant", "default", lambda p: p and p["status"].get("phase") == "Running",
               30)
    assert _wait(lambda: first in {u for u, h in (c.agent_request("warm-node", "GET", "/v1/node")
                                                  .get("probeHelpers") or {}).items()
                                   if h.get("parked")})
    k.delete(PODS, "tenant", "default", grace=0)
    k.wait_for(PODS, "tenant", "default", lambda p: p is None, 30)
    t0 = time.monotonic()
    k.patch(MI355XPOOLS, "pw", {"spec": {"replicas": 0}}, "default")
    wait_ready(k, "pw", 0, timeout=60)
    k.patch(MI355XPOOLS, "pw", {"spec": {"replicas": 1}}, "default")
    o = wait_ready(k, "pw", 1, timeout=60)
    took = time.monotonic() - t0
    assert o["status"]["devices"][0]["uuid"] != first  # the warm GPU
    m = c.agent_request("warm-node", "GET", "/metrics")
    assert _counter(m, "gpupool_agent_claim_helper_waits") == 0
    assert took < 1.5, took  # neither the release nor the claim waited out the 2 s init
    # both GPUs: the second one's probe waits for its helper (out of the probe deadline)
    k.patch(MI355XPOOLS, "pw", {"spec": {"replicas": 2}}, "default")
    wait_ready(k, "pw", 2, timeout=60)
