"""Demand-driven Mi355xPool (spec.autoscale, Mi355xPoolAutoscaler): pending pods and waiting
Mi355xJob gangs grow the pool immediately, bounded by maxReplicas; when demand falls the pool
shrinks after scaleDownDelaySeconds, releasing only idle GPUs (running pods keep theirs)."""
from __future__ import annotations

import time

import pytest

from gpupool.kube import MI355XJOBS, MI355XPOOLS, PODS

from .helpers import mi_pool, pause_pod, settled_events, wait_ready
from .test_jobs import job, phase_is

pytestmark = pytest.mark.slow
RES = "amd.com/gpu-auto"


def running(k, name):
    return k.wait_for(PODS, name, "default", lambda o: o and o["status"].get("phase") == "Running",
                      timeout=30)


def test_pool_follows_pod_and_job_demand(cluster_factory):
    k = cluster_factory().client
    k.create(MI355XPOOLS, mi_pool("auto", 0, resourceName=RES, drain={"gracePeriodSeconds": 1},
                                  autoscale={"enabled": True, "minReplicas": 0, "maxReplicas": 6,
                                             "scaleDownDelaySeconds": 2}), "default")
    wait_ready(k, "auto", 0)
    # two pending pods on an empty pool: it grows to 2 and the pods bind and run
    for n in ("w0", "w1"):
        k.create(PODS, pause_pod(n, resource=RES), "default")
    wait_ready(k, "auto", 2)
    keep = {running(k, n)["metadata"]["annotations"]["gpupool.amd.com/devices"] for n in ("w0", "w1")}
    # a 3 x 1 gang on the pool: 5 GPUs
    k.create(MI355XJOBS, job("g", 3, ["sleep", "600"], poolRef="auto"), "default")
    k.wait_for(MI355XJOBS, "g", "default", phase_is("Running"), timeout=30)
    wait_ready(k, "auto", 5)
    # demand 7 > maxReplicas 6: clamped
    k.create(PODS, pause_pod("big", resource=RES, n=2), "default")
    pool = wait_ready(k, "auto", 6)
    assert pool["metadata"]["annotations"]["gpupool.amd.com/autoscale-demand"] == "7"
    time.sleep(0.5)
    assert k.get(MI355XPOOLS, "auto", "default")["spec"]["replicas"] == 6
    # demand falls to 2: only after the delay, and w0/w1 keep their GPUs
    k.delete(MI355XJOBS, "g", "default")
    k.delete(PODS, "big", "default")
    t0 = time.monotonic()
    pool = wait_ready(k, "auto", 2, timeout=40)
    assert time.monotonic() - t0 >= 1.5
    still = {running(k, n)["metadata"]["annotations"]["gpupool.amd.com/devices"] for n in ("w0", "w1")}
    assert still == keep and keep <= {d["uuid"] for d in pool["status"]["devices"]}
    reasons = [e["reason"] for e in settled_events(k)
               if e["involvedObject"]["name"] == "auto"]
    assert "AutoscaledUp" in reasons and "AutoscaledDown" in reasons


def test_min_replicas_floor_and_disable(cluster_factory):
    k = cluster_factory().client
    k.create(MI355XPOOLS, mi_pool("warm", 0, resourceName=RES,
                                  autoscale={"enabled": True, "minReplicas": 2, "maxReplicas": 4,
                                             "scaleDownDelaySeconds": 0}), "default")
    wait_ready(k, "warm", 2)  # idle pool held at its floor
    # disabling hands spec.replicas back to the user: no further changes
    k.patch(MI355XPOOLS, "warm", {"spec": {"autoscale": {"enabled": False}, "replicas": 3}}, "default")
    wait_ready(k, "warm", 3)
    time.sleep(0.5)
    assert k.get(MI355XPOOLS, "warm", "default")["spec"]["replicas"] == 3


def test_scale_down_delay_counts_from_the_drop(cluster_factory):
    """A long steady state must not shorten the delay: after demand has been constant for longer
    than scaleDownDelaySeconds, a drop still waits the full delay before the pool shrinks."""
    k = cluster_factory().client
    k.create(MI355XPOOLS, mi_pool("steady", 0, resourceName=RES, drain={"gracePeriodSeconds": 1},
                                  autoscale={"enabled": True, "maxReplicas": 4,
                                             "scaleDownDelaySeconds": 3}), "default")
    for n in ("s0", "s1"):
        k.create(PODS, pause_pod(n, resource=RES), "default")
    wait_ready(k, "steady", 2)
    running(k, "s0")
    time.sleep(4.0)  # steady for longer than the delay
    k.delete(PODS, "s1", "default")
    t0 = time.monotonic()
    time.sleep(1.5)
    assert k.get(MI355XPOOLS, "steady", "default")["spec"]["replicas"] == 2
    wait_ready(k, "steady", 1, timeout=30)
    assert time.monotonic() - t0 >= 2.5


def test_two_pools_same_resource_do_not_double_count(cluster_factory):
    """A fixed pool of 4 and an autoscaled pool serve the same resource: 6 GPUs of pending pods
    grow the autoscaled pool to 2 (the fixed pool serves 4), not to 6 (which would claim idle
    GPUs for pods the other pool already serves)."""
    k = cluster_factory().client
    k.create(MI355XPOOLS, mi_pool("fixed", 4, resourceName=RES), "default")
    wait_ready(k, "fixed", 4)
    k.create(MI355XPOOLS, mi_pool("auto", 0, resourceName=RES,
                                  autoscale={"enabled": True, "minReplicas": 0, "maxReplicas": 8,
                                             "scaleDownDelaySeconds": 60}), "default")
    wait_ready(k, "auto", 0)
    for i in range(3):
        k.create(PODS, pause_pod(f"p{i}", resource=RES, n=2), "default")
    pool = wait_ready(k, "auto", 2)
    assert pool["metadata"]["annotations"]["gpupool.amd.com/autoscale-demand"] == "2"
    for i in range(3):
        running(k, f"p{i}")
    time.sleep(1.0)
    assert k.get(MI355XPOOLS, "auto", "default")["spec"]["replicas"] == 2


def test_two_autoscaled_pools_keep_their_running_pods(cluster_factory):
    """Two autoscaled pools of one resource; pods already run on the later pool ("zb", grown for
    them while it was the only one). Creating "za" (first in name order) must not hand it zb's
    demand: za stays at 0 while zb keeps its GPUs and pods, even past scaleDownDelaySeconds."""
    k = cluster_factory().client
    auto = {"enabled": True, "minReplicas": 0, "maxReplicas": 4, "scaleDownDelaySeconds": 0}
    k.create(MI355XPOOLS, mi_pool("zb", 0, resourceName=RES, autoscale=auto,
                                  drain={"gracePeriodSeconds": 1}), "default")
    for i in range(2):
        k.create(PODS, pause_pod(f"w{i}", resource=RES), "default")
    wait_ready(k, "zb", 2)
    for i in range(2):
        running(k, f"w{i}")
    # zb's status lists its pods (the agents' PodResources view) before za appears
    k.wait_for(MI355XPOOLS, "zb", "default", lambda o: sum(
        len(d.get("pods") or []) for d in o["status"]["devices"]) == 2, timeout=20)
    k.create(MI355XPOOLS, mi_pool("za", 0, resourceName=RES, autoscale=auto), "default")
    wait_ready(k, "za", 0)
    time.sleep(1.5)  # several autoscaler passes, scale-down delay 0
    assert k.get(MI355XPOOLS, "za", "default")["spec"]["replicas"] == 0
    zb = wait_ready(k, "zb", 2)
    assert sum(len(d.get("pods") or []) for d in zb["status"]["devices"]) == 2
    for i in range(2):
        assert k.get(PODS, f"w{i}", "default")["status"]["phase"] == "Running"
