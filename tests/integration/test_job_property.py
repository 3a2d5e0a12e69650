"""Property test for the gang scheduler (Mi355xJob): random submissions (sizes, priorities,
preemption on/off), deletions and suspend/resume on one 6-GPU pool. Invariants checked while the
scenario runs and after it settles:
  * never over-committed: the GPUs requested by live pods bound to the node never exceed its
    allocatable, and no pod is ever rejected by the kubelet for lack of a device;
  * gangs are all-or-nothing: a Running job has exactly `replicas` pods of its current attempt;
  * liveness: every job that fits the pool eventually succeeds (preempted and suspended ones too,
    once resumed), and preemption never counts as a failure restart.
"""
from __future__ import annotations

import os
import time

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from gpupool.kube import MI355XJOBS, MI355XPOOLS, NODES, PODS
from gpupool.testing.cluster import Cluster, NodeSpec

from .helpers import mi_pool, wait_ready

pytestmark = pytest.mark.slow

# more examples for a deeper search: GPUPOOL_PROPERTY_SCALE=5 python -m pytest ...
SCALE = max(1, int(os.environ.get("GPUPOOL_PROPERTY_SCALE", "1")))
RES = "amd.com/gpu"
CAP = 6

submit = st.tuples(st.just("submit"), st.integers(1, 3), st.integers(1, 2), st.integers(0, 3),
                   st.booleans())
ops = st.lists(st.one_of(submit, st.tuples(st.just("delete"), st.integers(0, 9)),
                         st.tuples(st.just("suspend"), st.integers(0, 9))), min_size=2, max_size=8)


@pytest.fixture(scope="module")
def shared(tmp_path_factory, native_built):
    c = Cluster(str(tmp_path_factory.mktemp("jobprop")), nodes=[NodeSpec("mi355x-node-0")])
    c.start()
    c.client.create(MI355XPOOLS, mi_pool("pool", CAP), "default")
    wait_ready(c.client, "pool", CAP)
    yield c
    c.stop()


def check_capacity(k, seen_reasons: set) -> None:
    alloc = int((k.get(NODES, "mi355x-node-0")["status"].get("allocatable") or {}).get(RES, "0"))
    used = 0
    for p in k.list(PODS, None)["items"]:
        ph = (p.get("status") or {}).get("phase", "Pending")
        if (p.get("status") or {}).get("reason", "").startswith("OutOf"):
            seen_reasons.add(p["status"]["reason"])
        if p["spec"].get("nodeName") and ph not in ("Succeeded", "Failed"):
            used += int(p["spec"]["containers"][0].get("resources", {}).get("limits", {}).get(RES, 0))
    assert used <= alloc, (used, alloc)


@settings(max_examples=12 * SCALE, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture,
                                                                 HealthCheck.too_slow])
@given(ops=ops)
def test_gang_scheduler_invariants(shared, ops):
    k = shared.client
    ns = f"j{int(time.time() * 1e6) % 10**9}"
    names: list[str] = []
    suspended: set[str] = set()
    rejected: set[str] = set()
    seq = 0
    for op in ops:
        if op[0] == "submit":
            _, replicas, gpus, prio, preempt = op
            name = f"job{seq}"
            seq += 1
            names.append(name)
            spec = {"replicas": replicas, "gpusPerReplica": gpus, "priority": prio,
                    "masterPort": 30000 + seq,
                    "template": {"spec": {"terminationGracePeriodSeconds": 1, "containers": [{
                        "name": "m", "command": ["sleep", "0.4"]}]}}}
            if preempt:
                spec["preemptionPolicy"] = "PreemptLowerPriority"
            k.create(MI355XJOBS, {"apiVersion": "compute.my.domain/v1alpha1", "kind": "Mi355xJob",
                                  "metadata": {"name": name}, "spec": spec}, ns)
        elif names:
            name = names[op[1] % len(names)]
            try:
                if op[0] == "delete":
                    k.delete(MI355XJOBS, name, ns)
                    names.remove(name)
                    suspended.discard(name)
                else:
                    k.patch(MI355XJOBS, name, {"spec": {"suspend": True}}, ns)
                    suspended.add(name)
            except Exception:
                pass  # already finished and TTL'd, or gone
        check_capacity(k, rejected)
        time.sleep(0.05)
    for name in list(suspended):
        k.patch(MI355XJOBS, name, {"spec": {"suspend": False}}, ns)
    deadline = time.time() + 60
    while True:
        check_capacity(k, rejected)
        jobs = {j["metadata"]["name"]: j for j in k.list(MI355XJOBS, ns)["items"]}
        for j in jobs.values():
            st_ = j.get("status") or {}
            if st_.get("phase") == "Running":
                cur = [p for p in k.list(PODS, ns, label_selector=f"gpupool.amd.com/job-name="
                                         f"{j['metadata']['name']}")["items"]
                       if p["metadata"]["labels"].get("gpupool.amd.com/attempt") == str(st_["attempt"])]
                assert len(cur) in (0, j["spec"]["replicas"]) or any(
                    p["metadata"].get("deletionTimestamp") or p["status"].get("phase") in
                    ("Succeeded", "Failed") for p in cur), (j["metadata"]["name"], len(cur))
        if all((j.get("status") or {}).get("phase") == "Succeeded" for j in jobs.values()):
            break
        assert time.time() < deadline, {n: (j.get("status") or {}).get("phase") for n, j in jobs.items()}
        time.sleep(0.1)
    assert not rejected, rejected
    for j in jobs.values():
        assert j["status"].get("restarts", 0) == 0, (j["metadata"]["name"], j["status"])
    for name in list(jobs):
        k.delete(MI355XJOBS, name, ns)
