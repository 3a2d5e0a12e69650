"""Mi355xPool end-to-end on the 8x MI355X fake node (BASELINE configs 3, 4, 5 and the failure
paths): apiserver-sim + C++ manager + node agent + ROCm device plugin + fake kubelet."""
from __future__ import annotations

import time

import pytest

from gpupool.kube import MI355XPOOLS, NODES, PODS, KubeError
from gpupool.testing.cluster import NodeSpec

from .helpers import cond_is, conds, mi_pool, pause_pod, ready_at, settled_events, wait_ready

pytestmark = pytest.mark.slow


@pytest.fixture
def node8(cluster_factory):
    return cluster_factory()


def agent_view(c, node="mi355x-node-0"):
    return c.agent_request(node, "GET", "/v1/node")


def test_config3_scale_up_1_to_8(node8):
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("p", 1), "default")
    wait_ready(k, "p", 1)
    seen = set()
    for r in (2, 4, 8):
        t0 = time.perf_counter()
        k.patch(MI355XPOOLS, "p", {"spec": {"replicas": r}}, "default")
        o = wait_ready(k, "p", r)
        assert time.perf_counter() - t0 < 30
        uuids = [d["uuid"] for d in o["status"]["devices"]]
        assert len(set(uuids)) == r and seen <= set(uuids)  # scale-up keeps existing GPUs
        seen = set(uuids)
        k.wait_for(NODES, "mi355x-node-0", None, lambda n, r=r: (n["status"].get("allocatable") or {})
                   .get("amd.com/gpu") == str(r), timeout=20)  # kubelet status is asynchronous
    view = agent_view(node8)
    assert sum(1 for d in view["devices"] if d.get("poolUID")) == 8
    assert conds(o)["Progressing"]["reason"] == "Stable"


def test_all_or_nothing_insufficient(node8):
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("big", 9), "default")
    o = k.wait_for(MI355XPOOLS, "big", "default",
                   cond_is("Progressing", "False", "InsufficientDevices"), timeout=20)
    assert o["status"]["readyReplicas"] == 0
    assert all(not d.get("poolUID") for d in agent_view(node8)["devices"])  # nothing claimed
    k.patch(MI355XPOOLS, "big", {"spec": {"replicas": 8}}, "default")
    wait_ready(k, "big", 8)


def test_config4_scale_down_8_to_4_with_drain(node8):
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("p", 8, drain={"gracePeriodSeconds": 1}), "default")
    o = wait_ready(k, "p", 8)
    for i in range(8):
        k.create(PODS, pause_pod(f"w{i}"), "default")
    for i in range(8):
        k.wait_for(PODS, f"w{i}", "default", lambda o: o and o["status"].get("phase") == "Running",
                   timeout=30)
    k.patch(MI355XPOOLS, "p", {"spec": {"replicas": 4}}, "default")
    o = wait_ready(k, "p", 4, timeout=60)
    kept = {d["uuid"] for d in o["status"]["devices"]}
    assert [d["index"] for d in o["status"]["devices"]] == [0, 1, 2, 3]  # highest indices drained
    pods = k.list(PODS, "default")["items"]
    assert len(pods) == 4  # exactly the pods on released GPUs were evicted
    for p in pods:
        assert p["metadata"]["annotations"]["gpupool.amd.com/devices"] in kept
    view = agent_view(node8)
    for d in view["devices"]:
        if d["uuid"] not in kept:
            assert d["state"] == "Free" and not d["pods"]  # no pod left on a released GPU
    reasons = {e["reason"] for e in settled_events(k)}
    assert {"DrainStarted", "PodEvicted", "GPUReleased"} <= reasons
    # finalizer-guarded delete: pods evicted, GPUs released, then the CR disappears
    k.delete(MI355XPOOLS, "p", "default")
    k.wait_for(MI355XPOOLS, "p", "default", lambda o: o is None, timeout=60)
    assert k.list(PODS, "default")["items"] == []
    assert all(d["state"] == "Free" for d in agent_view(node8)["devices"])


def test_drain_wakes_on_pod_exit_not_the_sample_period(cluster_factory):
    """A drain waits for the evicted pod to exit. The agent's pod watch (PodResources polled every
    20 ms while a GPU drains) bumps the pool when the pod is gone, so the release follows within
    tens of ms — not after the agent's sample period (5 s here) or the manager's 5 s view-cache
    age, which a view-driven refresh alone would wait for (BENCH r2t: 0.96 s at a 1 s period)."""
    c = cluster_factory(sample_interval=5.0)
    k = c.client
    k.create(MI355XPOOLS, mi_pool("p", 1, drain={"gracePeriodSeconds": 1}), "default")
    wait_ready(k, "p", 1)
    k.create(PODS, pause_pod("w0"), "default")
    k.wait_for(PODS, "w0", "default", lambda o: o and o["status"].get("phase") == "Running",
               timeout=30)
    time.sleep(0.3)  # let the Allocate pod-watch window lapse into steady state
    t0 = time.perf_counter()
    k.patch(MI355XPOOLS, "p", {"spec": {"replicas": 0}}, "default")
    wait_ready(k, "p", 0, timeout=20)
    dt = time.perf_counter() - t0
    assert k.list(PODS, "default")["items"] == []
    assert dt < 2.5, f"scale-down with drain took {dt:.2f} s"  # vs >= 5 s without the pod watch


def test_config5_two_pools_with_health_conditions(node8):
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("team-a", 4, resourceName="amd.com/gpu-team-a",
                                  replacePolicy="Keep"), "default")
    k.create(MI355XPOOLS, mi_pool("team-b", 4, resourceName="amd.com/gpu-team-b"), "default")
    a = wait_ready(k, "team-a", 4)
    b = wait_ready(k, "team-b", 4)
    ua = {d["uuid"] for d in a["status"]["devices"]}
    ub = {d["uuid"] for d in b["status"]["devices"]}
    assert not ua & ub  # no cross-pool claims
    # the kubelet publishes node allocatable asynchronously after ListAndWatch (as a real kubelet's
    # node-status sync does), so wait for it rather than racing it under load
    k.wait_for(NODES, "mi355x-node-0", None, lambda n: (
        (n["status"].get("allocatable") or {}).get("amd.com/gpu-team-a") == "4"
        and n["status"]["allocatable"].get("amd.com/gpu-team-b") == "4"), timeout=20)
    victim = sorted(a["status"]["devices"], key=lambda d: d["index"])[0]["uuid"]
    # xGMI link down on one team-a GPU
    node8.set_faults("mi355x-node-0", {"devices": {victim: {"xgmi": {
        "links": ["X", "U", "D", "U", "U", "U", "U", "U"]}}}})
    a = k.wait_for(MI355XPOOLS, "team-a", "default", cond_is("XGMILinksHealthy", "False",
                                                            "XGMILinkDown"), timeout=20)
    assert conds(a)["Degraded"]["status"] == "True" and a["status"]["readyReplicas"] == 3
    assert conds(k.get(MI355XPOOLS, "team-b", "default"))["XGMILinksHealthy"]["status"] == "True"
    # HBM ECC + thermal on the same GPU
    node8.set_faults("mi355x-node-0", {"devices": {victim: {
        "ecc": {"uncorrectable": 2}, "temps": {"hotspot": {"current": 104}}}}})
    a = k.wait_for(MI355XPOOLS, "team-a", "default",
                   lambda o: cond_is("HBMECCHealthy", "False")(o) and
                   cond_is("ThermalHealthy", "False")(o) and
                   cond_is("XGMILinksHealthy", "True")(o), timeout=20)
    dev = next(d for d in a["status"]["devices"] if d["uuid"] == victim)
    assert dev["health"] == "Unhealthy" and any("HBMUncorrectableECC" in r for r in dev["reasons"])
    node8.set_faults("mi355x-node-0", {})
    wait_ready(k, "team-a", 4)
    # device plugin: the unhealthy GPU was advertised Unhealthy while faulted -> now healthy again
    k.wait_for(NODES, "mi355x-node-0", None, lambda n: (n["status"].get("allocatable") or {}).get(
        "amd.com/gpu-team-a") == "4", timeout=20)  # kubelet node status follows asynchronously


def test_replace_on_failure(cluster_factory):
    c = cluster_factory(nodes=[NodeSpec("mi355x-node-0")])
    k = c.client
    k.create(MI355XPOOLS, mi_pool("p", 2), "default")
    o = wait_ready(k, "p", 2)
    bad = o["status"]["devices"][0]["uuid"]
    c.set_faults("mi355x-node-0", {"devices": {bad: {"ecc": {"uncorrectable": 5}}}})

    def replaced(o):
        u = {d["uuid"] for d in (o or {}).get("status", {}).get("devices", [])}
        return ready_at(2)(o) and bad not in u
    k.wait_for(MI355XPOOLS, "p", "default", replaced, timeout=30)
    view = c.agent_request("mi355x-node-0", "GET", "/v1/node")
    assert next(d for d in view["devices"] if d["uuid"] == bad)["state"] == "Quarantined"


def test_probe_failure_replaced(cluster_factory):
    c = cluster_factory(nodes=[NodeSpec("mi355x-node-0")])
    k = c.client
    # the first two GPUs (NUMA-packed choice) fail their probe
    c.set_faults("mi355x-node-0", {"devices": {"0": {"probeFail": True}, "1": {"probeFail": True}}})
    k.create(MI355XPOOLS, mi_pool("p", 2), "default")
    o = wait_ready(k, "p", 2, timeout=30)
    assert {d["index"] for d in o["status"]["devices"]}.isdisjoint({0, 1})
    reasons = {e["reason"] for e in settled_events(k)}
    assert "HealthDegraded" in reasons


def test_performance_floor_replaces_slow_gpu(cluster_factory):
    """spec.probe.minMfmaTflops: a GPU that computes correctly but at half speed (fault overlay
    probeScale, e.g. a throttled part) fails DeviceProbePassed and is replaced."""
    c = cluster_factory(nodes=[NodeSpec("mi355x-node-0")])
    k = c.client
    c.set_faults("mi355x-node-0", {"devices": {"0": {"probeScale": 0.5}}})
    k.create(MI355XPOOLS, mi_pool("p", 2, probe={"minMfmaTflops": 1000, "minHbmGBps": 3000}),
             "default")
    o = wait_ready(k, "p", 2, timeout=30)
    assert 0 not in {d["index"] for d in o["status"]["devices"]}
    assert all(d["probe"]["mfmaTflops"] >= 1000 for d in o["status"]["devices"])
    msgs = " ".join(e.get("message", "") for e in settled_events(k))
    assert "PerformanceBelowFloor" in msgs and "MFMA 600 TFLOP/s < floor 1000" in msgs


def test_manager_restart_readopts_claims(node8):
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("p", 3), "default")
    before = wait_ready(k, "p", 3)
    node8._kill("manager")
    node8.start_manager()
    time.sleep(0.5)
    after = wait_ready(k, "p", 3)
    assert [d["uuid"] for d in after["status"]["devices"]] == \
        [d["uuid"] for d in before["status"]["devices"]]


def test_agent_restart_keeps_ledger(node8):
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("p", 2), "default")
    before = wait_ready(k, "p", 2)
    node8._kill("agent-mi355x-node-0")
    node8.start_agent(node8.nodes[0])
    after = wait_ready(k, "p", 2, timeout=30)
    assert {d["uuid"] for d in after["status"]["devices"]} == \
        {d["uuid"] for d in before["status"]["devices"]}


def _interrupt_probe(node8, victim: str) -> None:
    """Kill the agent and leave ``victim``'s record in 'Probing', as a kill between the claim's
    reply and the ledger's background write of Probing -> Claimed does."""
    import json
    import os
    node8._kill("agent-mi355x-node-0")
    path = os.path.join(node8.workdir, "state-mi355x-node-0", "ledger.json")
    with open(path) as f:
        doc = json.load(f)
    doc["claims"][victim].update({"state": "Probing", "probe": None})
    with open(path, "w") as f:
        json.dump(doc, f)


def test_agent_crash_mid_probe_reprobes_and_keeps_a_healthy_gpu(node8):
    """A claim is committed as 'Probing' before the probe runs; an agent killed before the
    Claimed state reached the disk must neither leave the pool stuck Progressing=Probing nor
    replace a healthy GPU: the restarted agent runs the probe again and the GPU stays."""
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("p", 2), "default")
    before = wait_ready(k, "p", 2)
    uuids = {d["uuid"] for d in before["status"]["devices"]}
    victim = before["status"]["devices"][1]["uuid"]
    _interrupt_probe(node8, victim)
    node8.start_agent(node8.nodes[0])
    d = next(x for x in agent_view(node8)["devices"] if x["uuid"] == victim)
    assert d["state"] == "Claimed" and d["probe"]["passed"] and d["probe"]["rerunAtStart"], d
    after = wait_ready(k, "p", 2, timeout=30)
    assert {x["uuid"] for x in after["status"]["devices"]} == uuids


def test_agent_crash_mid_probe_replaces_a_gpu_that_fails_the_rerun(node8):
    """Same interrupted claim, but the GPU fails the probe the restarted agent runs: the record
    becomes a failed probe (ProbeInterrupted) and the pool replaces that GPU."""
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("p", 2), "default")
    before = wait_ready(k, "p", 2)
    victim = before["status"]["devices"][1]
    _interrupt_probe(node8, victim["uuid"])
    node8.set_faults("mi355x-node-0", {"devices": {str(victim["index"]): {"probeFail": True}}},
                     sample=False)
    node8.start_agent(node8.nodes[0])

    def replaced(o):
        return ready_at(2)(o) and victim["uuid"] not in {d["uuid"] for d in o["status"]["devices"]}
    k.wait_for(MI355XPOOLS, "p", "default", replaced, timeout=30)
    d = next(x for x in agent_view(node8)["devices"] if x["uuid"] == victim["uuid"])
    assert d["state"] == "Quarantined" and "ProbeInterrupted" in d["quarantine"]["reason"]
    msgs = " ".join(e.get("message", "") for e in settled_events(k))
    assert "ProbeInterrupted, re-run at agent start" in msgs, msgs


def _deleting(k, name):
    o = k.get(MI355XPOOLS, name, "default")
    assert o["metadata"].get("deletionTimestamp") and o["metadata"].get("finalizers"), o["metadata"]
    return o


def test_delete_with_agent_down_waits_for_release(node8):
    """Deleting a pool right after it turned ready, with its agent already dead: the finalizer
    stays until the agent answers and the GPUs are really released. (A pass running on an
    informer copy older than the pool's own status write saw no nodeName, skipped the dead
    node as 'not ours' and removed the finalizer — GPUs still claimed on the agent.)"""
    k = node8.client
    o = k.create(MI355XPOOLS, mi_pool("p", 2), "default")
    uid = o["metadata"]["uid"]
    wait_ready(k, "p", 2)
    node8._kill("agent-mi355x-node-0")
    k.delete(MI355XPOOLS, "p", "default")
    time.sleep(1.5)
    st = _deleting(k, "p")["status"]
    assert st.get("nodeName") == "mi355x-node-0", st
    node8.start_agent(node8.nodes[0])
    k.wait_for(MI355XPOOLS, "p", "default", lambda o: o is None, timeout=30)
    assert not [d for d in agent_view(node8)["devices"] if d.get("poolUID") == uid]


def test_agent_down_right_after_ready_claims_nowhere_else(cluster_factory):
    """Two nodes; the pool's agent dies just after the pool turned ready, and the pool is poked.
    The passes that follow may run on an informer copy from before the manager's own status write
    (no nodeName yet): they must still treat the pool's node as its home — blocked while that agent
    is down — not see 'no GPUs anywhere' and claim a second set on the other node."""
    c = cluster_factory(nodes=[NodeSpec("sn-a"), NodeSpec("sn-b")])
    k = c.client
    o = k.create(MI355XPOOLS, mi_pool("p", 2), "default")
    uid = o["metadata"]["uid"]
    home = wait_ready(k, "p", 2)["status"]["nodeName"]
    other = "sn-b" if home == "sn-a" else "sn-a"
    before = k.get(MI355XPOOLS, "p", "default")["status"]
    c._kill(f"agent-{home}")
    for i in range(5):
        k.patch(MI355XPOOLS, "p", {"metadata": {"labels": {"poke": str(i)}}}, "default")
        time.sleep(0.05)
    # throughout the outage the pool keeps what it last observed: its GPUs
    # (still held, pods and all), replicas and node; Ready is Unknown, readyReplicas 0 (the node's
    # device plugin is down with the agent: nothing new can be scheduled on them until it answers)
    saw_unknown = False
    deadline = time.monotonic() + 1.5
    while time.monotonic() < deadline:
        st = k.get(MI355XPOOLS, "p", "default")["status"]
        assert st.get("replicas") == 2, st
        assert [d["uuid"] for d in st["devices"]] == [d["uuid"] for d in before["devices"]], st
        assert st.get("nodeName") == home
        ready = conds({"status": st})["Ready"]
        if ready["status"] == "Unknown":
            saw_unknown = True
            assert ready["reason"] == "AgentUnreachable" and st["readyReplicas"] == 0, st
            assert {d["health"] for d in st["devices"]} == {"Unknown"}, st["devices"]
        time.sleep(0.01)
    assert saw_unknown
    assert not [d for d in agent_view(c, other)["devices"] if d.get("poolUID") == uid]
    assert k.get(MI355XPOOLS, "p", "default")["status"].get("nodeName") == home
    c.start_agent(next(n for n in c.nodes if n.name == home))  # back: verified and Ready again
    o = wait_ready(k, "p", 2)
    assert [d["uuid"] for d in o["status"]["devices"]] == [d["uuid"] for d in before["devices"]]


def test_lost_claim_reply_neither_leaks_nor_double_claims(cluster_factory):
    """Both agents die while claims are in flight (a pool scaled 1 -> 5 right after creation): a
    claim the agent committed to its ledger before the connection reset survives the restart,
    although the manager never got the reply. Such GPUs on a node the pool's status does not name
    must be released (or adopted) — not stay claimed for a live pool that never sees them."""
    c = cluster_factory(nodes=[NodeSpec("sn-a"), NodeSpec("sn-b")])
    k = c.client
    for it in range(3):
        ns = f"lost{it}"
        uid = k.create(MI355XPOOLS, mi_pool("p", 1), ns)["metadata"]["uid"]
        k.patch(MI355XPOOLS, "p", {"spec": {"replicas": 5}}, ns)
        for n in c.nodes:
            c._kill(f"agent-{n.name}")
        for n in c.nodes:
            c.start_agent(n)
        k.patch(MI355XPOOLS, "p", {"spec": {"replicas": 3}}, ns)
        o = k.wait_for(MI355XPOOLS, "p", ns, ready_at(3), timeout=60)
        held = {d["uuid"] for d in o["status"]["devices"]}
        deadline = time.time() + 10
        while True:
            on_agents = {d["uuid"] for n in c.nodes for d in agent_view(c, n.name)["devices"]
                         if d.get("poolUID") == uid}
            if on_agents == held or time.time() > deadline:
                break
            time.sleep(0.1)
        assert on_agents == held, (it, sorted(on_agents - held))
        k.delete(MI355XPOOLS, "p", ns)
        k.wait_for(MI355XPOOLS, "p", ns, lambda o: o is None, timeout=30)


def test_sweep_finds_claims_on_a_node_status_does_not_name(cluster_factory):
    """GPUs claimed for a live single-node pool on a node its status does not name — a lost claim
    reply from before a manager restart, which no in-memory record remembers (simulated here by
    claiming on the other agent directly). The sweep flags the node and wakes the pool, whose pass
    releases them; the pool itself is untouched."""
    c = cluster_factory(nodes=[NodeSpec("sn-a"), NodeSpec("sn-b")],
                        manager_args=["--orphan-sweep", "300ms"])
    k = c.client
    uid = k.create(MI355XPOOLS, mi_pool("p", 2), "default")["metadata"]["uid"]
    o = wait_ready(k, "p", 2)
    home = o["status"]["nodeName"]
    other = "sn-b" if home == "sn-a" else "sn-a"
    r = c.agent_request(other, "POST", "/v1/claims", {"poolUID": uid, "pool": "default/p", "count": 3})
    assert r["ok"] and len(r["devices"]) == 3
    deadline = time.time() + 15
    while [d for d in agent_view(c, other)["devices"] if d.get("poolUID") == uid]:
        assert time.time() < deadline, "stray claims never released"
        time.sleep(0.1)
    o = k.get(MI355XPOOLS, "p", "default")
    assert o["status"]["nodeName"] == home and o["status"]["readyReplicas"] == 2
    assert {d["uuid"] for d in o["status"]["devices"]} == \
        {d["uuid"] for d in agent_view(c, home)["devices"] if d.get("poolUID") == uid}


def test_delete_unplaced_pool_waits_for_unreachable_agent(node8):
    """A pool whose status names no node (here: never placed) is deleted while an agent is down:
    that agent could hold GPUs of the pool (a claim whose status write never landed), so the
    finalizer stays — with a status saying which agent it waits for — until it answers."""
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("big", 9), "default")  # more than the node has
    k.wait_for(MI355XPOOLS, "big", "default",
               lambda o: conds(o).get("Ready", {}).get("reason") == "InsufficientDevices", timeout=30)
    node8._kill("agent-mi355x-node-0")
    # past the manager's agent-view cache age (5 s): the dead agent's last answer has expired, so
    # the finalize pass must ask it — and gets no answer
    time.sleep(5.5)
    k.delete(MI355XPOOLS, "big", "default")

    def waiting(o):
        assert o is not None, "finalizer removed while the agent was unreachable"
        return "unreachable agent(s) on mi355x-node-0" in conds(o).get("Progressing", {}).get("message", "")
    k.wait_for(MI355XPOOLS, "big", "default", waiting, timeout=30)
    time.sleep(0.5)
    _deleting(k, "big")
    node8.start_agent(node8.nodes[0])
    k.wait_for(MI355XPOOLS, "big", "default", lambda o: o is None, timeout=30)


def test_orphan_sweep_releases_claims_of_deleted_pool(cluster_factory):
    c = cluster_factory(manager_args=["--orphan-sweep", "500ms"])
    k = c.client
    k.create(MI355XPOOLS, mi_pool("p", 2), "default")
    wait_ready(k, "p", 2)
    c._kill("manager")
    # force-delete the CR behind the operator's back (finalizer stripped)
    k.patch(MI355XPOOLS, "p", {"metadata": {"finalizers": []}}, "default")
    k.delete(MI355XPOOLS, "p", "default")
    c.start_manager()
    deadline = time.time() + 20
    while time.time() < deadline:
        if all(not d.get("poolUID") for d in c.agent_request("mi355x-node-0", "GET",
                                                             "/v1/node")["devices"]):
            break
        time.sleep(0.1)
    else:
        pytest.fail("orphaned claims were not released")


def test_leader_election_failover(cluster_factory):
    lease = ["--leader-elect", "--lease-duration", "2s", "--renew-deadline", "1500ms",
             "--retry-period", "200ms"]
    c = cluster_factory(manager_args=lease)
    k = c.client
    from gpupool.kube import LEASES
    # the port file appears before the first acquire: wait for the Lease itself
    first = k.wait_for(LEASES, "gpupool-manager-leader", "gpupool-system",
                       lambda o: bool(o) and bool(o["spec"].get("holderIdentity")), timeout=15,
                       poll=0.05)["spec"]["holderIdentity"]
    # a second manager stands by
    standby = c._spawn("manager2", [c.procs["manager"].args[0], "--apiserver", c.url,
                                    "--identity", "standby", "--progress-poll", "100ms"] + lease)
    time.sleep(0.5)
    assert k.get(LEASES, "gpupool-manager-leader", "gpupool-system")["spec"]["holderIdentity"] == first
    c._kill("manager")
    k.wait_for(LEASES, "gpupool-manager-leader", "gpupool-system",
               lambda o: o and o["spec"]["holderIdentity"] == "standby", timeout=15, poll=0.1)
    k.create(MI355XPOOLS, mi_pool("p", 1), "default")
    wait_ready(k, "p", 1)  # the new leader reconciles
    assert standby.poll() is None


def test_multinode_placement(cluster_factory):
    c = cluster_factory(nodes=[NodeSpec("node-a", count=4), NodeSpec("node-b", count=8)])
    k = c.client
    k.create(MI355XPOOLS, mi_pool("pinned", 2, nodeName="node-a"), "default")
    o = wait_ready(k, "pinned", 2)
    assert o["status"]["nodeName"] == "node-a"
    k.create(MI355XPOOLS, mi_pool("big", 6), "default")  # only node-b fits 6
    o = wait_ready(k, "big", 6)
    assert o["status"]["nodeName"] == "node-b"
    k.create(MI355XPOOLS, mi_pool("sel", 1, nodeSelector={"kubernetes.io/hostname": "node-a"}),
             "default")
    assert wait_ready(k, "sel", 1)["status"]["nodeName"] == "node-a"


def test_metrics_and_events_exposed(node8):
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("p", 2), "default")
    wait_ready(k, "p", 2)
    # the gauges are set right after the status write the watch just delivered: poll briefly
    deadline = time.monotonic() + 5
    while True:
        m = node8.manager_metrics()
        if 'gpupool_ready_replicas{kind="Mi355xPool",pool="default/p"} 2' in m or \
                time.monotonic() > deadline:
            break
        time.sleep(0.05)
    assert "gpupool_reconcile_total" in m and "gpupool_reconcile_to_ready_seconds_bucket" in m
    assert 'gpupool_ready_replicas{kind="Mi355xPool",pool="default/p"} 2' in m
    am = node8.agent_request.__self__  # cluster
    txt = am.agent_request("mi355x-node-0", "GET", "/v1/node")
    assert txt["backend"] == "fake"


def test_reconcile_traces(node8):
    """SURVEY §5 tracing: each reconcile pass is a trace with per-phase spans (incl. the node
    agent's own claim phases), served at /debug/traces and exported as a span histogram."""
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("tr", 2), "default")
    wait_ready(k, "tr", 2)
    # a pass's trace is committed after its status write, which the watch may deliver first
    deadline = time.monotonic() + 10
    while True:
        traces = node8.manager_traces(key="Mi355xPool/default/tr", n=50)
        claim = [t for t in traces if any(s["name"] == "agent:POST /v1/claims" for s in t["spans"])]
        if claim or time.monotonic() > deadline:
            break
        time.sleep(0.05)
    assert traces and all(t["key"] == "Mi355xPool/default/tr" for t in traces)
    assert len(claim) == 1, traces
    names = [s["name"] for s in claim[0]["spans"]]
    for want in ("observe", "agent.claim.select", "agent.claim.probe", "agent.claim.advertise",
                 "status"):
        assert want in names, names
    # the pool's node view: an RPC, or the view cache the agent's event feed keeps fresh
    assert "agent:GET /v1/node" in names or "agent:view-cache" in names, names
    assert claim[0]["totalMs"] >= max(s["ms"] for s in claim[0]["spans"]) - 1e-6
    assert len(claim[0]["reconcileID"]) == 16
    m = node8.manager_metrics()
    assert 'gpupool_reconcile_span_seconds_count{kind="Mi355xPool",span="observe"}' in m


def test_observe_served_from_the_agent_view_cache(node8):
    """Informer-style cache of the agents' node views: after the agent's event feed announced a
    change the manager prefetches the view, so the next reconcile observes without an RPC; a
    mutating RPC invalidates it, so status after acting still comes from the agent."""
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("vc", 1), "default")
    wait_ready(k, "vc", 1)
    time.sleep(0.3)  # the claim's event -> prefetch
    k.patch(MI355XPOOLS, "vc", {"spec": {"replicas": 3}}, "default")
    o = wait_ready(k, "vc", 3)
    hits = [ln for ln in node8.manager_metrics().splitlines()
            if ln.startswith("gpupool_agent_view_cache_hits_total{")]
    assert hits and float(hits[0].rsplit(" ", 1)[1]) >= 1, hits
    # scale down: cordon + release are POSTs (cache invalidated) -> the status is ground truth
    k.patch(MI355XPOOLS, "vc", {"spec": {"replicas": 1}}, "default")
    o = wait_ready(k, "vc", 1)
    view = agent_view(node8)
    assert {d["uuid"] for d in view["devices"] if d.get("pool") == "default/vc"} == \
        {d["uuid"] for d in o["status"]["devices"]}


def test_namespace_gpu_quota(node8):
    """a ResourceQuota caps the GPUs pools in a namespace may claim."""
    from gpupool.kube import Res
    quotas = Res("", "v1", "resourcequotas")
    k = node8.client
    k.create(quotas, {"metadata": {"name": "gpu-quota"},
                      "spec": {"hard": {"requests.amd.com/gpu": "3"}}}, "team")
    k.create(MI355XPOOLS, mi_pool("a", 2), "team")
    wait_ready(k, "a", 2, ns="team")
    k.create(MI355XPOOLS, mi_pool("b", 2), "team")
    o = k.wait_for(MI355XPOOLS, "b", "team", cond_is("Progressing", "False", "QuotaExceeded"),
                   timeout=20)
    assert o["status"].get("readyReplicas", 0) == 0 and "gpu-quota" in \
        conds(o)["Progressing"]["message"]
    k.patch(MI355XPOOLS, "b", {"spec": {"replicas": 1}}, "team")
    wait_ready(k, "b", 1, ns="team")  # 2 + 1 fits the quota


def test_node_preflight_and_partition_surface(node8):
    k = node8.client
    node = k.get(NODES, "mi355x-node-0")
    c = {x["type"]: x for x in node["status"]["conditions"]}
    assert c["ROCmReady"]["status"] == "True" and c["GPUPoolAgentReady"]["status"] == "True"
    assert node["metadata"]["labels"]["amd.com/gpu.family"] == "gfx950"
    assert node["metadata"]["labels"]["amd.com/compute-partition"] == "SPX"
    k.create(MI355XPOOLS, mi_pool("p", 1, partition={"compute": "SPX", "memory": "NPS1"}),
             "default")
    o = wait_ready(k, "p", 1)
    assert o["status"]["devices"][0]["partition"] == {"compute": "SPX", "memory": "NPS1"}
    # a pool requiring CPX mode cannot use these SPX GPUs (observed, never changed)
    k.create(MI355XPOOLS, mi_pool("cpx", 1, partition={"compute": "CPX"}), "default")
    k.wait_for(MI355XPOOLS, "cpx", "default", cond_is("Progressing", "False",
                                                      "InsufficientDevices"), timeout=20)


def test_invalid_spec_is_rejected(node8):
    with pytest.raises(KubeError):
        node8.client.create(MI355XPOOLS, mi_pool("neg", -1), "default")


def test_drain_respects_pod_disruption_budget(node8):
    """Scale-down drains through the Eviction API: a PodDisruptionBudget refusal (429) leaves the
    GPU draining (EvictionBlocked event, retried every pass) until the budget allows it."""
    from gpupool.kube import BY_KIND
    PDBS = BY_KIND["PodDisruptionBudget"]
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("p", 2, drain={"gracePeriodSeconds": 1, "timeoutSeconds": 300}),
             "default")
    wait_ready(k, "p", 2)
    for i in range(2):
        pod = pause_pod(f"trainer-{i}")
        pod["metadata"]["labels"] = {"app": "trainer"}
        k.create(PODS, pod, "default")
    for i in range(2):
        k.wait_for(PODS, f"trainer-{i}", "default",
                   lambda o: o and o["status"].get("phase") == "Running", timeout=30)
    k.create(PDBS, {"apiVersion": "policy/v1", "kind": "PodDisruptionBudget",
                    "metadata": {"name": "trainers"},
                    "spec": {"minAvailable": 2, "selector": {"matchLabels": {"app": "trainer"}}}},
             "default")
    k.patch(MI355XPOOLS, "p", {"spec": {"replicas": 1}}, "default")

    def blocked(_o):
        return any(e["reason"] == "EvictionBlocked" for e in settled_events(k))
    try:
        k.wait_for(MI355XPOOLS, "p", "default", blocked, timeout=20)
    except TimeoutError:  # diagnostics for a rare flake seen once under full-suite load
        ev = [(e["reason"], e.get("message", "")[:120]) for e in settled_events(k)]
        pods = [(p["metadata"]["name"], p["status"].get("phase"),
                 p["metadata"].get("annotations", {}).get("gpupool.amd.com/devices"))
                for p in k.list(PODS, "default")["items"]]
        view = [(d["index"], d["state"], d.get("pods")) for d in agent_view(node8)["devices"]
                if d.get("poolUID")]
        raise AssertionError(f"no EvictionBlocked: events={ev} pods={pods} agent={view}")
    time.sleep(0.5)
    o = k.get(MI355XPOOLS, "p", "default")
    assert len(k.list(PODS, "default")["items"]) == 2  # nobody evicted
    assert conds(o)["Progressing"]["reason"] == "ScalingDown" or \
        conds(o)["Progressing"]["reason"] == "Draining"
    # relax the budget: the next pass evicts and releases
    k.delete(PDBS, "trainers", "default")
    wait_ready(k, "p", 1, timeout=30)
    assert len(k.list(PODS, "default")["items"]) == 1


def test_periodic_recheck_replaces_degraded_gpu(cluster_factory):
    """spec.probe.recheckSeconds: an idle claimed GPU is re-probed; when it starts failing
    (fault overlay probeFail after the claim) it is cordoned, released and replaced."""
    c = cluster_factory(nodes=[NodeSpec("mi355x-node-0")])
    k = c.client
    k.create(MI355XPOOLS, mi_pool("p", 1, probe={"recheckSeconds": 1}), "default")
    o = wait_ready(k, "p", 1)
    first = o["status"]["devices"][0]
    t0 = time.monotonic()
    c.set_faults("mi355x-node-0", {"devices": {first["uuid"]: {"probeFail": True}}})

    def replaced(o):
        devs = (o or {}).get("status", {}).get("devices", [])
        return ready_at(1)(o) and devs and devs[0]["uuid"] != first["uuid"]
    k.wait_for(MI355XPOOLS, "p", "default", replaced, timeout=30)
    # event-driven: the agent's long-poll wakes the manager (not the 10 s resync)
    assert time.monotonic() - t0 < 6.0
    view = c.agent_request("mi355x-node-0", "GET", "/v1/node")
    assert next(d for d in view["devices"] if d["uuid"] == first["uuid"])["state"] == "Quarantined"


def test_xgmi_peer_check(cluster_factory):
    """spec.probe.xgmiPeerCheck: ring peer copies across the pool's GPUs; link bandwidth lands in
    status.devices[].probe.xgmiGBps and a failing link (fault overlay xgmiPeerFail) makes its
    sender fail the probe and get replaced."""
    c = cluster_factory(nodes=[NodeSpec("mi355x-node-0")])
    k = c.client
    c.set_faults("mi355x-node-0", {"devices": {"1": {"xgmiPeerFail": True}}})
    k.create(MI355XPOOLS, mi_pool("ring", 4, probe={"xgmiPeerCheck": True, "minXgmiGBps": 10}),
             "default")
    o = wait_ready(k, "ring", 4, timeout=30)
    devs = o["status"]["devices"]
    assert 1 not in {d["index"] for d in devs}
    assert all(d["probe"]["xgmiGBps"] > 10 for d in devs)
    msgs = " ".join(e.get("message", "") for e in settled_events(k))
    assert "XGMIPeerCheckFailed" in msgs


def test_gpu_maintenance_cordon(node8):
    """`gpuctl gpu cordon NODE GPU`: the pool holding the GPU replaces it (event-driven), the GPU is
    never claimed while cordoned (survives release), and `uncordon` returns it to the free set."""
    import os
    import subprocess
    import sys
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("p", 2), "default")
    o = wait_ready(k, "p", 2)
    victim = o["status"]["devices"][0]
    env = dict(os.environ, PYTHONPATH=node8.env["PYTHONPATH"], GPUPOOL_APISERVER=node8.url,
               GPUPOOL_AGENT_TOKEN_FILE=node8.agent_token_file)  # the admin's copy of the Secret

    def gpuctl(*a):
        r = subprocess.run([sys.executable, "-m", "gpupool.cli", *a], env=env, capture_output=True,
                           text=True, timeout=60)
        assert r.returncode == 0, r.stdout + r.stderr
        return r.stdout
    out = gpuctl("gpu", "cordon", "mi355x-node-0", str(victim["index"]), "--reason", "fw update")
    assert "cordoned" in out and "replaced" in out

    def replaced(o):
        u = {d["uuid"] for d in (o or {}).get("status", {}).get("devices", [])}
        return ready_at(2)(o) and victim["uuid"] not in u
    k.wait_for(MI355XPOOLS, "p", "default", replaced, timeout=15)
    dev = next(d for d in agent_view(node8)["devices"] if d["uuid"] == victim["uuid"])
    assert dev["state"] == "Maintenance" and "fw update" in dev["quarantine"]["reason"]
    # a scale-up never picks the cordoned GPU
    k.patch(MI355XPOOLS, "p", {"spec": {"replicas": 7}}, "default")
    o = wait_ready(k, "p", 7)
    assert victim["uuid"] not in {d["uuid"] for d in o["status"]["devices"]}
    gpuctl("gpu", "uncordon", "mi355x-node-0", victim["uuid"])
    assert next(d for d in agent_view(node8)["devices"] if d["uuid"] == victim["uuid"])["state"] == "Free"
    k.patch(MI355XPOOLS, "p", {"spec": {"replicas": 8}}, "default")
    wait_ready(k, "p", 8)


def test_many_pools_fill_every_gpu_across_nodes(cluster_factory):
    """32 one-GPU pools on 4 nodes x 8 GPUs: concurrent workers race for the tightest node; a
    pool that loses the race falls through to the next fitting node in the same pass, so every
    GPU ends up claimed exactly once."""
    c = cluster_factory(nodes=[NodeSpec(f"n{i}") for i in range(4)])
    k = c.client
    t0 = time.monotonic()
    for i in range(32):
        k.create(MI355XPOOLS, mi_pool(f"p{i}", 1), "default")
    deadline = time.monotonic() + 30
    while time.monotonic() < deadline:
        items = k.list(MI355XPOOLS, "default")["items"]
        if sum(1 for o in items if ready_at(1)(o)) == 32:
            break
        time.sleep(0.1)
    items = k.list(MI355XPOOLS, "default")["items"]
    assert sum(1 for o in items if ready_at(1)(o)) == 32, time.monotonic() - t0
    uuids = [o["status"]["devices"][0]["uuid"] for o in items]
    assert len(set(uuids)) == 32
    # placement spreads concurrent claims by the capacity the manager already committed (claims
    # made or in flight since each agent's last full view), so few lose a race for a node
    claims = full_views = 0
    for i in range(4):
        m = c.agent_request(f"n{i}", "GET", "/metrics")
        for line in m.splitlines():
            if line.startswith('gpupool_agent_rpc_requests_total{path="/v1/claims"}'):
                claims += int(line.rsplit(" ", 1)[1])
            if line.startswith('gpupool_agent_rpc_requests_total{path="/v1/node"}'):
                full_views += int(line.rsplit(" ", 1)[1])
    print("claim RPCs", claims, "node views", full_views)
    assert claims <= 32 + 8, claims
    k.create(MI355XPOOLS, mi_pool("extra", 1), "default")
    k.wait_for(MI355XPOOLS, "extra", "default",
               cond_is("Progressing", "False", "InsufficientDevices"), timeout=15)
    # freeing one GPU wakes the waiting pool without waiting for its requeue
    k.patch(MI355XPOOLS, "p0", {"spec": {"replicas": 0}}, "default")
    wait_ready(k, "extra", 1, timeout=15)


def test_agent_rpc_requires_the_shared_token(node8):
    """The agent's RPC refuses callers without the manager's shared secret (any pod
    could otherwise claim, cordon or release GPUs); /healthz and /metrics stay open."""
    from gpupool.kube import Client
    anon = Client("unix://" + node8.agent_socket("mi355x-node-0"))
    for method, path, body in (("POST", "/v1/claims", {"poolUID": "x", "count": 1}),
                               ("POST", "/v1/maintenance", {"gpu": "0", "on": True}),
                               ("POST", "/v1/release", {"poolUID": "x", "uuids": []}),
                               ("GET", "/v1/node", None)):
        with pytest.raises(KubeError) as ei:
            anon.request(method, path, body)
        assert ei.value.code == 401
    wrong = Client("unix://" + node8.agent_socket("mi355x-node-0"), "not-the-token")
    with pytest.raises(KubeError) as ei:
        wrong.request("POST", "/v1/claims", {"poolUID": "x", "count": 1})
    assert ei.value.code == 401
    assert "gpupool_device_healthy" in str(anon.request("GET", "/metrics"))
    assert agent_view(node8)["devices"]  # the harness (and the manager) hold the token
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("p", 1), "default")
    wait_ready(k, "p", 1)


def test_pool_spans_nodes(cluster_factory):
    """spec.maxNodes (the reference's pool of N machines, README.md:23-31, :199-209): a pool of 12
    on two 8-GPU nodes claims 8 + 4 (all-or-nothing per pass), is Ready with status.nodes listing
    both and every device carrying its node; scaling to 4 drains the smaller node first and ends
    on one node; maxNodes=1 pools still refuse what no single node fits; deletion releases the
    GPUs on every node through the finalizer."""
    c = cluster_factory(nodes=[NodeSpec("node-a"), NodeSpec("node-b")])
    k = c.client
    k.create(MI355XPOOLS, mi_pool("one", 12), "default")  # maxNodes defaults to 1
    k.wait_for(MI355XPOOLS, "one", "default", cond_is("Ready", "False", "InsufficientDevices"),
               timeout=30)
    k.delete(MI355XPOOLS, "one", "default")
    k.wait_for(MI355XPOOLS, "one", "default", lambda o: o is None, timeout=30)
    k.create(MI355XPOOLS, mi_pool("wide", 12, maxNodes=2), "default")
    o = wait_ready(k, "wide", 12, timeout=60)
    st = o["status"]
    assert sorted(st["nodes"]) == ["node-a", "node-b"]
    per = {}
    for d in st["devices"]:
        per[d["node"]] = per.get(d["node"], 0) + 1
    assert sorted(per.values()) == [4, 8] and st["nodeName"] == max(per, key=per.get)
    assert "on 2 nodes" in conds(o)["Ready"]["message"]
    views = {n: agent_view(c, n) for n in ("node-a", "node-b")}
    owned = {n: sum(1 for d in v["devices"] if d.get("pool") == "default/wide") for n, v in views.items()}
    assert owned == per  # the agents agree with the status, node by node
    small = min(per, key=per.get)
    k.patch(MI355XPOOLS, "wide", {"spec": {"replicas": 4}}, "default")
    o = wait_ready(k, "wide", 4, timeout=60)
    assert {d["node"] for d in o["status"]["devices"]} == {max(per, key=per.get)}
    assert sum(1 for d in agent_view(c, small)["devices"] if d.get("pool") == "default/wide") == 0
    # grows back onto the node it is on first (8 there), then the other
    k.patch(MI355XPOOLS, "wide", {"spec": {"replicas": 10}}, "default")
    o = wait_ready(k, "wide", 10, timeout=60)
    per = {}
    for d in o["status"]["devices"]:
        per[d["node"]] = per.get(d["node"], 0) + 1
    assert sorted(per.values()) == [2, 8]
    # maxNodes=3 cannot exceed what the cluster has: all-or-nothing, nothing partial
    k.create(MI355XPOOLS, mi_pool("rest", 8, maxNodes=3), "default")
    r = k.wait_for(MI355XPOOLS, "rest", "default", cond_is("Ready", "False", "InsufficientDevices"),
                   timeout=30)
    assert r["status"].get("replicas", 0) == 0
    k.delete(MI355XPOOLS, "wide", "default")
    k.wait_for(MI355XPOOLS, "wide", "default", lambda o: o is None, timeout=30)
    for n in ("node-a", "node-b"):
        assert not any(d.get("pool") == "default/wide" for d in agent_view(c, n)["devices"])
    wait_ready(k, "rest", 8, timeout=60)  # the freed GPUs are claimed by the waiting pool


def test_spanning_claim_is_all_or_nothing(cluster_factory):
    """A spanning scale-up whose second node refuses its part (here: the pool's stricter
    maxRetiredPages, which the node's free-GPU count does not know about) hands back the GPUs it
    already claimed on the first node in the same pass: nothing partial is left held."""
    c = cluster_factory(nodes=[NodeSpec("node-a"), NodeSpec("node-b", count=4)])
    c.set_faults("node-b", {"devices": {str(i): {"ras": {"retiredPages": 10}} for i in range(4)}})
    k = c.client
    k.create(MI355XPOOLS, mi_pool("strict", 12, maxNodes=2, health={"maxRetiredPages": 5}),
             "default")
    o = k.wait_for(MI355XPOOLS, "strict", "default",
                   cond_is("Ready", "False", "InsufficientDevices"), timeout=30)
    time.sleep(0.5)
    o = k.get(MI355XPOOLS, "strict", "default")
    assert o["status"].get("replicas", 0) == 0
    for n in ("node-a", "node-b"):
        assert not any(d.get("pool") == "default/strict" for d in agent_view(c, n)["devices"])
    msgs = " ".join(e.get("message", "") for e in settled_events(k))
    assert "other claims released" in msgs


def test_lagging_watch_cache_does_not_fail_reconciles(cluster_factory):
    """Informers can lag the apiserver (a loaded kube-apiserver's watch cache; here every watch
    event arrives 300 ms late). Passes that act on a stale object — the finalizer patch and the
    status write carry its resourceVersion — re-read it on 409 instead of failing into backoff, so
    a pool still converges promptly and the manager logs no failed reconcile."""
    c = cluster_factory(apiserver_args=["--watch-delay", "0.3"])
    k = c.client
    k.create(MI355XPOOLS, mi_pool("p", 1), "default")
    wait_ready(k, "p", 1, timeout=30)
    t0 = time.perf_counter()
    k.patch(MI355XPOOLS, "p", {"spec": {"replicas": 3}}, "default")
    wait_ready(k, "p", 3, timeout=30)
    assert time.perf_counter() - t0 < 5.0
    k.patch(MI355XPOOLS, "p", {"spec": {"replicas": 0}}, "default")
    wait_ready(k, "p", 0, timeout=30)
    k.delete(MI355XPOOLS, "p", "default")
    k.wait_for(MI355XPOOLS, "p", "default", lambda o: o is None, timeout=30)
    failed = [ln for ln in c.log("manager").splitlines() if "reconcile failed" in ln]
    assert not failed, failed[:3]


def test_cordoned_node_takes_no_new_claims(cluster_factory):
    """A cordoned Node (spec.unschedulable, `kubectl cordon`) keeps the GPUs its pools hold but
    takes no new claims: an unpinned pool is placed on another node, a pool pinned to the cordoned
    node waits (InsufficientDevices, reason in the message) until the node is uncordoned."""
    c = cluster_factory(nodes=[NodeSpec("node-a", count=4), NodeSpec("node-b", count=4)])
    k = c.client
    k.create(MI355XPOOLS, mi_pool("held", 1, nodeName="node-a"), "default")
    wait_ready(k, "held", 1)
    k.patch(NODES, "node-a", {"spec": {"unschedulable": True}}, None)
    # the manager learns of the cordon through its Node watch, asynchronously (as after a
    # `kubectl cordon`): a pool created in the same instant may still be placed on the node
    time.sleep(0.5)
    k.create(MI355XPOOLS, mi_pool("free", 2), "default")
    o = wait_ready(k, "free", 2)
    assert o["status"]["nodeName"] == "node-b"
    k.patch(MI355XPOOLS, "held", {"spec": {"replicas": 2}}, "default")
    o = k.wait_for(MI355XPOOLS, "held", "default",
                   cond_is("Progressing", "False", "InsufficientDevices"), timeout=20)
    assert "cordoned" in conds(o)["Progressing"]["message"]
    assert o["status"]["readyReplicas"] == 1  # its GPU stays
    k.patch(NODES, "node-a", {"spec": {"unschedulable": False}}, None)
    wait_ready(k, "held", 2, timeout=30)


def test_leader_election_tolerates_clock_skew(cluster_factory):
    """A live leader whose clock runs an hour behind renews with renewTimes far in the past: a
    standby times the lease from when *it* saw the record change (client-go observedTime), so it
    never takes over a lease that is still being renewed — and it does take over once the
    renewals stop."""
    import threading
    from gpupool.kube import LEASES
    c = cluster_factory(manager=False)
    k = c.client
    stale = "2001-01-01T00:00:%02d.000000Z"
    k.create(LEASES, {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                      "metadata": {"name": "gpupool-manager-leader"},
                      "spec": {"holderIdentity": "skewed-leader", "leaseDurationSeconds": 2,
                               "renewTime": stale % 0, "acquireTime": stale % 0}},
             "gpupool-system")
    stop = threading.Event()

    def renew():
        i = 0
        while not stop.wait(0.4):
            i += 1
            o = k.get(LEASES, "gpupool-manager-leader", "gpupool-system")
            if o["spec"]["holderIdentity"] != "skewed-leader":
                return
            o["spec"]["renewTime"] = stale % (i % 60)
            k.update(LEASES, o, "gpupool-system")
    t = threading.Thread(target=renew, daemon=True)
    t.start()
    c.manager_args = ["--leader-elect", "--lease-duration", "2s", "--renew-deadline", "1500ms",
                      "--retry-period", "200ms", "--identity", "standby"]
    c.start_manager()
    time.sleep(4.0)  # two lease durations: the skewed holder keeps renewing
    assert k.get(LEASES, "gpupool-manager-leader", "gpupool-system")["spec"]["holderIdentity"] == \
        "skewed-leader"
    stop.set()
    t.join()
    k.wait_for(LEASES, "gpupool-manager-leader", "gpupool-system",
               lambda o: o and o["spec"]["holderIdentity"] == "standby", timeout=10, poll=0.1)


def test_spanning_pool_keeps_unreachable_nodes(cluster_factory):
    """A pool spanning three nodes loses two agents: status.nodes keeps listing them (their GPUs
    and pods are still held), the pool reports AgentUnreachable and claims nothing elsewhere;
    when the agents return it is Ready again on the same three nodes."""
    nodes = [NodeSpec(f"sn-{i}", count=4) for i in range(3)]
    c = cluster_factory(nodes=nodes)
    k = c.client
    k.create(MI355XPOOLS, mi_pool("wide", 12, maxNodes=3), "default")
    o = wait_ready(k, "wide", 12, timeout=60)
    assert sorted(o["status"]["nodes"]) == ["sn-0", "sn-1", "sn-2"]
    before = {d["uuid"] for d in o["status"]["devices"]}
    c._kill("agent-sn-1")
    c._kill("agent-sn-2")
    o = k.wait_for(MI355XPOOLS, "wide", "default", lambda o: conds(o).get("Ready", {}).get(
        "reason") == "AgentUnreachable", timeout=60)
    time.sleep(1.0)  # a few more passes with both nodes down
    o = k.get(MI355XPOOLS, "wide", "default")
    assert sorted(o["status"]["nodes"]) == ["sn-0", "sn-1", "sn-2"], o["status"].get("nodes")
    for n in nodes[1:]:
        c.start_agent(n)
    o = wait_ready(k, "wide", 12, timeout=60)
    assert sorted(o["status"]["nodes"]) == ["sn-0", "sn-1", "sn-2"]
    assert {d["uuid"] for d in o["status"]["devices"]} == before


def test_kubelet_restart_readvertises_without_a_device_change(cluster_factory):
    """The kubelet restarts (its ListAndWatch stream ends, the plugin re-registers, a new stream
    opens): while it is gone the pool's GPUs are not advertised (readyReplicas 0); once the new
    stream has resent the same device list the pool is Ready again — no device change needed."""
    c = cluster_factory()
    k = c.client
    k.create(MI355XPOOLS, mi_pool("kr", 2), "default")
    wait_ready(k, "kr", 2)
    node = c.nodes[0]
    c._kill(f"kubelet-{node.name}")
    k.wait_for(MI355XPOOLS, "kr", "default",
               lambda o: (o.get("status") or {}).get("readyReplicas") == 0, timeout=30)
    c.start_kubelet(node)
    o = wait_ready(k, "kr", 2, timeout=30)
    assert all(d["advertised"] for d in o["status"]["devices"])


def test_spanning_pool_with_a_lost_claim_reply_can_be_deleted(cluster_factory):
    """A spanning pool (maxNodes > 1) whose claim reply is lost (the agent stalls past the
    manager's RPC timeout, then commits the claim) must still be deletable: the node it suspected
    answers every later pass (a spanning pool observes every node), so the suspicion is resolved
    and the finalizer comes off once its GPUs are released — not 'claim outcome unknown' forever."""
    stall = ["--inject-claim-delay", "2:1.5"]  # claims of >= 2 GPUs stall 1.5 s
    c = cluster_factory(nodes=[NodeSpec("sp-a", extra_args=stall), NodeSpec("sp-b", extra_args=stall)],
                        manager_args=["--agent-timeout", "600ms", "--orphan-sweep", "1s"])
    k = c.client
    uid = k.create(MI355XPOOLS, mi_pool("span", 10, maxNodes=2), "default")["metadata"]["uid"]
    deadline = time.time() + 20
    while not [d for n in ("sp-a", "sp-b") for d in agent_view(c, n)["devices"]
               if d.get("poolUID") == uid]:
        assert time.time() < deadline, "no stalled claim ever landed"
        time.sleep(0.1)
    k.delete(MI355XPOOLS, "span", "default")
    k.wait_for(MI355XPOOLS, "span", "default", lambda o: o is None, timeout=30)
    deadline = time.time() + 15  # a claim still stalled at deletion lands as an orphan: swept
    while [d for n in ("sp-a", "sp-b") for d in agent_view(c, n)["devices"] if d.get("poolUID") == uid]:
        assert time.time() < deadline, "GPUs of the deleted pool still held"
        time.sleep(0.2)
