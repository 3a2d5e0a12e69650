"""Property test (SURVEY.md §4.2 'Property' row): random sequences of replicas edits and device
faults on two pools sharing one 8-GPU node. After faults clear and the system settles:
  * readyReplicas == spec.replicas for both pools (when the total fits the node);
  * the pools' device sets are disjoint (never claims a device owned by another pool);
  * the agent's claims are exactly the union of the pools' status.devices;
  * the kubelet's allocatable per resource equals each pool's readyReplicas.
"""
from __future__ import annotations

import os
import time

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from gpupool.kube import MI355XPOOLS, NODES
from gpupool.testing.cluster import Cluster, NodeSpec

from .helpers import mi_pool, ready_at, settled_pools

pytestmark = pytest.mark.slow

# more examples for a deeper search: GPUPOOL_PROPERTY_SCALE=5 python -m pytest ...
SCALE = max(1, int(os.environ.get("GPUPOOL_PROPERTY_SCALE", "1")))

op = st.one_of(
    st.tuples(st.just("scale"), st.sampled_from(["pa", "pb"]), st.integers(0, 6)),
    st.tuples(st.just("fault"), st.integers(0, 7), st.sampled_from(["ecc", "xgmi", "thermal"])),
    st.tuples(st.just("clear"), st.just(0), st.just(0)),
)


@pytest.fixture(scope="module")
def shared(tmp_path_factory, native_built):
    c = Cluster(str(tmp_path_factory.mktemp("prop")),
                nodes=[NodeSpec("mi355x-node-0", extra_args=["--quarantine", "0.3"])],
                sample_interval=0.2)
    c.start()
    yield c
    c.stop()


FAULTS = {"ecc": {"ecc": {"uncorrectable": 1}},
          "xgmi": {"xgmi": {"links": ["X", "U", "D", "U", "U", "U", "U", "U"]}},
          "thermal": {"temps": {"hotspot": {"current": 110}}}}


@settings(max_examples=8 * SCALE, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture,
                                                                 HealthCheck.too_slow])
@given(ops=st.lists(op, min_size=1, max_size=6), final=st.tuples(st.integers(0, 4),
                                                                  st.integers(0, 4)))
def test_random_edits_and_faults_converge(shared, ops, final):
    c = shared
    k = c.client
    ns = f"p{int(time.time() * 1e6) % 10**9}"
    k.create(MI355XPOOLS, mi_pool("pa", 1, resourceName="amd.com/gpu-a"), ns)
    k.create(MI355XPOOLS, mi_pool("pb", 1, resourceName="amd.com/gpu-b"), ns)
    faults: dict = {}
    for kind, a, b in ops:
        if kind == "scale":
            k.patch(MI355XPOOLS, a, {"spec": {"replicas": b}}, ns)
        elif kind == "fault":
            faults[str(a)] = FAULTS[b]
            c.set_faults("mi355x-node-0", {"devices": faults})
        else:
            faults = {}
            c.set_faults("mi355x-node-0", {})
        time.sleep(0.05)
    c.set_faults("mi355x-node-0", {})
    ra, rb = final
    try:
        k.patch(MI355XPOOLS, "pa", {"spec": {"replicas": ra}}, ns)
        k.patch(MI355XPOOLS, "pb", {"spec": {"replicas": rb}}, ns)
        k.wait_for(MI355XPOOLS, "pa", ns, ready_at(ra), timeout=90)
        k.wait_for(MI355XPOOLS, "pb", ns, ready_at(rb), timeout=90)
        pools, claims = settled_pools(
            k, ns, {"pa": ra, "pb": rb},
            lambda: [c.agent_request("mi355x-node-0", "GET", "/v1/node")])
        ua = {d["uuid"] for d in pools["pa"]["status"]["devices"]}
        ub = {d["uuid"] for d in pools["pb"]["status"]["devices"]}
        assert ready_at(ra)(pools["pa"]) and ready_at(rb)(pools["pb"])
        assert not ua & ub
        assert claims == {"pa": ua, "pb": ub}
        deadline = time.time() + 10
        while True:  # kubelet's view converges through ListAndWatch
            alloc = k.get(NODES, "mi355x-node-0")["status"].get("allocatable", {})
            if alloc.get("amd.com/gpu-a", "0") == str(ra) and \
                    alloc.get("amd.com/gpu-b", "0") == str(rb):
                break
            assert time.time() < deadline, alloc
            time.sleep(0.05)
    finally:  # a failed example must not leave pools behind for the next one (same resources)
        for name in ("pa", "pb"):
            k.delete(MI355XPOOLS, name, ns)
        for name in ("pa", "pb"):
            k.wait_for(MI355XPOOLS, name, ns, lambda o: o is None, timeout=30)


span_op = st.one_of(
    st.tuples(st.just("scale"), st.sampled_from(["sa", "sb"]), st.integers(0, 6)),
    st.tuples(st.just("fault"), st.sampled_from(["node-a", "node-b"]), st.integers(0, 3)),
    st.tuples(st.just("clear"), st.just(""), st.just(0)),
)


@pytest.fixture(scope="module")
def two_nodes(tmp_path_factory, native_built):
    c = Cluster(str(tmp_path_factory.mktemp("prop2")),
                nodes=[NodeSpec(n, count=4, extra_args=["--quarantine", "0.3"])
                       for n in ("node-a", "node-b")],
                sample_interval=0.2)
    c.start()
    yield c
    c.stop()


@settings(max_examples=6 * SCALE, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture,
                                                                 HealthCheck.too_slow])
@given(ops=st.lists(span_op, min_size=1, max_size=6),
       final=st.tuples(st.integers(0, 5), st.integers(0, 3)))
def test_spanning_pools_converge(two_nodes, ops, final):
    """Two pools with spec.maxNodes=2 over two 4-GPU nodes under random edits and ECC faults:
    once faults clear, both are Ready at their final size (sum <= 8), never share a GPU, hold GPUs
    on at most 2 nodes, and the two agents' claims are exactly the union of the pools' devices."""
    c = two_nodes
    k = c.client
    ns = f"s{int(time.time() * 1e6) % 10**9}"
    k.create(MI355XPOOLS, mi_pool("sa", 1, maxNodes=2, resourceName="amd.com/gpu-sa"), ns)
    k.create(MI355XPOOLS, mi_pool("sb", 1, maxNodes=2, resourceName="amd.com/gpu-sb"), ns)
    faults: dict = {"node-a": {}, "node-b": {}}
    for kind, a, b in ops:
        if kind == "scale":
            k.patch(MI355XPOOLS, a, {"spec": {"replicas": b}}, ns)
        elif kind == "fault":
            faults[a][str(b)] = FAULTS["ecc"]
            c.set_faults(a, {"devices": faults[a]})
        else:
            faults = {"node-a": {}, "node-b": {}}
            for n in faults:
                c.set_faults(n, {})
        time.sleep(0.05)
    for n in ("node-a", "node-b"):
        c.set_faults(n, {})
    ra, rb = final
    try:
        k.patch(MI355XPOOLS, "sa", {"spec": {"replicas": ra}}, ns)
        k.patch(MI355XPOOLS, "sb", {"spec": {"replicas": rb}}, ns)
        k.wait_for(MI355XPOOLS, "sa", ns, ready_at(ra), timeout=90)
        k.wait_for(MI355XPOOLS, "sb", ns, ready_at(rb), timeout=90)
        pools, claims = settled_pools(
            k, ns, {"sa": ra, "sb": rb},
            lambda: [c.agent_request(n, "GET", "/v1/node") for n in ("node-a", "node-b")])
        ua = {d["uuid"] for d in pools["sa"]["status"]["devices"]}
        ub = {d["uuid"] for d in pools["sb"]["status"]["devices"]}
        assert ready_at(ra)(pools["sa"]) and ready_at(rb)(pools["sb"])
        assert not ua & ub
        for o in pools.values():
            assert len({d["node"] for d in o["status"]["devices"]}) <= 2
        assert claims == {"sa": ua, "sb": ub}
    finally:
        for name in ("sa", "sb"):
            k.delete(MI355XPOOLS, name, ns)
        for name in ("sa", "sb"):
            k.wait_for(MI355XPOOLS, name, ns, lambda o: o is None, timeout=30)


chaos_op = st.one_of(
    st.tuples(st.just("scale"), st.integers(0, 6)),
    st.tuples(st.just("pod"), st.integers(0, 1000)),
    st.tuples(st.just("restart-manager"), st.just(0)),
    st.tuples(st.just("restart-agent"), st.just(0)),
)


@pytest.fixture(scope="module")
def chaos(tmp_path_factory, native_built):
    c = Cluster(str(tmp_path_factory.mktemp("chaos")), nodes=[NodeSpec("mi355x-node-0")],
                sample_interval=0.2)
    c.start()
    yield c
    c.stop()


@settings(max_examples=5 * SCALE, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture,
                                                                 HealthCheck.too_slow])
@given(ops=st.lists(chaos_op, min_size=2, max_size=7), final=st.integers(0, 5))
def test_restarts_and_pods_never_strand_a_pod(chaos, ops, final):
    """Random replicas edits, GPU pods and restarts of the manager and of the node agent (the
    SURVEY §4.2 property row). Once settled: readyReplicas == spec.replicas, the agent's claims
    are exactly the pool's devices (restarts re-adopt from the ledger, nothing is double-claimed
    or leaked), and every pod still running sits on a GPU the pool holds — no GPU was released
    under a running pod."""
    from gpupool.kube import PODS
    from .helpers import pause_pod
    c = chaos
    k = c.client
    node = c.nodes[0]
    ns = f"c{int(time.time() * 1e6) % 10**9}"
    res = "amd.com/gpu-chaos"
    k.create(MI355XPOOLS, mi_pool("pc", 1, resourceName=res, drain={"gracePeriodSeconds": 1}), ns)
    for kind, v in ops:
        if kind == "scale":
            k.patch(MI355XPOOLS, "pc", {"spec": {"replicas": v}}, ns)
        elif kind == "pod":
            k.create(PODS, pause_pod(f"w{v}-{len(ns)}-{time.time_ns() % 10**6}", resource=res), ns)
        elif kind == "restart-manager":
            c._kill("manager")
            c.start_manager()
        else:
            c._kill(f"agent-{node.name}")
            c.start_agent(node)
        time.sleep(0.1)
    k.patch(MI355XPOOLS, "pc", {"spec": {"replicas": final}}, ns)
    o = k.wait_for(MI355XPOOLS, "pc", ns, ready_at(final), timeout=90)
    held = {d["uuid"] for d in o["status"]["devices"]}
    view = c.agent_request(node.name, "GET", "/v1/node")
    assert {d["uuid"] for d in view["devices"] if d.get("poolUID") == o["metadata"]["uid"]} == held
    deadline = time.time() + 15
    while True:  # evictions of pods on released GPUs complete asynchronously (grace 1 s)
        running = [p for p in k.list(PODS, ns)["items"]
                   if p["status"].get("phase") == "Running" and not p["metadata"].get("deletionTimestamp")]
        stray = [p["metadata"]["name"] for p in running
                 if not set((p["metadata"].get("annotations") or {})
                            .get("gpupool.amd.com/devices", "").split(",")) <= held]
        if not stray or time.time() > deadline:
            break
        time.sleep(0.1)
    assert not stray, (stray, held)
    for p in k.list(PODS, ns)["items"]:
        k.delete(PODS, p["metadata"]["name"], ns, grace=0)
    k.delete(MI355XPOOLS, "pc", ns)
    k.wait_for(MI355XPOOLS, "pc", ns, lambda x: x is None, timeout=60)


outage_op = st.one_of(
    st.tuples(st.just("scale"), st.integers(0, 5)),
    st.tuples(st.just("agent-down"), st.sampled_from(["on-a", "on-b"])),
    st.tuples(st.just("agent-up"), st.sampled_from(["on-a", "on-b"])),
    st.tuples(st.just("delete"), st.just("")),
    st.tuples(st.just("create"), st.just("")),
    st.tuples(st.just("wait"), st.sampled_from([0.0, 0.02, 0.2])),
    st.tuples(st.just("restart-manager"), st.just("")),
)


@pytest.fixture(scope="module")
def outage(tmp_path_factory, native_built):
    # the sweep runs every 2 s: a restarted manager forgets the claims whose reply it lost, and the
    # sweep is what finds those again
    c = Cluster(str(tmp_path_factory.mktemp("outage")), nodes=[NodeSpec("on-a"), NodeSpec("on-b")],
                sample_interval=0.2, manager_args=["--orphan-sweep", "2s"])
    c.start()
    yield c
    c.stop()


@settings(max_examples=6 * SCALE, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture,
                                                                 HealthCheck.too_slow])
@given(ops=st.lists(outage_op, min_size=3, max_size=9), final=st.integers(1, 4))
def test_agent_outages_never_leak_or_double_claim(outage, ops, final):
    """Random replicas edits, pool deletes / re-creates, manager restarts and agent outages that
    last over several operations, on two nodes. Once every agent is back and the pool settles: the
    live pool's GPUs on the agents are exactly its status.devices, all on one node; and no agent
    holds a GPU for a pool that no longer exists."""
    c = outage
    k = c.client
    ns = f"o{int(time.time() * 1e6) % 10**9}"
    by_name = {n.name: n for n in c.nodes}
    down: set[str] = set()
    uids: set[str] = set()
    exists = False

    def create():
        o = k.create(MI355XPOOLS, mi_pool("po", 1), ns)
        uids.add(o["metadata"]["uid"])

    create()
    exists = True
    for kind, v in ops:
        if kind == "scale" and exists:
            k.patch(MI355XPOOLS, "po", {"spec": {"replicas": v}}, ns)
        elif kind == "agent-down" and v not in down:
            c._kill(f"agent-{v}")
            down.add(v)
        elif kind == "agent-up" and v in down:
            c.start_agent(by_name[v])
            down.discard(v)
        elif kind == "delete" and exists:
            k.delete(MI355XPOOLS, "po", ns)
            exists = False
        elif kind == "create" and not exists:
            try:  # the deleted pool may still be finalizing (an agent is down): then it stays
                k.wait_for(MI355XPOOLS, "po", ns, lambda o: o is None, timeout=0.3)
            except TimeoutError:
                continue
            create()
            exists = True
        elif kind == "wait":
            time.sleep(v)
        elif kind == "restart-manager":
            c._kill("manager")
            c.start_manager()
    for n in sorted(down):
        c.start_agent(by_name[n])
    if not exists:
        k.wait_for(MI355XPOOLS, "po", ns, lambda o: o is None, timeout=60)
        create()
    k.patch(MI355XPOOLS, "po", {"spec": {"replicas": final}}, ns)
    o = k.wait_for(MI355XPOOLS, "po", ns, ready_at(final), timeout=90)
    live = o["metadata"]["uid"]
    deadline = time.time() + 8  # a stray claim from before a manager restart waits for a sweep
    while True:
        o = k.get(MI355XPOOLS, "po", ns)
        held = {d["uuid"] for d in o["status"]["devices"]}
        mine, stale = set(), []
        for n in c.nodes:
            for d in c.agent_request(n.name, "GET", "/v1/node")["devices"]:
                if d.get("poolUID") == live:
                    mine.add(d["uuid"])
                elif d.get("poolUID") in uids:
                    stale.append((n.name, d["uuid"], d.get("state")))
        if (mine == held and not stale) or time.time() > deadline:
            break
        time.sleep(0.2)
    assert ready_at(final)(o)
    assert len({d["node"] for d in o["status"]["devices"]}) == 1, o["status"]["devices"]
    assert mine == held
    assert not stale, f"GPUs still held for deleted pools of this example: {stale}"
    k.delete(MI355XPOOLS, "po", ns)
    k.wait_for(MI355XPOOLS, "po", ns, lambda x: x is None, timeout=60)
