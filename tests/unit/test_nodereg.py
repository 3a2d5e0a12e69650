"""The agent's Node registration and heartbeat (gpupool/agent/nodereg.py), without a running agent:
a NodeRegistrar against apiserver-sim, with kubelet writes interleaved between its calls."""
from __future__ import annotations

import itertools
import threading
import time

import pytest

from gpupool.agent.nodereg import NodeRegistrar
from gpupool.kube import NODES, Client, KubeError
from tests.unit.test_apiserver_http import SimThread


@pytest.fixture(scope="module")
def sim():
    return SimThread()


class Kubelet:
    """What the kubelet writes: Node creation, then allocatable + its Ready heartbeat, as a
    strategic merge patch (the real kubelet's PatchNodeStatus)."""

    def __init__(self, c: Client, node: str):
        self.c, self.node = c, node
        c.create(NODES, {"apiVersion": "v1", "kind": "Node", "metadata": {"name": node}})

    def status(self, gpus: int, beat: str) -> None:
        self.c.patch(NODES, self.node, {"status": {
            "allocatable": {"amd.com/gpu": str(gpus)},
            "conditions": [{"type": "Ready", "status": "True", "reason": "KubeletReady",
                            "lastHeartbeatTime": beat, "lastTransitionTime": "T-start"}]}},
            sub="status", ptype="strategic")


def _clock():
    n = itertools.count()
    return lambda: f"2026-10-18T00:00:{next(n):02d}Z"


def _registrar(c, node, state, clock=None):
    return NodeRegistrar(c, node, {"amd.com/gpu.product": "MI355X"},
                         {"gpupool.amd.com/agent-endpoint": "unix:///x.sock"},
                         lambda: dict(state), clock or _clock())


def _conds(c, node):
    return {x["type"]: x for x in c.get(NODES, node)["status"].get("conditions", [])}


def test_no_node_is_created_and_registration_waits_for_the_kubelet(sim):
    c = Client(sim.url)
    r = _registrar(c, "nr-wait", {"GPUPoolAgentReady": ("True", "AgentRunning", "")})
    assert r.heartbeat() is False and not r.registered
    with pytest.raises(KubeError):
        c.get(NODES, "nr-wait")  # the agent did not create it
    Kubelet(c, "nr-wait")
    assert r.heartbeat() is True
    node = c.get(NODES, "nr-wait")
    assert node["metadata"]["labels"]["amd.com/gpu.product"] == "MI355X"
    assert node["metadata"]["annotations"]["gpupool.amd.com/agent-endpoint"] == "unix:///x.sock"


def test_kubelet_writes_between_agent_calls_survive(sim):
    """The round-5 repro: a kubelet update (allocatable 0 -> 1, Ready heartbeat T0 -> T1) between
    two agent calls is kept, whatever the agent sends."""
    c = Client(sim.url)
    k = Kubelet(c, "nr-keep")
    k.status(0, "T0")
    r = _registrar(c, "nr-keep", {"GPUPoolAgentReady": ("True", "AgentRunning", ""),
                                  "ROCmReady": ("True", "PreflightPassed", "")})
    assert r.heartbeat()
    body = r.patch_body()   # the agent's next write is computed ...
    k.status(1, "T1")       # ... the kubelet writes ...
    c.patch(NODES, "nr-keep", body, sub="status", ptype="strategic")  # ... and it lands
    st = c.get(NODES, "nr-keep")["status"]
    assert st["allocatable"] == {"amd.com/gpu": "1"}
    conds = {x["type"]: x for x in st["conditions"]}
    assert conds["Ready"]["lastHeartbeatTime"] == "T1"
    assert set(conds) == {"Ready", "GPUPoolAgentReady", "ROCmReady"}
    # the agent's patch carries nothing but its own two conditions
    assert set(body) == {"status"} and set(body["status"]) == {"conditions"}
    assert {x["type"] for x in body["status"]["conditions"]} == {"GPUPoolAgentReady", "ROCmReady"}


def test_last_transition_time_moves_only_on_a_flip(sim):
    c = Client(sim.url)
    Kubelet(c, "nr-ltt")
    state = {"GPUPoolAgentReady": ("True", "AgentRunning", ""),
             "ROCmReady": ("True", "PreflightPassed", "")}
    r = _registrar(c, "nr-ltt", state)
    assert r.heartbeat()
    first = _conds(c, "nr-ltt")
    for _ in range(3):
        assert r.heartbeat()
    now = _conds(c, "nr-ltt")
    for t in ("ROCmReady", "GPUPoolAgentReady"):
        assert now[t]["lastTransitionTime"] == first[t]["lastTransitionTime"]
        assert now[t]["lastHeartbeatTime"] != first[t]["lastHeartbeatTime"]
    state["ROCmReady"] = ("False", "PreflightFailed", "kfd: missing")
    assert r.heartbeat()
    flipped = _conds(c, "nr-ltt")
    assert flipped["ROCmReady"]["lastTransitionTime"] != first["ROCmReady"]["lastTransitionTime"]
    assert flipped["GPUPoolAgentReady"]["lastTransitionTime"] == \
        first["GPUPoolAgentReady"]["lastTransitionTime"]
    assert r.heartbeat()
    assert _conds(c, "nr-ltt")["ROCmReady"]["lastTransitionTime"] == \
        flipped["ROCmReady"]["lastTransitionTime"]


def test_restarted_agent_keeps_transition_times(sim):
    c = Client(sim.url)
    Kubelet(c, "nr-restart")
    state = {"GPUPoolAgentReady": ("True", "AgentRunning", ""),
             "ROCmReady": ("True", "PreflightPassed", "")}
    assert _registrar(c, "nr-restart", state).heartbeat()
    before = _conds(c, "nr-restart")
    later = iter(f"2026-10-19T00:00:{i:02d}Z" for i in range(60))
    r2 = _registrar(c, "nr-restart", state, clock=lambda: next(later))  # a new process
    assert r2.heartbeat()
    after = _conds(c, "nr-restart")
    for t in state:
        assert after[t]["lastTransitionTime"] == before[t]["lastTransitionTime"]
        assert after[t]["lastHeartbeatTime"].startswith("2026-10-19")


def test_concurrent_kubelet_churn_never_goes_backwards(sim):
    """A kubelet thread raising allocatable and its heartbeat as fast as it can, beside an agent
    heartbeating as fast as it can: every watch event shows both non-decreasing."""
    c = Client(sim.url)
    k = Kubelet(c, "nr-churn")
    k.status(0, "B00000")
    rv = c.get(NODES, "nr-churn")["metadata"]["resourceVersion"]
    r = _registrar(Client(sim.url), "nr-churn",
                   {"GPUPoolAgentReady": ("True", "AgentRunning", ""),
                    "ROCmReady": ("True", "PreflightPassed", "")})
    stop = threading.Event()
    seen: list[tuple[int, str]] = []

    def watch():
        for ev in Client(sim.url).watch(NODES, resource_version=rv,
                                        field_selector="metadata.name=nr-churn", stop=stop,
                                        timeout_seconds=30):
            if ev["type"] != "MODIFIED":
                continue
            st = ev["object"]["status"]
            ready = next(x for x in st["conditions"] if x["type"] == "Ready")
            seen.append((int(st["allocatable"]["amd.com/gpu"]), ready["lastHeartbeatTime"]))

    def agent():
        while not stop.is_set():
            r.heartbeat()

    threads = [threading.Thread(target=watch, daemon=True), threading.Thread(target=agent,
                                                                              daemon=True)]
    for t in threads:
        t.start()
    for i in range(1, 200):
        k.status(i, f"B{i:05d}")
    deadline = time.monotonic() + 10
    while (not seen or seen[-1][0] != 199) and time.monotonic() < deadline:
        time.sleep(0.01)
    time.sleep(0.1)  # a few agent heartbeats after the kubelet's last write
    stop.set()
    threads[1].join(10)
    assert r.stats["heartbeats"] > 5
    assert len(seen) > 200
    assert all(a[0] <= b[0] and a[1] <= b[1] for a, b in zip(seen, seen[1:])), seen
    assert seen[-1][0] == 199


def test_agent_node_policy_in_the_simulator():
    """schema.agent_node_policy, enforced by apiserver-sim for the agent ServiceAccount: its own
    Node's agent conditions and agent-prefixed labels pass; another Node, the kubelet's status,
    spec and foreign labels are refused. Without the policy object nothing is checked."""
    from gpupool.api import schema
    from gpupool.kube import res_for
    s = SimThread(token="admin")
    extra = {"authentication.kubernetes.io/node-name": ["node-a"]}
    s.sim.users = {"agent-a": {"username": schema.AGENT_SA_USER, "extra": extra}}
    admin, agent = Client(s.url, "admin"), Client(s.url, "agent-a")
    for n in ("node-a", "node-b"):
        Kubelet(admin, n).status(8, "T0")
    other = _registrar(agent, "node-b", {"GPUPoolAgentReady": ("True", "AgentRunning", "")})
    assert other.heartbeat()  # no policy installed yet: RBAC alone lets it through
    for o in schema.agent_node_policy():
        admin.create(res_for(o), o)
    own = _registrar(agent, "node-a", {"GPUPoolAgentReady": ("True", "AgentRunning", ""),
                                       "ROCmReady": ("True", "PreflightPassed", "")})
    assert own.heartbeat() and own.registered
    other = _registrar(agent, "node-b", {"GPUPoolAgentReady": ("True", "AgentRunning", "")})
    assert not other.heartbeat()
    refused = [
        ("node-b", {"metadata": {"annotations": {"gpupool.amd.com/agent-endpoint": "http://x"}}},
         None, "merge"),
        ("node-a", {"status": {"allocatable": {"amd.com/gpu": "0"}}}, "status", "strategic"),
        ("node-a", {"status": {"conditions": [{"type": "Ready", "status": "False"}]}}, "status",
         "strategic"),
        ("node-a", {"spec": {"unschedulable": True}}, None, "merge"),
        ("node-a", {"metadata": {"labels": {"kubernetes.io/hostname": "evil"}}}, None, "merge"),
    ]
    for node, body, sub, ptype in refused:
        with pytest.raises(KubeError) as ei:
            agent.patch(NODES, node, body, sub=sub, ptype=ptype)
        assert ei.value.code == 403, (node, body)
    st = admin.get(NODES, "node-a")["status"]
    assert st["allocatable"] == {"amd.com/gpu": "8"}
    # the kubelet (admin here) is not subject to the policy
    Kubelet.status(type("K", (), {"c": admin, "node": "node-a"})(), 7, "T1")


def test_expired_tokens_are_refused():
    s = SimThread(token="admin")
    s.sim.users = {"short": {"username": "u", "expiresAt": time.time() + 0.3}}
    c = Client(s.url, "short")
    c.list(NODES)
    time.sleep(0.4)
    with pytest.raises(KubeError) as ei:
        c.list(NODES)
    assert ei.value.code == 401
