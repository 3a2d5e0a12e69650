"""60 s of agent Node heartbeats beside fake-kubelet status churn (the round-5 revert of
kubelet-owned Node status): the kubelet's allocatable and Ready heartbeat never go backwards, and
the agent's conditions keep their lastTransitionTime."""
from __future__ import annotations

import threading
import time

import pytest

from gpupool.kube import NODES, Client
from gpupool.testing.cluster import NodeSpec

pytestmark = pytest.mark.slow
NODE = "hb-node-0"


def test_heartbeats_never_revert_kubelet_status(cluster_factory):
    c = cluster_factory(nodes=[NodeSpec(NODE, extra_args=["--heartbeat-interval", "0.02"],
                                        kubelet_args=["--status-interval", "0.05"])],
                        manager=False)
    k = c.client
    k.wait_for(NODES, NODE, None, lambda n: (n or {}).get("status", {}).get("allocatable", {})
               .get("amd.com/gpu") is not None and any(x["type"] == "GPUPoolAgentReady" for x in
                                                  n["status"].get("conditions", [])), timeout=30)
    node0 = k.get(NODES, NODE)
    first = {x["type"]: x for x in node0["status"]["conditions"]}
    gpus0 = int(node0["status"]["allocatable"]["amd.com/gpu"])  # advertised (no pool: none)
    rv = k.get(NODES, NODE)["metadata"]["resourceVersion"]
    stop = threading.Event()
    seen: list[tuple[int, int, str]] = []
    bad: list = []

    def watch():
        w = Client(c.url)
        cur = rv
        while not stop.is_set():
            try:
                for ev in w.watch(NODES, resource_version=cur, stop=stop, timeout_seconds=20,
                                  field_selector=f"metadata.name={NODE}"):
                    if ev["type"] == "BOOKMARK":
                        cur = ev["object"]["metadata"]["resourceVersion"]
                        continue
                    if ev["type"] != "MODIFIED":
                        continue
                    o = ev["object"]
                    cur = o["metadata"]["resourceVersion"]
                    st = o["status"]
                    conds = {x["type"]: x for x in st.get("conditions", [])}
                    gpus = int(st["allocatable"].get("amd.com/gpu", "-1"))
                    churn = int(st["allocatable"].get("example.com/churn", "0"))
                    if "Ready" not in conds or gpus != gpus0:
                        bad.append(("kubelet status lost", st))
                    for t in ("GPUPoolAgentReady", "ROCmReady"):
                        if t in conds and conds[t]["lastTransitionTime"] != \
                                first[t]["lastTransitionTime"]:
                            bad.append(("lastTransitionTime moved", t, conds[t]))
                    seen.append((churn, gpus, conds.get("Ready", {}).get("lastHeartbeatTime", "")))
            except Exception:  # noqa: BLE001 — a dropped watch resumes from its last RV
                time.sleep(0.05)

    def churner():
        """A second status writer beside the kubelet (an extended-resource counter)."""
        cl = Client(c.url)
        i = 0
        while not stop.is_set():
            i += 1
            cl.patch(NODES, NODE, {"status": {"allocatable": {"example.com/churn": str(i)},
                                              "capacity": {"example.com/churn": str(i)}}},
                     sub="status", ptype="strategic")
            time.sleep(0.01)

    ts = [threading.Thread(target=watch, daemon=True), threading.Thread(target=churner,
                                                                         daemon=True)]
    for t in ts:
        t.start()
    time.sleep(60)
    stop.set()
    for t in ts:
        t.join(30)
    assert not bad, bad[:5]
    assert len(seen) > 1000, len(seen)
    assert all(a[0] <= b[0] and a[2] <= b[2] for a, b in zip(seen, seen[1:]))
    m = c.agent_request(NODE, "GET", "/metrics")
    beats = [ln for ln in m.splitlines() if ln.startswith("gpupool_agent_node_heartbeats ")]
    assert beats and float(beats[0].split()[1]) > 500, beats
