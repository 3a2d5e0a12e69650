"""HBM scrubber on the fake 8x MI355X node: idle GPUs are swept window by window over their whole
HBM, coverage persists in the ledger and surfaces in pool status, a bad window quarantines the GPU
(never claimed), and a claim always wins over an in-flight scrub."""
from __future__ import annotations

import json
import os
import time

import pytest

from gpupool.kube import MI355XPOOLS
from gpupool.testing.cluster import NodeSpec

from .helpers import cond_is, mi_pool, settled_events, wait_ready

pytestmark = pytest.mark.slow

SCRUB = ["--scrub-interval", "0.2", "--scrub-start-delay", "0", "--scrub-window", str(32 << 30),
         "--scrub-windows", "4", "--probe-sim-ms", "1"]


def view(cl, node="mi355x-node-0"):
    return cl.agent_request(node, "GET", "/v1/node")


def wait(pred, timeout=20.0):
    deadline = time.monotonic() + timeout
    while True:
        v = pred()
        if v:
            return v
        assert time.monotonic() < deadline, "timed out"
        time.sleep(0.05)


def test_idle_gpus_are_swept_and_coverage_reaches_status(cluster_factory):
    cl = cluster_factory(nodes=[NodeSpec("mi355x-node-0", extra_args=SCRUB)])
    # every free GPU completes at least one full sweep of its ~305 GB (9-10 windows of 32 GiB)
    wait(lambda: all((d.get("hbmSweep") or {}).get("passes", 0) >= 1 for d in view(cl)["devices"]))
    d0 = view(cl)["devices"][0]["hbmSweep"]
    assert d0["span"] > 300e9 and d0["windows"] >= 9
    # persisted with the ledger (survives an agent restart)
    with open(os.path.join(cl.workdir, "state-mi355x-node-0", "ledger.json")) as f:
        doc = json.load(f)
    assert len(doc["hbmSweep"]) == 8
    k = cl.client
    k.create(MI355XPOOLS, mi_pool("p", 2), "default")
    o = wait_ready(k, "p", 2)
    for dev in o["status"]["devices"]:
        assert dev["hbmCoverage"]["passes"] >= 1, dev
        assert dev["probe"]["cusVerified"] == dev["probe"]["cusExpected"] == 256, dev


def test_bad_hbm_window_quarantines_free_gpu(cluster_factory):
    cl = cluster_factory(nodes=[NodeSpec("mi355x-node-0", extra_args=SCRUB)])
    victim = view(cl)["devices"][5]["uuid"]
    cl.set_faults("mi355x-node-0", {"devices": {victim: {"hbmBadOffset": 200 << 30}}})
    d = wait(lambda: next((x for x in view(cl)["devices"]
                           if x["uuid"] == victim and x["state"] == "Quarantined"), None))
    assert "HBMSweepFailed" in d["quarantine"]["reason"]
    k = cl.client
    # the agent tells the cluster: a Warning Event on the Node
    ev = wait(lambda: next((e for e in settled_events(k)
                            if e.get("reason") == "HBMSweepFailed"), None))
    assert ev["involvedObject"] == {"kind": "Node", "name": "mi355x-node-0", "apiVersion": "v1"}
    assert ev["type"] == "Warning" and victim in ev["message"]
    k.create(MI355XPOOLS, mi_pool("all", 8), "default")
    o = k.wait_for(MI355XPOOLS, "all", "default",
                   cond_is("Progressing", "False", "InsufficientDevices"), timeout=20)
    assert o["status"]["readyReplicas"] == 0  # all-or-nothing: the quarantined GPU is never claimed
    k.patch(MI355XPOOLS, "all", {"spec": {"replicas": 7}}, "default")
    o = wait_ready(k, "all", 7)
    assert victim not in {x["uuid"] for x in o["status"]["devices"]}


def test_synchronous_scrub_rpc_and_claim_wins(cluster_factory):
    cl = cluster_factory(nodes=[NodeSpec("mi355x-node-0", extra_args=[
        "--scrub-interval", "0", "--scrub-window", str(64 << 30), "--probe-sim-ms", "1"])])
    r = cl.agent_request("mi355x-node-0", "POST", "/v1/scrub", {"gpu": "0", "windows": 2})
    assert r["ok"] and r["coverage"]["windows"] == 2 and r["coverage"]["cursor"] == 128 << 30
    r = cl.agent_request("mi355x-node-0", "POST", "/v1/scrub", {"gpu": "0", "windows": 3})
    assert r["coverage"]["passes"] == 1 and r["coverage"]["fraction"] == 1.0
    # a claimed GPU is not scrubbed (its workload owns the memory)
    k = cl.client
    k.create(MI355XPOOLS, mi_pool("p", 8), "default")
    o = wait_ready(k, "p", 8)
    u = o["status"]["devices"][3]["uuid"]
    r = cl.agent_request("mi355x-node-0", "POST", "/v1/scrub", {"gpu": u, "windows": 3})
    assert r["record"]["windows"] == 0 and r["coverage"] is None
