"""xGMI link coverage (the reference's "ownership and health must be exact", README.md:238-240, on
an 8x MI355X node where every GPU pair has its own xGMI link).

* every link a claim measures counts: an owned GPU's bad link into a newly claimed GPU fails the
  new GPU (it is replaced), not just the new GPUs' outgoing links;
* ring order rotates over the least recently checked pairs, so claims + idle rechecks cover all
  28 pairs of the node; per-pair results are persisted in the ledger and surfaced as
  status.devices[].xgmi.pairsCovered;
* a check that cannot run (no peer access, HIP error) is XGMILinksHealthy=Unknown
  (XGMIPeerCheckUnavailable), never a replace loop.
"""
from __future__ import annotations

import json
import os

import pytest

from gpupool.kube import MI355XPOOLS
from gpupool.testing.cluster import FIXTURE, NodeSpec

from .helpers import conds, mi_pool, ready_at, wait_ready

pytestmark = pytest.mark.slow
RING = {"xgmiPeerCheck": True}


def _agent(tmp_path, faults: dict | None = None):
    from gpupool.agent.agent import Agent, AgentConfig
    fp = tmp_path / "faults.json"
    fp.write_text(json.dumps(faults or {}))
    return Agent(AgentConfig(node="n0", backend="fake", fixture=FIXTURE,
                             state_dir=str(tmp_path / "s"), probe_mode="simulated",
                             probe_sim_ms=1, fsync=False, faults=str(fp), scrub_interval_s=0,
                             xgmi_recheck_s=0))


def _claim(a, pool: str, count: int):
    return a.claim({"poolUID": pool, "pool": f"default/{pool}", "count": count,
                    "resourceName": "amd.com/gpu", "policy": {}, "topologyPolicy": "xgmi-packed",
                    "probe": {"enabled": True, **RING}})


def _pair(a, i: int, j: int) -> dict | None:
    return next((v for k, v in a.xgmi_pairs.items()
                 if {a.by_uuid[u]["index"] for u in k.split("|")} == {i, j}), None)


def test_bad_link_from_an_owned_gpu_into_a_new_gpu_fails_the_new_gpu(tmp_path, native_built):
    """Incremental scale-up 4 -> 5 where every owned GPU's link *into* GPU 4 corrupts data while
    GPU 4's own outgoing links are fine: the ring over {0..3} + {4} necessarily carries one owned
    -> 4 link, and GPU 4 (the receiving new GPU) fails its probe. Before, only a new GPU's
    outgoing link counted, so this GPU passed."""
    a = _agent(tmp_path, {"devices": {str(i): {"xgmiBadPeers": [4]} for i in range(4)}})
    try:
        r = _claim(a, "p", 4)
        assert r["ok"] and sorted(d["index"] for d in r["devices"]) == [0, 1, 2, 3]
        assert all(d["probe"]["passed"] for d in r["devices"])
        r = _claim(a, "p", 1)
        assert [d["index"] for d in r["devices"]] == [4]
        probe = r["devices"][0]["probe"]
        assert not probe["passed"] and "XGMIPeerCheckFailed" in probe["error"], probe
        bad = [v for v in a.xgmi_pairs.values() if v["verdict"] == "bad"]
        assert len(bad) == 1 and a.by_uuid[bad[0]["dst"]]["index"] == 4
    finally:
        a.stop()


def test_scale_4_to_8_then_idle_rechecks_find_a_bad_link_between_owned_gpus(tmp_path, native_built):
    """4 -> 8 with the physical link 3 <-> 4 bad (both directions). If the claim ring measured
    that pair, GPU 4 (new) failed; whether or not it did, the rotating idle rechecks over the
    idle pool cover the pair within a few rings and fail a GPU on it."""
    a = _agent(tmp_path, {"devices": {"3": {"xgmiBadPeers": [4]}, "4": {"xgmiBadPeers": [3]}}})
    try:
        _claim(a, "p", 4)
        r = _claim(a, "p", 4)
        failed = {d["index"] for d in r["devices"] if not d["probe"]["passed"]}
        pair = _pair(a, 3, 4)
        if pair is not None:
            assert pair["verdict"] == "bad" and failed == {4}
        else:
            assert not failed
            for _ in range(4):
                a.xgmi_recheck(force=True)
            assert _pair(a, 3, 4)["verdict"] == "bad"
            view = {d["index"]: d for d in a.node_view()["devices"]}
            bad = {i for i in (3, 4) if not view[i]["probe"]["passed"]}
            assert len(bad) == 1 and "XGMIPeerCheckFailed" in view[bad.pop()]["probe"]["error"]
        assert len(a.xgmi_pairs) >= 12  # two claim rings: 4 + 8 links, no pair measured twice
    finally:
        a.stop()


def test_rotating_rings_cover_all_28_pairs_and_persist(tmp_path, native_built):
    a = _agent(tmp_path)
    try:
        for k in range(1, 5):
            out = a.xgmi_recheck(force=True)
            assert out["checked"] == 8 and not out["bad"]
        view = a.node_view()
        covered = {d["index"]: d["xgmiPairs"]["pairsCovered"] for d in view["devices"]}
        assert covered == {i: 7 for i in range(8)}, covered
        assert len(a.xgmi_pairs) == 28
    finally:
        a.stop()
    a.ledger.flush()
    doc = json.load(open(os.path.join(tmp_path, "s", "ledger.json")))
    assert len(doc["xgmiPairs"]) == 28
    b = _agent(tmp_path)  # a restarted agent keeps the coverage
    try:
        assert len(b.xgmi_pairs) == 28
    finally:
        b.stop()


def test_idle_recheck_quarantines_a_free_gpu_with_a_bad_link(tmp_path, native_built):
    a = _agent(tmp_path, {"devices": {"6": {"xgmiPeerFail": True}}})
    try:
        out = a.xgmi_recheck(force=True)
        assert len(out["bad"]) == 1 and "XGMIPeerCheckFailed" in out["bad"][0]
        state = {d["index"]: d["state"] for d in a.node_view()["devices"]}
        assert state[6] == "Quarantined" and sum(s == "Free" for s in state.values()) == 7
    finally:
        a.stop()


def test_unavailable_peer_check_is_unknown_not_a_replace(cluster_factory):
    c = cluster_factory(nodes=[NodeSpec("mi355x-node-0", extra_args=["--probe-sim-ms", "1"])])
    k = c.client
    c.set_faults("mi355x-node-0", {"devices": {"0": {"xgmiPeerUnavailable": True}}})
    k.create(MI355XPOOLS, mi_pool("ring", 2, probe=RING), "default")

    def unknown(o):
        x = conds(o).get("XGMILinksHealthy", {})
        return ready_at(2)(o) and x.get("status") == "Unknown" and \
            x.get("reason") == "XGMIPeerCheckUnavailable"
    o = k.wait_for(MI355XPOOLS, "ring", "default", unknown, timeout=30)
    assert sorted(d["index"] for d in o["status"]["devices"]) == [0, 1]  # nothing replaced
    d0 = next(d for d in o["status"]["devices"] if d["index"] == 0)
    assert d0["xgmi"]["peerCheckUnavailable"] is True and d0["xgmi"]["pairsTotal"] == 7
    assert conds(o)["Degraded"]["status"] == "False"


def test_pool_scale_4_to_5_replaces_the_gpu_behind_a_bad_incoming_link(cluster_factory):
    c = cluster_factory(nodes=[NodeSpec("mi355x-node-0", extra_args=["--probe-sim-ms", "1"])])
    k = c.client
    k.create(MI355XPOOLS, mi_pool("p", 4, probe=RING), "default")
    o = wait_ready(k, "p", 4, timeout=30)
    assert sorted(d["index"] for d in o["status"]["devices"]) == [0, 1, 2, 3]
    c.set_faults("mi355x-node-0", {"devices": {str(i): {"xgmiBadPeers": [4]} for i in range(4)}})
    k.patch(MI355XPOOLS, "p", {"spec": {"replicas": 5}}, "default")
    o = wait_ready(k, "p", 5, timeout=30)  # GPU 4 failed, was drained, and a spare replaced it
    assert 4 not in {d["index"] for d in o["status"]["devices"]}
    view = c.agent_request("mi355x-node-0", "GET", "/v1/node")
    g4 = next(d for d in view["devices"] if d["index"] == 4)
    assert g4["state"] == "Quarantined"
    assert all(d["xgmi"]["pairsCovered"] >= 2 for d in o["status"]["devices"])
    assert conds(o)["XGMILinksHealthy"]["status"] == "True"
