"""Retirement-aware HBM health, event-driven detection and MI355X partitions (CPU, fake backend).

* HBM page retirement (amdsmi_get_gpu_bad_page_info) gates claims: a GPU with more retired pages
  than ``spec.health.maxRetiredPages``, or any page pending retirement, is never claimed, and a
  claimed GPU whose pages go pending turns HBMECCHealthy=False.
* The fault overlay is an event source (inotify): a rewrite is applied without waiting for the
  periodic sample; ``notify: false`` leaves it to the sample (the path of a real ECC counter).
* CPX/NPS2 node (8 ASICs x 8 logical GPUs): a pool of 8 is packed on one ASIC; an ECC fault seen
  through one partition degrades all 8 partitions and the pool moves to a healthy ASIC
  (the HAMi/MIG-style sharing layer of /root/reference/GPU调度平台搭建.md:289-298).
"""
from __future__ import annotations

import json
import os
import shutil
import tempfile
import time

import pytest

from gpupool.agent.agent import Agent, AgentConfig
from gpupool.kube import MI355XPOOLS
from gpupool.ops import devlib
from gpupool.testing.cluster import NodeSpec

from .helpers import cond_is, conds, mi_pool, wait_ready

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FIXTURE = os.path.join(ROOT, "tests", "fixtures", "node_8x_mi355x.json")
CPX = os.path.join(ROOT, "tests", "fixtures", "node_8x_mi355x_cpx.json")


@pytest.fixture
def workdir():
    d = tempfile.mkdtemp(prefix="gph", dir="/tmp")
    yield d
    shutil.rmtree(d, ignore_errors=True)


def make_agent(d, fixture=FIXTURE, faults=None, **kw) -> Agent:
    cfg = AgentConfig(node="n0", backend="fake", fixture=fixture, state_dir=os.path.join(d, "state"),
                      probe_mode="simulated", probe_sim_ms=1, fsync=False, faults=faults or "",
                      scrub_interval_s=0, **kw)
    return Agent(cfg)


def claim(agent, uid="pool-1", count=1, policy=None):
    return agent.claim({"poolUID": uid, "pool": "default/p", "count": count,
                        "resourceName": "amd.com/gpu", "policy": policy or {},
                        "topologyPolicy": "xgmi-packed", "probe": {"enabled": True}})


def write_faults(path, faults):
    with open(path + ".tmp", "w") as f:
        json.dump(faults, f)
    os.replace(path + ".tmp", path)


def test_evaluate_retired_pending_and_lifetime_rules(native_built):
    dev = json.load(open(FIXTURE))["devices"][0]
    ok = devlib.evaluate(dev, dev, {})
    assert ok["healthy"] and ok["eccOk"]
    bad = {**dev, "ras": {**dev["ras"], "retiredPages": 65}}
    v = devlib.evaluate(bad, bad, {})
    assert not v["healthy"] and not v["eccOk"]
    assert any(r.startswith("HBMRetiredPages: 65") for r in v["reasons"]), v
    assert devlib.evaluate(bad, bad, {"health": {"maxRetiredPages": 100}})["healthy"]
    pend = {**dev, "ras": {**dev["ras"], "pendingPages": 1}}
    assert any(r.startswith("HBMPendingRetirement") for r in devlib.evaluate(pend, pend, {})["reasons"])
    unres = {**dev, "ras": {**dev["ras"], "unreservablePages": 2}}
    assert not devlib.evaluate(unres, unres, {"health": {"maxRetiredPages": 1000}})["healthy"]
    # a backend that cannot read bad pages does not make the GPU unhealthy
    nosup = {**dev, "ras": {"badPagesSupported": False}}
    assert devlib.evaluate(nosup, nosup, {})["healthy"]
    # historic uncorrectable errors: only with an explicit lifetime limit (the delta is 0 here)
    hist = {**dev, "ecc": {**dev["ecc"], "uncorrectable": 3}}
    assert devlib.evaluate(hist, hist, {})["healthy"]
    v = devlib.evaluate(hist, hist, {"health": {"maxLifetimeUncorrectableECC": 0}})
    assert not v["healthy"] and any("HBMUncorrectableECCHistory" in r for r in v["reasons"])
    # the health poll's UMC-only count is its own delta (never mixed with the all-blocks total)
    base = {**dev, "eccUmc": {"correctable": 0, "uncorrectable": 0, "deferred": 0}}
    now = {**base, "eccUmc": {"correctable": 0, "uncorrectable": 1, "deferred": 0}}
    v = devlib.evaluate(now, base, {})
    assert not v["eccOk"] and any("in HBM (UMC)" in r for r in v["reasons"]), v
    assert devlib.evaluate(now, now, {})["healthy"]


def test_retired_pages_make_a_gpu_unclaimable(workdir, native_built):
    faults = os.path.join(workdir, "faults.json")
    write_faults(faults, {"devices": {"0": {"ras": {"retiredPages": 200}}}})
    a = make_agent(workdir, faults=faults)
    try:
        r = claim(a, count=8)
        assert not r["ok"] and r["reason"] == "InsufficientDevices"
        r = claim(a, count=7)
        assert r["ok"] and 0 not in {d["index"] for d in r["devices"]}
        v = a.node_view()
        d0 = next(d for d in v["devices"] if d["index"] == 0)
        assert d0["state"] == "Free" and not d0["healthy"]
        assert any("HBMRetiredPages" in x for x in d0["verdict"]["reasons"])
        # a pool that tolerates more retired pages may take it
        assert claim(a, uid="pool-2", count=1, policy={"health": {"maxRetiredPages": 500}})["ok"]
    finally:
        a.stop()


def test_fault_overlay_event_applies_without_a_sample(workdir, native_built):
    faults = os.path.join(workdir, "faults.json")
    write_faults(faults, {})
    a = make_agent(workdir, faults=faults, sample_interval=3600, health_interval=0)
    a.start_background()
    try:
        assert claim(a, count=1)["ok"]
        u = next(iter(a.records))
        time.sleep(0.2)  # the watcher is armed
        samples0 = a.stats["samples"]
        t0 = time.monotonic()
        write_faults(faults, {"devices": {u: {"ecc": {"uncorrectable": 1}}}})
        while a.verdicts[u]["healthy"] and time.monotonic() - t0 < 5:
            time.sleep(0.005)
        dt = time.monotonic() - t0
        assert not a.verdicts[u]["healthy"] and dt < 1.0, dt
        assert a.stats["fault_events"] >= 1 and a.stats["samples"] > samples0
        assert a.node_view()["eventSources"].get("faultOverlay") is True
        assert any(e["type"] == "FaultOverlayChanged" for e in a.node_view()["recentEvents"])
        # notify=false: not an event; only the periodic sample (an hour away here) would see it
        write_faults(faults, {"devices": {u: {"ecc": {"uncorrectable": 0}}}, "notify": False})
        time.sleep(0.5)
        assert not a.verdicts[u]["healthy"]
        a.sample()
        assert a.verdicts[u]["healthy"]
        # the fake backend has no hardware event source: the watcher reports it and exits
        assert a.node_view()["eventSources"].get("device") is False
    finally:
        a.stop()


def test_health_poll_detects_a_silent_counter_change(workdir, native_built):
    """No event, no full sample (an hour away): the 50 ms health-only poll sees the ECC counter
    move, re-evaluates only what changed, and degrades the GPU."""
    faults = os.path.join(workdir, "faults.json")
    write_faults(faults, {})
    a = make_agent(workdir, faults=faults, sample_interval=3600, health_interval=0.05)
    a.start_background()
    try:
        assert claim(a, count=1)["ok"]
        u = next(iter(a.records))
        time.sleep(0.2)
        polls0, samples0 = a.stats["health_polls"], a.stats["samples"]
        t0 = time.monotonic()
        write_faults(faults, {"devices": {u: {"ecc": {"uncorrectable": 2}}}, "notify": False})
        while a.verdicts[u]["healthy"] and time.monotonic() - t0 < 5:
            time.sleep(0.005)
        assert not a.verdicts[u]["healthy"] and time.monotonic() - t0 < 1.0
        assert a.stats["health_polls"] > polls0 and a.stats["samples"] == samples0
        assert a.stats["fault_events"] == 0
    finally:
        a.stop()


def test_device_events_unsupported_on_fake_backend(native_built):
    d = devlib.DeviceLib("fake", fixture=FIXTURE, node="n0")
    t0 = time.monotonic()
    r = d.wait_events(2000)
    assert r == {"supported": False, "events": []} and time.monotonic() - t0 < 0.5
    assert d.wait_faults(10) == {"supported": False, "changed": False}


def test_cpx_partitions_packed_per_asic_and_faults_fan_out(workdir, native_built):
    a = make_agent(workdir, fixture=CPX)
    try:
        snap = a.node_view()
        assert len(snap["devices"]) == 64
        assert all(d["partition"]["compute"] == "CPX" for d in snap["devices"])
        r = claim(a, count=8)
        assert r["ok"]
        serials = {a.by_uuid[d["uuid"]]["asic"]["serial"] for d in r["devices"]}
        assert len(serials) == 1  # all 8 partitions of one ASIC (weight 5 < xGMI 15)
        # a second pool of 4 lands on a different ASIC, also packed
        r2 = claim(a, uid="pool-2", count=4)
        s2 = {a.by_uuid[d["uuid"]]["asic"]["serial"] for d in r2["devices"]}
        assert len(s2) == 1 and not s2 & serials
        # ECC fault seen through ONE partition of pool-2's ASIC: every partition of that ASIC
        # (4 claimed + 4 free) turns unhealthy; pool-1's ASIC is untouched
        victim = r2["devices"][0]["uuid"]
        a.by_uuid[victim] = {**a.by_uuid[victim], "ecc": {"correctable": 0, "uncorrectable": 1,
                                                          "deferred": 0}}
        with a.lock:
            a._evaluate_all()
        asic = a.by_uuid[victim]["asic"]["serial"]
        sib = [u for u, d in a.by_uuid.items() if d["asic"]["serial"] == asic]
        assert len(sib) == 8 and all(not a.verdicts[u]["healthy"] for u in sib)
        assert all(any(x.startswith("ASICFault: sibling partition") for x in a.verdicts[u]["reasons"])
                   for u in sib if u != victim)
        assert all(a.verdicts[d["uuid"]]["healthy"] for d in r["devices"])
        # the 4 free partitions of the faulted ASIC are not claimable
        r3 = claim(a, uid="pool-3", count=8)
        s3 = {a.by_uuid[d["uuid"]]["asic"]["serial"] for d in r3["devices"]}
        assert r3["ok"] and asic not in s3
    finally:
        a.stop()


@pytest.mark.slow
def test_cpx_pool_moves_off_an_asic_with_an_ecc_fault(cluster_factory):
    """A CPX-mode pool of 8 packs one ASIC; an uncorrectable ECC error through one partition
    degrades all 8 and the pool replaces them with the 8 partitions of a healthy ASIC."""
    c = cluster_factory(nodes=[NodeSpec("mi355x-node-0", fixture=CPX)])
    k = c.client
    k.create(MI355XPOOLS, mi_pool("cpx", 8, partition={"compute": "CPX"}), "default")
    o = wait_ready(k, "cpx", 8, timeout=60)
    view = {d["uuid"]: d for d in c.agent_request("mi355x-node-0", "GET", "/v1/node")["devices"]}
    first = {d["uuid"] for d in o["status"]["devices"]}
    assert len({view[u]["bdf"][:-1] for u in first}) == 1  # one ASIC (PCI functions .0-.7)
    victim = sorted(first)[3]
    c.set_faults("mi355x-node-0", {"devices": {victim: {"ecc": {"uncorrectable": 1}}}})

    def moved(o):
        u = {d["uuid"] for d in (o or {}).get("status", {}).get("devices", [])}
        return len(u) == 8 and not (u & first) and \
            (o or {}).get("status", {}).get("readyReplicas") == 8
    o = k.wait_for(MI355XPOOLS, "cpx", "default", moved, timeout=60)
    assert conds(o)["Ready"]["status"] == "True"
    view = {d["uuid"]: d for d in c.agent_request("mi355x-node-0", "GET", "/v1/node")["devices"]}
    assert all(view[u]["state"] == "Quarantined" for u in first)
    assert len({view[d["uuid"]]["bdf"][:-1] for d in o["status"]["devices"]}) == 1
    # the SPX requirement is refused on a CPX node (partition mode is observed, never changed)
    k.create(MI355XPOOLS, mi_pool("spx", 1, partition={"compute": "SPX"}), "default")
    k.wait_for(MI355XPOOLS, "spx", "default", cond_is("Ready", "False"), timeout=30)


@pytest.mark.slow
def test_utilisation_metrics_agent_and_pool(cluster_factory):
    """GPU utilisation export (GPU调度平台搭建.md:800): per-GPU gauges on the agent (with the pool
    label) and pool-level aggregates on the manager, from the fake backend's telemetry."""
    c = cluster_factory(nodes=[NodeSpec("mi355x-node-0")])
    k = c.client
    k.create(MI355XPOOLS, mi_pool("util", 2), "default")
    wait_ready(k, "util", 2)
    view = c.agent_request("mi355x-node-0", "GET", "/v1/node")
    tel = [d["telemetry"] for d in view["devices"] if d.get("pool") == "default/util"]
    assert len(tel) == 2 and all(t["memTotalBytes"] == 309220868096 for t in tel)
    text = c.agent_request("mi355x-node-0", "GET", "/metrics")  # text/plain on the RPC socket
    for name in ("gpupool_device_gfx_activity_percent", "gpupool_device_umc_activity_percent",
                 "gpupool_device_power_watts", "gpupool_device_vram_used_bytes",
                 "gpupool_device_vram_total_bytes", "gpupool_device_hbm_bad_pages"):
        assert name + "{" in text, name
    assert 'pool="default/util"' in text
    want = 2 * 309220868096

    def pool_gauge(metrics: str, name: str) -> float | None:
        for line in metrics.splitlines():
            if line.startswith(name + "{") and 'pool="default/util"' in line:
                return float(line.rsplit(" ", 1)[1])
        return None
    deadline = time.monotonic() + 20
    while time.monotonic() < deadline:
        m = c.manager_metrics()
        if pool_gauge(m, "gpupool_pool_vram_total_bytes") == want:
            break
        time.sleep(0.1)
    assert pool_gauge(m, "gpupool_pool_vram_total_bytes") == want
    assert pool_gauge(m, "gpupool_pool_power_watts") == 2 * 262
    assert pool_gauge(m, "gpupool_pool_gfx_activity_percent") == 0
    # gpuctl devices: partition, utilisation, VRAM, power and the event sources per GPU
    import subprocess
    r = subprocess.run([os.path.join(ROOT, "bin", "gpuctl"), "--server", c.url, "devices",
                        "mi355x-node-0"], capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, GPUPOOL_AGENT_TOKEN=c.agent_token))
    assert r.returncode == 0, r.stderr
    assert "events faultOverlay" in r.stdout and "GFX%" in r.stdout
    assert "0/288" in r.stdout and "262W" in r.stdout and "default/util" in r.stdout
    r = subprocess.run([os.path.join(ROOT, "bin", "gpuctl"), "--server", c.url, "top"],
                       capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, GPUPOOL_AGENT_TOKEN=c.agent_token))
    assert r.returncode == 0, r.stderr
    row = next(ln for ln in r.stdout.splitlines() if ln.startswith("default/util"))
    assert row.split()[1:] == ["2", "0", "0", "524", "1/576"], row
    dash = json.load(open(os.path.join(ROOT, "config", "prometheus", "grafana-dashboard.json")))
    exprs = " ".join(t["expr"] for p in dash["panels"] for t in p.get("targets", []))
    for name in ("gpupool_pool_gfx_activity_percent", "gpupool_device_vram_used_bytes",
                 "gpupool_ready_replicas", "gpupool_pod_vram_bytes", "gpupool_pod_gfx_busy_ratio",
                 "gpupool_namespace_quota_units", "gpupool_device_xgmi_pairs_covered",
                 "process_resident_memory_bytes", "process_threads"):
        assert name in exprs
