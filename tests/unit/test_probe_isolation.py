"""Probe isolation (gpupool/agent/probehost.py): the claim-time probe runs in per-GPU helper
processes with a deadline, so a GPU whose probe aborts its process or never returns cannot take the
node agent down or wedge its pool (the reference checks a GPU in a
throwaway pod, GPU调度平台搭建.md:134-138).

The helpers here run the simulated kernels (``helper-sim``): the same child processes, pipes,
deadlines and crash replacement as on MI355X, with the fault overlay's ``probeCrash`` (the helper
calls abort(), as HIP does on a GPU memory fault) and ``probeHang`` (the probe never returns)."""
from __future__ import annotations

import json
import os
import threading
import time

import pytest

from gpupool.agent.agent import Agent, AgentConfig
from gpupool.agent.ledger import Ledger

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FIXTURE = os.path.join(ROOT, "tests", "fixtures", "node_8x_mi355x.json")


def make_agent(tmp_path, faults: dict | None = None, count: int = 4) -> Agent:
    fp = str(tmp_path / "faults.json")
    json.dump(faults or {}, open(fp, "w"))
    cfg = AgentConfig(node="n0", backend="fake", fixture=FIXTURE, count=count,
                      state_dir=str(tmp_path / "state"), probe_mode="helper-sim", probe_sim_ms=2,
                      fsync=False, faults=fp, scrub_interval_s=0)
    return Agent(cfg)


def claim(agent, uid="pool-1", count=1, **probe):
    return agent.claim({"poolUID": uid, "pool": f"default/{uid}", "count": count,
                        "resourceName": "amd.com/gpu", "policy": {},
                        "topologyPolicy": "xgmi-packed", "probe": {"enabled": True, **probe}})


def wait(pred, timeout=10.0):
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        if pred():
            return True
        time.sleep(0.02)
    return pred()


@pytest.fixture
def agents():
    made = []
    yield made
    for a in made:
        a.stop()


def test_helpers_probe_and_the_agent_never_loads_the_probe_library(tmp_path, agents, native_built):
    a = make_agent(tmp_path)
    agents.append(a)
    # one helper per GPU, plus the fabric helper the agent starts and warms on a multi-GPU node
    assert wait(lambda: a.prober.helpers.alive("fabric") and a.prober.fabric_warm_ms is not None)
    pids = a.prober.helper_pids()
    assert len(pids) == 5 and os.getpid() not in pids
    assert a.prober.hip_devices() == 0  # helper-sim: no HIP anywhere
    starts = a.prober.helpers.stats["helper_starts"]
    r = claim(a, count=2)
    assert r["ok"] and all(d["probe"]["passed"] for d in r["devices"]), r
    assert all(d["probe"]["backend"] == "helper-sim" for d in r["devices"])
    # the claim's xGMI ring ran in the resident fabric helper: nothing was started for it
    assert a.prober.helpers.stats["helper_starts"] == starts
    # helpers' processes are the agent's own in per-pod accounting
    assert a._pod_of_pid(next(iter(pids))) == {"namespace": "", "pod": "gpupool-agent"}
    with open("/proc/self/maps") as f:
        assert "libmi355x_probe" not in f.read()


def test_probe_crash_fails_only_that_gpu_and_the_agent_survives(tmp_path, agents, native_built):
    """(a) the agent survives a mid-probe abort, (b) a claim on another GPU concurrently succeeds,
    (c) the aborted GPU's probe fails with ProbeCrashed and its release quarantines it."""
    a = make_agent(tmp_path, {"devices": {"0": {"probeCrash": True}}})
    agents.append(a)
    out = {}

    def other():  # a second pool claims concurrently; it gets a healthy GPU
        out["r2"] = claim(a, uid="pool-2", count=1)
    t = threading.Thread(target=other)
    r = claim(a, count=1)  # lowest index first: GPU 0
    t.start()
    t.join(10)
    d0 = r["devices"][0]
    assert d0["index"] == 0 and not d0["probe"]["passed"]
    assert d0["probe"]["error"].startswith("ProbeCrashed:"), d0["probe"]
    assert "SIGABRT" in d0["probe"]["error"]
    assert out["r2"]["ok"] and out["r2"]["devices"][0]["probe"]["passed"]
    # the agent is fine: views, metrics, and the crashed GPU's helper is replaced by a fresh one
    assert a.node_view()["devices"]
    assert wait(lambda: a.prober.helpers.alive(d0["uuid"]))
    assert a.prober.helpers.stats["helper_crashes"] == 1
    assert a.stats["probe_crashes"] == 1
    assert "gpupool_agent_probe_helper_crashes_total 1" in a.metrics_text()
    # the pool replaces it: drain -> release -> quarantined with the crash as the reason
    assert a.release("pool-1", [d0["uuid"]])["ok"]
    v = {d["uuid"]: d for d in a.node_view()["devices"]}[d0["uuid"]]
    assert v["state"] == "Quarantined" and "ProbeCrashed" in v["quarantine"]["reason"]


def test_hung_probe_answers_within_its_deadline(tmp_path, agents, native_built):
    """(e) a probe that never returns: the claim answers within timeoutSeconds + 1 s with
    ProbeTimeout; the hung helper is killed and replaced; the next GPU probes normally."""
    a = make_agent(tmp_path, {"devices": {"0": {"probeHang": True}}})
    agents.append(a)
    t0 = time.monotonic()
    r = claim(a, count=1, timeoutSeconds=1)
    dt = time.monotonic() - t0
    d0 = r["devices"][0]
    assert d0["index"] == 0 and dt < 1 + 1.0, dt
    assert d0["probe"]["error"].startswith("ProbeTimeout:"), d0["probe"]
    assert d0["state"] == "Claimed" and not d0["probe"]["passed"]
    assert a.stats["probe_timeouts"] == 1
    assert wait(lambda: a.prober.helpers.stats["helper_timeouts"] == 1)
    assert wait(lambda: a.prober.helpers.alive(d0["uuid"]))
    r2 = claim(a, uid="pool-2", count=1, timeoutSeconds=1)
    assert r2["devices"][0]["index"] == 1 and r2["devices"][0]["probe"]["passed"]


def _interrupted_state(tmp_path, attempts: dict) -> tuple[str, str, str]:
    """Claim GPUs 0-2, stop the agent, then rewrite the ledger as a process that died mid-claim
    leaves it: the records 'Probing', with the given probeAttempts (index -> n; absent: a record
    of an older agent, which counts as 1)."""
    a = make_agent(tmp_path)
    r = claim(a, count=3)
    uu = [d["uuid"] for d in sorted(r["devices"], key=lambda d: d["index"])]
    a.stop()
    led = Ledger(str(tmp_path / "state"), fsync=False)
    claims = led.load()
    for i, u in enumerate(uu):
        claims[u]["state"], claims[u]["probe"] = "Probing", None
        claims[u].pop("probeAttempts", None)
        if i in attempts:
            claims[u]["probeAttempts"] = attempts[i]
    led.commit(claims)
    return tuple(uu)


def test_restart_after_dying_mid_probe_never_crash_loops(tmp_path, agents, native_built):
    """(d) A restarted agent fails unprobed — ProbeInterrupted — a GPU whose probe already
    outlived one agent process (probeAttempts >= 2): a GPU that takes down whatever probes it
    cannot crash-loop the agent. A first interruption (the death was something else: the probe
    runs in a helper, which a GPU fault cannot take the agent down with) gets one re-probe, in the
    GPU's helper."""
    u0, u1, u2 = _interrupted_state(tmp_path, {0: 2, 1: 3, 2: 1})
    # had GPU 0 or 1 been probed again, its helper would abort: the result would say ProbeCrashed
    b = make_agent(tmp_path, {"devices": {"0": {"probeCrash": True}, "1": {"probeCrash": True}}})
    agents.append(b)
    for u in (u0, u1):
        p = b.records[u]["probe"]
        assert b.records[u]["state"] == "Claimed"
        assert not p["passed"] and p["error"].startswith("ProbeInterrupted:"), p
        assert "in a row" in p["error"]
    assert b.prober.helpers.stats["helper_crashes"] == 0  # neither was probed
    p2 = b.records[u2]["probe"]
    assert p2["passed"] and p2.get("rerunAtStart")  # first interruption: probed again, passes
    assert b.records[u2]["probeAttempts"] == 2


def test_the_reprobe_attempt_is_durable_before_the_reprobe_runs(tmp_path, agents, native_built,
                                                                 monkeypatch):
    """The restart's re-probe is counted on disk first: if the agent dies during it, the next
    restart finds probeAttempts 2 and fails the GPU unprobed. A record of an older agent (no
    counter) counts as a first attempt."""
    u0, _, _ = _interrupted_state(tmp_path, {})
    seen = {}
    from gpupool.agent.prober import Prober
    orig = Prober.probe_many

    def spy(self, devs, opts):
        on_disk = Ledger(str(tmp_path / "state"), fsync=False).load()
        seen.update({d["uuid"]: on_disk[d["uuid"]].get("probeAttempts") for d in devs})
        return orig(self, devs, opts)
    monkeypatch.setattr(Prober, "probe_many", spy)
    b = make_agent(tmp_path)
    agents.append(b)
    assert seen[u0] == 2 and b.records[u0]["probe"]["passed"]


def test_probing_record_past_its_deadline_is_reported_overdue(tmp_path, agents, native_built,
                                                              monkeypatch):
    """Defence in depth for a claim stuck outside the probe: a GPU still 'Probing' past
    timeoutSeconds + PROBE_GRACE_S is flagged probeOverdue in the node view, which the manager's
    plan_pool replaces (native/src/controller/reconciler.cc)."""
    a = make_agent(tmp_path)
    agents.append(a)
    monkeypatch.setattr(Agent, "PROBE_GRACE_S", 0.2)
    gate = threading.Event()
    orig = a.prober.probe_many
    monkeypatch.setattr(a.prober, "probe_many", lambda devs, opts: (gate.wait(10), orig(devs, opts))[1])
    t = threading.Thread(target=lambda: claim(a, count=1, timeoutSeconds=0.5))
    t.start()
    try:
        assert wait(lambda: any(d.get("state") == "Probing" for d in a.node_view()["devices"]), 5)
        view = lambda: [d for d in a.node_view()["devices"] if d.get("state") == "Probing"][0]  # noqa: E731
        assert not view().get("probeOverdue")
        assert wait(lambda: view().get("probeOverdue") is True, 3)
        assert view()["probingMs"] >= 700
    finally:
        gate.set()
        t.join(10)
    assert not any(d.get("probeOverdue") for d in a.node_view()["devices"])


def test_resident_fabric_helper_is_warm_before_ready_and_replaced_after_a_kill():
    """On a multi-GPU node the fabric helper starts with the GPU helpers, runs its warm ring
    before it reports ready, and — resident — is replaced (warm again) after it dies."""
    from gpupool.agent.probehost import HelperPool
    devs = [{"uuid": f"g{i}", "index": i} for i in range(3)]
    pool = HelperPool("sim", sim_ms=1, resident_fabric=True)
    try:
        pool.start(devs)
        assert wait(lambda: (pool.snapshot().get("fabric") or {}).get("warmMs") is not None)
        first = pool.snapshot()["fabric"]
        assert first["alive"] and first["warm"] == {"passed": True, "links": 6}, first  # 3 x 2 pairs
        pool.kill("fabric", "test kill")
        assert wait(lambda: (pool.snapshot().get("fabric") or {}).get("pid") not in (None, first["pid"])
                    and pool.alive("fabric"))
        assert pool.snapshot()["fabric"]["warmMs"] is not None
        assert pool.stats["helper_timeouts"] == 1  # kill() = a missed deadline
    finally:
        pool.stop()


def test_a_burst_of_parks_restarts_the_fabric_helper_once():
    """Parking several GPUs at once (a drain, a gang's pods starting) stops the resident fabric
    helper at once — it has a context on each of them — and starts it again once, over the GPUs
    still pod-free at the end of the burst; unparking them brings them back the same way."""
    from gpupool.agent.probehost import HelperPool
    devs = [{"uuid": f"g{i}", "index": i} for i in range(4)]
    pool = HelperPool("sim", sim_ms=1, resident_fabric=True)
    try:
        pool.start(devs)
        assert wait(lambda: pool.alive("fabric"))
        first = pool.snapshot()["fabric"]["pid"]
        starts = pool.stats["helper_starts"]
        for u in ("g0", "g1"):
            assert pool.park(u)
        assert not pool.alive("fabric")  # gone at once: it had a context on g0 and g1
        assert wait(lambda: pool.alive("fabric"))
        time.sleep(2 * pool.FABRIC_RESPAWN_DEBOUNCE_S)
        assert pool.snapshot()["fabric"]["pid"] != first
        assert pool.stats["helper_starts"] == starts + 1  # one start for the two parks
        assert pool.stats["fabric_respawns"] == 1
        assert wait(lambda: (pool.snapshot()["fabric"].get("warm") or {}).get("links") == 2)
        for u in ("g0", "g1"):
            pool.unpark(u)
        assert wait(lambda: pool.alive("fabric") and
                    (pool.snapshot()["fabric"].get("warm") or {}).get("links") == 12)
        time.sleep(2 * pool.FABRIC_RESPAWN_DEBOUNCE_S)
        assert pool.stats["fabric_respawns"] == 2
        assert wait(lambda: all(pool.alive(f"g{i}") for i in range(4)))
    finally:
        pool.stop()


def test_on_demand_fabric_helper_is_not_replaced():
    from gpupool.agent.probehost import HelperPool
    devs = [{"uuid": f"g{i}", "index": i} for i in range(2)]
    pool = HelperPool("sim", sim_ms=1, resident_fabric=False)
    try:
        pool.start(devs)
        assert "fabric" not in pool.snapshot()  # nothing until a ring asks
        h = pool.fabric(devs)
        assert h.wait_ready(10) and pool.alive("fabric")
        pool.kill("fabric", "test kill")
        assert wait(lambda: not pool.alive("fabric"))
        time.sleep(0.3)
        assert not pool.alive("fabric")
    finally:
        pool.stop()


def test_a_helper_whose_init_hangs_is_killed_at_its_ready_timeout():
    """A helper that never reports ready (a HIP init hung in the driver) is killed when its
    ready timeout passes, like a request past its deadline, and callers are not held past their
    own deadline meanwhile."""
    from gpupool.agent.probehost import Helper, HelperUnavailable
    exits = []
    h = Helper("g0", {"kind": "sim", "initHang": True}, on_exit=lambda h_, why, cause:
               exits.append((why, cause)), ready_timeout=1.5).start()
    t0 = time.monotonic()
    with pytest.raises(HelperUnavailable):
        h.call("ping", {}, timeout=0.3)
    assert time.monotonic() - t0 < 1.0
    assert wait(lambda: exits, timeout=10)
    why, cause = exits[0]
    assert cause == "timeout" and "not ready within 1.5 s" in why, exits
    assert h.dead and not h.ready_ok


def test_a_gpu_whose_helper_is_held_back_is_left_out_not_failed(tmp_path, agents, native_built):
    """A helper that exited twice in a row is replaced only after a backoff; meanwhile a claim
    leaves its GPU out (InsufficientDevices naming the helper when nothing else fits) instead of
    failing — and quarantining — a GPU whose probe could not run."""
    a = make_agent(tmp_path, count=2)
    agents.append(a)
    u0 = next(d["uuid"] for d in a.snap["devices"] if d["index"] == 0)
    pool = a.prober.helpers
    pid0 = pool.snapshot()[u0]["pid"]
    pool.kill(u0, "test kill 1")  # first exit: replaced at once
    assert wait(lambda: pool.snapshot().get(u0, {}).get("pid") not in (None, pid0)
                and pool.alive(u0))
    pool.kill(u0, "test kill 2")  # second within the window: 1 s backoff
    assert wait(lambda: not pool.available(u0), timeout=5)
    r = claim(a, count=2)
    assert not r["ok"] and r["reason"] == "InsufficientDevices", r
    assert "1 more wait for their probe helper" in r["message"], r
    r = claim(a, "pool-2", count=1)  # the other GPU is still claimable
    assert r["ok"] and [d["index"] for d in r["devices"]] == [1], r
    assert not a.ledger.quarantined()
    assert wait(lambda: pool.alive(u0), timeout=10)  # replaced after the backoff
    r = claim(a, "pool-3", count=1)
    assert r["ok"] and [d["index"] for d in r["devices"]] == [0], r


def test_an_idle_on_demand_fabric_helper_exits_and_is_not_counted_as_a_crash():
    """``--probe-fabric-idle S``: the fabric helper (contexts on every GPU) is let go after S idle
    seconds and started again by the next ring."""
    from gpupool.agent.probehost import HelperPool
    devs = [{"uuid": f"g{i}", "index": i} for i in range(2)]
    pool = HelperPool("sim", sim_ms=1, fabric_idle_s=0.5)
    try:
        pool.start(devs)
        h = pool.fabric(devs)
        assert h.wait_ready(10)
        pid = h.pid
        assert wait(lambda: not pool.alive("fabric"), timeout=10)
        assert pool.stats["helper_crashes"] == 0 and pool.stats["helper_timeouts"] == 0
        h2 = pool.fabric(devs)  # the next ring starts it again
        assert h2.wait_ready(10) and h2.pid != pid
    finally:
        pool.stop()


def test_a_claim_never_waits_for_a_warming_fabric_helper(monkeypatch):
    """The resident fabric helper warms (every pair's peer access) before it reports ready; a
    claim's ring arriving meanwhile reports the check unavailable at once instead of waiting —
    here the helper's init never finishes at all."""
    from gpupool.agent import probehost as ph
    from gpupool.agent.prober import Prober
    orig = ph.HelperPool._fabric_spec
    monkeypatch.setattr(ph.HelperPool, "_fabric_spec", lambda self: {**orig(self), "initHang": True})
    devs = [{"uuid": f"g{i}", "index": i, "hipUUID": f"GPU-{i}"} for i in range(2)]
    p = Prober("helper-sim", sim_ms=1, devices=devs)
    try:
        t0 = time.monotonic()
        links = p.peer_ring(devs, {"timeoutSeconds": 10})
        assert time.monotonic() - t0 < 1.0
        assert set(links) == {"g0", "g1"}
        for link in links.values():
            assert not link["passed"] and link["error"].startswith("ProbeUnavailable"), link
        from gpupool.agent.agent import Agent
        assert Agent._link_verdict(links["g0"], 0) == "unavailable"  # never a replace
    finally:
        p.helpers.stop()


def test_requests_sent_while_a_helper_starts_are_answered_promptly():
    """callers arriving while the watcher reads a starting helper's ready message (the
    pipe's reader role held) must not sleep out their deadline — the watcher hands the pipe on,
    and followers retry the reader role in short slices."""
    from gpupool.agent.probehost import Helper
    h = Helper("slow", {"kind": "sim", "single": True, "simMs": 1, "devices": 1,
                        "initDelayS": 0.4}).start()
    lat: list[float] = []
    errs: list[BaseException] = []

    def one():
        t0 = time.monotonic()
        try:
            h.call("ping", {}, 20.0)
            lat.append(time.monotonic() - t0)
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
    try:
        for _round in range(3):
            ts = [threading.Thread(target=one) for _ in range(6)]
            for t in ts:
                t.start()
            for t in ts:
                t.join(30)
        assert not errs, errs
        assert len(lat) == 18 and max(lat) < 2.0, lat
    finally:
        h.stop()


def test_parked_helper_holds_no_process_and_restarts_warm(tmp_path, agents, native_built):
    """Weak #5 (r5): a GPU with a tenant pod gets its probe helper stopped (parked) — requests
    for it are refused as unavailable, the fabric helper is restarted without it — and it comes
    back when the GPU is pod-free; release waits for it to be warm."""
    a = make_agent(tmp_path, count=3)
    agents.append(a)
    d0 = a.by_uuid[sorted(a.by_uuid, key=lambda u: a.by_uuid[u]["index"])[0]]
    pool = a.prober.helpers
    assert pool.alive(d0["uuid"])
    pid0 = next(v["pid"] for k, v in pool.snapshot().items() if k == d0["uuid"])
    a._sync_parking({d0["uuid"]: [{"namespace": "default", "name": "tenant"}]})
    assert d0["uuid"] in a.prober.parked() and not pool.alive(d0["uuid"])
    assert pid0 not in a.prober.helper_pids()
    assert not a.prober.can_probe(d0)
    fab = pool.snapshot().get("fabric") or {}
    assert wait(lambda: (pool.snapshot().get("fabric") or {}).get("alive"))
    assert {d["uuid"] for d in pool._fabric_devs} == set(a.by_uuid) - {d0["uuid"]}
    view = a.device_view(d0["uuid"], {})
    assert view["probeHelper"] == "Parked"
    r = a.prober.probe_many([d0], {"enabled": True})[0]
    assert not r["passed"] and r["error"].startswith("ProbeUnavailable")
    # pods gone: the helper restarts (a fresh pid) and rejoins the fabric helper's GPUs
    a._sync_parking({})
    assert d0["uuid"] not in a.prober.parked()
    assert pool.wait_ready(d0["uuid"], 30) < 30_000 and pool.alive(d0["uuid"])
    assert pid0 not in a.prober.helper_pids()
    assert wait(lambda: {d["uuid"] for d in pool._fabric_devs} == set(a.by_uuid))
    assert claim(a, "pool-x", 3)["ok"]
    assert fab is not None


def test_recheck_of_a_parked_or_unavailable_gpu_is_postponed_not_failed(tmp_path, agents,
                                                                         native_built):
    """a periodic recheck (or the one after a GPU reset) that cannot run — the helper
    is held back or parked — keeps the previous verdict instead of failing the GPU."""
    a = make_agent(tmp_path, count=2)
    agents.append(a)
    out = claim(a, "pool-r", 1, recheckSeconds=0.01)
    assert out["ok"]
    u = out["devices"][0]["uuid"]
    a._sync_parking({u: [{"namespace": "default", "name": "tenant"}]})
    dev = dict(a.by_uuid[u])
    opts = {"enabled": True}
    a._rechecking.add(u)
    a._recheck_one(u, dev, opts, out["devices"][0]["poolUID"] if "poolUID" in out["devices"][0]
                   else "pool-r", after_reset=True)
    rec = a.records[u]
    assert rec["probe"]["passed"], rec["probe"]
    assert a.stats.get("rechecks_postponed") == 1
    assert a.recheck_probes(force=True) == []  # pods / parked: nothing started
