"""Node agent + ROCm device plugin conformance against the fake kubelet, all in-process
(SURVEY.md §4.2 'Device plugin' row): Registration, ListAndWatch health transitions, Allocate
contents, GetPreferredAllocation, PodResources, kubelet restart -> re-registration, ledger
persistence, quarantine, all-or-nothing + topology-aware claims."""
from __future__ import annotations

import json
import os
import time

import grpc
import pytest

from gpupool.agent.agent import Agent, AgentConfig
from gpupool.agent.deviceplugin.proto import DP, PR, Stub, unix_target

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FIXTURE = os.path.join(ROOT, "tests", "fixtures", "node_8x_mi355x.json")


@pytest.fixture
def sockdir():
    import shutil
    import tempfile
    d = tempfile.mkdtemp(prefix="gpa", dir="/tmp")
    yield d
    shutil.rmtree(d, ignore_errors=True)


def make_agent(tmp_path, sockdir, plugin=True, faults=None, **kw):
    cfg = AgentConfig(node="n0", backend="fake", fixture=FIXTURE, state_dir=str(tmp_path / "state"),
                      plugin_dir=os.path.join(sockdir, "dp") if plugin else "",
                      pod_resources=os.path.join(sockdir, "pr", "kubelet.sock") if plugin else "",
                      probe_mode="simulated", probe_sim_ms=1, fsync=False,
                      faults=faults or "", **kw)
    return Agent(cfg)


def claim(agent, uid="pool-1", count=2, resource="amd.com/gpu", policy=None):
    return agent.claim({"poolUID": uid, "pool": "default/p", "count": count,
                        "resourceName": resource, "policy": policy or {},
                        "topologyPolicy": "xgmi-packed", "probe": {"enabled": True}})


def test_claim_all_or_nothing_and_topology(tmp_path, sockdir, native_built):
    a = make_agent(tmp_path, sockdir, plugin=False)
    r = claim(a, count=3)
    assert r["ok"] and sorted(d["index"] for d in r["devices"]) == [0, 1, 2]  # NUMA-0 packed
    r2 = claim(a, uid="pool-2", count=6)
    assert not r2["ok"] and r2["reason"] == "InsufficientDevices"
    assert sum(1 for d in a.node_view()["devices"] if d.get("poolUID")) == 3  # nothing partial
    r3 = claim(a, uid="pool-1", count=1)  # grows next to its NUMA-0 devices
    assert r3["devices"][0]["index"] == 3


def test_ledger_survives_restart_and_quarantine(tmp_path, sockdir, native_built):
    faults = str(tmp_path / "faults.json")
    json.dump({"devices": {"0": {"probeFail": True}}}, open(faults, "w"))
    a = make_agent(tmp_path, sockdir, plugin=False, faults=faults)
    r = claim(a, count=2)
    bad = [d for d in r["devices"] if not d["probe"]["passed"]]
    assert len(bad) == 1 and bad[0]["index"] == 0
    b = make_agent(tmp_path, sockdir, plugin=False, faults=faults)  # "restart": reload ledger
    assert {u for u, rec in b.records.items()} == {d["uuid"] for d in r["devices"]}
    out = b.release("pool-1", [bad[0]["uuid"]])
    assert out["ok"]
    view = {d["uuid"]: d for d in b.node_view()["devices"]}
    assert view[bad[0]["uuid"]]["state"] == "Quarantined"
    r2 = claim(b, uid="pool-2", count=6)  # 8 - 1 claimed - 1 quarantined = 6 free
    assert r2["ok"] and bad[0]["uuid"] not in {d["uuid"] for d in r2["devices"]}
    assert not claim(b, uid="pool-3", count=1)["ok"]


def test_release_refuses_gpu_with_pods(tmp_path, sockdir, native_built, monkeypatch):
    a = make_agent(tmp_path, sockdir, plugin=False)
    r = claim(a, count=1)
    u = r["devices"][0]["uuid"]
    monkeypatch.setattr(a, "_pods_by_device", lambda **_: {u: [{"namespace": "d", "name": "p"}]})
    out = a.release("pool-1", [u])
    assert not out["ok"] and out["reason"] == "PodsRunning"
    assert u in a.records


def test_health_sampling_follows_fault_overlay(tmp_path, sockdir, native_built):
    faults = str(tmp_path / "faults.json")
    a = make_agent(tmp_path, sockdir, plugin=False, faults=faults)
    r = claim(a, count=1)
    u = r["devices"][0]["uuid"]
    json.dump({"devices": {u: {"temps": {"hotspot": {"current": 101}}}}}, open(faults, "w"))
    changed = a.sample()
    assert "pool-1" in changed
    v = {d["uuid"]: d for d in a.node_view()["devices"]}[u]
    assert not v["healthy"] and not v["verdict"]["thermalOk"]
    gen, pools = a.changed_since(0)
    assert gen >= 1 and "pool-1" in pools
    os.remove(faults)
    a.sample()
    assert {d["uuid"]: d for d in a.node_view()["devices"]}[u]["healthy"]


class MiniKubelet:
    """Just the kubelet's Registration service + a ListAndWatch consumer."""

    def __init__(self, plugin_dir, wipe: bool = False):
        import concurrent.futures as cf
        from gpupool.agent.deviceplugin.proto import service_handler
        self.dir = plugin_dir
        self.registrations = []
        if wipe:  # a real kubelet's device manager removes every socket in the directory at start
            for name in os.listdir(plugin_dir) if os.path.isdir(plugin_dir) else []:
                if name.endswith(".sock"):
                    os.unlink(os.path.join(plugin_dir, name))
        self.server = grpc.server(cf.ThreadPoolExecutor(4))
        self.server.add_generic_rpc_handlers((service_handler("v1beta1.Registration",
                                                              {"Register": self.Register}),))
        os.makedirs(plugin_dir, exist_ok=True)
        self.server.add_insecure_port(unix_target(os.path.join(plugin_dir, "kubelet.sock")))
        self.server.start()

    def Register(self, req, ctx):
        self.registrations.append((req.version, req.endpoint, req.resource_name,
                                   req.options.get_preferred_allocation_available))
        return DP.Empty()

    def stop(self):
        # wait for the teardown: gRPC removes its unix socket file when the listener is destroyed,
        # which, done asynchronously, deleted a restarted kubelet's new socket (a test-only race)
        self.server.stop(0).wait(5)
        try:
            os.unlink(os.path.join(self.dir, "kubelet.sock"))
        except FileNotFoundError:
            pass


def test_device_plugin_conformance(tmp_path, sockdir, native_built):
    dp_dir = os.path.join(sockdir, "dp")
    kubelet = MiniKubelet(dp_dir)
    a = make_agent(tmp_path, sockdir)
    try:
        r = claim(a, count=2)
        deadline = time.time() + 5  # the plugin registers from its own thread
        while not kubelet.registrations and time.time() < deadline:
            time.sleep(0.02)
        assert kubelet.registrations == [("v1beta1", "gpupool-amd-com_gpu.sock", "amd.com/gpu", True)]
        ch = grpc.insecure_channel(unix_target(os.path.join(dp_dir, "gpupool-amd-com_gpu.sock")))
        stub = Stub(ch, "v1beta1.DevicePlugin")
        assert stub.GetDevicePluginOptions(DP.Empty()).get_preferred_allocation_available
        stream = stub.ListAndWatch(DP.Empty())
        first = next(stream)
        ids = {d.ID: d.health for d in first.devices}
        assert set(ids) == {d["uuid"] for d in r["devices"]} and set(ids.values()) == {"Healthy"}
        assert all(d.topology.nodes[0].ID == 0 for d in first.devices)
        # advertised bit set once the stream delivered them
        deadline = time.time() + 5
        while time.time() < deadline and not all(d["advertised"] for d in a.node_view()["devices"]
                                                   if d.get("poolUID")):
            time.sleep(0.02)
        assert all(d["advertised"] for d in a.node_view()["devices"] if d.get("poolUID"))
        # Allocate: ROCR_VISIBLE_DEVICES + /dev/kfd + render nodes
        u0 = r["devices"][0]["uuid"]
        resp = stub.Allocate(DP.AllocateRequest(container_requests=[{"devices_ids": [u0]}]))
        cr = resp.container_responses[0]
        assert cr.envs["ROCR_VISIBLE_DEVICES"] == r["devices"][0]["hipUUID"]
        assert cr.envs["GPUPOOL_NUM_GPUS"] == cr.envs["PET_NPROC_PER_NODE"] == "1"
        assert [d.host_path for d in cr.devices] == ["/dev/kfd", r["devices"][0]["renderNode"]]
        assert all(d.permissions == "rw" for d in cr.devices)
        # Allocate of a non-pool device is refused
        free = next(d["uuid"] for d in a.node_view()["devices"] if not d.get("poolUID"))
        with pytest.raises(grpc.RpcError) as e:
            stub.Allocate(DP.AllocateRequest(container_requests=[{"devices_ids": [free]}]))
        assert e.value.code() == grpc.StatusCode.FAILED_PRECONDITION
        # cordon -> the device turns Unhealthy on the stream
        a.cordon("pool-1", [u0])
        upd = next(stream)
        assert {d.ID: d.health for d in upd.devices}[u0] == "Unhealthy"
        pref = stub.GetPreferredAllocation(DP.PreferredAllocationRequest(container_requests=[
            {"available_deviceIDs": [d["uuid"] for d in r["devices"]], "allocation_size": 1}]))
        assert len(pref.container_responses[0].deviceIDs) == 1
        # kubelet restart -> plugin re-registers by itself
        kubelet.stop()
        kubelet = MiniKubelet(dp_dir)
        deadline = time.time() + 5
        while time.time() < deadline and not kubelet.registrations:
            time.sleep(0.05)
        assert kubelet.registrations and kubelet.registrations[0][2] == "amd.com/gpu"
        stream.cancel()
        ch.close()
    finally:
        a.stop()
        kubelet.stop()


def test_podresources_roundtrip(tmp_path, sockdir):
    """The fake kubelet's PodResources server and the agent's client agree on the wire format."""
    import concurrent.futures as cf

    from gpupool.agent.deviceplugin.proto import service_handler
    from gpupool.agent.podresources import list_pod_devices
    sock = os.path.join(sockdir, "pr.sock")

    def List(req, ctx):
        resp = PR.ListPodResourcesResponse()
        pr = resp.pod_resources.add(name="p", namespace="ns")
        c = pr.containers.add(name="c")
        c.devices.add(resource_name="amd.com/gpu", device_ids=["u1", "u2"])
        return resp
    s = grpc.server(cf.ThreadPoolExecutor(2))
    s.add_generic_rpc_handlers((service_handler("v1.PodResourcesLister", {"List": List}),))
    s.add_insecure_port(unix_target(sock))
    s.start()
    try:
        out = list_pod_devices(sock)
        assert set(out) == {"u1", "u2"} and out["u1"][0]["name"] == "p"
    finally:
        s.stop(0)


def test_probe_performance_floors():
    from gpupool.agent.prober import Prober
    ok = {"passed": True, "hbm": {"GBps": 4900.0}, "mfma": {"tflops": 1200.0, "enabled": True}}
    import copy
    r = Prober.apply_floors(copy.deepcopy(ok), {}, {"minHbmGBps": 4000, "minMfmaTflops": 1000})
    assert r["passed"]
    r = Prober.apply_floors(copy.deepcopy(ok), {"probeScale": 0.5}, {"minMfmaTflops": 1000})
    assert not r["passed"] and r["error"].startswith("PerformanceBelowFloor: MFMA 600")
    r = Prober.apply_floors(copy.deepcopy(ok), {"faults": {"probeScale": 0.7}},
                            {"minHbmGBps": 4000})
    assert not r["passed"] and "HBM 3430 GB/s < floor 4000" in r["error"]
    # floors off (0) and MFMA disabled: never fail on perf
    r = Prober.apply_floors({"passed": True, "hbm": {"GBps": 1.0}, "mfma": {"enabled": False}},
                            {}, {"minHbmGBps": 0, "minMfmaTflops": 500})
    assert r["passed"]
    # a failed probe keeps its own error
    bad = {"passed": False, "error": "HBM mismatch", "hbm": {"GBps": 1.0}}
    assert Prober.apply_floors(bad, {}, {"minHbmGBps": 4000})["error"] == "HBM mismatch"


def test_claiming_pool_events_held_until_released(tmp_path, sockdir, native_built):
    """A claim RPC holds its pool's change events (the reply carries that state) and emits one
    bump when the handler releases them; other pools' events pass through meanwhile."""
    a = make_agent(tmp_path, sockdir, plugin=False)
    g0, _ = a.changed_since(-1)
    r = a.claim({"poolUID": "held", "pool": "default/p", "count": 1, "resourceName": "amd.com/gpu",
                 "policy": {}, "probe": {"enabled": True}}, hold_events=True)
    assert r["ok"]
    a._bump({"held", "other"})  # e.g. a health flip during the claim: "other" goes out now
    g1, pools = a.changed_since(g0)
    assert "other" in pools and "held" not in pools
    a.release_events("held")
    g2, pools = a.changed_since(g1)
    assert g2 == g1 + 1 and pools == ["held"]
    a.release_events("held")  # idempotent: nothing more
    assert a.changed_since(g2)[0] == g2
    # without the hold (direct callers) the claim releases its own hold when it returns
    assert claim(a, uid="plain", count=1)["ok"]
    assert not a._claiming and not a._deferred


def test_new_listandwatch_stream_restores_advertised(tmp_path, sockdir, native_built):
    """A kubelet restart drops its ListAndWatch stream (the advertised bits clear: nothing is
    known to be advertised) and opens a new one: the new stream's first message — the same device
    list version — must mark the GPUs advertised again, without waiting for a device change."""
    dp_dir = os.path.join(sockdir, "dp")
    kubelet = MiniKubelet(dp_dir)
    a = make_agent(tmp_path, sockdir)
    try:
        r = claim(a, count=2)
        mine = {d["uuid"] for d in r["devices"]}

        def advertised() -> set:
            return {d["uuid"] for d in a.node_view()["devices"] if d.get("advertised")}

        def wait(pred, timeout=5.0):
            deadline = time.time() + timeout
            while time.time() < deadline and not pred():
                time.sleep(0.02)
            return pred()
        sock = os.path.join(dp_dir, "gpupool-amd-com_gpu.sock")
        assert wait(lambda: os.path.exists(sock))
        ch = grpc.insecure_channel(unix_target(sock))
        stream = Stub(ch, "v1beta1.DevicePlugin").ListAndWatch(DP.Empty())
        next(stream)
        assert wait(lambda: advertised() == mine)
        stream.cancel()
        ch.close()
        assert wait(lambda: advertised() == set())  # no stream: nothing counts as advertised
        ch2 = grpc.insecure_channel(unix_target(sock))
        stream2 = Stub(ch2, "v1beta1.DevicePlugin").ListAndWatch(DP.Empty())
        first = next(stream2)
        assert {d.ID for d in first.devices if d.health == "Healthy"} == mine
        assert wait(lambda: advertised() == mine), advertised()
        stream2.cancel()
        ch2.close()
    finally:
        a.stop()
        kubelet.stop()


def test_kubelet_restart_that_wipes_the_plugin_dir(tmp_path, sockdir, native_built):
    """A starting kubelet removes every socket in the device-plugin directory, the plugin's own
    endpoint included, and dials that endpoint when the plugin registers. So the plugin must notice
    its socket is gone, serve again on a fresh one and re-register — after which the new kubelet
    can open ListAndWatch on it."""
    dp_dir = os.path.join(sockdir, "dp")
    kubelet = MiniKubelet(dp_dir)
    a = make_agent(tmp_path, sockdir)
    sock = os.path.join(dp_dir, "gpupool-amd-com_gpu.sock")
    try:
        r = claim(a, count=1)
        deadline = time.time() + 5
        while not kubelet.registrations and time.time() < deadline:
            time.sleep(0.02)
        assert kubelet.registrations
        kubelet.stop()
        kubelet = MiniKubelet(dp_dir, wipe=True)
        assert not os.path.exists(sock)
        deadline = time.time() + 5
        while time.time() < deadline and not (kubelet.registrations and os.path.exists(sock)):
            time.sleep(0.05)
        assert kubelet.registrations and os.path.exists(sock), (kubelet.registrations, os.listdir(dp_dir))
        ch = grpc.insecure_channel(unix_target(sock))
        first = next(Stub(ch, "v1beta1.DevicePlugin").ListAndWatch(DP.Empty()))
        assert {d.ID for d in first.devices} == {r["devices"][0]["uuid"]}
        ch.close()
    finally:
        a.stop()
        kubelet.stop()


def test_plugin_reregisters_promptly_after_a_kubelet_outage(tmp_path, sockdir, native_built):
    """While the kubelet is away, gRPC backs off reconnecting to its socket (1 s, growing). The
    plugin's Register after the kubelet returns must not inherit that backoff from the channel it
    keeps to watch the kubelet: it dials a fresh connection, so the new kubelet hears from the
    plugin within the monitor's poll period, not a backoff later."""
    dp_dir = os.path.join(sockdir, "dp")
    kubelet = MiniKubelet(dp_dir)
    a = make_agent(tmp_path, sockdir)
    try:
        claim(a, count=1)
        deadline = time.time() + 5
        while not kubelet.registrations and time.time() < deadline:
            time.sleep(0.02)
        assert kubelet.registrations
        kubelet.stop()
        time.sleep(1.5)  # long enough for a reconnect backoff to reach 1 s
        kubelet = MiniKubelet(dp_dir)
        t0 = time.monotonic()
        while not kubelet.registrations and time.monotonic() - t0 < 10:
            time.sleep(0.01)
        took = time.monotonic() - t0
        assert kubelet.registrations and took < 0.8, took
    finally:
        a.stop()
        kubelet.stop()


def test_allocate_mounts_the_hbm_limit_read_only(tmp_path, sockdir, native_built):
    """An isolated slot's Allocate: the pod-wide account (counters) read-write, the limit the
    agent fixed read-only beside it — and a one-sample over-budget reading never evicts."""
    a = make_agent(tmp_path, sockdir, plugin=False)
    r = claim(a, count=1, policy={"sharing": {"replicasPerGPU": 2, "hbmBytesPerSlot": 8 << 30,
                                              "overBudgetAction": "Evict"}})
    u = r["devices"][0]["uuid"]
    spec = a.allocate_spec("amd.com/gpu", [f"{u}::0"])
    m = {x["container_path"]: x for x in spec["mounts"]}
    assert m[a.SHARE_ACCOUNT_PATH]["read_only"] is False
    assert m[a.SHARE_LIMIT_PATH]["read_only"] is True
    assert open(m[a.SHARE_LIMIT_PATH]["host_path"]).read() == f"GPLIMIT1 {8 << 30}\n"
    assert spec["envs"]["GPUPOOL_SHARE_LIMIT"] == a.SHARE_LIMIT_PATH
    # budget checks: one over-budget sample flags, the second evicts (no API server: counted only)
    a._pods_cache = (0.0, {u: [{"namespace": "d", "name": "rogue"}]})
    usage = {u: [{"namespace": "d", "pod": "rogue", "vramBytes": 20 << 30}]}
    assert a._check_slot_budgets(usage) and not a.stats.get("over_budget_evictions")
    a._check_slot_budgets({u: [dict(usage[u][0])]})
    assert a.stats["over_budget_evictions"] == 1
    a._check_slot_budgets({u: [dict(usage[u][0])]})  # once per pod
    assert a.stats["over_budget_evictions"] == 1


def test_account_for_gpus_without_hip_uuid_is_version_1(tmp_path, sockdir, native_built):
    """a GPU without a hipUUID cannot be matched by identity — a version-2 account
    would match nothing and the pod-wide budget would silently become per-process. The agent
    writes a version-1 (ordinal) account instead."""
    from gpupool.agent.slots import read_account
    a = make_agent(tmp_path, sockdir, plugin=False)
    r = claim(a, count=1, policy={"sharing": {"replicasPerGPU": 2, "hbmBytesPerSlot": 8 << 30}})
    u = r["devices"][0]["uuid"]
    a.by_uuid[u] = {**a.by_uuid[u], "hipUUID": ""}
    path = a._share_account([f"{u}::0"], 8 << 30, [u])
    acct = read_account(path)
    assert acct["version"] == 1 and acct["limit"] == 8 << 30 and acct["slots"] == [f"{u}::0"]
    assert acct["created"] > 0  # the GC grace still applies


def test_cu_masks_are_per_gpu_for_a_pod_spanning_slots_of_two_gpus(tmp_path, sockdir, native_built):
    """a pod holding slot 0 of GPU A and slot 1 of GPU B gets slot 0's CUs on A and slot
    1's on B (GPUPOOL_CU_MASKS by HIP UUID), not their union on both."""
    a = make_agent(tmp_path, sockdir, plugin=False)
    r = claim(a, count=2, policy={"sharing": {"replicasPerGPU": 2, "cuPerSlot": 128}})
    ua, ub = (d["uuid"] for d in sorted(r["devices"], key=lambda d: d["index"]))
    env = a.allocate_spec("amd.com/gpu", [f"{ua}::0", f"{ub}::1"])["envs"]
    ha, hb = a.by_uuid[ua]["hipUUID"], a.by_uuid[ub]["hipUUID"]
    masks = dict(x.split("=") for x in env["GPUPOOL_CU_MASKS"].split(";"))
    assert masks == {ha: "0-127", hb: "128-255"}, masks
    assert env["GPUPOOL_CU_MASK"] == "0-255"  # the union: fallback for a GPU the library cannot name
    assert env["GPUPOOL_CU_XCDS"] == "8"
