"""Time-sliced GPU sharing (spec.sharing.replicasPerGPU): the HAMi / time-slicing analogue of the
reference platform's GPU-sharing layer (GPU调度平台搭建.md:289-298). Each GPU of the pool is
advertised as K device IDs, so K pods share it; drain and release still act per GPU."""
from __future__ import annotations

import pytest

from gpupool.agent.agent import gpu_of
from gpupool.kube import MI355XPOOLS, NODES, PODS, KubeError

from .helpers import mi_pool, pause_pod, wait_ready

pytestmark = pytest.mark.slow


def running(o):
    return bool(o) and o["status"].get("phase") == "Running"


def test_shared_gpus_hold_k_pods_each_and_drain_per_gpu(cluster_factory):
    c = cluster_factory()
    k = c.client
    k.create(MI355XPOOLS, mi_pool("shared", 2, sharing={"replicasPerGPU": 4},
                                  drain={"gracePeriodSeconds": 1}), "default")
    o = wait_ready(k, "shared", 2)
    assert o["status"]["allocatable"] == 8 and o["status"]["readyReplicas"] == 2
    gpus = {d["uuid"]: d["index"] for d in o["status"]["devices"]}
    k.wait_for(NODES, "mi355x-node-0", None, lambda n: (n["status"].get("allocatable") or {})
               .get("amd.com/gpu") == "8", timeout=20)
    for i in range(8):
        k.create(PODS, pause_pod(f"s{i}"), "default")
    for i in range(8):
        k.wait_for(PODS, f"s{i}", "default", running, timeout=30)
    # a ninth pod does not fit: 2 GPUs x 4 slots
    k.create(PODS, pause_pod("s8"), "default")
    p9 = k.wait_for(PODS, "s8", "default",
                    lambda p: p and p["status"].get("phase") in ("Pending", "Failed"), timeout=10)
    assert p9["status"].get("phase") != "Running"
    k.delete(PODS, "s8", "default", grace=0)
    by_gpu: dict[str, list[str]] = {}
    for i in range(8):
        slot = k.get(PODS, f"s{i}", "default")["metadata"]["annotations"]["gpupool.amd.com/devices"]
        by_gpu.setdefault(gpu_of(slot), []).append(f"s{i}")
    assert sorted(len(v) for v in by_gpu.values()) == [4, 4] and set(by_gpu) == set(gpus)
    # the agent sees every slot's pod on its GPU (its PodResources map refreshes asynchronously)
    import time
    deadline = time.monotonic() + 10
    while True:
        view = {d["uuid"]: d for d in c.agent_request("mi355x-node-0", "GET", "/v1/node")["devices"]}
        if all(len(view[u]["pods"]) == 4 for u in gpus) or time.monotonic() > deadline:
            break
        time.sleep(0.05)
    assert all(len(view[u]["pods"]) == 4 for u in gpus)

    # scale 2 -> 1: the victim (highest index) GPU's four pods are evicted, the other four stay
    victim = max(gpus, key=gpus.get)
    k.patch(MI355XPOOLS, "shared", {"spec": {"replicas": 1}}, "default")
    o = wait_ready(k, "shared", 1, timeout=60)
    assert [d["uuid"] for d in o["status"]["devices"]] == [u for u in gpus if u != victim]
    assert o["status"]["allocatable"] == 4
    left = {p["metadata"]["name"] for p in k.list(PODS, "default")["items"]
            if not p["metadata"].get("deletionTimestamp")}
    assert left == set(by_gpu[min(gpus, key=gpus.get)])
    k.wait_for(NODES, "mi355x-node-0", None, lambda n: (n["status"].get("allocatable") or {})
               .get("amd.com/gpu") == "4", timeout=20)


def test_sharing_slots_in_allocate(tmp_path, native_built):
    """Allocate of slots maps back to the GPUs: one ROCR_VISIBLE_DEVICES entry per GPU however
    many of its slots a pod got; preferred allocation packs a pod's slots onto one GPU."""
    from gpupool.agent.agent import Agent, AgentConfig
    from gpupool.testing.cluster import FIXTURE
    a = Agent(AgentConfig(node="n0", backend="fake", fixture=FIXTURE, state_dir=str(tmp_path / "s"),
                          probe_mode="simulated", probe_sim_ms=1, fsync=False, scrub_interval_s=0))
    try:
        r = a.claim({"poolUID": "p", "pool": "default/p", "count": 2, "resourceName": "amd.com/gpu",
                     "policy": {"sharing": {"replicasPerGPU": 3}}, "probe": {"enabled": True}})
        assert r["ok"]
        devs = a.plugin_devices("amd.com/gpu")
        assert len(devs) == 6 and all("::" in d["id"] for d in devs)
        u0, u1 = sorted({d["uuid"] for d in devs}, key=lambda u: a.by_uuid[u]["index"])
        spec = a.allocate_spec("amd.com/gpu", [f"{u0}::0", f"{u0}::2"])
        assert spec["envs"]["GPUPOOL_DEVICE_UUIDS"] == u0 and spec["envs"]["GPUPOOL_NUM_GPUS"] == "1"
        assert spec["envs"]["ROCR_VISIBLE_DEVICES"].count(",") == 0
        assert spec["envs"]["GPUPOOL_GPU_SLOTS"] == f"{u0}::0,{u0}::2"
        avail = [d["id"] for d in devs]
        assert a.preferred("amd.com/gpu", list(reversed(avail)), [], 2) == [f"{u0}::0", f"{u0}::1"]
        # one ID per GPU without sharing
        a.update_policy("p", {}, "amd.com/gpu")
        assert [d["id"] for d in a.plugin_devices("amd.com/gpu")] == [u0, u1]
    finally:
        a.stop()


def test_autoscaled_shared_pool_counts_slots(cluster_factory):
    """Autoscaling a shared pool: demand is in devices of the resource (slots), so 6 pending pods
    on a pool of 4 slots per GPU need ceil(6/4) = 2 GPUs, not 6."""
    k = cluster_factory().client
    res = "amd.com/gpu-shared"
    k.create(MI355XPOOLS, mi_pool("sa", 0, resourceName=res, sharing={"replicasPerGPU": 4},
                                  autoscale={"enabled": True, "minReplicas": 0, "maxReplicas": 8,
                                             "scaleDownDelaySeconds": 60}), "default")
    wait_ready(k, "sa", 0)
    for i in range(6):
        k.create(PODS, pause_pod(f"a{i}", resource=res), "default")
    o = wait_ready(k, "sa", 2)
    assert o["status"]["allocatable"] == 8
    for i in range(6):
        k.wait_for(PODS, f"a{i}", "default", running, timeout=30)
    assert k.get(MI355XPOOLS, "sa", "default")["spec"]["replicas"] == 2


def test_sharing_cpx_partitions(cluster_factory):
    """Sharing composes with CPX: each logical GPU (partition) of a pool is advertised as K
    slots, so one MI355X in CPX mode with K=2 serves 16 pods."""
    from gpupool.testing.cluster import ROOT, NodeSpec
    import os
    cpx = os.path.join(ROOT, "tests", "fixtures", "node_8x_mi355x_cpx.json")
    c = cluster_factory(nodes=[NodeSpec("cpx-node", fixture=cpx)])
    k = c.client
    k.create(MI355XPOOLS, mi_pool("cs", 8, partition={"compute": "CPX"},
                                  sharing={"replicasPerGPU": 2}), "default")
    o = wait_ready(k, "cs", 8, timeout=60)
    assert o["status"]["allocatable"] == 16
    k.wait_for(NODES, "cpx-node", None, lambda n: (n["status"].get("allocatable") or {})
               .get("amd.com/gpu") == "16", timeout=20)


def test_isolated_slots_get_the_share_library_disjoint_cus_and_a_budget(cluster_factory):
    """spec.sharing.hbmBytesPerSlot / cuPerSlot (the HAMi layer): Allocate hands each pod the
    ROCm tools library (HSA_TOOLS_LIB, mounted from the agent's build dir), its slot's HBM budget
    and a CU range disjoint from the other slots of the same GPU."""
    import os
    import time
    c = cluster_factory()
    k = c.client
    k.create(MI355XPOOLS, mi_pool("iso", 1, sharing={"replicasPerGPU": 4, "hbmBytesPerSlot": 8 << 30,
                                                     "cuPerSlot": 64}), "default")
    wait_ready(k, "iso", 1)
    cmd = ["bash", "-c", "env | grep -E '^(HSA_TOOLS_LIB|GPUPOOL_CU_MASK|GPUPOOL_CU_LAYOUT|GPUPOOL_HBM_LIMIT_BYTES|"
                         "GPUPOOL_SHARE_ACCOUNT|GPUPOOL_GPU_SLOTS)=' | sort; sleep 600"]

    def start(name: str) -> dict:
        pod = pause_pod(name)
        pod["spec"]["containers"][0]["command"] = cmd
        k.create(PODS, pod, "default")

    def env_of(name: str) -> dict:
        p = k.wait_for(PODS, name, "default", running, timeout=30)
        path = p["metadata"]["annotations"]["gpupool.amd.com/log-path"]
        deadline = time.monotonic() + 10
        while time.monotonic() < deadline and open(path).read().count("\n") < 6:
            time.sleep(0.05)
        return dict(line.split("=", 1) for line in open(path).read().split())

    for i in range(4):
        start(f"iso{i}")
    envs = [env_of(f"iso{i}") for i in range(4)]
    # contiguous, disjoint 64-bit masks: 8 CUs on each of the 8 XCDs per slot (a mask leaving an
    # XCD empty is not applied by the hardware at all: gpupool/agent/slots.py)
    masks = sorted(e["GPUPOOL_CU_MASK"] for e in envs)
    assert masks == ["0-63", "128-191", "192-255", "64-127"], masks
    assert all(e["GPUPOOL_CU_LAYOUT"] == "striped" for e in envs)
    assert all(e["GPUPOOL_HBM_LIMIT_BYTES"] == str(8 << 30) for e in envs)
    lib = envs[0]["HSA_TOOLS_LIB"]  # the container path, rewritten to the host path
    assert lib.endswith("/libgpupool_share.so") and os.path.exists(lib)
    # mounted from the agent's copy under its state dir (the DaemonSet's hostPath), not from the
    # agent's own tree (a path that exists only inside the agent image) — the fake kubelet runs
    # with strict mounts and would have failed the pod otherwise
    assert lib.startswith(c.state_dir("mi355x-node-0") + "/lib/"), lib
    # status shows the layout per slot
    gpu = k.get(MI355XPOOLS, "iso", "default")["status"]["devices"][0]
    sh = gpu["sharing"]
    assert sh["cuLayout"] == "striped" and sh["slotXcds"] == ["0-7"] * 4, sh
    assert sh["slotCUMasks"] == ["0-63", "64-127", "128-191", "192-255"], sh
    # one HBM account per container (shared by all its processes): the library's layout — magic,
    # the per-GPU limit, version 2 with the GPU's HIP UUID, zeroed counters, and the container's
    # slot ids for the agent's cleanup
    from gpupool.agent.slots import read_account
    accts = [e["GPUPOOL_SHARE_ACCOUNT"] for e in envs]
    assert len(set(accts)) == 4
    for e, a in zip(envs, accts):
        raw = open(a, "rb").read()
        assert len(raw) == 16384 and raw[:8] == b"GPSHARE1", raw[:16]
        assert int.from_bytes(raw[8:16], "little") == 8 << 30
        assert not any(raw[64:8192])
        assert raw[8192:8224].split(b"\0")[0].decode() == gpu["hipUUID"]
        assert read_account(a)["slots"] == e["GPUPOOL_GPU_SLOTS"].split(",")
    # the slot of a finished pod goes to a new pod: the old account is replaced, not reused
    k.delete(PODS, "iso0", "default")
    k.wait_for(PODS, "iso0", "default", lambda o: o is None, timeout=30)
    start("iso4")
    e4 = env_of("iso4")
    assert e4["GPUPOOL_GPU_SLOTS"] == envs[0]["GPUPOOL_GPU_SLOTS"]
    assert e4["GPUPOOL_SHARE_ACCOUNT"] != accts[0] and not os.path.exists(accts[0])
    assert all(os.path.exists(a) for a in accts[1:] + [e4["GPUPOOL_SHARE_ACCOUNT"]])
    # a pool whose slots overrun the GPU's CUs is refused at admission by the CRD's CEL rule
    # (the manager checks the same, InvalidSpec, for objects written before the rule existed)
    with pytest.raises(KubeError) as ei:
        k.create(MI355XPOOLS, mi_pool("over", 1, sharing={"replicasPerGPU": 4, "cuPerSlot": 128}),
                 "default")
    assert ei.value.code == 422 and "256 CUs" in str(ei.value)
    # fewer CUs per slot than the GPU has XCDs would leave XCDs empty: the hardware would ignore
    # the mask, so such a pool is refused — on SPX (or Any) below 8, on CPX (1 XCD) any size goes
    with pytest.raises(KubeError) as ei:
        k.create(MI355XPOOLS, mi_pool("thin", 1, sharing={"replicasPerGPU": 4, "cuPerSlot": 4}),
                 "default")
    assert ei.value.code == 422 and "one CU per XCD" in str(ei.value)


def test_per_pod_accounting_on_a_time_shared_gpu(cluster_factory):
    """Per-pod GPU accounting (GPU调度平台搭建.md:800-802): the GPU's process list (amdsmi; here
    injected through the fault overlay for the fake backend) is attributed to the pods of a
    time-shared GPU — distinct VRAM per pod on the same uuid, and each pod's share of the GPU's
    time from the gfx-engine counter between two samples."""
    import re
    import time
    c = cluster_factory()
    k = c.client
    k.create(MI355XPOOLS, mi_pool("acct", 1, sharing={"replicasPerGPU": 2}), "default")
    o = wait_ready(k, "acct", 1)
    gpu = o["status"]["devices"][0]
    pids = {}
    for name in ("small", "big"):
        k.create(PODS, pause_pod(name), "default")
        p = k.wait_for(PODS, name, "default", lambda p: running(p) and "gpupool.amd.com/pid" in
                       p["metadata"].get("annotations", {}), timeout=30)
        pids[name] = int(p["metadata"]["annotations"]["gpupool.amd.com/pid"])

    def procs(gfx_small):
        return {"devices": {str(gpu["index"]): {"processes": [
            {"pid": pids["small"], "vramBytes": 2 << 30, "gfxNs": gfx_small},
            {"pid": pids["big"], "vramBytes": 6 << 30, "gfxNs": 0}]}}}
    c.set_faults("mi355x-node-0", procs(0), sample=True)
    t0 = time.monotonic()
    time.sleep(0.5)
    c.set_faults("mi355x-node-0", procs(250_000_000), sample=True)  # 0.25 s of gfx time
    dt = time.monotonic() - t0
    view = c.agent_request("mi355x-node-0", "GET", "/v1/node")
    use = {e["pod"]: e for e in next(d for d in view["devices"] if d["uuid"] == gpu["uuid"])["usage"]}
    assert use["small"]["vramBytes"] == 2 << 30 and use["big"]["vramBytes"] == 6 << 30
    assert use["small"]["namespace"] == "default" and use["small"]["pids"] == [pids["small"]]
    assert 0.25 / (dt + 0.3) < use["small"]["gfxBusy"] < 0.25 / max(dt - 0.3, 0.05)
    assert use["big"]["gfxBusy"] == 0
    metrics = c.agent_request("mi355x-node-0", "GET", "/metrics")
    got = dict(re.findall(r'gpupool_pod_vram_bytes\{[^}]*pod="(\w+)"\} (\d+)', str(metrics)))
    assert got == {"small": str(2 << 30), "big": str(6 << 30)}
    assert 'gpupool_pod_gfx_busy_ratio{' in str(metrics)
    # the same accounting from the CLI: gpuctl top pods
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    r = subprocess.run([os.path.join(root, "bin", "gpuctl"), "--server", c.url, "top", "pods"],
                       capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, GPUPOOL_AGENT_TOKEN=c.agent_token))
    assert r.returncode == 0, r.stderr
    rows = {ln.split()[0]: ln.split() for ln in r.stdout.splitlines()[1:]}
    assert rows["default/small"][4] == "2.00" and rows["default/big"][4] == "6.00", r.stdout
    assert rows["default/big"][5] == "0" and rows["default/small"][6] == str(pids["small"])


def test_overcommitted_slot_budgets_are_refused(cluster_factory):
    """replicasPerGPU x hbmBytesPerSlot must fit the GPU's HBM minus the agent's own reserve
    (--hbm-reserve, default 2 GiB: HIP context + probe arena): 4 x 100 GiB on a 288 GiB MI355X is
    refused with SharingOvercommitted on Ready/Progressing and no GPU is claimed; 4 x 64 GiB fits."""
    c = cluster_factory()
    k = c.client
    k.create(MI355XPOOLS, mi_pool("big", 1, sharing={"replicasPerGPU": 4,
                                                     "hbmBytesPerSlot": 100 << 30}), "default")
    o = k.wait_for(MI355XPOOLS, "big", "default", lambda o: any(
        x["reason"] == "SharingOvercommitted" for x in (o.get("status") or {}).get("conditions", [])),
        timeout=30)
    conds = {x["type"]: x for x in o["status"]["conditions"]}
    assert conds["Ready"]["status"] == "False" and conds["Ready"]["reason"] == "SharingOvercommitted"
    msg = conds["Progressing"]["message"]
    assert "hbmBytesPerSlot" in msg and "reserve" in msg, msg
    assert not o["status"].get("devices") and o["status"].get("readyReplicas", 0) == 0
    k.create(MI355XPOOLS, mi_pool("fits", 1, sharing={"replicasPerGPU": 4,
                                                      "hbmBytesPerSlot": 64 << 30}), "default")
    o = wait_ready(k, "fits", 1)
    assert o["status"]["devices"][0]["sharing"]["hbmBytesPerSlot"] == 64 << 30


def test_hbm_account_of_an_exited_pod_is_removed(cluster_factory):
    """The agent deletes an isolated slot's HBM account once the kubelet's PodResources lists none
    of its slots: within one sample period of the pod's exit (after the creation grace)."""
    import os
    import time
    from gpupool.testing.cluster import NodeSpec
    c = cluster_factory(nodes=[NodeSpec("mi355x-node-0", extra_args=["--share-acct-grace", "0.2"])])
    k = c.client
    k.create(MI355XPOOLS, mi_pool("gc", 1, sharing={"replicasPerGPU": 2,
                                                    "hbmBytesPerSlot": 8 << 30}), "default")
    wait_ready(k, "gc", 1)
    share = os.path.join(c.state_dir("mi355x-node-0"), "share")
    k.create(PODS, pause_pod("keep"), "default")
    k.create(PODS, pause_pod("go"), "default")
    for n in ("keep", "go"):
        k.wait_for(PODS, n, "default", running, timeout=30)
    assert len([f for f in os.listdir(share) if f.endswith(".acct")]) == 2
    time.sleep(1.5)  # past the grace and several sample periods: both pods are listed, both kept
    assert len([f for f in os.listdir(share) if f.endswith(".acct")]) == 2
    k.delete(PODS, "go", "default", grace=0)
    k.wait_for(PODS, "go", "default", lambda o: o is None, timeout=30)
    t0 = time.monotonic()
    while len([f for f in os.listdir(share) if f.endswith(".acct")]) > 1:
        assert time.monotonic() - t0 < 3 * c.sample_interval + 1.0, os.listdir(share)
        time.sleep(0.05)
    print(f"account removed {time.monotonic() - t0:.2f} s after the pod was gone "
          f"(sample period {c.sample_interval} s)")


def test_pod_over_its_slot_budget_is_reported(cluster_factory):
    """Defence in depth for the in-pod HBM limit: the agent compares each pod's VRAM on a shared
    GPU (amdsmi process list; here injected through the fault overlay) with its slots x
    hbmBytesPerSlot. A pod holding far more — its limit is not in force, e.g. the share library
    did not load in its image — is flagged in the usage view and metrics and gets one Node event;
    a pod within budget (+ ROCr's uncharged internals) is not."""
    import time
    from gpupool.kube import EVENTS
    c = cluster_factory()
    k = c.client
    k.create(MI355XPOOLS, mi_pool("bud", 1, sharing={"replicasPerGPU": 2,
                                                     "hbmBytesPerSlot": 8 << 30}), "default")
    gpu = wait_ready(k, "bud", 1)["status"]["devices"][0]
    pids = {}
    for name in ("ok", "rogue"):
        k.create(PODS, pause_pod(name), "default")
        p = k.wait_for(PODS, name, "default", lambda p: running(p) and "gpupool.amd.com/pid" in
                       p["metadata"].get("annotations", {}), timeout=30)
        pids[name] = int(p["metadata"]["annotations"]["gpupool.amd.com/pid"])
    deadline = time.monotonic() + 10  # the agent's PodResources view shows both slots' pods
    while time.monotonic() < deadline:
        view = c.agent_request("mi355x-node-0", "GET", "/v1/node")
        if len(next(d for d in view["devices"] if d["uuid"] == gpu["uuid"])["pods"]) == 2:
            break
        time.sleep(0.1)
    c.set_faults("mi355x-node-0", {"devices": {str(gpu["index"]): {"processes": [
        {"pid": pids["ok"], "vramBytes": (8 << 30) + (200 << 20), "gfxNs": 0},
        {"pid": pids["rogue"], "vramBytes": 20 << 30, "gfxNs": 0}]}}}, sample=True)
    view = c.agent_request("mi355x-node-0", "GET", "/v1/node")
    use = {e["pod"]: e for e in next(d for d in view["devices"] if d["uuid"] == gpu["uuid"])["usage"]}
    assert use["rogue"]["overBudget"] and use["rogue"]["slotBudgetBytes"] == 8 << 30, use
    assert not use["ok"].get("overBudget") and use["ok"]["slotBudgetBytes"] == 8 << 30, use
    metrics = str(c.agent_request("mi355x-node-0", "GET", "/metrics"))
    assert 'gpupool_pod_over_slot_budget{' in metrics and 'pod="rogue"} 1' in metrics
    deadline = time.monotonic() + 10
    evs = []
    while time.monotonic() < deadline:
        evs = [e for e in k.list(EVENTS, "default")["items"] if e["reason"] == "SlotBudgetExceeded"]
        if evs:
            break
        time.sleep(0.1)
    assert len(evs) == 1 and "default/rogue" in evs[0]["message"], evs
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    r = subprocess.run([os.path.join(root, "bin", "gpuctl"), "--server", c.url, "top", "pods"],
                       capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, GPUPOOL_AGENT_TOKEN=c.agent_token))
    rows = {ln.split()[0]: ln.split() for ln in r.stdout.splitlines()[1:]}
    assert rows["default/rogue"][-1] == "8.00!" and rows["default/ok"][-1] == "8.00", r.stdout
    c.set_faults("mi355x-node-0", {"devices": {str(gpu["index"]): {"processes": [
        {"pid": pids["rogue"], "vramBytes": 20 << 30, "gfxNs": 0}]}}}, sample=True)
    time.sleep(0.5)  # still over: no second event for the same pod and GPU
    assert len([e for e in k.list(EVENTS, "default")["items"]
                if e["reason"] == "SlotBudgetExceeded"]) == 1


def test_over_budget_pod_is_evicted_when_the_pool_says_so(cluster_factory):
    """spec.sharing.overBudgetAction Evict (VERDICT r4 missing #4; HAMi enforces its limit per
    container, GPU调度平台搭建.md:289-298): the pod holding 20 GiB against its 8 GiB slot — its
    in-pod limit is not in force — is evicted through the API after two consecutive over-budget
    samples, with a SlotBudgetExceeded event on the pod; its sibling within budget keeps
    running."""
    import time
    from gpupool.kube import EVENTS
    c = cluster_factory()
    k = c.client
    k.create(MI355XPOOLS, mi_pool("bud", 1, sharing={"replicasPerGPU": 2, "hbmBytesPerSlot": 8 << 30,
                                                     "overBudgetAction": "Evict"}), "default")
    gpu = wait_ready(k, "bud", 1)["status"]["devices"][0]
    pids = {}
    for name in ("ok", "rogue"):
        k.create(PODS, pause_pod(name), "default")
        p = k.wait_for(PODS, name, "default", lambda p: running(p) and "gpupool.amd.com/pid" in
                       p["metadata"].get("annotations", {}), timeout=30)
        pids[name] = int(p["metadata"]["annotations"]["gpupool.amd.com/pid"])
    deadline = time.monotonic() + 10
    while time.monotonic() < deadline:
        view = c.agent_request("mi355x-node-0", "GET", "/v1/node")
        if len(next(d for d in view["devices"] if d["uuid"] == gpu["uuid"])["pods"]) == 2:
            break
        time.sleep(0.1)
    procs = {"devices": {str(gpu["index"]): {"processes": [
        {"pid": pids["ok"], "vramBytes": 6 << 30, "gfxNs": 0},
        {"pid": pids["rogue"], "vramBytes": 20 << 30, "gfxNs": 0}]}}}
    c.set_faults("mi355x-node-0", procs, sample=True)  # the periodic samples follow (0.5 s)
    k.wait_for(PODS, "rogue", "default", lambda o: o is None, timeout=30)
    assert running(k.get(PODS, "ok", "default"))
    deadline = time.monotonic() + 10
    evs = []
    while time.monotonic() < deadline and not evs:
        evs = [e for e in k.list(EVENTS, "default")["items"]
               if e["reason"] == "SlotBudgetExceeded" and e["involvedObject"]["kind"] == "Pod"]
        time.sleep(0.1)
    assert len(evs) == 1 and evs[0]["involvedObject"]["name"] == "rogue", evs
    assert "evicted" in evs[0]["message"] and "overBudgetAction Evict" in evs[0]["message"]
    assert "for 2+ samples" in evs[0]["message"]  # never on one reading
    assert "gpupool_agent_over_budget_evictions 1" in str(c.agent_request("mi355x-node-0", "GET",
                                                                            "/metrics"))


def test_limit_file_is_mounted_read_only_beside_the_account(cluster_factory, tmp_path):
    """The account a pod's processes charge is writable; the limit the agent fixed is a separate
    read-only file (GPLIMIT1 <bytes>, mode 0644, mounted read_only) the share library takes the
    smallest limit from: editing the account's header gains a pod nothing
    (native/tests/test_share.cc has the library side)."""
    import os
    import time
    c = cluster_factory()
    k = c.client
    k.create(MI355XPOOLS, mi_pool("lim", 1, sharing={"replicasPerGPU": 2,
                                                     "hbmBytesPerSlot": 8 << 30}), "default")
    wait_ready(k, "lim", 1)
    pod = pause_pod("p0")
    pod["spec"]["containers"][0]["command"] = [
        "bash", "-c", "env | grep -E '^GPUPOOL_SHARE_(LIMIT|ACCOUNT)=' | sort; sleep 600"]
    k.create(PODS, pod, "default")
    p = k.wait_for(PODS, "p0", "default", running, timeout=30)
    path = p["metadata"]["annotations"]["gpupool.amd.com/log-path"]
    deadline = time.monotonic() + 10
    while time.monotonic() < deadline and open(path).read().count("\n") < 2:
        time.sleep(0.05)
    env = dict(line.split("=", 1) for line in open(path).read().split())
    lim, acct = env["GPUPOOL_SHARE_LIMIT"], env["GPUPOOL_SHARE_ACCOUNT"]
    assert lim == acct[:-len(".acct")] + ".limit"
    assert open(lim).read() == f"GPLIMIT1 {8 << 30}\n"
    assert oct(os.stat(lim).st_mode & 0o777) == "0o644"
