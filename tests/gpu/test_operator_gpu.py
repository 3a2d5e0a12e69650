"""Real-MI355X operator tests (BASELINE config 2 + workload/drain/fault paths on hardware)."""
from __future__ import annotations

import json
import os
import time

import pytest

from gpupool.kube import MI355XPOOLS, PODS
from gpupool.testing.cluster import NodeSpec

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def ready_at(r):
    def pred(o):
        st = (o or {}).get("status") or {}
        return st.get("observedGeneration") == (o or {}).get("metadata", {}).get("generation") and \
            st.get("readyReplicas") == r and len(st.get("devices", [])) == r and \
            any(x["type"] == "Ready" and x["status"] == "True" for x in st.get("conditions", []))
    return pred


def pool(name, r, **spec):
    return {"apiVersion": "compute.my.domain/v1alpha1", "kind": "Mi355xPool",
            "metadata": {"name": name}, "spec": {"replicas": r, **spec}}


def test_devlib_amdsmi_matches_cli(native_built):
    from gpupool.ops import devlib
    a = devlib.DeviceLib("amdsmi", node="t").snapshot()
    c = devlib.DeviceLib("cli", node="t").snapshot()
    assert [d["uuid"] for d in a["devices"]] == [d["uuid"] for d in c["devices"]]
    for da, dc in zip(a["devices"], c["devices"]):
        assert da["hipUUID"] == dc["hipUUID"] and da["bdf"] == dc["bdf"]
        assert da["xgmi"]["links"] == dc["xgmi"]["links"]
        assert da["asic"]["gfx"] == "gfx950"
        v = devlib.evaluate(da, da, {})
        assert v["healthy"], v


def test_config2_pool_ready_on_real_gpu(cluster_factory):
    c = cluster_factory(nodes=[NodeSpec("gpu-node", backend="amdsmi", probe="helper")])
    k = c.client
    t0 = time.perf_counter()
    k.create(MI355XPOOLS, pool("p", 1), "default")
    obj = k.wait_for(MI355XPOOLS, "p", "default", ready_at(1), timeout=60)
    dt = time.perf_counter() - t0
    assert dt < 30.0  # BASELINE target
    d = obj["status"]["devices"][0]
    assert d["health"] == "Healthy" and d["advertised"] and d["probe"]["passed"]
    assert d["probe"]["backend"] == "helper" and d["probe"]["hbmGBps"] > 1000
    conds = {x["type"]: x["status"] for x in obj["status"]["conditions"]}
    assert conds["XGMILinksHealthy"] == "True" and conds["HBMECCHealthy"] == "True"
    assert conds["ThermalHealthy"] == "True" and conds["DeviceProbePassed"] == "True"
    # the kubelet reports device-plugin capacity in Node status asynchronously (coalesced)
    node = k.wait_for(__import__("gpupool.kube", fromlist=["NODES"]).NODES, "gpu-node", None,
                      lambda n: (n["status"].get("allocatable") or {}).get("amd.com/gpu") == "1",
                      timeout=10)
    assert node["status"]["allocatable"]["amd.com/gpu"] == "1"


def test_workload_pod_runs_on_allotted_gpu_then_drain(cluster_factory, tmp_path):
    c = cluster_factory(nodes=[NodeSpec("gpu-node", backend="amdsmi", probe="helper")])
    k = c.client
    k.create(MI355XPOOLS, pool("p", 1), "default")
    obj = k.wait_for(MI355XPOOLS, "p", "default", ready_at(1), timeout=60)
    hip_uuid = obj["status"]["devices"][0]["hipUUID"]
    k.create(PODS, {"metadata": {"name": "train"}, "spec": {"restartPolicy": "Never", "containers": [{
        "name": "train", "command": ["python", "examples/fmnist_train.py", "--epochs", "1",
                                     "--synthetic", "--steps", "60", "--output", str(tmp_path)],
        "resources": {"limits": {"amd.com/gpu": 1}}}]}}, "default")
    done = k.wait_for(PODS, "train", "default",
                      lambda o: o and o.get("status", {}).get("phase") in ("Succeeded", "Failed"),
                      timeout=240)
    logp = done["metadata"]["annotations"]["gpupool.amd.com/log-path"]
    log = open(logp).read()
    assert done["status"]["phase"] == "Succeeded", log[-3000:]
    events = [json.loads(x) for x in log.splitlines() if x.startswith("{")]
    start = next(e for e in events if e["event"] == "start")
    assert start["rocr_visible"] == hip_uuid          # exactly the allotted GPU
    assert start["arch"].startswith("gfx950")
    assert os.path.exists(tmp_path / "fashion_mnist_cnn.pth")
    # a long-running pod on the GPU, then scale to 0: cordon -> evict -> release
    k.create(PODS, {"metadata": {"name": "hold"}, "spec": {"terminationGracePeriodSeconds": 2,
                                                          "containers": [{
        "name": "hold", "command": ["sleep", "600"], "resources": {"limits": {"amd.com/gpu": 1}}}]}},
        "default")
    k.wait_for(PODS, "hold", "default", lambda o: o and o["status"].get("phase") == "Running", 60)
    k.patch(MI355XPOOLS, "p", {"spec": {"replicas": 0}}, "default")
    k.wait_for(PODS, "hold", "default", lambda o: o is None, timeout=60)  # evicted + deleted
    k.wait_for(MI355XPOOLS, "p", "default", ready_at(0), timeout=60)


def test_fault_overlay_on_real_hardware(cluster_factory):
    c = cluster_factory(nodes=[NodeSpec("gpu-node", backend="amdsmi", probe="helper")])
    k = c.client
    k.create(MI355XPOOLS, pool("p", 1, replacePolicy="Keep"), "default")
    obj = k.wait_for(MI355XPOOLS, "p", "default", ready_at(1), timeout=60)
    uuid = obj["status"]["devices"][0]["uuid"]
    c.set_faults("gpu-node", {"devices": {uuid: {"ecc": {"uncorrectable": 10 ** 6}}}})

    def degraded(o):
        conds = {x["type"]: x for x in (o or {}).get("status", {}).get("conditions", [])}
        return conds.get("HBMECCHealthy", {}).get("status") == "False" and \
            conds.get("Degraded", {}).get("status") == "True" and o["status"]["readyReplicas"] == 0
    k.wait_for(MI355XPOOLS, "p", "default", degraded, timeout=30)
    c.set_faults("gpu-node", {})
    k.wait_for(MI355XPOOLS, "p", "default", ready_at(1), timeout=30)


def test_performance_floor_on_real_gpu(cluster_factory):
    """spec.probe.minMfmaTflops above what any MI355X reaches: the (correct) GPU fails
    DeviceProbePassed with PerformanceBelowFloor and the pool does not report Ready."""
    c = cluster_factory(nodes=[NodeSpec("gpu-node", backend="amdsmi", probe="helper")])
    k = c.client
    k.create(MI355XPOOLS, pool("slow", 1, probe={"minMfmaTflops": 100000}, replacePolicy="Keep"),
             "default")

    def probe_failed(o):
        return any(x["type"] == "DeviceProbePassed" and x["status"] == "False"
                   for x in ((o or {}).get("status") or {}).get("conditions", []))
    o = k.wait_for(MI355XPOOLS, "slow", "default", probe_failed, timeout=60)
    msg = next(x["message"] for x in o["status"]["conditions"] if x["type"] == "DeviceProbePassed")
    assert "PerformanceBelowFloor" in msg and "TFLOP/s" in msg
    assert o["status"].get("readyReplicas", 0) == 0


def test_mi355xjob_torchrun_worker_on_pool_gpu(cluster_factory, tmp_path):
    """Mi355xJob on real hardware: the gang is placed on the pool's GPU, the pod gets the job's
    rendezvous env, and torchrun (driven by PET_*/MASTER_*) starts a distributed-mode worker on
    exactly the allotted GPU (GPU调度平台搭建.md:300-306, :623-635, :638-675). One GPU per box here,
    so world size is 1; multi-rank rendezvous is covered by the CPU job tests. Attempt 1 fails on
    purpose at step 25 and the restarted gang resumes from its checkpoint (spec.checkpointDir)."""
    from gpupool.kube import MI355XJOBS
    c = cluster_factory(nodes=[NodeSpec("gpu-node", backend="amdsmi", probe="helper")])
    k = c.client
    k.create(MI355XPOOLS, pool("p", 1), "default")
    obj = k.wait_for(MI355XPOOLS, "p", "default", ready_at(1), timeout=60)
    hip_uuid = obj["status"]["devices"][0]["hipUUID"]
    script = ("exec python -m torch.distributed.run --nnodes $PET_NNODES "
              "--nproc-per-node $PET_NPROC_PER_NODE --node-rank $PET_NODE_RANK "
              "--master-addr $MASTER_ADDR --master-port $MASTER_PORT "
              f"examples/fmnist_train.py --mode distributed --synthetic --epochs 1 --steps 40 "
              f"--checkpoint_every 10 --fail_at_step 25 --output {tmp_path}")
    k.create(MI355XJOBS, {"apiVersion": "compute.my.domain/v1alpha1", "kind": "Mi355xJob",
                          "metadata": {"name": "ddp"},
                          "spec": {"replicas": 1, "gpusPerReplica": 1, "poolRef": "p",
                                   "masterPort": 29731, "backoffLimit": 1,
                                   "checkpointDir": str(tmp_path / "ckpt"),
                                   "template": {"spec": {"containers": [{
                                       "name": "main", "command": ["bash", "-c", script]}]}}}},
             "default")
    done = k.wait_for(MI355XJOBS, "ddp", "default",
                      lambda o: ((o or {}).get("status") or {}).get("phase") in ("Succeeded", "Failed"),
                      timeout=240)
    pod = k.list(PODS, "default", label_selector="gpupool.amd.com/job-name=ddp")["items"][0]
    log = open(pod["metadata"]["annotations"]["gpupool.amd.com/log-path"]).read()
    assert done["status"]["phase"] == "Succeeded", (done["status"], log[-3000:])
    events = [json.loads(x) for x in log.splitlines() if x.startswith("{")]
    start = next(e for e in events if e["event"] == "start")
    assert start["mode"] == "distributed" and start["world"] == 1
    assert start["device"] == "cuda:0" and start["arch"].startswith("gfx950")
    assert start["rocr_visible"] == hip_uuid
    # attempt 1 died at step 25; the restarted gang resumed from the step-20 checkpoint on the GPU
    assert done["status"]["restarts"] == 1
    resume = next(e for e in events if e["event"] == "resume")
    assert resume["step"] == 20
    assert next(e for e in events if e["event"] == "done")["steps"] == 40
    assert done["status"]["replicaStatuses"][0]["devices"]
    assert os.path.exists(tmp_path / "fashion_mnist_cnn.pth")


def test_autoscaled_pool_grows_for_pending_gpu_pod(cluster_factory, tmp_path):
    """spec.autoscale on real hardware: an empty pool grows to 1 when a pod asks for its GPU,
    the GPU is probed and advertised, the pod runs on it, and the pool shrinks back once the pod
    has finished."""
    c = cluster_factory(nodes=[NodeSpec("gpu-node", backend="amdsmi", probe="helper")])
    k = c.client
    k.create(MI355XPOOLS, pool("auto", 0, autoscale={"enabled": True, "maxReplicas": 1,
                                                     "scaleDownDelaySeconds": 0}), "default")
    k.wait_for(MI355XPOOLS, "auto", "default", ready_at(0), timeout=60)
    k.create(PODS, {"metadata": {"name": "train"}, "spec": {"restartPolicy": "Never", "containers": [{
        "name": "train", "command": ["python", "examples/fmnist_train.py", "--epochs", "1",
                                     "--synthetic", "--steps", "20", "--output", str(tmp_path)],
        "resources": {"limits": {"amd.com/gpu": 1}}}]}}, "default")
    obj = k.wait_for(MI355XPOOLS, "auto", "default", ready_at(1), timeout=60)
    assert obj["status"]["devices"][0]["probe"]["passed"]
    done = k.wait_for(PODS, "train", "default",
                      lambda o: o and o.get("status", {}).get("phase") in ("Succeeded", "Failed"),
                      timeout=240)
    log = open(done["metadata"]["annotations"]["gpupool.amd.com/log-path"]).read()
    assert done["status"]["phase"] == "Succeeded", log[-3000:]
    assert '"arch": "gfx950' in log
    k.wait_for(MI355XPOOLS, "auto", "default", ready_at(0), timeout=60)


def test_hbm_scrub_on_real_gpu_and_claim_is_not_blocked(cluster_factory):
    """The agent's HBM scrubber on the MI355X: two 16 GiB windows of the all-free-HBM buffer are
    pattern-tested through the RPC, coverage lands in the agent view; a claim issued right after
    (while the ~280 GB buffer is being freed, ~3 s) is Ready in well under a second, and the pod
    Allocate path waits for the free. status.devices[] carries the CU census and coverage."""
    c = cluster_factory(nodes=[NodeSpec("gpu-node", backend="amdsmi", probe="helper", extra_args=[
        "--scrub-interval", "0", "--scrub-window", str(16 << 30)])])
    r = c.agent_request("gpu-node", "POST", "/v1/scrub", {"gpu": "0", "windows": 2})
    assert r["ok"], r
    cov = r["coverage"]
    assert cov["windows"] == 2 and cov["cursor"] == 32 << 30 and cov["span"] > 200e9, cov
    assert cov["lastBadBits"] == 0 and cov["lastGBps"] > 3000, cov
    k = c.client
    t0 = time.perf_counter()
    k.create(MI355XPOOLS, pool("p", 1), "default")
    obj = k.wait_for(MI355XPOOLS, "p", "default", ready_at(1), timeout=60)
    dt = time.perf_counter() - t0
    if dt >= 1.0 or os.environ.get("GPUPOOL_SCRUB_DIAG"):  # keep the evidence: which span waited
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        with open(os.path.join(ROOT, "gpurun_out", f"scrub_claim_diag_{int(time.time())}.json"),
                  "w") as f:
            json.dump({"dt": dt, "traces": c.manager_traces(key="Mi355xPool/default/p", n=16),
                       "agent_log": c.log("agent-gpu-node")[-20000:],
                       "manager_log": c.log("manager")[-20000:]}, f, indent=1)
    assert dt < 1.0, dt
    d = obj["status"]["devices"][0]
    assert d["probe"]["cusVerified"] == d["probe"]["cusExpected"] == 256, d
    assert d["hbmCoverage"]["span"] > 200e9, d


def test_amdsmi_ras_event_source_and_utilisation_on_real_gpu(native_built):
    """On the MI355X: the bad-page (RAS) read, VRAM in use and the amdsmi event subscription work
    through libmi355x_dev, and GFX activity / VRAM used rise while a bf16 GEMM workload runs in
    another process (what the agent exports as gpupool_device_* utilisation)."""
    import subprocess
    import sys
    from gpupool.ops import devlib
    lib = devlib.DeviceLib("amdsmi", node="t")
    d0 = lib.snapshot()["devices"][0]
    ras = d0["ras"]
    assert isinstance(ras.get("badPagesSupported"), bool), ras
    if ras["badPagesSupported"]:
        assert min(ras["retiredPages"], ras["pendingPages"], ras["unreservablePages"]) >= 0
    assert d0["memTotalBytes"] > 250e9 and d0.get("memUsedBytes", -1) >= 0
    assert devlib.evaluate(d0, d0, {})["healthy"]  # the box's GPU passes the retirement rules
    ev = lib.wait_events(50)
    print("RAS", json.dumps(ras), "events", json.dumps(ev), "memUsed", d0.get("memUsedBytes"))
    assert isinstance(ev.get("supported"), bool) and ev.get("events") == []
    code = ("import torch,time,sys\n"
            "a=torch.randn(8192,8192,device='cuda',dtype=torch.bfloat16)\n"
            "(a@a).sum().item(); print('READY',flush=True); t=time.time()\n"
            "while time.time()-t<4: (a@a).sum().item()\n")
    p = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, text=True)
    peak_gfx, peak_used = 0, 0
    try:
        assert p.stdout.readline().strip() == "READY"
        t0 = time.time()
        while time.time() - t0 < 3.5:
            s = lib.snapshot()["devices"][0]
            peak_gfx = max(peak_gfx, int((s.get("activity") or {}).get("gfx") or 0))
            peak_used = max(peak_used, int(s.get("memUsedBytes") or 0))
            time.sleep(0.1)
    finally:
        p.wait(timeout=90)
    print("peak gfx activity", peak_gfx, "peak VRAM used", peak_used)
    assert p.returncode == 0
    # (VRAM "used" right after another test's process exit can still include memory the driver
    # has not finished clearing, so compare against the workload's own footprint, not a baseline)
    assert peak_gfx > 0 and peak_used >= 8192 * 8192 * 2


def test_agent_exports_events_and_utilisation_on_real_gpu(cluster_factory):
    c = cluster_factory(nodes=[NodeSpec("gpu-node", backend="amdsmi", probe="helper")])
    k = c.client
    k.create(MI355XPOOLS, pool("u", 1), "default")
    k.wait_for(MI355XPOOLS, "u", "default", ready_at(1), timeout=60)
    deadline = time.monotonic() + 10
    view = c.agent_request("gpu-node", "GET", "/v1/node")
    while "device" not in view["eventSources"] and time.monotonic() < deadline:
        time.sleep(0.1)
        view = c.agent_request("gpu-node", "GET", "/v1/node")
    print("eventSources", view["eventSources"])
    assert view["eventSources"].get("faultOverlay") is True and "device" in view["eventSources"]
    d = next(x for x in view["devices"] if x.get("pool") == "default/u")
    assert d["telemetry"]["memTotalBytes"] > 250e9 and d["telemetry"]["powerW"] > 0
    text = c.agent_request("gpu-node", "GET", "/metrics")
    assert 'gpupool_device_power_watts{' in text and 'pool="default/u"' in text
    deadline = time.monotonic() + 20
    while 'gpupool_pool_vram_total_bytes{kind="Mi355xPool",pool="default/u"}' not in \
            c.manager_metrics() and time.monotonic() < deadline:
        time.sleep(0.2)
    assert 'gpupool_pool_vram_total_bytes{kind="Mi355xPool",pool="default/u"}' in c.manager_metrics()


def test_rccl_check_harness_on_real_gpu():
    """The collective check bench.py runs per rank when N > 1 (RCCL over xGMI on the 8-GPU node):
    on one MI355X it initialises RCCL (backend "nccl") and all-reduces a bf16 buffer exactly."""
    import socket
    import subprocess
    import sys
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    p = subprocess.run([sys.executable, "-m", "gpupool.parallel.rccl_check", "--rank", "0",
                        "--world", "1", "--master-port", str(port), "--bytes", str(64 << 20),
                        "--iters", "5"], capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    out = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
    assert out["exact"] and out["backend"] == "nccl" and out["world"] == 1


def test_time_sliced_pods_share_the_real_gpu(cluster_factory):
    """spec.sharing.replicasPerGPU on hardware: the one MI355X is advertised as 3 slots and three
    pods compute on it at the same time (each a torch matmul loop through the ROCR_VISIBLE_DEVICES
    the plugin handed it), all seeing the same GPU."""
    c = cluster_factory(nodes=[NodeSpec("gpu-node", backend="amdsmi", probe="helper")])
    k = c.client
    k.create(MI355XPOOLS, pool("shared", 1, sharing={"replicasPerGPU": 3}), "default")
    obj = k.wait_for(MI355XPOOLS, "shared", "default", ready_at(1), timeout=60)
    assert obj["status"]["allocatable"] == 3
    hip_uuid = obj["status"]["devices"][0]["hipUUID"]
    code = ("import json, os, time, torch\n"
            "x = torch.randn(2048, 2048, device='cuda', dtype=torch.bfloat16)\n"
            "t0 = time.time(); n = 0\n"
            "while time.time() - t0 < 3: x = (x @ x).clamp_(-1, 1); n += 1\n"
            "torch.cuda.synchronize()\n"
            "print(json.dumps({'rocr': os.environ.get('ROCR_VISIBLE_DEVICES'), 'iters': n,"
            " 'slots': os.environ.get('GPUPOOL_GPU_SLOTS'),"
            " 'arch': torch.cuda.get_device_properties(0).gcnArchName}))\n")
    for i in range(3):
        k.create(PODS, {"metadata": {"name": f"share{i}"}, "spec": {"restartPolicy": "Never",
                        "containers": [{"name": "c", "command": ["python", "-c", code],
                                        "resources": {"limits": {"amd.com/gpu": 1}}}]}}, "default")
    outs = []
    for i in range(3):
        done = k.wait_for(PODS, f"share{i}", "default",
                          lambda o: o and o.get("status", {}).get("phase") in ("Succeeded", "Failed"),
                          timeout=240)
        log = open(done["metadata"]["annotations"]["gpupool.amd.com/log-path"]).read()
        assert done["status"]["phase"] == "Succeeded", log[-3000:]
        outs.append(json.loads([x for x in log.splitlines() if x.startswith("{")][-1]))
    assert all(o["rocr"] == hip_uuid and o["arch"].startswith("gfx950") and o["iters"] > 0
               for o in outs), outs
    assert len({o["slots"] for o in outs}) == 3  # three different slots of the one GPU


def test_isolated_slots_and_per_pod_accounting_on_the_real_gpu(cluster_factory):
    """The HAMi layer end to end on hardware: a pool sharing the MI355X as 2 isolated slots
    (8 GiB HBM and 128 CUs each). Pod "small" holds 2 GiB, pod "big" 6 GiB and is refused 4 GiB
    more (its slot's budget), both see an 8 GiB GPU; meanwhile the agent's per-pod accounting
    (amdsmi process list -> pod) shows both pods on the same uuid with their distinct VRAM."""
    c = cluster_factory(nodes=[NodeSpec("gpu-node", backend="amdsmi", probe="helper")])
    k = c.client
    k.create(MI355XPOOLS, pool("iso", 1, sharing={"replicasPerGPU": 2, "hbmBytesPerSlot": 8 << 30,
                                                  "cuPerSlot": 128}), "default")
    obj = k.wait_for(MI355XPOOLS, "iso", "default", ready_at(1), timeout=60)
    uuid = obj["status"]["devices"][0]["uuid"]
    code = ("import json, os, sys, time, torch\n"
            "hold, more = int(sys.argv[1]), int(sys.argv[2])\n"
            "a = torch.ones(hold, dtype=torch.uint8, device='cuda'); torch.cuda.synchronize()\n"
            "try:\n"
            "    b = torch.ones(more, dtype=torch.uint8, device='cuda'); torch.cuda.synchronize(); r = 'ok'\n"
            "except torch.OutOfMemoryError:\n"
            "    r = 'oom'\n"
            "print(json.dumps({'more': r, 'total': torch.cuda.mem_get_info(0)[1],"
            " 'mask': os.environ.get('GPUPOOL_CU_MASK')}), flush=True)\n"
            "time.sleep(20)\n")
    for name, hold, more in (("small", 2 << 30, 1 << 30), ("big", 6 << 30, 4 << 30)):
        k.create(PODS, {"metadata": {"name": name}, "spec": {"restartPolicy": "Never", "containers": [
            {"name": "c", "command": ["python", "-c", code, str(hold), str(more)],
             "resources": {"limits": {"amd.com/gpu": 1}}}]}}, "default")
    outs = {}
    for name in ("small", "big"):
        p = k.wait_for(PODS, name, "default", lambda o: o and o["status"].get("phase") == "Running"
                       and "gpupool.amd.com/log-path" in o["metadata"].get("annotations", {}),
                       timeout=60)
        path = p["metadata"]["annotations"]["gpupool.amd.com/log-path"]
        deadline = time.monotonic() + 60
        while time.monotonic() < deadline and "{" not in open(path).read():
            time.sleep(0.2)
        log = open(path).read()
        outs[name] = json.loads([x for x in log.splitlines() if x.startswith("{")][-1])
    assert outs["small"]["more"] == "ok" and outs["big"]["more"] == "oom", outs
    assert outs["small"]["total"] == outs["big"]["total"] == 8 << 30, outs
    assert {outs["small"]["mask"], outs["big"]["mask"]} == {"0-127", "128-255"}, outs
    # per-pod accounting from the amdsmi process list, attributed through the pods' environment
    deadline = time.monotonic() + 15
    use = {}
    while time.monotonic() < deadline:
        c.agent_request("gpu-node", "POST", "/v1/sample", {})
        view = c.agent_request("gpu-node", "GET", "/v1/node")
        use = {e["pod"]: e for e in next(d for d in view["devices"] if d["uuid"] == uuid).get("usage", [])}
        if {"small", "big"} <= set(use) and use["big"]["vramBytes"] >= 6 << 30:
            break
        time.sleep(0.5)
    print({k2: (v["vramBytes"], v.get("gfxBusy")) for k2, v in use.items()})
    assert 2 << 30 <= use["small"]["vramBytes"] < 6 << 30, use
    assert 6 << 30 <= use["big"]["vramBytes"] <= 8 << 30, use
    for name in ("small", "big"):
        k.delete(PODS, name, "default", grace=0)


def _maps(pid: int) -> str:
    with open(f"/proc/{pid}/maps") as f:
        return f.read()


def test_probe_runs_in_a_helper_never_in_the_agent(cluster_factory):
    """The claim-time probe's HIP runs in the GPU's probe helper: the agent process (device plugin,
    health, claims for every GPU of the node) never maps libmi355x_probe.so, the helper does."""
    c = cluster_factory(nodes=[NodeSpec("gpu-node", backend="amdsmi", probe="helper")])
    k = c.client
    k.create(MI355XPOOLS, pool("p", 1), "default")
    obj = k.wait_for(MI355XPOOLS, "p", "default", ready_at(1), timeout=60)
    assert obj["status"]["devices"][0]["probe"]["passed"]
    agent_pid = c.procs["agent-gpu-node"].pid
    assert "libmi355x_probe" not in _maps(agent_pid)
    view = c.agent_request("gpu-node", "GET", "/v1/node")
    helpers = {k2: v for k2, v in view["probeHelpers"].items() if k2 != "fabric"}
    assert helpers and all(v["alive"] for v in helpers.values()), helpers
    for v in helpers.values():
        assert "libmi355x_probe" in _maps(v["pid"])
    print("helpers", helpers)


def _probe_cond(o):
    return next((x for x in ((o or {}).get("status") or {}).get("conditions", [])
                 if x["type"] == "DeviceProbePassed"), {})


def test_probe_helper_crash_on_the_real_gpu_leaves_the_agent_serving(cluster_factory):
    """A probe that aborts its process (what HIP does on a GPU memory fault; injected with the
    overlay's probeCrash) on the MI355X: the pool's DeviceProbePassed turns False with reason
    ProbeCrashed, the agent keeps answering, a fresh helper with a HIP context on the GPU replaces
    the dead one, and once the fault is gone the GPU passes again."""
    c = cluster_factory(nodes=[NodeSpec("gpu-node", backend="amdsmi", probe="helper",
                                        extra_args=["--quarantine", "1"])])
    k = c.client
    c.set_faults("gpu-node", {"devices": {"0": {"probeCrash": True}}})
    k.create(MI355XPOOLS, pool("p", 1, replacePolicy="Keep"), "default")
    o = k.wait_for(MI355XPOOLS, "p", "default",
                   lambda o: _probe_cond(o).get("status") == "False", timeout=60)
    cond = _probe_cond(o)
    assert cond["reason"] == "ProbeCrashed" and "SIGABRT" in cond["message"], cond
    view = c.agent_request("gpu-node", "GET", "/v1/node")  # the agent is alive and serving
    uuid = o["status"]["devices"][0]["uuid"]
    deadline = time.monotonic() + 60
    while not (view["probeHelpers"].get(uuid) or {}).get("alive") and time.monotonic() < deadline:
        time.sleep(0.2)
        view = c.agent_request("gpu-node", "GET", "/v1/node")
    assert view["probeHelpers"][uuid]["alive"], view["probeHelpers"]
    assert "SIGABRT" in view["probeHelpers"][uuid]["lastExit"]
    c.set_faults("gpu-node", {})
    k.delete(MI355XPOOLS, "p", "default")
    k.wait_for(MI355XPOOLS, "p", "default", lambda o: o is None, timeout=60)
    time.sleep(1.5)  # the 1 s quarantine of the crashed GPU runs out
    k.create(MI355XPOOLS, pool("q", 1), "default")
    obj = k.wait_for(MI355XPOOLS, "q", "default", ready_at(1), timeout=60)
    assert obj["status"]["devices"][0]["probe"]["passed"]


def test_hung_probe_on_the_real_gpu_is_cut_at_its_deadline(cluster_factory):
    """A probe that never returns (overlay probeHang) with spec.probe.timeoutSeconds 2: the claim
    is answered within the deadline + 1 s, DeviceProbePassed says ProbeTimeout, the hung helper
    is killed and replaced."""
    c = cluster_factory(nodes=[NodeSpec("gpu-node", backend="amdsmi", probe="helper")])
    k = c.client
    c.set_faults("gpu-node", {"devices": {"0": {"probeHang": True}}})
    t0 = time.monotonic()
    k.create(MI355XPOOLS, pool("p", 1, replacePolicy="Keep", probe={"timeoutSeconds": 2}), "default")
    o = k.wait_for(MI355XPOOLS, "p", "default",
                   lambda o: _probe_cond(o).get("status") == "False", timeout=60)
    dt = time.monotonic() - t0
    cond = _probe_cond(o)
    assert cond["reason"] == "ProbeTimeout", cond
    assert dt < 2 + 1 + 1.0, dt  # deadline + 1 s (+ the manager's own round trips)
    c.set_faults("gpu-node", {})
    view = c.agent_request("gpu-node", "GET", "/v1/node")
    uuid = o["status"]["devices"][0]["uuid"]
    deadline = time.monotonic() + 60
    while not (view["probeHelpers"].get(uuid) or {}).get("alive") and time.monotonic() < deadline:
        time.sleep(0.2)
        view = c.agent_request("gpu-node", "GET", "/v1/node")
    assert view["probeHelpers"][uuid]["alive"], view["probeHelpers"]


def test_pod_that_escapes_its_hbm_limit_is_evicted_on_the_real_gpu(cluster_factory):
    """spec.sharing.overBudgetAction Evict on hardware: a pod that drops the share library
    (``env -u HSA_TOOLS_LIB``) and allocates 12 GiB against its 8 GiB slot is seen from outside
    (amdsmi process list -> pod) and evicted within 3 samples; its sibling, within budget through
    the library, keeps running."""
    c = cluster_factory(nodes=[NodeSpec("gpu-node", backend="amdsmi", probe="helper")])
    k = c.client
    k.create(MI355XPOOLS, pool("iso", 1, sharing={"replicasPerGPU": 2, "hbmBytesPerSlot": 8 << 30,
                                                  "overBudgetAction": "Evict"}), "default")
    k.wait_for(MI355XPOOLS, "iso", "default", ready_at(1), timeout=60)
    hold = ("import sys, time, torch\n"
            "a = torch.ones(int(sys.argv[1]), dtype=torch.uint8, device='cuda')\n"
            "torch.cuda.synchronize(); print('HOLDING', flush=True); time.sleep(120)\n")
    specs = {"ok": ["python", "-c", hold, str(2 << 30)],
             "rogue": ["env", "-u", "HSA_TOOLS_LIB", "python", "-c", hold, str(12 << 30)]}
    for name, cmd in specs.items():
        k.create(PODS, {"metadata": {"name": name}, "spec": {
            "restartPolicy": "Never", "terminationGracePeriodSeconds": 2,
            "containers": [{"name": "c", "command": cmd,
                            "resources": {"limits": {"amd.com/gpu": 1}}}]}}, "default")
    held = {}
    deadline = time.monotonic() + 90
    while len(held) < 2 and time.monotonic() < deadline:
        for name in specs:
            p = k.get(PODS, name, "default")
            path = (p or {}).get("metadata", {}).get("annotations", {}).get("gpupool.amd.com/log-path")
            if name not in held and path and os.path.exists(path) and "HOLDING" in open(path).read():
                held[name] = time.monotonic()
        time.sleep(0.1)
    assert set(held) == {"ok", "rogue"}, held
    k.wait_for(PODS, "rogue", "default", lambda o: o is None, timeout=60)
    dt = time.monotonic() - held["rogue"]
    print(f"rogue evicted {dt:.2f} s after it held 12 GiB (sample period {c.sample_interval} s)")
    assert dt < 3 * c.sample_interval + 5.0, dt  # 3 samples + the pod's termination grace
    assert k.get(PODS, "ok", "default")["status"]["phase"] == "Running"
    k.delete(PODS, "ok", "default", grace=0)


def test_fabric_helper_rings_on_the_real_gpu(native_built):
    """The xGMI ring as the agent runs it: in the fabric helper (its own process, HIP on every
    listed GPU; with 2+ GPUs it runs a warm ring before it reports ready), then a claim-size ring
    answered by the same helper. On a 1-GPU box the ring [gpu, gpu] runs its links as local
    copies through the same code and protocol."""
    from gpupool.agent.prober import Prober
    from gpupool.ops import devlib
    devs = [d for d in devlib.DeviceLib("amdsmi", node="t").snapshot()["devices"]
            if d.get("hipUUID")][:1]
    assert devs, "no GPU with a hipUUID"
    p = Prober("helper", devices=devs)
    try:
        ring = [devs[0], devs[0]]
        t0 = time.monotonic()
        fab = p.helpers.fabric(ring)  # 1 GPU: not resident, started on demand, warmed before ready
        assert fab.wait_ready(60), fab.ready_error
        assert p.fabric_warm_ms is not None, p.helpers.snapshot()
        fabric_pid = p.helpers.snapshot()["fabric"]["pid"]
        assert "libmi355x_probe" in _maps(fabric_pid)
        starts = p.helpers.stats["helper_starts"]
        links = p.peer_ring(ring, {"xgmiBytes": 16 << 20, "timeoutSeconds": 10})
        link = links[devs[0]["uuid"]]
        assert link["passed"] and link["badBits"] == 0 and link["GBps"] > 50, link
        assert p.helpers.stats["helper_starts"] == starts  # the warmed helper answered
        assert p.helpers.snapshot()["fabric"]["pid"] == fabric_pid
        print(f"fabric warm {p.fabric_warm_ms:.0f} ms, ring {link['GBps']:.0f} GB/s, "
              f"total {time.monotonic() - t0:.1f} s")
    finally:
        p.helpers.stop()


def test_probe_helper_parked_while_a_tenant_holds_the_gpu(cluster_factory):
    """Round-5 weak #5 on hardware: while a pod holds the pool's GPU the agent keeps no HIP
    context there (its probe helper is parked: no agent process in the GPU's process list), the
    GPU's VRAM in use is the tenant's alone, and after the pod the helper comes back warm before
    release returns the GPU."""
    c = cluster_factory(nodes=[NodeSpec("gpu-node", backend="amdsmi", probe="helper")])
    k = c.client
    k.create(MI355XPOOLS, pool("p", 1, drain={"gracePeriodSeconds": 2}), "default")
    obj = k.wait_for(MI355XPOOLS, "p", "default", ready_at(1), timeout=60)
    gpu = obj["status"]["devices"][0]["uuid"]

    def dev():
        v = c.agent_request("gpu-node", "GET", "/v1/node")
        return next(d for d in v["devices"] if d["uuid"] == gpu), v

    def agent_vram(d):
        return sum(e["vramBytes"] for e in d.get("usage") or [] if e["pod"] == "gpupool-agent")

    deadline = time.monotonic() + 30
    while time.monotonic() < deadline and agent_vram(dev()[0]) == 0:
        time.sleep(0.5)
    before = agent_vram(dev()[0])
    assert before > 256 << 20, dev()[0].get("usage")  # the helper's context (+ probe arena)
    k.create(PODS, {"metadata": {"name": "tenant"}, "spec": {
        "terminationGracePeriodSeconds": 2, "containers": [{
            "name": "t", "command": ["python", "-c",
                                     "import torch, time; x = torch.empty(1 << 28, device='cuda');"
                                     " torch.cuda.synchronize(); print('holding', flush=True);"
                                     " time.sleep(600)"],
            "resources": {"limits": {"amd.com/gpu": 1}}}]}}, "default")
    k.wait_for(PODS, "tenant", "default", lambda o: o and o["status"].get("phase") == "Running", 120)
    deadline = time.monotonic() + 120
    d = None
    while time.monotonic() < deadline:
        d, view = dev()
        tenant = [e for e in d.get("usage") or [] if e["pod"] == "tenant"]
        if d.get("probeHelper") == "Parked" and agent_vram(d) == 0 and tenant and \
                tenant[0]["vramBytes"] >= 1 << 30:
            break
        time.sleep(0.5)
    assert d.get("probeHelper") == "Parked", d
    assert agent_vram(d) == 0, d.get("usage")           # no agent process on the tenant's GPU
    assert not (view.get("probeHelpers") or {}).get(gpu, {}).get("alive")
    tenant_vram = sum(e["vramBytes"] for e in d["usage"] if e["pod"] == "tenant")
    used = d["telemetry"]["memUsedBytes"]
    # what is in use is the tenant's (the driver's own reservation aside): the agent's ~1 GiB is
    # back with the tenant
    assert used - tenant_vram < 512 << 20, (used, tenant_vram, d["usage"])
    k.patch(MI355XPOOLS, "p", {"spec": {"replicas": 0}}, "default")
    k.wait_for(PODS, "tenant", "default", lambda o: o is None, timeout=60)
    k.wait_for(MI355XPOOLS, "p", "default", ready_at(0), timeout=120)
    deadline = time.monotonic() + 60  # the release hands the GPU back while the helper restarts
    while time.monotonic() < deadline:
        d, view = dev()
        if (view.get("probeHelpers") or {}).get(gpu, {}).get("alive"):
            break
        time.sleep(0.2)
    assert (view.get("probeHelpers") or {}).get(gpu, {}).get("alive"), view.get("probeHelpers")
    # claimable again: the claim's probe runs in the restarted helper
    k.patch(MI355XPOOLS, "p", {"spec": {"replicas": 1}}, "default")
    k.wait_for(MI355XPOOLS, "p", "default", ready_at(1), timeout=60)
    m = c.agent_request("gpu-node", "GET", "/metrics")
    lines = [ln for ln in m.splitlines() if ln.startswith(("gpupool_agent_release_helpers",
                                                           "gpupool_agent_claim_helper",
                                                           "gpupool_agent_probe_helper_"))]
    print("PARKING", json.dumps({"agentVramBeforeBytes": before, "tenantVramBytes": tenant_vram,
                                 "memUsedWithTenantBytes": used, "helperCounters": lines}))
    assert any(ln.startswith("gpupool_agent_probe_helper_unparks_total 1") for ln in lines)
    # the manager's RPCs to this agent were authenticated with the per-node MAC (edsig v2)
    assert 'gpupool_agent_rpc_signature_versions_total{version="v2"}' in m
