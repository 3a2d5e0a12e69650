"""Mi355xJob end-to-end on the fake 8x MI355X node: gang placement over pool-advertised GPUs,
torchrun/PET rendezvous env, gang restarts, queue order, deadline/TTL/cleanup, and the GoHai-style
``gpuctl trainjob`` verbs (reference GPU调度平台搭建.md:503-550 CLI, :638-675 Volcano Job,
:300-306 + :623 Kubeflow PET env)."""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

import pytest
import yaml

from gpupool.kube import MI355XJOBS, MI355XPOOLS, PODS, KubeError

from .helpers import conds, mi_pool, settled_events, wait_ready

pytestmark = pytest.mark.slow

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
def _free_port() -> int:
    """A rendezvous port no other DDP job on this host holds: pods run as host processes, and
    fixed per-worker bases collided between two test sessions running at once."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def job(name: str, replicas: int, command: list[str], gpus: int = 1, **spec) -> dict:
    return {"apiVersion": "compute.my.domain/v1alpha1", "kind": "Mi355xJob",
            "metadata": {"name": name},
            "spec": {"replicas": replicas, "gpusPerReplica": gpus, "masterPort": _free_port(),
                     "template": {"spec": {"terminationGracePeriodSeconds": 1,
                                           "containers": [{"name": "main", "command": command}]}},
                     **spec}}


def phase_is(*phases):
    return lambda o: bool(o) and (o.get("status") or {}).get("phase") in phases


def job_pods(k, name, ns="default"):
    return k.list(PODS, ns, label_selector=f"gpupool.amd.com/job-name={name}")["items"]


def env_of(pod) -> dict:
    return {e["name"]: e.get("value") for e in pod["spec"]["containers"][0].get("env", [])}


@pytest.fixture
def node8(cluster_factory):
    return cluster_factory()


def test_ddp_job_gang_runs_to_success(node8, tmp_path):
    """Two workers x 1 GPU of a pool run real DDP (gloo on CPU here) through the job's env."""
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("pool", 2), "default")
    wait_ready(k, "pool", 2)
    cmd = [sys.executable, os.path.join(ROOT, "examples", "fmnist_train.py"), "--synthetic",
           "--cpu", "--samples", "256", "--batch_size", "32", "--steps", "3", "--epochs", "1",
           "--output", str(tmp_path / "out")]
    k.create(MI355XJOBS, job("ddp", 2, cmd, poolRef="pool"), "default")
    o = k.wait_for(MI355XJOBS, "ddp", "default", phase_is("Succeeded", "Failed"), timeout=120)
    assert o["status"]["phase"] == "Succeeded", o["status"]
    st = o["status"]
    assert st["succeeded"] == 2 and st["restarts"] == 0 and st["attempt"] == 1
    c = conds(o)
    assert c["Scheduled"]["status"] == "True" and c["Succeeded"]["status"] == "True"
    devs = [r["devices"] for r in st["replicaStatuses"]]
    assert len(devs) == 2 and len(set(devs)) == 2  # distinct pool GPUs
    # completed pods are kept (cleanPodPolicy Running); rank 1 rendezvoused at rank 0's pod IP
    pods = {p["metadata"]["labels"]["gpupool.amd.com/replica-index"]: p for p in job_pods(k, "ddp")}
    e0, e1 = env_of(pods["0"]), env_of(pods["1"])
    assert e0["RANK"] == "0" and e1["RANK"] == "1" and e1["WORLD_SIZE"] == "2"
    assert e1["MASTER_ADDR"] == "127.0.0.1" and e0["PET_NNODES"] == "2"
    assert pods["1"]["spec"]["containers"][0]["resources"]["limits"]["amd.com/gpu"] == "1"
    log = open(pods["0"]["metadata"]["annotations"]["gpupool.amd.com/log-path"]).read()
    assert '"world": 2' in log or "'world': 2" in log, log[-2000:]
    deadline = time.time() + 10  # the manager's event recorder is asynchronous
    while True:
        reasons = [e["reason"] for e in settled_events(k)]
        if "JobSucceeded" in reasons or time.time() > deadline:
            break
        time.sleep(0.05)
    assert "GangScheduled" in reasons and "JobSucceeded" in reasons


def test_gang_is_all_or_nothing_and_queue_is_ordered(node8):
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("pool", 3), "default")
    wait_ready(k, "pool", 3)
    # can never fit (4 > 3 GPUs in the cluster): stays Unschedulable, creates nothing, blocks nobody
    k.create(MI355XJOBS, job("huge", 4, ["sleep", "30"]), "default")
    o = k.wait_for(MI355XJOBS, "huge", "default",
                   lambda o: conds(o).get("Scheduled", {}).get("reason") == "Unschedulable", timeout=20)
    assert o["status"]["phase"] == "Pending" and not job_pods(k, "huge")
    k.create(MI355XJOBS, job("a", 2, ["sleep", "2"]), "default")
    k.wait_for(MI355XJOBS, "a", "default", phase_is("Running"), timeout=30)
    # b needs 2 (1 free): waits; c needs 1 and would fit, but is queued behind b
    k.create(MI355XJOBS, job("b", 2, ["sleep", "1"]), "default")
    time.sleep(0.05)
    k.create(MI355XJOBS, job("c", 1, ["sleep", "1"]), "default")
    k.wait_for(MI355XJOBS, "c", "default",
               lambda o: conds(o).get("Scheduled", {}).get("reason") == "QueuedBehind", timeout=20)
    assert not job_pods(k, "c") and not job_pods(k, "b")
    for n in ("a", "b", "c"):
        o = k.wait_for(MI355XJOBS, n, "default", phase_is("Succeeded", "Failed"), timeout=60)
        assert o["status"]["phase"] == "Succeeded", (n, o["status"])
    # queue order is placement order (GangScheduled events, resourceVersion order): startTime is
    # when every worker runs, and c's one pod can be Running before both of b's placed beside it
    evs = sorted(settled_events(k), key=lambda e: int(e["metadata"]["resourceVersion"]))
    placed = [e["involvedObject"]["name"] for e in evs
              if e["reason"] == "GangScheduled" and e["involvedObject"]["name"] in ("a", "b", "c")]
    assert placed.index("a") < placed.index("b") < placed.index("c"), placed
    # a higher priority jumps the queue
    k.create(MI355XJOBS, job("hold", 3, ["sleep", "2"]), "default")
    k.wait_for(MI355XJOBS, "hold", "default", phase_is("Running"), timeout=30)
    k.create(MI355XJOBS, job("low", 1, ["sleep", "1"]), "default")
    time.sleep(0.05)
    k.create(MI355XJOBS, job("high", 3, ["sleep", "1"], priority=10), "default")
    for n in ("hold", "high", "low"):
        k.wait_for(MI355XJOBS, n, "default", phase_is("Succeeded"), timeout=60)
    # placement order from the GangScheduled events (each written once: resourceVersion order)
    evs = sorted(settled_events(k), key=lambda e: int(e["metadata"]["resourceVersion"]))
    placed = [e["involvedObject"]["name"] for e in evs
              if e["reason"] == "GangScheduled" and e["involvedObject"]["name"] in ("high", "low")]
    assert placed.index("high") < placed.index("low"), placed
    assert k.get(MI355XJOBS, "huge", "default")["status"]["phase"] == "Pending"


def test_gang_restart_then_backoff_limit(node8):
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("pool", 2), "default")
    wait_ready(k, "pool", 2)
    # rank 1 fails on the first attempt only -> the whole gang restarts once, then succeeds
    flaky = ["bash", "-c", 'if [ "$GPUPOOL_JOB_ATTEMPT" = 1 ] && [ "$RANK" = 1 ]; then exit 3; fi; sleep 0.5']
    k.create(MI355XJOBS, job("flaky", 2, flaky), "default")
    o = k.wait_for(MI355XJOBS, "flaky", "default", phase_is("Succeeded", "Failed"), timeout=60)
    assert o["status"]["phase"] == "Succeeded" and o["status"]["restarts"] == 1, o["status"]
    reasons = [e["reason"] for e in settled_events(k)
               if e["involvedObject"]["name"] == "flaky"]
    assert "GangRestarting" in reasons
    # always failing with backoffLimit 1: two attempts, then Failed/BackoffLimitExceeded
    k.create(MI355XJOBS, job("bad", 2, ["bash", "-c", "exit 7"], backoffLimit=1), "default")
    o = k.wait_for(MI355XJOBS, "bad", "default", phase_is("Succeeded", "Failed"), timeout=60)
    c = conds(o)
    assert o["status"]["phase"] == "Failed" and c["Failed"]["reason"] == "BackoffLimitExceeded"
    assert o["status"]["attempt"] == 2 and "exit code 7" in c["Failed"]["message"]
    # restartPolicy Never: the first failure is final
    k.create(MI355XJOBS, job("never", 1, ["false"], restartPolicy="Never"), "default")
    o = k.wait_for(MI355XJOBS, "never", "default", phase_is("Failed"), timeout=30)
    assert conds(o)["Failed"]["reason"] == "PodFailed" and o["status"]["attempt"] == 1


def test_deadline_ttl_and_delete_cleanup(node8):
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("pool", 2), "default")
    wait_ready(k, "pool", 2)
    k.create(MI355XJOBS, job("slow", 2, ["sleep", "60"], activeDeadlineSeconds=1), "default")
    o = k.wait_for(MI355XJOBS, "slow", "default", phase_is("Failed"), timeout=30)
    assert conds(o)["Failed"]["reason"] == "DeadlineExceeded"
    k.wait_for(PODS, "slow-worker-0", "default", lambda p: p is None, timeout=30)  # cleanPodPolicy
    # ttlSecondsAfterFinished: the job object goes away after it finished
    k.create(MI355XJOBS, job("ttl", 1, ["true"], ttlSecondsAfterFinished=0), "default")
    k.wait_for(MI355XJOBS, "ttl", "default", lambda o: o is None, timeout=30)
    # deleting a running job deletes its pods first (finalizer), freeing the GPUs
    k.create(MI355XJOBS, job("run", 2, ["sleep", "600"]), "default")
    k.wait_for(MI355XJOBS, "run", "default", phase_is("Running"), timeout=30)
    k.delete(MI355XJOBS, "run", "default")
    k.wait_for(MI355XJOBS, "run", "default", lambda o: o is None, timeout=30)
    assert not job_pods(k, "run")
    k.create(MI355XJOBS, job("after", 2, ["true"]), "default")  # both GPUs are free again
    k.wait_for(MI355XJOBS, "after", "default", phase_is("Succeeded"), timeout=30)


def test_pool_scale_down_evicts_worker_and_gang_waits(node8):
    """Elastic interplay: scaling the pool down drains a GPU under a running gang; the lost pod
    restarts the gang, which then waits (Unschedulable) until the pool grows back."""
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("pool", 2, drain={"gracePeriodSeconds": 1}), "default")
    wait_ready(k, "pool", 2)
    k.create(MI355XJOBS, job("train", 2, ["sleep", "600"], poolRef="pool"), "default")
    k.wait_for(MI355XJOBS, "train", "default", phase_is("Running"), timeout=30)
    k.patch(MI355XPOOLS, "pool", {"spec": {"replicas": 1}}, "default")
    o = k.wait_for(MI355XJOBS, "train", "default",
                   lambda o: conds(o).get("Scheduled", {}).get("reason") == "Unschedulable"
                   and o["status"].get("restarts", 0) >= 0 and o["status"]["phase"] == "Restarting",
                   timeout=60)
    assert conds(o)["Restarting"]["status"] == "True"
    wait_ready(k, "pool", 1)
    k.patch(MI355XPOOLS, "pool", {"spec": {"replicas": 2}}, "default")
    o = k.wait_for(MI355XJOBS, "train", "default", phase_is("Running"), timeout=60)
    assert o["status"]["attempt"] == 2 and o["status"]["restarts"] == 1


def test_invalid_job_is_rejected(node8):
    k = node8.client
    with pytest.raises(KubeError):
        k.create(MI355XJOBS, job("zero", 0, ["true"]), "default")
    with pytest.raises(KubeError):
        k.create(MI355XJOBS, job("pol", 1, ["true"], restartPolicy="Always"), "default")


def test_gpuctl_trainjob_verbs(node8, tmp_path):
    """GoHai CLI flow (GPU调度平台搭建.md:503-550): template -> create --dry-run -> create ->
    list -> logs -> template -s (export) -> create --bare -> delete."""
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("pool", 1), "default")
    wait_ready(k, "pool", 1)

    def gpuctl(*args, check=True):
        r = subprocess.run([os.path.join(ROOT, "bin", "gpuctl"), "--server",
                            node8.url, *args], capture_output=True, text=True, timeout=60)
        if check:
            assert r.returncode == 0, r.stderr
        return r.stdout
    tpl = yaml.safe_load(gpuctl("trainjob", "template"))
    assert tpl["mode"] == "single" and tpl["spec"]["singleInstanceType"].endswith("1gpu")
    tpl.update({"title": "CLI Demo_1", "command": "echo hello-from-$RANK", "mode": "Single"})
    f = tmp_path / "train_job_template.yaml"
    f.write_text(yaml.safe_dump(tpl))
    dry = yaml.safe_load(gpuctl("trainjob", "create", "-f", str(f), "--dry-run"))
    assert dry["kind"] == "Mi355xJob" and dry["metadata"]["name"] == "cli-demo-1"
    assert dry["spec"]["replicas"] == 1 and dry["spec"]["gpusPerReplica"] == 1
    assert "created" in gpuctl("trainjob", "create", "-f", str(f))
    k.wait_for(MI355XJOBS, "cli-demo-1", "default", phase_is("Succeeded"), timeout=30)
    assert "cli-demo-1" in gpuctl("trainjob", "list") and "Succeeded" in gpuctl("trainjob", "list")
    deadline = time.monotonic() + 15  # the kubelet annotates the log path asynchronously
    while "hello-from-0" not in (out := gpuctl("trainjob", "logs", "cli-demo-1")) and \
            time.monotonic() < deadline:
        time.sleep(0.2)
    assert "hello-from-0" in out
    exported = yaml.safe_load(gpuctl("trainjob", "template", "-s", "cli-demo-1"))
    assert exported["command"] == "echo hello-from-$RANK" and exported["title"] == "CLI Demo_1"
    bare = tmp_path / "job_full.yaml"
    bare.write_text(yaml.safe_dump(job("bare", 1, ["true"])))
    assert "created" in gpuctl("trainjob", "create", "-f", str(bare), "--bare")
    k.wait_for(MI355XJOBS, "bare", "default", phase_is("Succeeded"), timeout=30)
    gpuctl("trainjob", "delete", "bare")
    k.wait_for(MI355XJOBS, "bare", "default", lambda o: o is None, timeout=30)


def test_a_container_that_exits_at_once_runs_once_and_stays_succeeded(node8):
    """A container that exits before its pod's Running status is written: the exit is reported
    after it (the phase never goes back from Succeeded to Running, which made the job's cleanup
    delete the finished pod), and the pod is not admitted again by a watch event that still shows
    it Pending/Running (its log would then hold the output twice)."""
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("pool", 8), "default")
    wait_ready(k, "pool", 8)
    names = [f"quick-{i}" for i in range(8)]
    for n in names:
        k.create(MI355XJOBS, job(n, 1, ["echo", f"ran-{n}"], poolRef="pool"), "default")
    for n in names:
        k.wait_for(MI355XJOBS, n, "default", phase_is("Succeeded"), timeout=30)
    time.sleep(0.5)  # a late Running write or a second run would show by now
    for n in names:
        pods = job_pods(k, n)
        assert len(pods) == 1 and pods[0]["status"]["phase"] == "Succeeded", (n, pods)
        log_path = pods[0]["metadata"]["annotations"]["gpupool.amd.com/log-path"]
        with open(log_path) as f:
            assert f.read().split() == [f"ran-{n}"], n


def test_priority_preemption_picks_fewest_lowest_victims(node8):
    """Volcano preempt / PriorityClass semantics: a PreemptLowerPriority gang that does not fit
    stops only the lowest-priority jobs it needs, holds its reservation until their pods are gone,
    and the victims re-queue without spending their backoffLimit."""
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("pool", 4), "default")
    wait_ready(k, "pool", 4)
    k.create(MI355XJOBS, job("low", 2, ["sleep", "600"], priority=1), "default")
    k.create(MI355XJOBS, job("mid", 2, ["sleep", "600"], priority=5), "default")
    for n in ("low", "mid"):
        k.wait_for(MI355XJOBS, n, "default", phase_is("Running"), timeout=30)
    # Never (the default): a higher-priority gang just waits
    k.create(MI355XJOBS, job("polite", 2, ["sleep", "1"], priority=9), "default")
    o = k.wait_for(MI355XJOBS, "polite", "default",
                   lambda o: conds(o).get("Scheduled", {}).get("reason") == "Unschedulable", timeout=20)
    k.delete(MI355XJOBS, "polite", "default")
    k.wait_for(MI355XJOBS, "polite", "default", lambda o: o is None, timeout=30)
    # 2 GPUs needed: preempting "low" (priority 1) is enough, "mid" keeps running
    k.create(MI355XJOBS, job("urgent", 2, ["sleep", "1"], priority=10,
                             preemptionPolicy="PreemptLowerPriority"), "default")
    o = k.wait_for(MI355XJOBS, "urgent", "default", phase_is("Running", "Succeeded"), timeout=30)
    low = k.get(MI355XJOBS, "low", "default")
    assert low["status"]["phase"] in ("Restarting", "Pending"), low["status"]
    assert conds(low)["Restarting"]["reason"] == "Preempted"
    assert low["status"]["preemptions"] == 1 and low["status"]["restarts"] == 0
    mid = k.get(MI355XJOBS, "mid", "default")
    assert mid["status"]["phase"] == "Running" and not mid["status"].get("preemptions")
    reasons = {(e["involvedObject"]["name"], e["reason"]) for e in settled_events(k)}
    assert ("urgent", "Preempting") in reasons and ("low", "Preempted") in reasons
    # the preemptor never overlapped a victim's pod on a GPU
    devs_u = {r.get("devices") for r in
              k.wait_for(MI355XJOBS, "urgent", "default", phase_is("Succeeded"), timeout=30)
              ["status"]["replicaStatuses"]}
    assert len(devs_u) == 2
    # once urgent is done the victim is placed again and runs (attempt 2, still 0 restarts)
    low = k.wait_for(MI355XJOBS, "low", "default", phase_is("Running"), timeout=30)
    assert low["status"]["attempt"] == 2 and low["status"]["restarts"] == 0
    # equal priority is never preempted
    k.create(MI355XJOBS, job("peer", 2, ["sleep", "1"], priority=5,
                             preemptionPolicy="PreemptLowerPriority"), "default")
    o = k.wait_for(MI355XJOBS, "peer", "default", phase_is("Running", "Succeeded"), timeout=30)
    assert k.get(MI355XJOBS, "mid", "default")["status"]["phase"] == "Running"
    assert k.get(MI355XJOBS, "low", "default")["status"]["preemptions"] == 2


def test_suspend_frees_gpus_and_resume_requeues(node8):
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("pool", 2), "default")
    wait_ready(k, "pool", 2)
    k.create(MI355XJOBS, job("s", 2, ["sleep", "600"], activeDeadlineSeconds=3600), "default")
    k.wait_for(MI355XJOBS, "s", "default", phase_is("Running"), timeout=30)
    k.patch(MI355XJOBS, "s", {"spec": {"suspend": True}}, "default")
    o = k.wait_for(MI355XJOBS, "s", "default", lambda o: phase_is("Suspended")(o) and not job_pods(k, "s"),
                   timeout=30)
    assert conds(o)["Suspended"]["status"] == "True" and not o["status"].get("startTime")
    # its GPUs are usable by another gang meanwhile
    k.create(MI355XJOBS, job("other", 2, ["true"]), "default")
    k.wait_for(MI355XJOBS, "other", "default", phase_is("Succeeded"), timeout=30)
    r = subprocess.run([os.path.join(ROOT, "bin", "gpuctl"), "--server", node8.url, "trainjob",
                        "resume", "s"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "resumed" in r.stdout, r.stderr
    o = k.wait_for(MI355XJOBS, "s", "default", phase_is("Running"), timeout=30)
    assert conds(o)["Suspended"]["reason"] == "Resumed" and o["status"]["restarts"] == 0
    assert o["status"]["attempt"] == 2


def test_queue_admission_capability_state_and_status(node8):
    """Volcano Queue semantics on Mi355xQueue: a named queue must exist, its capability bounds the
    GPUs its placed jobs hold (even with free GPUs), Closed stops new placements, and the queue's
    status reports job counts and allocated GPUs."""
    from gpupool.kube import MI355XQUEUES
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("pool", 4), "default")
    wait_ready(k, "pool", 4)
    k.create(MI355XJOBS, job("orphan", 1, ["true"], queue="research"), "default")
    k.wait_for(MI355XJOBS, "orphan", "default",
               lambda o: conds(o).get("Scheduled", {}).get("reason") == "QueueNotFound", timeout=20)
    k.create(MI355XQUEUES, {"apiVersion": "compute.my.domain/v1alpha1", "kind": "Mi355xQueue",
                            "metadata": {"name": "research"},
                            "spec": {"capability": {"amd.com/gpu": 2}}}, None)
    k.wait_for(MI355XJOBS, "orphan", "default", phase_is("Succeeded"), timeout=30)  # queue wakes it
    for n in ("qa", "qb", "qc"):
        k.create(MI355XJOBS, job(n, 1, ["sleep", "600"], queue="research"), "default")
        time.sleep(0.05)
    for n in ("qa", "qb"):
        k.wait_for(MI355XJOBS, n, "default", phase_is("Running"), timeout=30)
    o = k.wait_for(MI355XJOBS, "qc", "default",
                   lambda o: conds(o).get("Scheduled", {}).get("reason") == "QueueOverCapacity",
                   timeout=20)
    assert "capability 2" in conds(o)["Scheduled"]["message"]
    # other queues still use the two free GPUs
    k.create(MI355XJOBS, job("dflt", 2, ["true"]), "default")
    k.wait_for(MI355XJOBS, "dflt", "default", phase_is("Succeeded"), timeout=30)
    q = k.wait_for(MI355XQUEUES, "research", None, lambda q: (q.get("status") or {}).get("running") == 2
                   and q["status"].get("pending") == 1 and q["status"].get("completed") == 1,
                   timeout=20)
    assert q["status"]["allocated"] == {"amd.com/gpu": 2} and q["status"]["state"] == "Open"
    metrics = node8.manager_metrics()
    assert 'gpupool_queue_jobs{phase="Running",queue="research"} 2' in metrics
    assert 'gpupool_queue_allocated_gpus{queue="research",resource="amd.com/gpu"} 2' in metrics
    assert "gpupool_job_gang_wait_seconds_bucket" in metrics
    r = subprocess.run([os.path.join(ROOT, "bin", "gpuctl"), "--server", node8.url, "get", "mxq"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "research" in r.stdout and "Open" in r.stdout, r.stdout + r.stderr
    # Closed: freed capability is not used; reopening admits the waiting job
    k.patch(MI355XQUEUES, "research", {"spec": {"state": "Closed"}}, None)
    k.delete(MI355XJOBS, "qa", "default")
    k.wait_for(MI355XJOBS, "qc", "default",
               lambda o: conds(o).get("Scheduled", {}).get("reason") == "QueueClosed", timeout=20)
    k.patch(MI355XQUEUES, "research", {"spec": {"state": "Open"}}, None)
    k.wait_for(MI355XJOBS, "qc", "default", phase_is("Running"), timeout=30)
    q = k.wait_for(MI355XQUEUES, "research", None,
                   lambda q: (q.get("status") or {}).get("running") == 2, timeout=20)
    assert q["status"]["pending"] == 0


def test_cross_queue_preemption_respects_reclaimable(node8):
    from gpupool.kube import MI355XQUEUES
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("pool", 2), "default")
    wait_ready(k, "pool", 2)
    k.create(MI355XQUEUES, {"apiVersion": "compute.my.domain/v1alpha1", "kind": "Mi355xQueue",
                            "metadata": {"name": "prod"}, "spec": {"reclaimable": False}}, None)
    k.create(MI355XJOBS, job("svc", 2, ["sleep", "600"], queue="prod", priority=0), "default")
    k.wait_for(MI355XJOBS, "svc", "default", phase_is("Running"), timeout=30)
    k.create(MI355XJOBS, job("burst", 2, ["true"], priority=10,
                             preemptionPolicy="PreemptLowerPriority"), "default")
    k.wait_for(MI355XJOBS, "burst", "default",
               lambda o: conds(o).get("Scheduled", {}).get("reason") == "Unschedulable", timeout=20)
    assert k.get(MI355XJOBS, "svc", "default")["status"]["phase"] == "Running"
    k.patch(MI355XQUEUES, "prod", {"spec": {"reclaimable": True}}, None)  # wakes waiting jobs
    k.wait_for(MI355XJOBS, "burst", "default", phase_is("Succeeded"), timeout=30)
    assert k.get(MI355XJOBS, "svc", "default")["status"]["preemptions"] == 1


def test_gang_spans_nodes_with_torchrun_env(cluster_factory):
    """A 2 x 4-GPU gang on two 4-GPU nodes: one pod per node, rank 0 on the first, PET_* env for
    torchrun with nnodes 2 / nproc-per-node 4, and every worker pointed at rank 0's pod IP."""
    from gpupool.testing.cluster import NodeSpec
    c = cluster_factory(nodes=[NodeSpec("node-a", count=4), NodeSpec("node-b", count=4)])
    k = c.client
    k.create(MI355XPOOLS, mi_pool("pa", 4, nodeName="node-a"), "default")
    k.create(MI355XPOOLS, mi_pool("pb", 4, nodeName="node-b"), "default")
    wait_ready(k, "pa", 4)
    wait_ready(k, "pb", 4)
    k.create(MI355XJOBS, job("wide", 2, ["sleep", "600"], gpus=4), "default")
    o = k.wait_for(MI355XJOBS, "wide", "default", phase_is("Running"), timeout=30)
    assert sorted(s["node"] for s in o["status"]["placement"]) == ["node-a", "node-b"]
    pods = {p["metadata"]["labels"]["gpupool.amd.com/replica-index"]: p for p in job_pods(k, "wide")}
    assert {pods["0"]["spec"]["nodeName"], pods["1"]["spec"]["nodeName"]} == {"node-a", "node-b"}
    e0, e1 = env_of(pods["0"]), env_of(pods["1"])
    assert e0["PET_NNODES"] == e1["PET_NNODES"] == "2"
    assert e0["PET_NPROC_PER_NODE"] == "4" and e1["PET_NODE_RANK"] == "1"
    assert e1["MASTER_ADDR"] == pods["0"]["status"]["podIP"]
    for p in pods.values():
        assert len(p["metadata"]["annotations"]["gpupool.amd.com/devices"].split(",")) == 4
    # the cluster is full: a 1-GPU job waits, and gets a GPU once the gang is deleted
    k.create(MI355XJOBS, job("small", 1, ["true"]), "default")
    k.wait_for(MI355XJOBS, "small", "default",
               lambda o: conds(o).get("Scheduled", {}).get("reason") == "Unschedulable", timeout=20)
    k.delete(MI355XJOBS, "wide", "default")
    k.wait_for(MI355XJOBS, "small", "default", phase_is("Succeeded"), timeout=30)


def test_elastic_gang_min_available(node8):
    """Volcano minAvailable: a 4-replica job with minAvailable 2 starts with the 3 GPUs free, its
    world size (status.workers, PET_NNODES, WORLD_SIZE) is 3, and it succeeds with 3 workers; with
    fewer than minAvailable GPUs free it waits."""
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("pool", 3), "default")
    wait_ready(k, "pool", 3)
    k.create(MI355XJOBS, job("el", 4, ["sleep", "1"], minAvailable=2), "default")
    o = k.wait_for(MI355XJOBS, "el", "default", phase_is("Running", "Succeeded"), timeout=30)
    assert o["status"]["workers"] == 3 and len(o["status"]["placement"]) == 3
    pods = job_pods(k, "el")
    assert len(pods) == 3
    for p in pods:
        e = env_of(p)
        assert e["WORLD_SIZE"] == "3" and e["PET_NNODES"] == "3"
    o = k.wait_for(MI355XJOBS, "el", "default", phase_is("Succeeded"), timeout=30)
    assert o["status"]["succeeded"] == 3
    # 2 of 3 GPUs busy: a minAvailable-2 gang cannot start on the 1 left
    k.create(MI355XJOBS, job("busy", 2, ["sleep", "600"]), "default")
    k.wait_for(MI355XJOBS, "busy", "default", phase_is("Running"), timeout=30)
    k.create(MI355XJOBS, job("el2", 4, ["true"], minAvailable=2), "default")
    o = k.wait_for(MI355XJOBS, "el2", "default",
                   lambda o: conds(o).get("Scheduled", {}).get("reason") == "Unschedulable", timeout=20)
    assert "gang of 2..4" in conds(o)["Scheduled"]["message"]
    k.delete(MI355XJOBS, "busy", "default")
    o = k.wait_for(MI355XJOBS, "el2", "default", phase_is("Succeeded"), timeout=30)
    # the gang starts as soon as minAvailable GPUs are free: busy's two pods end one by one, so it
    # sees 2 or (when both endings land in one pass) 3 — elastic, never below minAvailable
    assert 2 <= o["status"]["workers"] <= 3 and o["status"]["succeeded"] == o["status"]["workers"]


def test_gpu_fault_under_running_gang_restarts_it_on_healthy_gpus(node8):
    """Failure handling end to end: an uncorrectable ECC error on a GPU under a running gang makes
    the pool replace that GPU (drain evicts the worker), the job restarts the whole gang (PodLost)
    and runs again on healthy GPUs only."""
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("pool", 2, drain={"gracePeriodSeconds": 1}), "default")
    wait_ready(k, "pool", 2)
    k.create(MI355XJOBS, job("tr", 2, ["sleep", "600"], poolRef="pool"), "default")
    o = k.wait_for(MI355XJOBS, "tr", "default", phase_is("Running"), timeout=30)
    victim = o["status"]["replicaStatuses"][0]["devices"]
    node8.set_faults("mi355x-node-0", {"devices": {victim: {"ecc": {"uncorrectable": 2}}}})
    o = k.wait_for(MI355XJOBS, "tr", "default",
                   lambda o: phase_is("Running")(o) and o["status"]["attempt"] == 2, timeout=60)
    assert o["status"]["restarts"] == 1
    assert conds(o)["Restarting"]["reason"] == "Restarted"
    assert any(e["reason"] == "GangRestarting" and e["involvedObject"]["name"] == "tr"
               for e in settled_events(k))
    devs = {r["devices"] for r in o["status"]["replicaStatuses"]}
    assert victim not in devs and len(devs) == 2
    node8.set_faults("mi355x-node-0", {})


def test_gpuctl_get_watch_streams_rows(node8):
    """`gpuctl get mxp NAME -w` (kubectl get -w, GPU调度平台搭建.md:682): the table, then a row per
    change until the watch times out."""
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("wp", 1), "default")
    wait_ready(k, "wp", 1)
    proc = subprocess.Popen([os.path.join(ROOT, "bin", "gpuctl"), "--server", node8.url, "get", "mxp",
                             "wp", "-w", "--watch-timeout", "4"], stdout=subprocess.PIPE, text=True)
    # the table is printed before the watch starts: change the pool only once it is out (a
    # loaded host can take more than a second to start the CLI)
    head = [proc.stdout.readline(), proc.stdout.readline()]
    k.patch(MI355XPOOLS, "wp", {"spec": {"replicas": 3}}, "default")
    wait_ready(k, "wp", 3)
    out, _ = proc.communicate(timeout=30)
    lines = [x for x in head + out.splitlines() if x.strip()]
    assert lines[0].startswith("NAME") and "wp" in lines[1]
    assert any(x.split()[:3] == ["wp", "3", "3"] for x in lines[2:]), "".join(head) + out


def test_gpuctl_login_contexts_whoami(node8, tmp_path):
    """GoHai CLI identity verbs (GPU调度平台搭建.md:461-482): login stores a token in a context,
    config get-contexts lists them, whoami reports the server/namespace/credential in use."""
    env = {**os.environ, "GPUPOOL_CONFIG": str(tmp_path / "cfg.yaml")}

    def gpuctl(*args, stdin=None):
        r = subprocess.run([os.path.join(ROOT, "bin", "gpuctl"), *args], capture_output=True,
                           text=True, timeout=60, env=env, input=stdin)
        assert r.returncode == 0, r.stdout + r.stderr
        return r.stdout
    gpuctl("config", "set-context", "lab", "--server", node8.url, "--namespace", "team-a")
    assert "logged in: context lab" in gpuctl("login", "--context-name", "lab", stdin="tok-123\n")
    cfg = yaml.safe_load(open(tmp_path / "cfg.yaml"))
    assert cfg["contexts"]["lab"]["token"] == "tok-123" and cfg["current-context"] == "lab"
    assert "*   lab" in gpuctl("config", "get-contexts")
    who = gpuctl("whoami")
    assert node8.url in who and "team-a" in who and "bearer token" in who and "reachable:  yes" in who


def test_restarted_gang_resumes_from_checkpoint(node8, tmp_path):
    """Elastic recovery end to end: a 2-rank DDP job with spec.checkpointDir checkpoints every 5
    steps; attempt 1 dies at step 12, the gang restarts and attempt 2 resumes at step 10 (the
    last checkpoint), not at 0, and finishes the 20 steps."""
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("pool", 2), "default")
    wait_ready(k, "pool", 2)
    cmd = [sys.executable, os.path.join(ROOT, "examples", "fmnist_train.py"), "--synthetic",
           "--cpu", "--samples", "2048", "--batch_size", "32", "--steps", "20", "--epochs", "1",
           "--checkpoint_every", "5", "--fail_at_step", "12", "--output", str(tmp_path / "out")]
    k.create(MI355XJOBS, job("ck", 2, cmd, poolRef="pool", checkpointDir=str(tmp_path / "ckpt")),
             "default")
    o = k.wait_for(MI355XJOBS, "ck", "default", phase_is("Succeeded", "Failed"), timeout=180)
    assert o["status"]["phase"] == "Succeeded" and o["status"]["restarts"] == 1, o["status"]
    pod0 = next(p for p in job_pods(k, "ck")
                if p["metadata"]["labels"]["gpupool.amd.com/replica-index"] == "0")
    assert env_of(pod0)["GPUPOOL_CHECKPOINT_DIR"] == str(tmp_path / "ckpt")
    log = open(pod0["metadata"]["annotations"]["gpupool.amd.com/log-path"]).read()
    events = [json.loads(x) for x in log.splitlines() if x.startswith("{")]
    resume = next(e for e in events if e["event"] == "resume")
    done = next(e for e in events if e["event"] == "done")
    assert resume["step"] == 10 and done["steps"] == 20 and done["world"] == 2


def test_reference_job_manifests_apply_unchanged(node8, tmp_path):
    """A user of the reference platform keeps their manifests: `gpuctl apply -f` of a Volcano Job
    (GPU调度平台搭建.md:643-672 shape) and of a Kubeflow PyTorchJob converts each to a Mi355xJob
    gang on pool GPUs, which runs to success (the PyTorchJob as real 2-rank DDP; here gloo on
    CPU). Only the command is swapped for a CPU-runnable one."""
    k = node8.client
    k.create(MI355XPOOLS, mi_pool("pool", 2), "default")
    wait_ready(k, "pool", 2)
    train = [sys.executable, os.path.join(ROOT, "examples", "fmnist_train.py"), "--synthetic",
             "--cpu", "--samples", "256", "--batch_size", "32", "--steps", "3", "--epochs", "1",
             "--output", str(tmp_path / "out")]
    vc = yaml.safe_load(open(os.path.join(ROOT, "config", "samples", "foreign",
                                          "volcano_fashion_mnist_job.yaml")))
    ct = vc["spec"]["tasks"][0]["template"]["spec"]["containers"][0]
    ct["command"], ct["args"] = train, []
    pt = yaml.safe_load(open(os.path.join(ROOT, "config", "samples", "foreign",
                                          "kubeflow_pytorchjob.yaml")))
    for spec in pt["spec"]["pytorchReplicaSpecs"].values():
        spec["template"]["spec"]["containers"][0]["command"] = train
    files = []
    for name, doc in (("vc.yaml", vc), ("ptj.yaml", pt)):
        p = tmp_path / name
        p.write_text(yaml.safe_dump(doc))
        files.append(str(p))
    env = dict(os.environ, PYTHONPATH=ROOT, GPUPOOL_APISERVER=node8.url)
    for f in files:
        r = subprocess.run([sys.executable, "-m", "gpupool.cli", "apply", "-f", f], cwd=ROOT,
                           env=env, capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr
        assert "to Mi355xJob" in r.stderr and "mi355xjob" in r.stdout, (r.stdout, r.stderr)
    o = k.wait_for(MI355XJOBS, "fashion-mnist-job", "default", phase_is("Succeeded", "Failed"),
                   timeout=120)
    assert o["status"]["phase"] == "Succeeded", o["status"]
    assert o["metadata"]["annotations"]["gpupool.amd.com/converted-from"] == \
        "batch.volcano.sh/v1alpha1/Job"
    o = k.wait_for(MI355XJOBS, "fmnist-ddp", "default", phase_is("Succeeded", "Failed"),
                   timeout=180)
    assert o["status"]["phase"] == "Succeeded" and o["status"]["succeeded"] == 2, o["status"]
    pods = {p["metadata"]["labels"]["gpupool.amd.com/replica-index"]: p
            for p in job_pods(k, "fmnist-ddp")}
    assert env_of(pods["1"])["WORLD_SIZE"] == "2" and env_of(pods["0"])["RANK"] == "0"
