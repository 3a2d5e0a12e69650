"""The real multithreaded manager (informers, work-queue workers, agent long-poll watchers, event
recorder, metrics server) under ThreadSanitizer and ASan+UBSan through a scale/drain/fault/delete
scenario ('TSan covers the informer/workqueue/worker threads')."""
from __future__ import annotations

import os

import pytest

from gpupool.kube import MI355XJOBS, MI355XPOOLS, PODS

from .helpers import mi_pool, pause_pod, wait_ready
from tests.conftest import make_native

pytestmark = pytest.mark.slow
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@pytest.mark.parametrize("san", ["tsan", "asan"])
def test_manager_scenario_under_sanitizer(san, cluster_factory):
    r = make_native("host", san, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    os.environ["TSAN_OPTIONS"] = "halt_on_error=0:report_signal_unsafe=0"
    os.environ["ASAN_OPTIONS"] = "detect_leaks=0"
    c = cluster_factory(manager_bin=os.path.join(ROOT, "build", f"native-{san}", "gpupool-manager"),
                        manager_args=["--workers", "4", "--orphan-sweep", "300ms"])
    k = c.client
    k.create(MI355XPOOLS, mi_pool("a", 4, drain={"gracePeriodSeconds": 1}), "default")
    k.create(MI355XPOOLS, mi_pool("b", 2, resourceName="amd.com/gpu-b"), "default")
    wait_ready(k, "a", 4, timeout=60)
    wait_ready(k, "b", 2, timeout=60)
    k.create(PODS, pause_pod("w"), "default")
    k.wait_for(PODS, "w", "default", lambda o: o and o["status"].get("phase") == "Running", 30)
    c.set_faults("mi355x-node-0", {"devices": {"0": {"ecc": {"uncorrectable": 3}}}})
    k.patch(MI355XPOOLS, "a", {"spec": {"replicas": 1}}, "default")
    wait_ready(k, "a", 1, timeout=60)
    c.set_faults("mi355x-node-0", {})
    # Mi355xJob gang on pool b's GPUs: placement under the scheduling mutex, pod-informer driven
    # status, one gang restart (the first attempt fails), then success and TTL deletion
    k.create(MI355XJOBS, {"apiVersion": "compute.my.domain/v1alpha1", "kind": "Mi355xJob",
                          "metadata": {"name": "j"},
                          "spec": {"replicas": 2, "poolRef": "b", "backoffLimit": 2,
                                   "ttlSecondsAfterFinished": 1, "template": {"spec": {
                                       "terminationGracePeriodSeconds": 1, "containers": [{
                                           "name": "m", "command": ["bash", "-c",
                                                                    '[ "$GPUPOOL_JOB_ATTEMPT" != 1 ]'
                                                                    ]}]}}}}, "default")
    o = k.wait_for(MI355XJOBS, "j", "default", lambda o: o and (o.get("status") or {}).get(
        "phase") in ("Succeeded", "Failed"), timeout=60)
    assert o["status"]["phase"] == "Succeeded" and o["status"]["restarts"] == 1, o["status"]
    k.wait_for(MI355XJOBS, "j", "default", lambda o: o is None, timeout=60)
    # priority preemption: "hi" stops "lo" (capacity check on the victims' pods), "lo" resumes
    def gang(name, prio, cmd, **extra):
        return {"apiVersion": "compute.my.domain/v1alpha1", "kind": "Mi355xJob",
                "metadata": {"name": name},
                "spec": {"replicas": 2, "poolRef": "b", "priority": prio, **extra,
                         "template": {"spec": {"terminationGracePeriodSeconds": 1,
                                               "containers": [{"name": "m", "command": cmd}]}}}}
    k.create(MI355XJOBS, gang("lo", 0, ["sleep", "600"]), "default")
    k.wait_for(MI355XJOBS, "lo", "default", lambda o: (o.get("status") or {}).get("phase") == "Running",
               timeout=60)
    k.create(MI355XJOBS, gang("hi", 5, ["true"], preemptionPolicy="PreemptLowerPriority"), "default")
    k.wait_for(MI355XJOBS, "hi", "default", lambda o: (o.get("status") or {}).get("phase") == "Succeeded",
               timeout=60)
    lo = k.wait_for(MI355XJOBS, "lo", "default", lambda o: (o.get("status") or {}).get("phase") == "Running"
                    and o["status"].get("preemptions") == 1, timeout=60)
    for name in ("lo", "hi"):
        k.delete(MI355XJOBS, name, "default")
    # autoscaler: a pending pod grows an empty autoscaled pool, deleting it shrinks it again
    k.create(MI355XPOOLS, mi_pool("auto", 0, resourceName="amd.com/gpu-auto",
                                  drain={"gracePeriodSeconds": 1},
                                  autoscale={"enabled": True, "maxReplicas": 2,
                                             "scaleDownDelaySeconds": 0}), "default")
    k.create(PODS, pause_pod("aw", resource="amd.com/gpu-auto"), "default")
    wait_ready(k, "auto", 1, timeout=60)
    k.delete(PODS, "aw", "default")
    wait_ready(k, "auto", 0, timeout=60)
    k.delete(MI355XPOOLS, "auto", "default")
    # quota admission under concurrency: three pools created at once race for a quota of 3
    # (reservations under the quota mutex, settled after each status write)
    import threading
    from gpupool.kube import Res
    k.create(Res("", "v1", "resourcequotas"), {"metadata": {"name": "q"},
                                               "spec": {"hard": {"amd.com/gpu-q": "3"}}}, "quota")
    ts = [threading.Thread(target=k.create, args=(MI355XPOOLS, mi_pool(
        n, 2, resourceName="amd.com/gpu-q"), "quota")) for n in ("qa", "qb", "qc")]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    from .helpers import cond_is, ready_at
    objs = [k.wait_for(MI355XPOOLS, n, "quota", lambda o: ready_at(2)(o) or cond_is(
        "Progressing", "False", "QuotaExceeded")(o), timeout=60) for n in ("qa", "qb", "qc")]
    assert sum(1 for o in objs if ready_at(2)(o)) == 1
    for n in ("qa", "qb", "qc"):
        k.delete(MI355XPOOLS, n, "quota")
    for name in ("a", "b"):
        k.delete(MI355XPOOLS, name, "default")
    for name in ("a", "b"):
        k.wait_for(MI355XPOOLS, name, "default", lambda o: o is None, timeout=60)
    for n in ("qa", "qb", "qc"):
        k.wait_for(MI355XPOOLS, n, "quota", lambda o: o is None, timeout=60)
    c._kill("manager")
    log = c.log("manager")
    assert "WARNING: ThreadSanitizer" not in log, log[-8000:]
    assert "ERROR: AddressSanitizer" not in log and "runtime error:" not in log, log[-8000:]


def test_credential_reload_under_tsan(cluster_factory, tmp_path):
    """The rotating-token path (TokenSource re-read on 401 while informer watches, workers and
    agent feeds share it) under ThreadSanitizer, through two apiserver-token rotations."""
    r = make_native("host", "tsan", timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    os.environ["TSAN_OPTIONS"] = "halt_on_error=0:report_signal_unsafe=0"
    from .rotation import run_rotation
    out = run_rotation(cluster_factory, tmp_path,
                       manager_bin=os.path.join(ROOT, "build", "native-tsan", "gpupool-manager"))
    assert out["errors"] == 0 and out["reloads"] >= 2 and out["auth_401s"] > 0, out
    log = (tmp_path / "cluster0" / "manager.log").read_text()
    assert b"__tsan_init" in open(os.path.join(ROOT, "build", "native-tsan", "gpupool-manager"),
                                  "rb").read()  # really the TSan build
    assert "WARNING: ThreadSanitizer" not in log, log[-8000:]
