"""Scenario runners behind ``bench.py`` — one per BASELINE.json config that has a number.

* ``cycle(n)``        configs 2/3: one pool, replicas 0 -> n timed to Ready at the new generation,
                      ground truth checked at n, then n -> 0 (reference scale-up loop,
                      README.md:199-209, plus the re-observe the reference lacks, :225);
* ``scale_down(n)``   config 4: n GPUs each running a pod, replicas n -> n//2 timed until the pool
                      is Ready at n//2 with the victims drained (pods evicted) and released
                      (reference scale-down loop README.md:210-222, which deletes without drain);
* ``two_pools(n)``    config 5: pools A and B of n//2 GPUs each, created together, timed until
                      both are Ready; per-pool ground truth; no device in both;
* ``health(pool)``    config 5 health Conditions: an uncorrectable-ECC fault on one claimed GPU
                      -> HBMECCHealthy=False + Degraded=True, timed three ways: detected by the
                      agent's 100 ms health poll (as a real ECC counter change is),
                      delivered as an event (overlay rewrite -> inotify, like an amdsmi event),
                      and with a forced sample (reaction only); then cleared -> Ready again.

Every pool in a run owns its own extended resource so the kubelet's per-resource view is an
independent ownership oracle (``ground_truth.pool_truth``).
"""
from __future__ import annotations

import statistics
import time
from dataclasses import dataclass, field

from ..kube import AZUREVMPOOLS, MI355XPOOLS, PODS, SECRETS, KubeError
from . import ground_truth as gt


def conds(o: dict | None) -> dict:
    return {x["type"]: x for x in ((o or {}).get("status") or {}).get("conditions", [])}


def ready_at(r: int):
    def pred(o):
        if not o:
            return False
        st = o.get("status") or {}
        return st.get("observedGeneration") == o["metadata"]["generation"] and \
            st.get("readyReplicas") == r and len(st.get("devices", [])) == r and \
            conds(o).get("Ready", {}).get("status") == "True"
    return pred


def pctl(xs: list[float], q: float) -> float | None:
    if not xs:
        return None
    s = sorted(xs)
    return s[min(len(s) - 1, int(q * len(s)))]


def summary(xs: list[float], ok: int | None = None) -> dict:
    out = {"n": len(xs), "p50_s": round(statistics.median(xs), 4) if xs else None,
           "p90_s": round(pctl(xs, 0.9), 4) if xs else None,
           "max_s": round(max(xs), 4) if xs else None}
    if ok is not None:
        out["accuracy"] = ok / len(xs) if xs else None
    return out


@dataclass
class BenchRun:
    cluster: object
    node: object                  # gpupool.testing.cluster.NodeSpec
    real: bool
    hbm_bytes: int = 1 << 30
    timeout: float = 120.0
    ns: str = "default"
    baseline_cli: dict = field(default_factory=dict)
    healthy: set = field(default_factory=set)
    gt_s: float = 0.0             # time spent in ground-truth reads (reported separately)

    @property
    def c(self):
        return self.cluster.client

    @property
    def pr_socket(self) -> str:
        import os
        return os.path.join(self.cluster.kubelet_root(self.node), "pod-resources", "kubelet.sock")

    @property
    def state_dir(self) -> str:
        import os
        return os.path.join(self.cluster.workdir, f"state-{self.node.name}")

    # ------------------------------------------------------------ ground truth
    def refresh_health(self) -> set[str]:
        """Independent device health (amd-smi CLI on hardware; fixture + overlay files on the
        fake backend). The CLI costs ~0.7 s, so it is read once per bench step, not per cycle."""
        t0 = time.perf_counter()
        if self.real:
            st = gt.cli_state()
            if not self.baseline_cli:
                self.baseline_cli = st
            self.healthy = gt.healthy_from_cli(st, self.baseline_cli)
        else:
            self.healthy = gt.healthy_uuids_fixture(self.node.fixture,
                                                    self.cluster.faults_path(self.node.name),
                                                    self.node.name)
        self.gt_s += time.perf_counter() - t0
        return self.healthy

    def truth(self, pool: dict) -> dict:
        t0 = time.perf_counter()
        try:
            return gt.pool_truth(self.pr_socket, pool["spec"]["resourceName"], self.healthy,
                                 self.state_dir, pool["metadata"]["uid"])
        finally:
            self.gt_s += time.perf_counter() - t0

    def wait_truth(self, pool: dict, want: int, timeout: float = 5.0) -> dict:
        """The kubelet learns the device set through ListAndWatch asynchronously (like a real
        kubelet); give it a bounded moment to converge before judging accuracy."""
        deadline = time.monotonic() + timeout
        while True:
            t = self.truth(pool)
            if (t["ready"] == want and t.get("ledgerAgrees", True)) or time.monotonic() > deadline:
                return t
            time.sleep(0.01)

    # ------------------------------------------------------------ pools
    def make_pool(self, name: str, resource: str, replicas: int = 0, **spec) -> dict:
        body = {"apiVersion": "compute.my.domain/v1alpha1", "kind": "Mi355xPool",
                "metadata": {"name": name},
                "spec": {"replicas": replicas, "nodeName": self.node.name,
                         "resourceName": resource,
                         "drain": {"gracePeriodSeconds": 1},
                         "probe": {"enabled": True, "hbmBytes": self.hbm_bytes, "mfma": True},
                         **spec}}
        try:
            return self.c.create(MI355XPOOLS, body, self.ns)
        except KubeError as e:
            if e.code != 409:
                raise
            return self.c.get(MI355XPOOLS, name, self.ns)

    def scale(self, name: str, r: int, wait: bool = True) -> dict | None:
        self.c.patch(MI355XPOOLS, name, {"spec": {"replicas": r}}, self.ns)
        if wait:
            return self.c.wait_for(MI355XPOOLS, name, self.ns, ready_at(r), timeout=self.timeout)
        return None

    def delete_pool(self, name: str) -> None:
        try:
            self.c.delete(MI355XPOOLS, name, self.ns)
        except KubeError as e:
            if e.code != 404:
                raise
        self.c.wait_for(MI355XPOOLS, name, self.ns, lambda o: o is None, timeout=self.timeout)

    # ------------------------------------------------------------ config 2/3
    def cycle(self, pool: dict, n: int) -> dict:
        name = pool["metadata"]["name"]
        patch_at = time.time()  # wall clock, to place the manager's trace of this cycle
        t0 = time.perf_counter()
        obj = self.scale(name, n)
        t_ready = time.perf_counter() - t0
        ready_at_wall = patch_at + t_ready
        truth = self.wait_truth(pool, n)
        ok = truth["ready"] == obj["status"]["readyReplicas"] == n and truth.get("ledgerAgrees", True)
        self.scale(name, 0)
        return {"n": n, "readySeconds": t_ready, "ok": ok, "truth": truth,
                "patchAt": patch_at, "readyAtWall": ready_at_wall,
                "probeMs": [round(d.get("probe", {}).get("ms", 0.0), 3)
                            for d in obj["status"]["devices"]]}

    # ------------------------------------------------------------ config 4
    def _pods(self, prefix: str, n: int, resource: str) -> list[str]:
        names = []
        for i in range(n):
            nm = f"{prefix}-{i}"
            self.c.create(PODS, {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": nm},
                                 "spec": {"terminationGracePeriodSeconds": 1,
                                          "containers": [{"name": "main", "command": ["sleep", "600"],
                                                          "resources": {"limits": {resource: 1}}}]}},
                          self.ns)
            names.append(nm)
        for nm in names:
            self.c.wait_for(PODS, nm, self.ns,
                            lambda o: bool(o) and o["status"].get("phase") == "Running",
                            timeout=self.timeout)
        return names

    def _delete_pods(self, names: list[str]) -> None:
        for nm in names:
            try:
                self.c.delete(PODS, nm, self.ns, grace=0)
            except KubeError as e:
                if e.code != 404:
                    raise
        for nm in names:
            self.c.wait_for(PODS, nm, self.ns, lambda o: o is None, timeout=self.timeout)

    def scale_down(self, pool: dict, n: int, step: int) -> dict:
        """n GPUs busy with one pod each -> replicas n//2: cordon, evict, wait, release."""
        name, res = pool["metadata"]["name"], pool["spec"]["resourceName"]
        keep = n // 2
        self.scale(name, n)
        pods = self._pods(f"sd{step}", n, res)
        t0 = time.perf_counter()
        obj = self.scale(name, keep)
        dt = time.perf_counter() - t0
        kept = {d["uuid"] for d in obj["status"]["devices"]}
        truth = self.wait_truth(pool, keep)
        left = [p for p in self.c.list(PODS, self.ns)["items"]
                if p["metadata"]["name"] in pods and not p["metadata"].get("deletionTimestamp")]
        on_released = [p["metadata"]["name"] for p in left
                       if not set((p["metadata"].get("annotations") or {})
                                  .get("gpupool.amd.com/devices", "").split(",")) <= kept]
        ok = truth["ready"] == obj["status"]["readyReplicas"] == keep and \
            truth.get("ledgerAgrees", True) and not on_released and len(left) == keep
        self._delete_pods([p["metadata"]["name"] for p in left])
        self.scale(name, 0)
        return {"from": n, "to": keep, "seconds": dt, "ok": ok, "evicted": n - len(left),
                "podsOnReleasedGPUs": on_released, "truth": truth}

    # ------------------------------------------------------------ config 5
    def two_pools(self, n: int, step: int) -> dict:
        half = n // 2
        a = self.make_pool(f"team-a-{step}", "amd.com/gpu-team-a", 0)
        b = self.make_pool(f"team-b-{step}", "amd.com/gpu-team-b", 0)
        t0 = time.perf_counter()
        self.scale(a["metadata"]["name"], half, wait=False)
        self.scale(b["metadata"]["name"], half, wait=False)
        oa = self.c.wait_for(MI355XPOOLS, a["metadata"]["name"], self.ns, ready_at(half),
                             timeout=self.timeout)
        ob = self.c.wait_for(MI355XPOOLS, b["metadata"]["name"], self.ns, ready_at(half),
                             timeout=self.timeout)
        dt = time.perf_counter() - t0
        ta, tb = self.wait_truth(a, half), self.wait_truth(b, half)
        ua = {d["uuid"] for d in oa["status"]["devices"]}
        ub = {d["uuid"] for d in ob["status"]["devices"]}
        ok = ta["ready"] == tb["ready"] == half and not (ua & ub) and \
            ta.get("ledgerAgrees", True) and tb.get("ledgerAgrees", True)
        self.delete_pool(a["metadata"]["name"])
        self.delete_pool(b["metadata"]["name"])
        return {"pools": [half, half], "seconds": dt, "ok": ok, "crossPoolDevices": len(ua & ub),
                "truth": {"a": ta, "b": tb}}

    # ------------------------------------------------------------ config 1
    def azure_pool(self, step: int, replicas: int = 0) -> dict:
        """BASELINE config 1: an AzureVmPool (the reference's own kind) created from scratch on the
        same manager with the in-process cloud: create -> Ready (finalizer added, credentials
        resolved, VMs listed by tag), then delete -> gone (finalizer-guarded cleanup)."""
        import base64
        if step == 0:
            data = {k: base64.b64encode(v.encode()).decode() for k, v in {
                "AZURE_CLIENT_ID": "00000000-0000-0000-0000-000000000001",
                "AZURE_CLIENT_SECRET": "bench", "AZURE_TENANT_ID": "00000000-0000-0000-0000-000000000002",
                "AZURE_SUBSCRIPTION_ID": "00000000-0000-0000-0000-000000000003"}.items()}
            try:
                self.c.create(SECRETS, {"apiVersion": "v1", "kind": "Secret",
                                        "metadata": {"name": "azure-credentials"}, "data": data},
                              self.ns)
            except KubeError as e:
                if e.code != 409:
                    raise
        name = f"az-bench-{step}"
        body = {"apiVersion": "compute.my.domain/v1alpha1", "kind": "AzureVmPool",
                "metadata": {"name": name},
                "spec": {"replicas": replicas, "resourceGroupName": "bench-rg", "location": "eastus",
                         "vmSize": "Standard_ND_MI300X_v5", "vnetName": "vnet", "subnetName": "default",
                         "imageReference": {"publisher": "Canonical", "offer": "ubuntu-24_04-lts",
                                            "sku": "server", "version": "latest"},
                         "azureCredentialSecret": "azure-credentials"}}

        def ready(o):
            st = (o or {}).get("status") or {}
            c = {x["type"]: x for x in st.get("conditions", [])}
            return bool(o) and st.get("observedGeneration") == o["metadata"]["generation"] and \
                st.get("readyReplicas", 0) == replicas and len(st.get("vms") or []) == replicas and \
                c.get("Ready", {}).get("status") == "True"
        t0 = time.perf_counter()
        self.c.create(AZUREVMPOOLS, body, self.ns)
        o = self.c.wait_for(AZUREVMPOOLS, name, self.ns, ready, timeout=self.timeout)
        t_ready = time.perf_counter() - t0
        fin = "compute.my.domain/device-release" in (o["metadata"].get("finalizers") or [])
        t1 = time.perf_counter()
        self.c.delete(AZUREVMPOOLS, name, self.ns)
        self.c.wait_for(AZUREVMPOOLS, name, self.ns, lambda x: x is None, timeout=self.timeout)
        return {"seconds": t_ready, "deleteSeconds": time.perf_counter() - t1,
                "ok": fin and o["status"]["readyReplicas"] == replicas}

    def agent_stats(self) -> dict:
        """The agent's own counters (gpupool_agent_*): sample / health-poll cost, events."""
        text = self.cluster.agent_request(self.node.name, "GET", "/metrics")
        st = {}
        for line in str(text).splitlines():
            if line.startswith("gpupool_agent_") and "{" not in line:
                k, v = line.split(" ", 1)
                st[k[len("gpupool_agent_"):]] = float(v)
        out = {"health_polls": int(st.get("health_polls", 0)),
               "samples": int(st.get("samples", 0)),
               "device_events": int(st.get("device_events", 0)),
               "fault_events": int(st.get("fault_events", 0))}
        if st.get("health_polls"):
            out["health_poll_ms_avg"] = round(st["health_poll_ms_sum"] / st["health_polls"], 3)
        if st.get("samples"):
            out["sample_ms_avg"] = round(st["sample_ms_sum"] / st["samples"], 3)
        return out

    def health(self, pool: dict, steps: int) -> dict:
        """Fault -> condition on one claimed GPU of ``pool`` (replacePolicy Keep, so the faulty
        GPU stays and the Conditions are what changes)."""
        name = pool["metadata"]["name"]
        self.c.patch(MI355XPOOLS, name, {"spec": {"replicas": 1, "replacePolicy": "Keep"}}, self.ns)
        obj = self.c.wait_for(MI355XPOOLS, name, self.ns, ready_at(1), timeout=self.timeout)
        victim = obj["status"]["devices"][0]["uuid"]

        def cond(o, t):
            return conds(o).get(t, {}).get("status")
        faulted = (lambda o: cond(o, "HBMECCHealthy") == "False" and cond(o, "Degraded") == "True")
        cleared = (lambda o: cond(o, "HBMECCHealthy") == "True" and ready_at(1)(o))
        out: dict[str, list[float]] = {"detect": [], "event": [], "react": [], "recover": []}
        for i in range(steps):
            for key, forced, notify in (("detect", False, False), ("event", False, True),
                                        ("react", True, False)):
                t0 = time.perf_counter()
                self.cluster.set_faults(self.node.name,
                                        {"devices": {victim: {"ecc": {"uncorrectable": 1 + i}}}},
                                        sample=forced, notify=notify)
                self.c.wait_for(MI355XPOOLS, name, self.ns, faulted, timeout=self.timeout)
                out[key].append(time.perf_counter() - t0)
                t0 = time.perf_counter()
                self.cluster.set_faults(self.node.name, {}, sample=True)
                self.c.wait_for(MI355XPOOLS, name, self.ns, cleared, timeout=self.timeout)
                out["recover"].append(time.perf_counter() - t0)
        self.c.patch(MI355XPOOLS, name, {"spec": {"replicas": 0, "replacePolicy": "Replace"}},
                     self.ns)
        self.c.wait_for(MI355XPOOLS, name, self.ns, ready_at(0), timeout=self.timeout)
        return {
            # detection included, polled: the counter change is seen by the agent's health-only
            # poll (amdsmi signals no ECC event), nothing forces or announces it
            "fault_to_condition_p50_s": summary(out["detect"])["p50_s"],
            "fault_to_condition_max_s": summary(out["detect"])["max_s"],
            # detection included, event-driven: the fault arrives as an event (overlay rewrite
            # via inotify, the same path an amdsmi thermal/reset event takes)
            "event_to_condition_p50_s": summary(out["event"])["p50_s"],
            "event_to_condition_max_s": summary(out["event"])["max_s"],
            # reaction only: a forced agent sample, then long-poll -> reconcile -> status
            "forced_sample_to_condition_p50_s": summary(out["react"])["p50_s"],
            "fault_cleared_to_ready_p50_s": summary(out["recover"])["p50_s"],
            "steps": steps,
        }
