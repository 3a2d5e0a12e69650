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

import os
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
    deadline: float = 0.0         # time.monotonic() wall budget end (0 = none): caps every wait
    phase: str = ""               # what the scenario is doing now (named in error records)
    last_patch_rtt: float = 0.0   # seconds, the last scale PATCH's request -> response

    def _to(self) -> float:
        """Per-wait timeout: the per-transition limit, cut to what the wall budget has left."""
        if not self.deadline:
            return self.timeout
        return max(1.0, min(self.timeout, self.deadline - time.monotonic()))

    def recover(self, name: str, timeout: float) -> bool:
        """After a failed scenario step: scale ``name`` back to 0 and wait (bounded) for it, so
        the next measurement starts from a clean pool. False if the pool did not get there."""
        self.phase = "recover"
        try:
            self.c.patch(MI355XPOOLS, name, {"spec": {"replicas": 0}}, self.ns)
            self.c.wait_for(MI355XPOOLS, name, self.ns, ready_at(0), timeout=max(1.0, timeout))
            return True
        except Exception:
            return False

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
        """Diagnostic only: poll the truth until it agrees (bounded), to report how long the
        kubelet side took to settle when the first read disagreed."""
        deadline = time.monotonic() + timeout
        while True:
            t = self.truth(pool)
            if (t["ready"] == want and t.get("ledgerAgrees", True)) or time.monotonic() > deadline:
                return t
            time.sleep(0.01)

    def truth_at_ready(self, pool: dict, want: int) -> dict:
        """Ground truth read ONCE, immediately when the pool reads Ready — no grace period: the
        accuracy the bench reports is whether status.readyReplicas agreed with the kubelet's
        PodResources allocatable (∩ independently healthy ∩ the agent's ledger) at that instant.
        If it did not, the truth is polled on (``settleMs``, a diagnostic) to show how far behind
        the kubelet was."""
        t0 = time.perf_counter()
        first = self.truth(pool)
        agrees = first["ready"] == want and first.get("ledgerAgrees", True)
        out = {**first, "firstReadAgrees": agrees}
        if not agrees:
            final = self.wait_truth(pool, want)
            out["settleMs"] = round((time.perf_counter() - t0) * 1e3, 2)
            out["settled"] = final["ready"] == want and final.get("ledgerAgrees", True)
        return out

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
        t0 = time.perf_counter()
        self.c.patch(MI355XPOOLS, name, {"spec": {"replicas": r}}, self.ns)
        self.last_patch_rtt = time.perf_counter() - t0  # the apiserver's PATCH round trip
        if wait:
            return self.c.wait_for(MI355XPOOLS, name, self.ns, ready_at(r), timeout=self._to())
        return None

    def delete_pool(self, name: str) -> None:
        try:
            self.c.delete(MI355XPOOLS, name, self.ns)
        except KubeError as e:
            if e.code != 404:
                raise
        self.c.wait_for(MI355XPOOLS, name, self.ns, lambda o: o is None, timeout=self._to())

    # ------------------------------------------------------------ config 2/3
    def cycle(self, pool: dict, n: int) -> dict:
        name = pool["metadata"]["name"]
        patch_at = time.time()  # wall clock, to place the manager's trace of this cycle
        t0 = time.perf_counter()
        self.phase = "scale_up"
        obj = self.scale(name, n)
        t_ready = time.perf_counter() - t0
        patch_rtt = self.last_patch_rtt
        ready_at_wall = patch_at + t_ready
        self.phase = "ground_truth"
        truth = self.truth_at_ready(pool, n)
        ok = truth["firstReadAgrees"] and obj["status"]["readyReplicas"] == n
        self.phase = "release"
        self.scale(name, 0)
        return {"n": n, "readySeconds": t_ready, "ok": ok, "truth": truth,
                "truthFirstReadAgrees": truth["firstReadAgrees"],
                "indices": [d.get("index") for d in obj["status"]["devices"]],
                "patchAt": patch_at, "readyAtWall": ready_at_wall, "patchRttMs": patch_rtt * 1e3,
                "probeMs": [round(d.get("probe", {}).get("ms", 0.0), 3)
                            for d in obj["status"]["devices"]],
                # the xGMI peer ring of this claim (n >= 2): GB/s of each GPU's outgoing link as
                # measured, and how many of the GPU's peer pairs have ever been checked
                "xgmiGBps": [round(float((d.get("probe") or {})["xgmiGBps"]), 1)
                             for d in obj["status"]["devices"]
                             if isinstance((d.get("probe") or {}).get("xgmiGBps"), (int, float))],
                "xgmiPairs": [[(d.get("xgmi") or {}).get("pairsCovered", 0),
                               (d.get("xgmi") or {}).get("pairsTotal", 0)]
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
                            timeout=self._to())
        return names

    def _delete_pods(self, names: list[str]) -> None:
        for nm in names:
            try:
                self.c.delete(PODS, nm, self.ns, grace=0)
            except KubeError as e:
                if e.code != 404:
                    raise
        for nm in names:
            self.c.wait_for(PODS, nm, self.ns, lambda o: o is None, timeout=self._to())

    def scale_down(self, pool: dict, n: int, step: int) -> dict:
        """n GPUs busy with one pod each -> replicas n//2: cordon, evict, wait, release."""
        name, res = pool["metadata"]["name"], pool["spec"]["resourceName"]
        keep = n // 2
        self.phase = "scale_up"
        m_up = self._agent_counters()
        self.scale(name, n)  # right after the previous step's release (its helpers restarting)
        m_up1 = self._agent_counters()
        self.phase = "start_pods"
        pods = self._pods(f"sd{step}", n, res)
        m0 = self._agent_counters()
        t0 = time.perf_counter()
        self.phase = "scale_down"
        obj = self.scale(name, keep)
        dt = time.perf_counter() - t0
        m1 = self._agent_counters()
        kept = {d["uuid"] for d in obj["status"]["devices"]}
        truth = self.truth_at_ready(pool, keep)
        left = [p for p in self.c.list(PODS, self.ns)["items"]
                if p["metadata"]["name"] in pods and not p["metadata"].get("deletionTimestamp")]
        on_released = [p["metadata"]["name"] for p in left
                       if not set((p["metadata"].get("annotations") or {})
                                  .get("gpupool.amd.com/devices", "").split(",")) <= kept]
        ok = truth["firstReadAgrees"] and obj["status"]["readyReplicas"] == keep and \
            not on_released and len(left) == keep
        self.phase = "cleanup"
        self._delete_pods([p["metadata"]["name"] for p in left])
        self.scale(name, 0)
        waits = m_up1.get("claim_helper_waits", 0) - m_up.get("claim_helper_waits", 0)
        return {"from": n, "to": keep, "seconds": dt, "ok": ok, "evicted": n - len(left),
                "podsOnReleasedGPUs": on_released, "truth": truth,
                # helper parking: the pods' GPUs had their probe helpers stopped while the pods
                # ran; release hands them back at once while the helpers restart, and the claim
                # that opened this step (right after the previous step's release) waited this
                # long when it had to take a GPU whose helper was still starting
                "helpersParked": m1.get("probe_helper_parks_total", 0) -
                m0.get("probe_helper_parks_total", 0),
                "helpersRestartingAtRelease": m1.get("release_helpers_restarting", 0) -
                m0.get("release_helpers_restarting", 0),
                "claimHelperWaits": waits,
                "claimHelperWaitMs": round((m_up1.get("claim_helper_wait_ms_sum", 0) -
                                            m_up.get("claim_helper_wait_ms_sum", 0)) / waits, 2)
                if waits else None}

    def _agent_counters(self) -> dict[str, float]:
        out: dict[str, float] = {}
        try:
            text = self.cluster.agent_request(self.node.name, "GET", "/metrics")
        except Exception:  # noqa: BLE001 - evidence only
            return out
        for ln in text.splitlines():
            if ln.startswith("gpupool_agent_") and "{" not in ln and " " in ln:
                k, _, v = ln.rpartition(" ")
                try:
                    out[k[len("gpupool_agent_"):]] = float(v)
                except ValueError:
                    pass
        return out

    # ------------------------------------------------------------ config 5
    def two_pools(self, n: int, step: int) -> dict:
        half = n // 2
        self.phase = "create"
        a = self.make_pool(f"team-a-{step}", "amd.com/gpu-team-a", 0)
        b = self.make_pool(f"team-b-{step}", "amd.com/gpu-team-b", 0)
        t0 = time.perf_counter()
        self.phase = "scale_up"
        self.scale(a["metadata"]["name"], half, wait=False)
        self.scale(b["metadata"]["name"], half, wait=False)
        oa = self.c.wait_for(MI355XPOOLS, a["metadata"]["name"], self.ns, ready_at(half),
                             timeout=self._to())
        ob = self.c.wait_for(MI355XPOOLS, b["metadata"]["name"], self.ns, ready_at(half),
                             timeout=self._to())
        dt = time.perf_counter() - t0
        ta, tb = self.truth_at_ready(a, half), self.truth_at_ready(b, half)
        self.phase = "cleanup"
        ua = {d["uuid"] for d in oa["status"]["devices"]}
        ub = {d["uuid"] for d in ob["status"]["devices"]}
        ok = ta["firstReadAgrees"] and tb["firstReadAgrees"] and not (ua & ub)
        self.delete_pool(a["metadata"]["name"])
        self.delete_pool(b["metadata"]["name"])
        return {"pools": [half, half], "seconds": dt, "ok": ok, "crossPoolDevices": len(ua & ub),
                "truth": {"a": ta, "b": tb}}

    def cleanup(self, pool: dict | None, scenario: str, step: int, timeout: float) -> bool:
        """Best-effort undo of a failed secondary scenario (its pods, its extra pools), then the
        main pool back to 0. False if the main pool could not be brought back."""
        deadline = time.monotonic() + max(1.0, timeout)
        try:
            if scenario == "scale_down":
                for p in self.c.list(PODS, self.ns)["items"]:
                    if p["metadata"]["name"].startswith(f"sd{step}-"):
                        try:
                            self.c.delete(PODS, p["metadata"]["name"], self.ns, grace=0)
                        except KubeError:
                            pass
            elif scenario == "two_pools":
                for nm in (f"team-a-{step}", f"team-b-{step}"):
                    try:
                        self.c.delete(MI355XPOOLS, nm, self.ns)
                    except KubeError:
                        pass
                for nm in (f"team-a-{step}", f"team-b-{step}"):
                    self.c.wait_for(MI355XPOOLS, nm, self.ns, lambda o: o is None,
                                    timeout=max(1.0, deadline - time.monotonic()))
        except Exception:
            pass
        if pool is None:
            return True
        return self.recover(pool["metadata"]["name"], deadline - time.monotonic())

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
        o = self.c.wait_for(AZUREVMPOOLS, name, self.ns, ready, timeout=self._to())
        t_ready = time.perf_counter() - t0
        fin = "compute.my.domain/device-release" in (o["metadata"].get("finalizers") or [])
        t1 = time.perf_counter()
        self.c.delete(AZUREVMPOOLS, name, self.ns)
        self.c.wait_for(AZUREVMPOOLS, name, self.ns, lambda x: x is None, timeout=self._to())
        return {"seconds": t_ready, "deleteSeconds": time.perf_counter() - t1,
                "ok": fin and o["status"]["readyReplicas"] == replicas}

    # ------------------------------------------------------------ accuracy under faults
    FAULT_KINDS = ("xgmi_down", "hotspot_critical", "hotspot_below", "vram_emergency",
                   "ecc_uncorrectable", "ecc_correctable_at_limit", "ecc_correctable_over",
                   "retired_at_limit", "retired_over", "pending", "missing")

    def _fault(self, kind: str, dev: dict, health: dict) -> dict:
        ecc = dev.get("ecc") or {}
        temps = dev.get("temps") or {}
        crit = lambda s, k="critical", d=100: (temps.get(s) or {}).get(k, d)  # noqa: E731
        if kind == "xgmi_down":
            links = list((dev.get("xgmi") or {}).get("links") or ["X"] + ["U"] * 7)
            j = next((i for i, x in enumerate(links) if x != "X"), 0)
            links[j] = "D"
            return {"xgmi": {"links": links}}
        if kind == "hotspot_critical":
            return {"temps": {"hotspot": {"current": crit("hotspot")}}}
        if kind == "hotspot_below":  # one degree under the limit: still healthy
            return {"temps": {"hotspot": {"current": crit("hotspot") - 1}}}
        if kind == "vram_emergency":
            return {"temps": {"vram": {"current": crit("vram", "emergency", 125)}}}
        if kind == "ecc_uncorrectable":
            return {"ecc": {"uncorrectable": ecc.get("uncorrectable", 0) + 1}}
        if kind == "ecc_correctable_at_limit":
            return {"ecc": {"correctable": ecc.get("correctable", 0) + health["maxCorrectableECC"]}}
        if kind == "ecc_correctable_over":
            return {"ecc": {"correctable": ecc.get("correctable", 0) +
                            health["maxCorrectableECC"] + 1}}
        if kind == "retired_at_limit":
            return {"ras": {"badPagesSupported": True, "retiredPages": health["maxRetiredPages"]}}
        if kind == "retired_over":
            return {"ras": {"badPagesSupported": True, "retiredPages": health["maxRetiredPages"] + 1}}
        if kind == "pending":
            return {"ras": {"badPagesSupported": True, "pendingPages": 1}}
        if kind == "missing":
            return {"present": False}
        raise ValueError(kind)

    def _state_now(self) -> dict[str, dict]:
        """Device state from the independent source, before any fault overlay."""
        return gt.cli_state() if self.real else gt.fixture_state(self.node.fixture, self.node.name)

    def accuracy_under_faults(self, n: int, steps: int, seed: int = 0,
                              truth_policy: dict | None = None, settle_s: float = 5.0,
                              hold_s: float = 0.25) -> dict:
        """readyReplicas vs ground truth after every step of a random fault / clear sequence on
        the GPUs of a dedicated pool (replacePolicy Keep, so ownership is fixed and health is what
        moves). The truth is ``ground_truth.device_healthy`` over the independent device state
        (fixture or amd-smi CLI) + the injected overlay, under the pool's spec.health read back
        from the API server (or ``truth_policy``, to prove a mismatching rule is caught). A step
        counts as accurate when status.readyReplicas equals the truth — and the kubelet holds
        exactly the truly healthy GPUs — within ``settle_s`` of the fault, and stays so for
        ``hold_s``."""
        import random
        rng = random.Random(seed)
        self.phase = "create"
        pool = self.make_pool("acc-pool", "amd.com/gpu-acc", n, replacePolicy="Keep",
                              health={"maxCorrectableECC": 10, "maxRetiredPages": 4,
                                      "maxPendingPages": 0},
                              probe={"enabled": True, "hbmBytes": min(self.hbm_bytes, 256 << 20),
                                     "mfma": False, "xgmiPeerCheck": False})
        name = pool["metadata"]["name"]
        self.phase = "scale_up"
        obj = self.c.wait_for(MI355XPOOLS, name, self.ns, ready_at(n), timeout=self._to())
        policy = truth_policy if truth_policy is not None else obj["spec"]
        health = {**gt.HEALTH_DEFAULTS, **(obj["spec"].get("health") or {})}
        self.phase = "ground_truth"
        base = self._state_now()                       # ECC baseline = state at claim
        deadline = time.monotonic() + 10  # the kubelet learns the devices asynchronously
        while True:
            owned = gt.kubelet_allocatable(self.pr_socket).get("amd.com/gpu-acc", set())
            if len(owned) >= n or time.monotonic() > deadline:
                break
            time.sleep(0.01)
        ledger0 = set().union(*gt.ledger_claims(self.state_dir, obj["metadata"]["uid"])) \
            if os.path.exists(os.path.join(self.state_dir, "ledger.json")) else set()
        samples: list[dict] = []
        t_conv: list[float] = []
        for i in range(steps):
            self.phase = f"fault_step_{i}"
            if i % 3 == 2 or not owned:
                overlay, kinds = {}, {}
            else:
                victims = rng.sample(sorted(owned), k=min(len(owned), rng.choice((1, 1, 2))))
                kinds = {u: rng.choice(self.FAULT_KINDS) for u in victims}
                overlay = {"devices": {u: self._fault(k, base.get(u, {}), health)
                                       for u, k in kinds.items()}}
            t0 = time.perf_counter()
            # delivered as an event (inotify) like a real amdsmi event; the forced sample makes
            # the write a fence: when it returns the agent has applied the new state
            self.cluster.set_faults(self.node.name, overlay, sample=True, notify=True)
            cur = gt.apply_overlay(base, overlay)
            truth_ok = {u for u in owned if gt.device_healthy(cur.get(u, {"present": False}),
                                                              base.get(u), policy)[0]}
            # agreement must hold for ``hold_s`` (a stale pre-fault status that happens to equal
            # the new truth is not a correct answer: the operator would move off it)
            deadline = time.monotonic() + settle_s + hold_s
            first_agree = None
            while True:
                o = self.c.get(MI355XPOOLS, name, self.ns)
                ready = (o.get("status") or {}).get("readyReplicas")
                adv = gt.kubelet_allocatable(self.pr_socket).get("amd.com/gpu-acc", set())
                now = time.monotonic()
                if ready == len(truth_ok) and adv == truth_ok:
                    if first_agree is None:
                        first_agree = (now, time.perf_counter() - t0)
                    elif now - first_agree[0] >= hold_s:
                        break
                else:
                    first_agree = None
                if now > deadline:
                    break
                time.sleep(0.01)
            agree = first_agree is not None and time.monotonic() - first_agree[0] >= hold_s
            if agree:
                t_conv.append(first_agree[1])
            samples.append({"step": i, "faults": {u[-8:]: k for u, k in kinds.items()},
                            "truth": len(truth_ok), "readyReplicas": ready,
                            "kubeletHealthy": len(adv), "ok": agree})
        self.phase = "cleanup"
        self.cluster.set_faults(self.node.name, {}, sample=True)
        ledger1 = set().union(*gt.ledger_claims(self.state_dir, obj["metadata"]["uid"])) \
            if os.path.exists(os.path.join(self.state_dir, "ledger.json")) else set()
        self.delete_pool(name)
        ok = sum(x["ok"] for x in samples)
        return {"accuracy": ok / len(samples) if samples else None, "samples": len(samples),
                "pool_replicas": n, "ownership_stable": ledger1 == ledger0 or not ledger0,
                "converge_p50_s": round(statistics.median(t_conv), 4) if t_conv else None,
                "converge_max_s": round(max(t_conv), 4) if t_conv else None,
                "fault_kinds": list(self.FAULT_KINDS),
                "mismatches": [x for x in samples if not x["ok"]][:5]}

    def footprint(self) -> dict:
        """Resident memory (MiB), threads and open fds of the node agent and the manager, from
        their /metrics process_* lines: taken before and after the timed region, a leak or a
        thread pile-up over many claim/release cycles shows as growth."""
        out = {}
        for who, get in (("agent", lambda: self.cluster.agent_request(self.node.name, "GET", "/metrics")),
                         ("manager", self.cluster.manager_metrics)):
            try:
                vals = {}
                for line in str(get()).splitlines():
                    if line.startswith("process_"):
                        k, _, v = line.partition(" ")
                        vals[k] = float(v)
                out[who] = {"rss_mib": round(vals.get("process_resident_memory_bytes", 0) / 2**20, 1),
                            "threads": int(vals.get("process_threads", 0)),
                            "open_fds": int(vals.get("process_open_fds", 0)),
                            "cpu_s": round(vals.get("process_cpu_seconds_total", 0.0), 2)}
                if who == "agent":
                    # HIP contexts the agent holds, and every GPU's VRAM in use (amdsmi): with N
                    # devices initialised, what the agent costs each GPU and the node
                    import re
                    text = str(get())
                    m = re.search(r"^gpupool_agent_hip_devices (\d+)", text, re.M)
                    out[who]["hip_devices"] = int(m.group(1)) if m else None
                    # the per-GPU probe helpers (child processes: their RSS is not the agent's)
                    m = re.search(r"^gpupool_agent_probe_helpers_rss_bytes (\d+)", text, re.M)
                    if m:
                        out[who]["helpers_rss_mib"] = round(int(m.group(1)) / 2**20, 1)
                        m = re.search(r"^gpupool_agent_probe_helpers_pss_bytes (\d+)", text, re.M)
                        if m:
                            out[who]["helpers_pss_mib"] = round(int(m.group(1)) / 2**20, 1)
                        # the xGMI fabric helper's warm-up over every directed GPU pair (2+ GPUs)
                        fw = {k: re.search(rf"^gpupool_agent_probe_fabric_warm_{k} ([0-9.]+)",
                                           text, re.M) for k in ("ms", "links", "passed")}
                        if fw["ms"]:
                            out[who]["fabric_warm"] = {
                                "ms": float(fw["ms"].group(1)),
                                "links": int(float(fw["links"].group(1))) if fw["links"] else None,
                                "passed": fw["passed"].group(1) == "1" if fw["passed"] else None}
                        m = re.search(r"^gpupool_agent_probe_helpers (\d+)", text, re.M)
                        out[who]["helpers"] = int(m.group(1)) if m else None
                    out[who]["vram_used_mib"] = {
                        int(i): round(float(v) / 2**20, 1) for i, v in re.findall(
                            r'^gpupool_device_vram_used_bytes\{[^}]*index="(\d+)"[^}]*\} ([0-9.e+]+)',
                            text, re.M)}
            except Exception as e:  # never fail the bench over a diagnostic
                out[who] = {"error": repr(e)[:200]}
        return out

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
        # the agent's own time per claim RPC (request parsed -> reply written): the manager's
        # "agent:POST /v1/claims" span minus this is socket transport + the manager's side
        import re
        m = re.search(r'gpupool_agent_rpc_requests_total\{path="/v1/claims"\} (\d+)', str(text))
        ms = re.search(r'gpupool_agent_rpc_seconds_sum\{path="/v1/claims"\} ([0-9.]+)', str(text))
        if m and ms and int(m.group(1)):
            out["claim_rpc_server_ms_avg"] = round(float(ms.group(1)) * 1e3 / int(m.group(1)), 3)
        return out

    def health(self, pool: dict, steps: int) -> dict:
        """Fault -> condition on one claimed GPU of ``pool`` (replacePolicy Keep, so the faulty
        GPU stays and the Conditions are what changes)."""
        name = pool["metadata"]["name"]
        self.c.patch(MI355XPOOLS, name, {"spec": {"replicas": 1, "replacePolicy": "Keep"}}, self.ns)
        obj = self.c.wait_for(MI355XPOOLS, name, self.ns, ready_at(1), timeout=self._to())
        victim = obj["status"]["devices"][0]["uuid"]

        def cond(o, t):
            return conds(o).get(t, {}).get("status")
        faulted = (lambda o: cond(o, "HBMECCHealthy") == "False" and cond(o, "Degraded") == "True")
        cleared = (lambda o: cond(o, "HBMECCHealthy") == "True" and ready_at(1)(o))
        out: dict[str, list[float]] = {"detect": [], "event": [], "react": [], "recover": []}
        checks = []  # readyReplicas vs the independent truth after every fault and every clear
        base = self._state_now()

        def check(overlay: dict, o: dict) -> None:
            cur = gt.apply_overlay(base, overlay)
            truth = int(gt.device_healthy(cur.get(victim, {"present": False}),
                                          base.get(victim), o["spec"])[0])
            checks.append(truth == (o.get("status") or {}).get("readyReplicas"))
        for i in range(steps):
            for key, forced, notify in (("detect", False, False), ("event", False, True),
                                        ("react", True, False)):
                t0 = time.perf_counter()
                fault = {"devices": {victim: {"ecc": {"uncorrectable": 1 + i}}}}
                self.cluster.set_faults(self.node.name, fault, sample=forced, notify=notify)
                o = self.c.wait_for(MI355XPOOLS, name, self.ns, faulted, timeout=self._to())
                out[key].append(time.perf_counter() - t0)
                check(fault, o)
                t0 = time.perf_counter()
                self.cluster.set_faults(self.node.name, {}, sample=True)
                o = self.c.wait_for(MI355XPOOLS, name, self.ns, cleared, timeout=self._to())
                out["recover"].append(time.perf_counter() - t0)
                check({}, o)
        self.c.patch(MI355XPOOLS, name, {"spec": {"replicas": 0, "replacePolicy": "Replace"}},
                     self.ns)
        self.c.wait_for(MI355XPOOLS, name, self.ns, ready_at(0), timeout=self._to())
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
            # readyReplicas == independent truth (device state + injected overlay, pool policy)
            # once the condition reported the fault / the clear
            "readyReplicas_accuracy": sum(checks) / len(checks) if checks else None,
            "accuracy_samples": len(checks),
            "steps": steps,
        }
