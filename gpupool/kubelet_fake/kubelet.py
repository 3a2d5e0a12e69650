"""Fake kubelet: the kubelet side of the device-plugin contract plus a minimal pod runtime.

There is no kubelet/kind/docker in this environment, so device-plugin conformance
and drain semantics are exercised against this process:

* Registration gRPC server on ``<plugin_dir>/kubelet.sock``; on Register it dials the plugin's
  endpoint and consumes ListAndWatch, keeping per-resource device health;
* Node status: ``capacity``/``allocatable`` for every registered extended resource;
* pod admission for pods bound to this node: picks device IDs (GetPreferredAllocation when the
  plugin offers it), calls Allocate, then runs ``containers[0].command`` as a host process with the
  returned env (ROCR_VISIBLE_DEVICES …) — i.e. the reference's `--gpus=1` smoke pod and the
  training job (GPU调度平台搭建.md:134-138, :638-675) run for real on the allotted MI355X;
* graceful termination: a pod with ``deletionTimestamp`` (delete or eviction) gets SIGTERM, then
  SIGKILL after its grace period, its devices are freed, and the pod object is deleted;
* PodResources v1 ``List`` / ``GetAllocatableResources`` for the node agent;
* an optional scheduler loop binding unscheduled pods that fit this node's allocatable.
"""
from __future__ import annotations

import concurrent.futures as cf
import datetime as _dt
import logging
import os
import shlex
import signal
import subprocess
import threading
import time
from dataclasses import dataclass, field

import grpc

from ..agent.deviceplugin.proto import (API_VERSION, DP, KUBELET_SOCKET, PR, Stub,
                                        fresh_channel, service_handler, unix_target)
from ..api import schema
from ..kube import NODES, PODS, Client, KubeError

log = logging.getLogger("gpupool.kubelet")


def now_rfc3339() -> str:
    return _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


@dataclass
class PluginConn:
    resource: str
    endpoint: str
    options: object
    devices: dict[str, str] = field(default_factory=dict)  # ID -> health
    numa: dict[str, int] = field(default_factory=dict)
    channel: grpc.Channel | None = None
    stub: Stub | None = None
    updates: int = 0


@dataclass
class RunningPod:
    ns: str
    name: str
    uid: str
    devices: dict[str, list[str]]  # resource -> device IDs
    container: str
    proc: subprocess.Popen | None = None
    log_path: str = ""
    restarts: int = 0
    terminating: bool = False
    running_written: bool = False  # its Running status is in the API: the exit may be reported


class FakeKubelet:
    def __init__(self, node: str, apiserver: str, plugin_dir: str, pod_resources_socket: str,
                 workdir: str | None = None, log_dir: str | None = None, token: str | None = None,
                 schedule: bool = True, extra_env: dict | None = None,
                 node_status_delay: float = 0.02, host_paths: list[str] | None = None,
                 status_interval: float = 10.0):
        self.node = node
        self.client = Client(apiserver, token)
        self.apiserver = apiserver
        self.plugin_dir = plugin_dir
        self.pr_socket = pod_resources_socket
        self.workdir = workdir or os.getcwd()
        self.log_dir = log_dir or os.path.join(plugin_dir, "..", "pod-logs")
        self.schedule = schedule
        self.extra_env = extra_env or {}
        # strict mounts: the host paths that exist on this "node" for a device plugin to hand out
        # (the agent DaemonSet's same-path hostPath volumes). A container runtime resolves an
        # Allocate's mount and device host paths on the HOST; one the agent only has inside its
        # own container fails CreateContainer — so does it here. None: anything goes.
        self.host_paths = [os.path.abspath(p) for p in host_paths] if host_paths else None
        self.plugins: dict[str, PluginConn] = {}
        self.pods: dict[str, RunningPod] = {}          # pod uid -> running pod
        # pods whose containers already ran to completion: an event that still shows one of them
        # Running (the watch delivers it between the exit and the Succeeded status write) must
        # not admit it again — a pod's containers run once (restartPolicy Never / OnFailure)
        self.finished: set[str] = set()
        self.assigned: dict[str, str] = {}             # device ID -> pod uid
        self.lock = threading.RLock()
        # serialises node-status snapshots with their PATCH: two ListAndWatch streams updating at
        # once must not land an older snapshot after a newer one
        self.status_lock = threading.Lock()
        self.stop_ev = threading.Event()
        self._sched_kick = threading.Event()  # unscheduled pod seen or capacity changed
        # Device-plugin updates reach Node status asynchronously and coalesced, as in a real
        # kubelet (there: the periodic node-status sync, 10 s by default); a burst of
        # ListAndWatch updates becomes one PATCH that does not queue in front of the control
        # plane's own writes on the apiserver.
        self.node_status_delay = node_status_delay
        # the periodic node-status sync (kubelet --node-status-update-frequency, 10 s): the Ready
        # condition's heartbeat plus capacity/allocatable, as a strategic merge patch
        self.status_interval = status_interval
        self._ready_since = ""
        self.status_writes = 0
        self._status_kick = threading.Event()
        self.threads: list[threading.Thread] = []
        self.reg_server: grpc.Server | None = None
        self.pr_server: grpc.Server | None = None
        os.makedirs(plugin_dir, exist_ok=True)
        os.makedirs(os.path.dirname(os.path.abspath(pod_resources_socket)), exist_ok=True)
        os.makedirs(self.log_dir, exist_ok=True)

    # ============================================================ gRPC servers
    def start(self) -> None:
        ksock = os.path.join(self.plugin_dir, KUBELET_SOCKET)
        # like the kubelet's device manager at start: remove every socket in the plugin directory
        # — stale plugin endpoints included; plugins take that as the signal to serve again and
        # re-register
        for name in os.listdir(self.plugin_dir):
            if name.endswith(".sock"):
                try:
                    os.unlink(os.path.join(self.plugin_dir, name))
                except FileNotFoundError:
                    pass
        try:
            os.unlink(self.pr_socket)
        except FileNotFoundError:
            pass
        self.reg_server = grpc.server(cf.ThreadPoolExecutor(max_workers=8))
        self.reg_server.add_generic_rpc_handlers((service_handler("v1beta1.Registration",
                                                                  {"Register": self.Register}),))
        self.reg_server.add_insecure_port(unix_target(ksock))
        self.reg_server.start()
        self.pr_server = grpc.server(cf.ThreadPoolExecutor(max_workers=8))
        self.pr_server.add_generic_rpc_handlers((service_handler("v1.PodResourcesLister", {
            "List": self.List, "GetAllocatableResources": self.GetAllocatableResources}),))
        self.pr_server.add_insecure_port(unix_target(self.pr_socket))
        self.pr_server.start()
        self._ensure_node()
        for fn, name in ((self._pod_loop, "pods"), (self._reaper, "reaper"),
                         (self._node_status_loop, "node-status")):
            t = threading.Thread(target=fn, daemon=True, name=name)
            t.start()
            self.threads.append(t)
        if self.schedule:
            for fn, name in ((self._scheduler_loop, "scheduler"),
                             (self._unscheduled_watch, "sched-watch")):
                t = threading.Thread(target=fn, daemon=True, name=name)
                t.start()
                self.threads.append(t)
        log.info("fake kubelet %s up (plugins %s, podresources %s)", self.node, self.plugin_dir,
                 self.pr_socket)

    def stop(self) -> None:
        self.stop_ev.set()
        with self.lock:
            for rp in self.pods.values():
                self._kill(rp, 0)
        if self.reg_server:
            self.reg_server.stop(0.2)
        if self.pr_server:
            self.pr_server.stop(0.2)

    def Register(self, request, context):
        if request.version != API_VERSION:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT,
                          f"unsupported device plugin API version {request.version}")
        conn = PluginConn(resource=request.resource_name, endpoint=request.endpoint,
                          options=request.options)
        # a private subchannel pool: the plugin's previous process may have died on this very
        # socket path, and a shared subchannel would make this connection wait out its backoff
        conn.channel = fresh_channel(os.path.join(self.plugin_dir, request.endpoint))
        conn.stub = Stub(conn.channel, "v1beta1.DevicePlugin")
        with self.lock:
            old = self.plugins.get(request.resource_name)
            self.plugins[request.resource_name] = conn
        if old and old.channel:
            old.channel.close()
        t = threading.Thread(target=self._list_and_watch, args=(conn,), daemon=True,
                             name=f"lw-{request.resource_name}")
        t.start()
        log.info("plugin registered: %s at %s", request.resource_name, request.endpoint)
        return DP.Empty()

    def _list_and_watch(self, conn: PluginConn) -> None:
        backoff = 0.05
        while not self.stop_ev.is_set():
            with self.lock:
                if self.plugins.get(conn.resource) is not conn:
                    return  # superseded by a re-registration
            try:
                for resp in conn.stub.ListAndWatch(DP.Empty()):
                    with self.lock:
                        conn.devices = {d.ID: d.health for d in resp.devices}
                        conn.numa = {d.ID: (d.topology.nodes[0].ID if d.topology.nodes else 0)
                                     for d in resp.devices}
                        conn.updates += 1
                    self._status_kick.set()
                    self._sched_kick.set()  # new or healthier devices may fit a pending pod
                    backoff = 0.05
                    if self.stop_ev.is_set():
                        return
            except grpc.RpcError as e:
                log.debug("ListAndWatch %s ended: %s", conn.resource, e.code())
            time.sleep(backoff)
            backoff = min(backoff * 2, 2.0)

    def List(self, request, context):
        resp = PR.ListPodResourcesResponse()
        with self.lock:
            for rp in self.pods.values():
                pr = resp.pod_resources.add(name=rp.name, namespace=rp.ns)
                c = pr.containers.add(name=rp.container)
                for res, ids in rp.devices.items():
                    c.devices.add(resource_name=res, device_ids=ids)
        return resp

    def GetAllocatableResources(self, request, context):
        resp = PR.AllocatableResourcesResponse()
        with self.lock:
            for res, conn in self.plugins.items():
                ids = [i for i, h in conn.devices.items() if h == "Healthy"]
                resp.devices.add(resource_name=res, device_ids=ids)
        return resp

    # ============================================================ node
    def _ensure_node(self) -> None:
        try:
            self.client.create(NODES, {"apiVersion": "v1", "kind": "Node",
                                       "metadata": {"name": self.node,
                                                    "labels": {"kubernetes.io/hostname": self.node}}})
        except KubeError as e:
            if e.code != 409:
                raise
        self._update_node_status()

    def _node_status_loop(self) -> None:
        next_sync = time.monotonic() + self.status_interval
        while not self.stop_ev.is_set():
            wait = max(0.0, min(0.5, next_sync - time.monotonic()))
            if not self._status_kick.wait(wait):
                if time.monotonic() >= next_sync:
                    next_sync = time.monotonic() + self.status_interval
                    self._update_node_status()
                continue
            time.sleep(self.node_status_delay)  # coalesce a burst of plugin updates
            self._status_kick.clear()
            self._update_node_status()

    def _update_node_status(self) -> None:
        """capacity/allocatable of every registered resource + the kubelet's own conditions
        (Ready with its heartbeat), as one strategic merge patch of Node status — conditions merge
        by type, so conditions other components own (the agent's) are left as they are."""
        from ..apiserver_sim.store import now_rfc3339
        with self.status_lock:
            with self.lock:
                cap = {r: str(len(c.devices)) for r, c in self.plugins.items()}
                alloc = {r: str(sum(1 for h in c.devices.values() if h == "Healthy"))
                         for r, c in self.plugins.items()}
            now = now_rfc3339()
            self._ready_since = self._ready_since or now
            conds = [{"type": t, "status": "False", "reason": f"KubeletHasNo{t}",
                      "message": f"kubelet has no {t}", "lastHeartbeatTime": now,
                      "lastTransitionTime": self._ready_since}
                     for t in ("MemoryPressure", "DiskPressure", "PIDPressure")]
            conds.append({"type": "Ready", "status": "True", "reason": "KubeletReady",
                          "message": "kubelet is posting ready status", "lastHeartbeatTime": now,
                          "lastTransitionTime": self._ready_since})
            try:
                self.client.patch(NODES, self.node, {"status": {
                    "capacity": {"cpu": "64", "memory": "1Ti", "pods": "110", **cap},
                    "allocatable": {"cpu": "64", "memory": "1Ti", "pods": "110", **alloc},
                    "conditions": conds}}, sub="status", ptype="strategic")
                self.status_writes += 1
            except KubeError as e:
                log.warning("node status patch failed: %s", e)

    def allocatable(self) -> dict[str, list[str]]:
        with self.lock:
            return {r: [i for i, h in c.devices.items() if h == "Healthy" and i not in self.assigned]
                    for r, c in self.plugins.items()}

    # ============================================================ pods
    def _pod_loop(self) -> None:
        rv = None
        while not self.stop_ev.is_set():
            try:
                if rv is None:
                    lst = self.client.list(PODS, field_selector=f"spec.nodeName={self.node}")
                    for p in lst["items"]:
                        self._handle_pod(p)
                    # a relist is the truth: pods deleted while the watch was down are gone
                    listed = {p["metadata"]["uid"] for p in lst["items"]}
                    with self.lock:
                        gone = [u for u in self.pods if u not in listed]
                        self.finished &= listed
                    for u in gone:
                        self._forget(u)
                    rv = lst["metadata"]["resourceVersion"]
                for ev in self.client.watch(PODS, resource_version=rv,
                                            field_selector=f"spec.nodeName={self.node}",
                                            stop=self.stop_ev, timeout_seconds=60):
                    if ev["type"] == "ERROR":
                        rv = None
                        break
                    rv = ev["object"]["metadata"].get("resourceVersion", rv)
                    if ev["type"] == "BOOKMARK":
                        continue
                    if ev["type"] == "DELETED":
                        self._forget(ev["object"]["metadata"]["uid"])
                    else:
                        self._handle_pod(ev["object"])
            except Exception as e:
                if not self.stop_ev.is_set():
                    log.warning("pod watch error: %s", e)
                time.sleep(0.2)
                rv = None

    def _requests(self, pod: dict) -> dict[str, int]:
        req: dict[str, int] = {}
        for c in pod["spec"].get("containers", []):
            lim = (c.get("resources") or {}).get("limits") or {}
            for k, v in lim.items():
                if "/" in k:
                    req[k] = req.get(k, 0) + int(v)
        return req

    MIRROR = "kubernetes.io/config.mirror"

    def _handle_pod(self, pod: dict) -> None:
        md = pod["metadata"]
        uid = md["uid"]
        if self.MIRROR in (md.get("annotations") or {}):
            return  # a static pod's mirror: the process runs outside this runtime (the agent)
        if md.get("deletionTimestamp"):
            with self.lock:
                rp = self.pods.get(uid)
            if rp is None:
                self._delete_pod(md["namespace"], md["name"], uid)
                return
            if not rp.terminating:
                rp.terminating = True
                grace = int(md.get("deletionGracePeriodSeconds",
                                   pod["spec"].get("terminationGracePeriodSeconds", 30)))
                threading.Thread(target=self._terminate, args=(rp, grace), daemon=True).start()
            return
        phase = pod.get("status", {}).get("phase", "Pending")
        with self.lock:
            known = uid in self.pods or uid in self.finished
        if known or phase in ("Succeeded", "Failed"):
            return
        self._admit(pod)

    def _admit(self, pod: dict) -> None:
        md = pod["metadata"]
        ns, name, uid = md["namespace"], md["name"], md["uid"]
        reqs = self._requests(pod)
        devices: dict[str, list[str]] = {}
        envs: dict[str, str] = {}
        with self.lock:
            for res, n in reqs.items():
                conn = self.plugins.get(res)
                avail = [i for i, h in (conn.devices.items() if conn else []) if h == "Healthy"
                         and i not in self.assigned]
                if conn is None or len(avail) < n:
                    self._fail(pod, f"OutOf{res}", f"Node didn't have enough resource: {res}, "
                               f"requested: {n}, available: {len(avail)}")
                    return
                ids = avail[:n]
                if conn.options.get_preferred_allocation_available:
                    try:
                        pref = conn.stub.GetPreferredAllocation(DP.PreferredAllocationRequest(
                            container_requests=[{"available_deviceIDs": avail,
                                                 "allocation_size": n}]), timeout=5)
                        got = list(pref.container_responses[0].deviceIDs)
                        if len(got) == n and all(g in avail for g in got):
                            ids = got
                    except grpc.RpcError as e:
                        log.warning("GetPreferredAllocation failed: %s", e)
                try:
                    resp = conn.stub.Allocate(DP.AllocateRequest(
                        container_requests=[{"devices_ids": ids}]), timeout=10)
                except grpc.RpcError as e:
                    self._fail(pod, "UnexpectedAdmissionError", f"Allocate failed: {e.details()}")
                    return
                cr = resp.container_responses[0]
                bad = self._off_node_paths(cr)
                if bad:
                    self._fail(pod, "CreateContainerError",
                               f"host path(s) {', '.join(bad)} of the device plugin's Allocate do "
                               f"not exist on node {self.node}")
                    return
                # the pod runs as a host process (no mount namespace): a device-plugin mount is
                # realised by pointing its container paths at the host paths
                rewrite = [(m.container_path, m.host_path) for m in cr.mounts
                           if m.container_path != m.host_path]
                for k, v in dict(cr.envs).items():
                    for cp, hp in rewrite:
                        if v.startswith(cp):
                            v = hp + v[len(cp):]
                    envs[k] = v
                for i in ids:
                    self.assigned[i] = uid
                devices[res] = ids
            container = (pod["spec"].get("containers") or [{"name": "main"}])[0]
            rp = RunningPod(ns, name, uid, devices, container.get("name", "main"))
            self.pods[uid] = rp
        self._start_process(rp, pod, envs)

    def _off_node_paths(self, cr) -> list[str]:
        """Allocate host paths (mounts, device nodes) outside the node's declared host paths."""
        if self.host_paths is None:
            return []
        paths = [m.host_path for m in cr.mounts] + [d.host_path for d in cr.devices]

        def on_node(p: str) -> bool:
            p = os.path.abspath(p)
            return any(p == r or p.startswith(r.rstrip("/") + "/") for r in self.host_paths)
        return [p for p in paths if not on_node(p)]

    def _start_process(self, rp: RunningPod, pod: dict, envs: dict[str, str]) -> None:
        container = (pod["spec"].get("containers") or [{}])[0]
        cmd = list(container.get("command") or []) + list(container.get("args") or [])
        if not cmd:
            cmd = ["sleep", "infinity"]  # a "pause" container: holds its GPUs until deleted
        env = dict(os.environ)
        env.update(self.extra_env)
        for e in container.get("env") or []:
            if "value" in e:
                env[e["name"]] = str(e["value"])
        env.update(envs)
        env["POD_NAME"], env["POD_NAMESPACE"] = rp.name, rp.ns
        rp.log_path = os.path.join(self.log_dir, f"{rp.ns}_{rp.name}.log")
        logf = open(rp.log_path, "ab")
        try:
            rp.proc = subprocess.Popen(cmd, cwd=self.workdir, env=env, stdout=logf,
                                       stderr=subprocess.STDOUT, start_new_session=True)
        except OSError as e:
            logf.close()
            self._fail(pod, "RunContainerError", str(e))
            with self.lock:
                self._free(rp)
            return
        logf.close()
        log.info("started pod %s/%s pid %d devices %s", rp.ns, rp.name, rp.proc.pid, rp.devices)
        try:  # `gpuctl logs` finds the container log through this annotation
            self.client.patch(PODS, rp.name, {"metadata": {"annotations": {
                "gpupool.amd.com/log-path": rp.log_path,
                "gpupool.amd.com/pid": str(rp.proc.pid),
                schema.ANN_POD_DEVICES: ",".join(i for ids in rp.devices.values() for i in ids)}}},
                ns=rp.ns)
        except KubeError:
            pass
        try:
            self._set_status(rp.ns, rp.name, "Running", ready=True, extra={
                "podIP": "127.0.0.1", "hostIP": "127.0.0.1", "startTime": now_rfc3339()})
        finally:
            rp.running_written = True

    def _reaper(self) -> None:
        while not self.stop_ev.wait(0.1):
            with self.lock:
                pods = list(self.pods.values())
            for rp in pods:
                # a container that exits before its Running status is written is reported after it,
                # so the pod's phase never goes back from Succeeded/Failed to Running
                if rp.proc is None or rp.terminating or not rp.running_written:
                    continue
                rc = rp.proc.poll()
                if rc is None:
                    continue
                phase = "Succeeded" if rc == 0 else "Failed"
                with self.lock:
                    self._free(rp)
                    self.pods.pop(rp.uid, None)
                    self.finished.add(rp.uid)
                self._set_status(rp.ns, rp.name, phase, ready=False, exit_code=rc)
                log.info("pod %s/%s exited %d", rp.ns, rp.name, rc)

    def _terminate(self, rp: RunningPod, grace: int) -> None:
        self._kill(rp, grace)
        with self.lock:
            self._free(rp)
            self.pods.pop(rp.uid, None)
        self._delete_pod(rp.ns, rp.name, rp.uid)

    def _kill(self, rp: RunningPod, grace: int) -> None:
        if rp.proc is None or rp.proc.poll() is not None:
            return
        try:
            os.killpg(rp.proc.pid, signal.SIGTERM)
        except ProcessLookupError:
            return
        try:
            rp.proc.wait(timeout=max(grace, 0.05))
        except subprocess.TimeoutExpired:
            try:
                os.killpg(rp.proc.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            rp.proc.wait(timeout=10)

    def _free(self, rp: RunningPod) -> None:
        for ids in rp.devices.values():
            for i in ids:
                if self.assigned.get(i) == rp.uid:
                    del self.assigned[i]
        self._sched_kick.set()  # freed devices may fit a pending pod

    def _forget(self, uid: str) -> None:
        with self.lock:
            self.finished.discard(uid)
            rp = self.pods.pop(uid, None)
            if rp:
                self._kill(rp, 0)
                self._free(rp)

    def _delete_pod(self, ns: str, name: str, uid: str) -> None:
        try:
            self.client.delete(PODS, name, ns, grace=0, preconditions={"uid": uid})
        except KubeError as e:
            if e.code not in (404, 409):
                log.warning("final pod delete failed: %s", e)

    def _fail(self, pod: dict, reason: str, msg: str) -> None:
        md = pod["metadata"]
        log.warning("pod %s/%s rejected: %s", md["namespace"], md["name"], msg)
        self._set_status(md["namespace"], md["name"], "Failed", ready=False,
                         extra={"reason": reason, "message": msg})

    def _set_status(self, ns: str, name: str, phase: str, ready: bool, exit_code: int | None = None,
                    extra: dict | None = None) -> None:
        st: dict = {"phase": phase, "conditions": [
            {"type": "Ready", "status": "True" if ready else "False",
             "lastTransitionTime": now_rfc3339()}]}
        cs = {"name": "main", "ready": ready, "restartCount": 0}
        if exit_code is not None:
            cs["state"] = {"terminated": {"exitCode": exit_code, "finishedAt": now_rfc3339()}}
        else:
            cs["state"] = {"running": {"startedAt": now_rfc3339()}}
        st["containerStatuses"] = [cs]
        st.update(extra or {})
        try:
            self.client.patch(PODS, name, {"status": st}, ns=ns, sub="status")
        except KubeError as e:
            if e.code != 404:
                log.warning("pod status patch failed: %s", e)

    # ============================================================ scheduler
    def _unscheduled_watch(self) -> None:
        """Watch unscheduled pods (kube-scheduler's informer) and wake the scheduling pass, rather
        than listing them every 50 ms: 20 LISTs/s per fake node loaded the apiserver-sim that the
        timed reconciles share."""
        rv = None
        while not self.stop_ev.is_set():
            try:
                if rv is None:
                    rv = self.client.list(PODS, field_selector="spec.nodeName=")["metadata"][
                        "resourceVersion"]
                    self._sched_kick.set()
                for ev in self.client.watch(PODS, resource_version=rv, field_selector="spec.nodeName=",
                                            stop=self.stop_ev, timeout_seconds=60):
                    if ev["type"] == "ERROR":
                        rv = None
                        break
                    rv = ev["object"]["metadata"].get("resourceVersion", rv)
                    if ev["type"] in ("ADDED", "MODIFIED"):
                        self._sched_kick.set()
            except Exception as e:
                if not self.stop_ev.is_set():
                    log.warning("unscheduled-pod watch error: %s", e)
                time.sleep(0.2)
                rv = None

    def _scheduler_loop(self) -> None:
        while not self.stop_ev.is_set():
            self._sched_kick.wait(1.0)  # woken by the watch or a capacity change; 1 s resync
            self._sched_kick.clear()
            if self.stop_ev.is_set():
                break
            try:
                pending = self.client.list(PODS, field_selector="spec.nodeName=")["items"]
            except Exception:
                continue
            if not pending:
                continue
            # like kube-scheduler's assumed pods: GPUs of pods already bound here but not yet
            # admitted (and of pods bound earlier in this pass) are not free
            try:
                bound = self.client.list(PODS, field_selector=f"spec.nodeName={self.node}")["items"]
            except Exception:
                continue
            with self.lock:
                admitted = set(self.pods)
            assumed: dict[str, int] = {}
            for b in bound:
                if b["metadata"].get("uid") in admitted or \
                        b.get("status", {}).get("phase") in ("Succeeded", "Failed"):
                    continue
                for r, n in self._requests(b).items():
                    assumed[r] = assumed.get(r, 0) + n
            for pod in pending:
                if pod["metadata"].get("deletionTimestamp"):
                    continue
                if pod.get("status", {}).get("phase", "Pending") != "Pending":
                    continue
                sel = pod["spec"].get("nodeSelector") or {}
                if sel.get("kubernetes.io/hostname", self.node) != self.node:
                    continue
                free = self.allocatable()
                req = self._requests(pod)
                if all(len(free.get(r, [])) - assumed.get(r, 0) >= n for r, n in req.items()):
                    pod["spec"]["nodeName"] = self.node
                    try:
                        self.client.update(PODS, pod, pod["metadata"]["namespace"])
                        for r, n in req.items():
                            assumed[r] = assumed.get(r, 0) + n
                    except KubeError:
                        pass  # another kubelet bound it first (409) or it is gone


def pod_command(cmdline: str) -> list[str]:
    return shlex.split(cmdline)
