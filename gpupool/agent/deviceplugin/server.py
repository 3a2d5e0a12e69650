"""ROCm device plugin (kubelet DevicePlugin v1beta1) — SURVEY B3.

The reference installs NVIDIA's plugin and requests ``nvidia.com/gpu`` (GPU调度平台搭建.md:128-132,
:665-667). Here each extended resource used by a pool (default ``amd.com/gpu``) gets one plugin
endpoint ``<plugin_dir>/gpupool-<resource>.sock`` registered with the kubelet:

* ListAndWatch streams the pool-claimed GPUs for that resource: Healthy iff claimed, not draining,
  healthy under the owning pool's policy and probe-passed; a cordoned (draining) GPU turns
  Unhealthy so the kubelet places no new pods on it. Every send records which devices were
  advertised Healthy — the agent's ``advertised`` bit that readyReplicas requires. The stream is
  served in gRPC's non-blocking mode: the handler keeps the stream's send callback and returns,
  and whoever changed the device list sends on it — a claim on its own thread (it writes the
  update and sees it delivered without a hop through a stream thread), everything else through
  the plugin's sender thread, so a sampler or health thread never blocks on the kubelet.
* Allocate returns /dev/kfd + /dev/dri/renderD<N> DeviceSpecs and ``ROCR_VISIBLE_DEVICES`` set to
  the GPUs' ROCr UUIDs (``GPU-<serial>``), so a container sees exactly its GPUs.
* GetPreferredAllocation picks xGMI/NUMA-close sets with libmi355x_dev's selector.
* The kubelet socket is watched; a kubelet restart (new socket, the watch channel to it dropping,
  or — as a real kubelet does at start — our own endpoint socket removed, which restarts the
  plugin's server) triggers re-registration.
"""
from __future__ import annotations

import concurrent.futures as cf
import logging
import os
import threading
import time
from typing import TYPE_CHECKING

import grpc

from .proto import API_VERSION, DP, KUBELET_SOCKET, Stub, fresh_channel, service_handler, unix_target

if TYPE_CHECKING:  # pragma: no cover
    from ..agent import Agent

log = logging.getLogger("gpupool.agent.deviceplugin")


def socket_name(resource: str) -> str:
    return "gpupool-" + resource.replace("/", "_").replace(".", "-") + ".sock"


class _Stream:
    """One kubelet ListAndWatch stream: gRPC's send callback (blocks until the message is
    written), the last version sent, and whether a thread is sending on it right now."""
    __slots__ = ("send", "context", "sent", "busy", "alive")

    def __init__(self, send, context):
        self.send, self.context = send, context
        self.sent, self.busy, self.alive = -1, False, True


class DevicePluginServer:
    def __init__(self, agent: "Agent", resource: str, plugin_dir: str):
        self.agent = agent
        self.resource = resource
        self.plugin_dir = plugin_dir
        self.sock = os.path.join(plugin_dir, socket_name(resource))
        self.server: grpc.Server | None = None
        self.version = 0
        self.cv = threading.Condition()
        self.stopped = False
        self.streams = 0
        self.registered = False
        self._kubelet_ino = None
        self._mon: threading.Thread | None = None
        self._sender: threading.Thread | None = None
        self._live: set[_Stream] = set()
        self._wake = False  # the sender thread has work
        self._pending: tuple | None = None  # (version, ListAndWatchResponse, healthy uuids)
        self._mark_mu = threading.Lock()
        self._marked = -1
        # a device list is built and numbered under one lock: two notifies built in one order and
        # numbered in the other left the NEWEST version carrying the OLDER list — a claim whose
        # GPUs the other claim's list lacked was never advertised (scripts/scale_bench.py, 128
        # nodes: concurrent claims on one agent, pools stuck at 0/2 ready)
        self._build_mu = threading.Lock()

    # ------------------------------------------------------------ lifecycle
    def _serve(self) -> None:
        """(Re)create the plugin's gRPC server on its socket."""
        try:
            os.unlink(self.sock)
        except FileNotFoundError:
            pass
        server = grpc.server(cf.ThreadPoolExecutor(max_workers=16,
                                                   thread_name_prefix=f"dp-{self.resource}"))

        def list_and_watch(request, context, send):
            return self.ListAndWatch(request, context, send)
        list_and_watch.experimental_non_blocking = True  # handler gets gRPC's send callback
        server.add_generic_rpc_handlers((service_handler("v1beta1.DevicePlugin", {
            "GetDevicePluginOptions": self.GetDevicePluginOptions,
            "ListAndWatch": list_and_watch,
            "GetPreferredAllocation": self.GetPreferredAllocation,
            "Allocate": self.Allocate,
            "PreStartContainer": self.PreStartContainer,
        }),))
        server.add_insecure_port(unix_target(self.sock))
        server.start()
        self.server = server
        self._sock_ino = self._sock_identity(self.sock)

    def _reserve(self) -> None:
        """A starting kubelet removes every socket in the device-plugin directory (its signal to
        plugins to re-register): the endpoint it would dial for our registration is gone. Stop the
        old server — and wait for it: gRPC unlinks its socket path when the listener is torn
        down, which done late would delete the new socket — then serve again on a fresh socket."""
        old = self.server
        if old is not None:
            old.stop(0).wait(5)
        log.info("device-plugin socket %s was removed (kubelet restart): serving again", self.sock)
        self._serve()

    def start(self) -> None:
        self._sock_ino = None
        self._serve()
        self._sender = threading.Thread(target=self._send_loop, daemon=True,
                                        name=f"dp-send-{self.resource}")
        self._sender.start()
        self._streams_lost = False
        self._kch, self._kcb = None, None
        self.register()  # synchronous first registration; the monitor handles kubelet restarts
        self._mon = threading.Thread(target=self._monitor_kubelet, daemon=True,
                                     name=f"dp-mon-{self.resource}")
        self._mon.start()

    def stop(self) -> None:
        self.stopped = True
        with self.cv:
            # end idle streams with an OK status (the kubelet reconnects); a stream with a send
            # in flight is left to server.stop, which cancels it
            idle = [st for st in self._live if not st.busy and st.alive]
            for st in idle:
                st.busy = True  # no new send may start on it now
            self.cv.notify_all()
        for st in idle:
            try:
                st.send(None)
            except Exception:
                pass
        kch = getattr(self, "_kch", None)
        if kch is not None:
            self._retire_channel(kch, self._kcb)
        if self.server:
            self.server.stop(grace=0.5)
        try:
            os.unlink(self.sock)
        except FileNotFoundError:
            pass

    def register(self) -> bool:
        ksock = os.path.join(self.plugin_dir, KUBELET_SOCKET)
        if not os.path.exists(ksock):
            return False
        try:
            with fresh_channel(ksock) as ch:
                opts = DP.DevicePluginOptions(pre_start_required=False,
                                              get_preferred_allocation_available=True)
                Stub(ch, "v1beta1.Registration").Register(
                    DP.RegisterRequest(version=API_VERSION, endpoint=os.path.basename(self.sock),
                                       resource_name=self.resource, options=opts), timeout=5)
            self.registered = True
            self._kubelet_ino = self._sock_identity(ksock)
            self._watch_kubelet(ksock)
            log.info("registered %s with kubelet at %s", self.resource, ksock)
            return True
        except (grpc.RpcError, OSError) as e:
            log.warning("register %s failed: %s", self.resource, e)
            return False

    def _watch_kubelet(self, ksock: str) -> None:
        """A kubelet restart shows as a new socket identity — unless the new socket reuses the
        inode within one ctime tick (tmpfs). So a channel to the kubelet is also kept connected:
        when it drops out of READY the kubelet went away, and the monitor re-registers once a
        kubelet answers again. No idle timeout: a quiet kubelet is not a restarted one."""
        old, old_cb = getattr(self, "_kch", None), getattr(self, "_kcb", None)
        ch = fresh_channel(ksock, [("grpc.client_idle_timeout_ms", 2**31 - 1)])
        was_ready = [False]

        def on_state(state) -> None:
            if self._kch is not ch or self.stopped:
                return  # a replaced or closed watch channel says nothing about the kubelet
            if state == grpc.ChannelConnectivity.READY:
                was_ready[0] = True
            elif was_ready[0]:
                was_ready[0] = False
                self._streams_lost = True
        self._kch, self._kcb = ch, on_state
        ch.subscribe(on_state, try_to_connect=True)
        if old is not None:
            self._retire_channel(old, old_cb)

    @staticmethod
    def _retire_channel(ch, cb) -> None:
        """Unsubscribe, then close once gRPC's connectivity-polling thread has seen that nothing is
        subscribed (it re-checks every 0.2 s): closing a channel under that thread makes its next
        poll raise 'Cannot monitor channel state: Channel closed!' and die with a traceback."""
        if cb is not None:
            try:
                ch.unsubscribe(cb)
            except Exception:
                pass
        t = threading.Timer(0.5, ch.close)
        t.daemon = True
        t.start()

    def _monitor_kubelet(self) -> None:
        ksock = os.path.join(self.plugin_dir, KUBELET_SOCKET)
        while not self.stopped:
            own = self._sock_identity(self.sock)
            if own is None or own != self._sock_ino:  # our endpoint was removed: serve it again
                try:
                    self._reserve()
                    self._kubelet_ino = None  # and register with whichever kubelet is there
                except Exception:
                    log.exception("restarting the device-plugin server failed")
            ident = self._sock_identity(ksock)
            if ident is None:
                self.registered = False  # kubelet gone: register again when it comes back
            elif ident != self._kubelet_ino or (self._streams_lost and not self.stopped):
                if self.register():  # a kubelet that is not answering yet keeps the signal
                    self._streams_lost = False
            time.sleep(0.2)

    @staticmethod
    def _sock_identity(path: str):
        # (inode, ctime) — a recreated socket may reuse the inode number on tmpfs
        try:
            st = os.stat(path)
        except FileNotFoundError:
            return None
        return (st.st_ino, st.st_ctime_ns)

    # Strict by default: a GPU counts as advertised (and so towards readyReplicas) only once the
    # ListAndWatch write carrying it has completed on a live kubelet stream — readyReplicas never
    # runs ahead of what the kubelet was told. Opt-in fast mode (GPUPOOL_ADVERTISE_ON_SUBMIT=1):
    # ``notify(sync=True)`` (the claim path) marks the list advertised as soon as it is handed to a
    # live stream's sender, saving gRPC's write acknowledgement (0.24–0.35 ms per claim,
    # profiles/r4g_advertise_ab.json) at the cost of that guarantee (a stream that turns out dead
    # clears the bits again, but a reader may have seen them meanwhile).
    ADVERTISE_ON_SUBMIT = os.environ.get("GPUPOOL_ADVERTISE_ON_SUBMIT", "0") == "1"

    def notify(self, sync: bool = False) -> None:
        """Publish the current device list, built on the caller's thread, through the sender
        thread. ``sync`` (the claim path): the caller then finds its GPUs advertised at once if
        a live kubelet stream will carry the list (ADVERTISE_ON_SUBMIT), else it sends on this
        thread and returns once written. Never before a stream exists: a pod placed on a GPU the
        kubelet has not heard of would fail admission."""
        early = sync and self.ADVERTISE_ON_SUBMIT
        with self._build_mu:
            resp, healthy = self._devices_msg()
            with self.cv:
                self.version += 1
                ver = self.version
                self._pending = (ver, resp, healthy)
                live = [st for st in self._live if st.alive]
                if not sync or early:
                    self._wake = True
                    self.cv.notify_all()
        if early:
            if live:
                self._mark(ver, healthy)
            return
        if sync:
            for st in live:
                self._drive(st)

    def _drive(self, st: _Stream) -> None:
        """Send the newest device list on ``st`` until it has sent the current version; returns
        at once if another thread is sending on it (that thread re-checks the version before it
        lets go, under the same lock notify() bumps it under, so no update is left unsent)."""
        with self.cv:
            if st.busy or not st.alive:
                return
            st.busy = True
        try:
            while True:
                with self.cv:
                    ver = self.version
                    if st.sent >= ver or not st.alive or self.stopped:
                        st.busy = False
                        return
                    pend = self._pending if self._pending and self._pending[0] == ver else None
                if pend is None:  # first message of a new stream
                    resp, healthy = self._devices_msg()
                else:
                    resp, healthy = pend[1], pend[2]
                st.send(resp)  # returns once gRPC has written the message
                st.sent = ver
                if st.context.is_active():
                    self._mark(ver, healthy)
                else:
                    st.alive = False
        except BaseException:
            with self.cv:
                st.busy = False
            raise

    def _send_loop(self) -> None:
        while not self.stopped:
            with self.cv:
                while not self._wake and not self.stopped:
                    self.cv.wait(timeout=1.0)
                self._wake = False
                live = list(self._live)
            for st in live:
                try:
                    self._drive(st)
                except Exception:
                    log.exception("ListAndWatch send failed")

    def _mark(self, version: int, healthy: set[str] | None) -> None:
        """A stream wrote device list ``version`` (``healthy`` = its Healthy GPUs), or ended
        (``None``: with no stream left nothing counts as advertised). Versions only move forward —
        a late send of an older list never undoes a newer one — but the same version may mark
        again: a new stream (a restarted kubelet) starts by resending the current list."""
        with self._mark_mu:
            if healthy is not None:
                if version < self._marked:
                    return
                self._marked = version
            self.agent.mark_advertised(self.resource, healthy)

    # ------------------------------------------------------------ API
    def GetDevicePluginOptions(self, request, context):
        return DP.DevicePluginOptions(pre_start_required=False,
                                      get_preferred_allocation_available=True)

    def _devices_msg(self) -> tuple[DP.ListAndWatchResponse, set[str]]:
        resp = DP.ListAndWatchResponse()
        healthy = set()
        for d in self.agent.plugin_devices(self.resource):
            dev = resp.devices.add()
            dev.ID = d.get("id") or d["uuid"]
            dev.health = "Healthy" if d["advertisable"] else "Unhealthy"
            if d.get("numa") is not None:
                dev.topology.nodes.add().ID = int(d["numa"])
            if d["advertisable"]:
                healthy.add(d["uuid"])
        return resp, healthy

    def ListAndWatch(self, request, context, send):
        """Non-blocking handler: register the stream, send it the current list, return. The
        stream stays open until the kubelet goes away or the plugin stops."""
        st = _Stream(send, context)

        def gone():
            st.alive = False
            with self.cv:
                if st in self._live:
                    self._live.discard(st)
                    self.streams -= 1
                last = not self._live
            # only when no stream is left does nothing count as advertised: a restarted kubelet's
            # new stream may already have marked its list when the old stream's callback fires
            if last:
                self._mark(self.version, None)
                # every stream ended: the kubelet went away (or restarted). Its new socket can
                # carry the old (inode, ctime) on tmpfs when it comes back within one timestamp
                # tick, so the monitor also re-registers on this signal
                self._streams_lost = True
        with self.cv:
            self._live.add(st)
            self.streams += 1
        if not context.add_callback(gone):  # already terminated
            gone()
            return
        self._drive(st)

    def GetPreferredAllocation(self, request, context):
        out = DP.PreferredAllocationResponse()
        for creq in request.container_requests:
            ids = self.agent.preferred(self.resource, list(creq.available_deviceIDs),
                                       list(creq.must_include_deviceIDs), creq.allocation_size)
            out.container_responses.add().deviceIDs.extend(ids)
        return out

    def Allocate(self, request, context):
        out = DP.AllocateResponse()
        for creq in request.container_requests:
            try:
                spec = self.agent.allocate_spec(self.resource, list(creq.devices_ids))
            except ValueError as e:
                context.abort(grpc.StatusCode.FAILED_PRECONDITION, str(e))
            c = out.container_responses.add()
            for k, v in spec["envs"].items():
                c.envs[k] = v
            for k, v in spec["annotations"].items():
                c.annotations[k] = v
            for dspec in spec["devices"]:
                c.devices.add(container_path=dspec, host_path=dspec, permissions="rw")
            for m in spec.get("mounts") or []:  # e.g. libgpupool_share.so for isolated sharing
                c.mounts.add(container_path=m["container_path"], host_path=m["host_path"],
                             read_only=bool(m.get("read_only", True)))
        return out

    def PreStartContainer(self, request, context):
        return DP.PreStartContainerResponse()
