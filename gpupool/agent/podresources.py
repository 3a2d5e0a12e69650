"""kubelet PodResources v1 client: which pods hold which device IDs (used for drain decisions).

One persistent gRPC channel per socket: building a channel + HTTP/2 connection per call cost
1.6-3 ms on the MI355X box after an idle gap (profiles/r2d_agent_rpc_latency.json), which sat on
every ``GET /v1/node`` of the claim path."""
from __future__ import annotations

import threading

import grpc

from .deviceplugin.proto import PR, Stub, fresh_channel


class PodResourcesClient:
    def __init__(self, socket_path: str):
        self.socket_path = socket_path
        self._lock = threading.Lock()
        self._ch: grpc.Channel | None = None
        self._stub = None

    def _lister(self):
        with self._lock:
            if self._stub is None:
                self._ch = fresh_channel(self.socket_path)  # a reset must really reconnect
                self._stub = Stub(self._ch, "v1.PodResourcesLister")
            return self._stub

    def _reset(self) -> None:
        with self._lock:
            if self._ch is not None:
                self._ch.close()
            self._ch, self._stub = None, None

    def list_pod_devices(self, timeout: float = 2.0) -> dict[str, list[dict]]:
        """device ID -> [{"namespace","name","container","resource"}]."""
        try:
            resp = self._lister().List(PR.ListPodResourcesRequest(), timeout=timeout)
        except grpc.RpcError:
            self._reset()  # kubelet restarted: reconnect on the next call
            raise
        out: dict[str, list[dict]] = {}
        for pr in resp.pod_resources:
            for c in pr.containers:
                for dev in c.devices:
                    for did in dev.device_ids:
                        out.setdefault(did, []).append({"namespace": pr.namespace, "name": pr.name,
                                                        "container": c.name,
                                                        "resource": dev.resource_name})
        return out

    def close(self) -> None:
        self._reset()


def list_pod_devices(socket_path: str, timeout: float = 2.0) -> dict[str, list[dict]]:
    """One-shot form (tools, tests)."""
    c = PodResourcesClient(socket_path)
    try:
        return c.list_pod_devices(timeout)
    finally:
        c.close()
