"""kubelet PodResources v1 client: which pods hold which device IDs (used for drain decisions)."""
from __future__ import annotations

import grpc

from .deviceplugin.proto import PR, Stub, unix_target


def list_pod_devices(socket_path: str, timeout: float = 2.0) -> dict[str, list[dict]]:
    """device ID -> [{"namespace","name","container","resource"}]."""
    out: dict[str, list[dict]] = {}
    with grpc.insecure_channel(unix_target(socket_path)) as ch:
        resp = Stub(ch, "v1.PodResourcesLister").List(PR.ListPodResourcesRequest(), timeout=timeout)
    for pr in resp.pod_resources:
        for c in pr.containers:
            for dev in c.devices:
                for did in dev.device_ids:
                    out.setdefault(did, []).append({"namespace": pr.namespace, "name": pr.name,
                                                    "container": c.name,
                                                    "resource": dev.resource_name})
    return out
