"""Codegen-free gRPC plumbing for the kubelet DevicePlugin v1beta1 and PodResources v1 APIs.

``grpc_tools`` is not installed and protoc-3.13-generated ``_pb2.py`` modules do not load under the
protobuf 7 runtime, so the ``.proto`` files in this directory are compiled once to descriptor sets
(``protoc --descriptor_set_out``; see ``regenerate()``) and the message classes are built at import
time from those descriptors with ``message_factory.GetMessageClass``. Services are exposed as
generic method handlers (server) and multicallables (client), which is all grpcio needs.
"""
from __future__ import annotations

import os
import shutil
import subprocess
from typing import Callable

import grpc
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

HERE = os.path.dirname(os.path.abspath(__file__))
_POOL = descriptor_pool.DescriptorPool()


def _load(desc_name: str) -> None:
    with open(os.path.join(HERE, desc_name), "rb") as f:
        fds = descriptor_pb2.FileDescriptorSet.FromString(f.read())
    for fdp in fds.file:
        _POOL.Add(fdp)


_load("deviceplugin.desc")
_load("podresources.desc")


def msg(full_name: str):
    return message_factory.GetMessageClass(_POOL.FindMessageTypeByName(full_name))


class DP:
    """v1beta1 message classes."""
    DevicePluginOptions = msg("v1beta1.DevicePluginOptions")
    RegisterRequest = msg("v1beta1.RegisterRequest")
    Empty = msg("v1beta1.Empty")
    ListAndWatchResponse = msg("v1beta1.ListAndWatchResponse")
    TopologyInfo = msg("v1beta1.TopologyInfo")
    NUMANode = msg("v1beta1.NUMANode")
    Device = msg("v1beta1.Device")
    PreStartContainerRequest = msg("v1beta1.PreStartContainerRequest")
    PreStartContainerResponse = msg("v1beta1.PreStartContainerResponse")
    PreferredAllocationRequest = msg("v1beta1.PreferredAllocationRequest")
    PreferredAllocationResponse = msg("v1beta1.PreferredAllocationResponse")
    ContainerPreferredAllocationResponse = msg("v1beta1.ContainerPreferredAllocationResponse")
    AllocateRequest = msg("v1beta1.AllocateRequest")
    AllocateResponse = msg("v1beta1.AllocateResponse")
    ContainerAllocateResponse = msg("v1beta1.ContainerAllocateResponse")
    Mount = msg("v1beta1.Mount")
    DeviceSpec = msg("v1beta1.DeviceSpec")


class PR:
    """podresources v1 message classes."""
    ListPodResourcesRequest = msg("v1.ListPodResourcesRequest")
    ListPodResourcesResponse = msg("v1.ListPodResourcesResponse")
    PodResources = msg("v1.PodResources")
    ContainerResources = msg("v1.ContainerResources")
    ContainerDevices = msg("v1.ContainerDevices")
    AllocatableResourcesRequest = msg("v1.AllocatableResourcesRequest")
    AllocatableResourcesResponse = msg("v1.AllocatableResourcesResponse")


API_VERSION = "v1beta1"
KUBELET_SOCKET = "kubelet.sock"
DEVICE_PLUGIN_PATH = "/var/lib/kubelet/device-plugins"
POD_RESOURCES_SOCKET = "/var/lib/kubelet/pod-resources/kubelet.sock"

# (service, method) -> (request class, response class, server-streaming?)
METHODS = {
    ("v1beta1.Registration", "Register"): (DP.RegisterRequest, DP.Empty, False),
    ("v1beta1.DevicePlugin", "GetDevicePluginOptions"): (DP.Empty, DP.DevicePluginOptions, False),
    ("v1beta1.DevicePlugin", "ListAndWatch"): (DP.Empty, DP.ListAndWatchResponse, True),
    ("v1beta1.DevicePlugin", "GetPreferredAllocation"): (DP.PreferredAllocationRequest,
                                                        DP.PreferredAllocationResponse, False),
    ("v1beta1.DevicePlugin", "Allocate"): (DP.AllocateRequest, DP.AllocateResponse, False),
    ("v1beta1.DevicePlugin", "PreStartContainer"): (DP.PreStartContainerRequest,
                                                   DP.PreStartContainerResponse, False),
    ("v1.PodResourcesLister", "List"): (PR.ListPodResourcesRequest, PR.ListPodResourcesResponse,
                                        False),
    ("v1.PodResourcesLister", "GetAllocatableResources"): (PR.AllocatableResourcesRequest,
                                                           PR.AllocatableResourcesResponse, False),
}


def service_handler(service: str, impl: dict[str, Callable]) -> grpc.GenericRpcHandler:
    """Build a generic handler for ``service`` from {method_name: fn(request, context)}."""
    handlers = {}
    for (svc, method), (req, resp, streaming) in METHODS.items():
        if svc != service or method not in impl:
            continue
        if streaming:
            handlers[method] = grpc.unary_stream_rpc_method_handler(
                impl[method], request_deserializer=req.FromString,
                response_serializer=resp.SerializeToString)
        else:
            handlers[method] = grpc.unary_unary_rpc_method_handler(
                impl[method], request_deserializer=req.FromString,
                response_serializer=resp.SerializeToString)
    return grpc.method_handlers_generic_handler(service, handlers)


class Stub:
    """Client stub: ``Stub(channel, "v1beta1.DevicePlugin").Allocate(req)``."""

    def __init__(self, channel: grpc.Channel, service: str):
        for (svc, method), (req, resp, streaming) in METHODS.items():
            if svc != service:
                continue
            path = f"/{svc}/{method}"
            if streaming:
                fn = channel.unary_stream(path, request_serializer=req.SerializeToString,
                                          response_deserializer=resp.FromString)
            else:
                fn = channel.unary_unary(path, request_serializer=req.SerializeToString,
                                         response_deserializer=resp.FromString)
            setattr(self, method, fn)


def unix_target(path: str) -> str:
    return "unix://" + os.path.abspath(path)


# gRPC Python shares subchannels between channels to one target through a process-wide pool: a
# new channel to a socket whose previous listener died inherits that subchannel's reconnect
# backoff (1 s, growing towards 2 min while the peer stays away) and fails UNAVAILABLE until it
# expires — a re-registration or a fresh ListAndWatch after a kubelet or agent restart then waits
# out the old connection's backoff. Channels that mean "connect now" take a private pool, as
# every new connection in Go's gRPC (the kubelet's) is.
FRESH_CHANNEL = [("grpc.use_local_subchannel_pool", 1)]


def fresh_channel(path: str, options: list | None = None):
    import grpc
    return grpc.insecure_channel(unix_target(path), options=FRESH_CHANNEL + list(options or []))


def regenerate(check: bool = False) -> bool:
    """Recompile the descriptor sets with protoc (torch ships one). Returns True if up to date."""
    protoc = shutil.which("protoc")
    if protoc is None:
        try:
            import torch
            cand = os.path.join(os.path.dirname(torch.__file__), "bin", "protoc")
            protoc = cand if os.path.exists(cand) else None
        except ImportError:
            protoc = None
    if protoc is None:
        return True
    fresh = True
    for name in ("deviceplugin", "podresources"):
        out = os.path.join(HERE, f"{name}.desc")
        tmp = out + ".new"
        subprocess.run([protoc, f"--descriptor_set_out={tmp}", f"{name}.proto"], cwd=HERE, check=True)
        with open(tmp, "rb") as f:
            new = f.read()
        old = open(out, "rb").read() if os.path.exists(out) else b""
        if new != old:
            fresh = False
            if not check:
                os.replace(tmp, out)
                continue
        os.remove(tmp)
    return fresh
