"""kubelet PodResources API v1 — the client the validator uses to see which GPUs tenants hold.

kubelet serves ``k8s.io/kubelet/pkg/apis/podresources/v1`` (package ``v1``) on
``/var/lib/kubelet/pod-resources/kubelet.sock``:

* ``PodResourcesLister.List(ListPodResourcesRequest) returns ListPodResourcesResponse`` — every
  pod's containers with the device IDs each got from a device plugin;
* ``PodResourcesLister.GetAllocatableResources`` — the devices kubelet could hand out.

The validator must not load GPUs that kubelet has already given to a pod (a validator restart —
Renovate bump of the operator image, node reboot, eviction — would otherwise run GEMM / stress /
RCCL on GPUs serving ``coder-llm``); the reference's isolation contract is one pod per GPU
(reference README.md:301-387).  As in ``deviceplugin_api.py`` there is no ``protoc`` here, so the
FileDescriptorProto is assembled field by field with the upstream field numbers (identical wire
format) and exposed through grpcio's generic stubs/handlers.
"""
from __future__ import annotations

from typing import Callable, Dict, Iterable, Optional, Set

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PACKAGE = "v1"
SOCKET = "/var/lib/kubelet/pod-resources/kubelet.sock"

_F = descriptor_pb2.FieldDescriptorProto
_T = {"string": _F.TYPE_STRING, "int64": _F.TYPE_INT64, "uint64": _F.TYPE_UINT64}

_MESSAGES = {
    "ListPodResourcesRequest": [],
    "ListPodResourcesResponse": [("pod_resources", 1, "PodResources", "rep")],
    "PodResources": [("name", 1, "string", "opt"), ("namespace", 2, "string", "opt"),
                     ("containers", 3, "ContainerResources", "rep")],
    "ContainerResources": [("name", 1, "string", "opt"), ("devices", 2, "ContainerDevices", "rep"),
                           ("cpu_ids", 3, "int64", "rep"), ("memory", 4, "ContainerMemory", "rep")],
    "ContainerDevices": [("resource_name", 1, "string", "opt"), ("device_ids", 2, "string", "rep"),
                         ("topology", 3, "TopologyInfo", "opt")],
    "ContainerMemory": [("memory_type", 1, "string", "opt"), ("size", 2, "uint64", "opt"),
                        ("topology", 3, "TopologyInfo", "opt")],
    "TopologyInfo": [("nodes", 1, "NUMANode", "rep")],
    "NUMANode": [("ID", 1, "int64", "opt")],
    "AllocatableResourcesRequest": [],
    "AllocatableResourcesResponse": [("devices", 1, "ContainerDevices", "rep"),
                                     ("cpu_ids", 2, "int64", "rep"),
                                     ("memory", 3, "ContainerMemory", "rep")],
}

SERVICES = {
    "PodResourcesLister": [
        ("List", "ListPodResourcesRequest", "ListPodResourcesResponse"),
        ("GetAllocatableResources", "AllocatableResourcesRequest", "AllocatableResourcesResponse"),
    ],
}


def _build_file() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name="amdk8s/podresources/v1/api.proto", package=PACKAGE,
                                            syntax="proto3")
    for name, fields in _MESSAGES.items():
        m = fd.message_type.add(name=name)
        for fname, num, ftype, label in fields:
            f = m.field.add(name=fname, number=num, json_name=fname)
            f.label = _F.LABEL_REPEATED if label == "rep" else _F.LABEL_OPTIONAL
            if ftype in _T:
                f.type = _T[ftype]
            else:
                f.type = _F.TYPE_MESSAGE
                f.type_name = f".{PACKAGE}.{ftype}"
    for sname, methods in SERVICES.items():
        s = fd.service.add(name=sname)
        for mname, inp, out in methods:
            s.method.add(name=mname, input_type=f".{PACKAGE}.{inp}", output_type=f".{PACKAGE}.{out}")
    return fd


_POOL = descriptor_pool.DescriptorPool()
_POOL.Add(_build_file())
_FD = _POOL.FindFileByName("amdk8s/podresources/v1/api.proto")
_BY_NAME = {n: message_factory.GetMessageClass(_FD.message_types_by_name[n]) for n in _MESSAGES}

ListPodResourcesRequest = _BY_NAME["ListPodResourcesRequest"]
ListPodResourcesResponse = _BY_NAME["ListPodResourcesResponse"]
PodResources = _BY_NAME["PodResources"]
ContainerResources = _BY_NAME["ContainerResources"]
ContainerDevices = _BY_NAME["ContainerDevices"]
AllocatableResourcesRequest = _BY_NAME["AllocatableResourcesRequest"]
AllocatableResourcesResponse = _BY_NAME["AllocatableResourcesResponse"]


def method_path(method: str, service: str = "PodResourcesLister") -> str:
    return f"/{PACKAGE}.{service}/{method}"


def generic_handler(impl: Dict[str, Callable], service: str = "PodResourcesLister"):
    """grpcio handler (for the fake kubelet in tests) from {method: callable(request, context)}."""
    import grpc

    handlers = {}
    for mname, inp, out in SERVICES[service]:
        if mname in impl:
            handlers[mname] = grpc.unary_unary_rpc_method_handler(
                impl[mname], request_deserializer=_BY_NAME[inp].FromString,
                response_serializer=_BY_NAME[out].SerializeToString)
    return grpc.method_handlers_generic_handler(f"{PACKAGE}.{service}", handlers)


def list_pod_resources(socket: str = SOCKET, timeout: float = 10.0):
    """One ``List`` call over the kubelet's unix socket."""
    import grpc

    with grpc.insecure_channel("unix://" + socket) as ch:
        call = ch.unary_unary(method_path("List"),
                              request_serializer=ListPodResourcesRequest.SerializeToString,
                              response_deserializer=ListPodResourcesResponse.FromString)
        return call(ListPodResourcesRequest(), timeout=timeout)


def allocated_device_ids(resp, resource: str) -> Dict[str, str]:
    """{kubelet device ID: "namespace/pod"} of every device of ``resource`` held by a container."""
    out: Dict[str, str] = {}
    for pod in resp.pod_resources:
        for c in pod.containers:
            for dev in c.devices:
                if dev.resource_name == resource:
                    for i in dev.device_ids:
                        out[i] = f"{pod.namespace}/{pod.name}"
    return out


def allocated(resource: str, socket: str = SOCKET, timeout: float = 10.0,
              exclude_pods: Iterable[str] = ()) -> Optional[Dict[str, str]]:
    """Allocated device IDs of ``resource`` (None when the PodResources socket is absent)."""
    import os

    if not os.path.exists(socket):
        return None
    skip: Set[str] = set(exclude_pods)
    return {k: v for k, v in allocated_device_ids(list_pod_resources(socket, timeout), resource).items()
            if v not in skip}
