"""kubelet Device Plugin API v1beta1 — protobuf messages and gRPC plumbing, built without protoc.

The kubelet speaks ``k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1`` (package ``v1beta1``):

* service ``Registration`` (served by kubelet on ``/var/lib/kubelet/device-plugins/kubelet.sock``):
  ``Register(RegisterRequest) returns (Empty)``
* service ``DevicePlugin`` (served by the plugin on its own socket in the same directory):
  ``GetDevicePluginOptions``, ``ListAndWatch`` (server stream), ``GetPreferredAllocation``,
  ``Allocate``, ``PreStartContainer``.

The reference never implements this — NVIDIA's plugin ships inside the GPU Operator chart
(SURVEY.md §2.2 X3).  ``grpc_tools``/``protoc`` are not available in the build image, so the
FileDescriptorProto is assembled field by field here (field numbers and names follow the upstream
api.proto, so the wire format is identical) and message classes come from protobuf's
message_factory.  Services are exposed to grpcio through generic method handlers.
"""
from __future__ import annotations

from typing import Callable, Dict

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PACKAGE = "v1beta1"
VERSION = "v1beta1"
KUBELET_SOCKET = "kubelet.sock"
DEVICE_PLUGIN_PATH = "/var/lib/kubelet/device-plugins"
HEALTHY = "Healthy"
UNHEALTHY = "Unhealthy"

_F = descriptor_pb2.FieldDescriptorProto
_T = {
    "string": _F.TYPE_STRING,
    "bool": _F.TYPE_BOOL,
    "int64": _F.TYPE_INT64,
    "int32": _F.TYPE_INT32,
}

# name -> list of (field_name, number, type, label) ; type is a scalar name or ".v1beta1.Msg"
_MESSAGES = {
    "DevicePluginOptions": [("pre_start_required", 1, "bool", "opt"),
                            ("get_preferred_allocation_available", 2, "bool", "opt")],
    "RegisterRequest": [("version", 1, "string", "opt"), ("endpoint", 2, "string", "opt"),
                        ("resource_name", 3, "string", "opt"),
                        ("options", 4, "DevicePluginOptions", "opt")],
    "Empty": [],
    "ListAndWatchResponse": [("devices", 1, "Device", "rep")],
    "TopologyInfo": [("nodes", 1, "NUMANode", "rep")],
    "NUMANode": [("ID", 1, "int64", "opt")],
    "Device": [("ID", 1, "string", "opt"), ("health", 2, "string", "opt"),
               ("topology", 3, "TopologyInfo", "opt")],
    "PreStartContainerRequest": [("devices_ids", 1, "string", "rep")],
    "PreStartContainerResponse": [],
    "PreferredAllocationRequest": [("container_requests", 1, "ContainerPreferredAllocationRequest", "rep")],
    "ContainerPreferredAllocationRequest": [("available_deviceIDs", 1, "string", "rep"),
                                            ("must_include_deviceIDs", 2, "string", "rep"),
                                            ("allocation_size", 3, "int32", "opt")],
    "PreferredAllocationResponse": [("container_responses", 1, "ContainerPreferredAllocationResponse", "rep")],
    "ContainerPreferredAllocationResponse": [("deviceIDs", 1, "string", "rep")],
    "AllocateRequest": [("container_requests", 1, "ContainerAllocateRequest", "rep")],
    "ContainerAllocateRequest": [("devices_ids", 1, "string", "rep")],
    "CDIDevice": [("name", 1, "string", "opt")],
    "AllocateResponse": [("container_responses", 1, "ContainerAllocateResponse", "rep")],
    "ContainerAllocateResponse": [("envs", 1, "map", "rep"), ("mounts", 2, "Mount", "rep"),
                                  ("devices", 3, "DeviceSpec", "rep"),
                                  ("annotations", 4, "map", "rep"),
                                  ("cdi_devices", 5, "CDIDevice", "rep")],
    "Mount": [("container_path", 1, "string", "opt"), ("host_path", 2, "string", "opt"),
              ("read_only", 3, "bool", "opt")],
    "DeviceSpec": [("container_path", 1, "string", "opt"), ("host_path", 2, "string", "opt"),
                   ("permissions", 3, "string", "opt")],
}

# service -> [(method, input, output, server_streaming)]
SERVICES = {
    "Registration": [("Register", "RegisterRequest", "Empty", False)],
    "DevicePlugin": [
        ("GetDevicePluginOptions", "Empty", "DevicePluginOptions", False),
        ("ListAndWatch", "Empty", "ListAndWatchResponse", True),
        ("GetPreferredAllocation", "PreferredAllocationRequest", "PreferredAllocationResponse", False),
        ("Allocate", "AllocateRequest", "AllocateResponse", False),
        ("PreStartContainer", "PreStartContainerRequest", "PreStartContainerResponse", False),
    ],
}


def _camel(s: str) -> str:
    return "".join(p[:1].upper() + p[1:] for p in s.split("_"))


def _build_file() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name="amdk8s/deviceplugin/v1beta1/api.proto",
                                            package=PACKAGE, syntax="proto3")
    for name, fields in _MESSAGES.items():
        m = fd.message_type.add(name=name)
        for fname, num, ftype, label in fields:
            f = m.field.add(name=fname, number=num)
            f.label = _F.LABEL_REPEATED if label == "rep" else _F.LABEL_OPTIONAL
            if ftype == "map":  # map<string,string> → nested XxxEntry{key=1,value=2} w/ map_entry
                entry = m.nested_type.add(name=_camel(fname) + "Entry")
                entry.options.map_entry = True
                entry.field.add(name="key", number=1, type=_F.TYPE_STRING, label=_F.LABEL_OPTIONAL)
                entry.field.add(name="value", number=2, type=_F.TYPE_STRING, label=_F.LABEL_OPTIONAL)
                f.type = _F.TYPE_MESSAGE
                f.type_name = f".{PACKAGE}.{name}.{entry.name}"
            elif ftype in _T:
                f.type = _T[ftype]
            else:
                f.type = _F.TYPE_MESSAGE
                f.type_name = f".{PACKAGE}.{ftype}"
            f.json_name = fname
    for sname, methods in SERVICES.items():
        s = fd.service.add(name=sname)
        for mname, inp, out, stream in methods:
            s.method.add(name=mname, input_type=f".{PACKAGE}.{inp}", output_type=f".{PACKAGE}.{out}",
                         server_streaming=stream)
    return fd


_POOL = descriptor_pool.DescriptorPool()
_FILE = _POOL.Add(_build_file())
_FD = _POOL.FindFileByName("amdk8s/deviceplugin/v1beta1/api.proto")


def _cls(name: str):
    return message_factory.GetMessageClass(_FD.message_types_by_name[name])


DevicePluginOptions = _cls("DevicePluginOptions")
RegisterRequest = _cls("RegisterRequest")
Empty = _cls("Empty")
ListAndWatchResponse = _cls("ListAndWatchResponse")
TopologyInfo = _cls("TopologyInfo")
NUMANode = _cls("NUMANode")
Device = _cls("Device")
PreStartContainerRequest = _cls("PreStartContainerRequest")
PreStartContainerResponse = _cls("PreStartContainerResponse")
PreferredAllocationRequest = _cls("PreferredAllocationRequest")
ContainerPreferredAllocationRequest = _cls("ContainerPreferredAllocationRequest")
PreferredAllocationResponse = _cls("PreferredAllocationResponse")
ContainerPreferredAllocationResponse = _cls("ContainerPreferredAllocationResponse")
AllocateRequest = _cls("AllocateRequest")
ContainerAllocateRequest = _cls("ContainerAllocateRequest")
CDIDevice = _cls("CDIDevice")
AllocateResponse = _cls("AllocateResponse")
ContainerAllocateResponse = _cls("ContainerAllocateResponse")
Mount = _cls("Mount")
DeviceSpec = _cls("DeviceSpec")

_BY_NAME = {n: _cls(n) for n in _MESSAGES}


def method_path(service: str, method: str) -> str:
    return f"/{PACKAGE}.{service}/{method}"


def generic_handler(service: str, impl: Dict[str, Callable]):
    """grpcio generic handler for ``service`` from a {method_name: callable(request, context)} dict."""
    import grpc

    handlers = {}
    for mname, inp, out, stream in SERVICES[service]:
        if mname not in impl:
            continue
        req_cls, resp_cls = _BY_NAME[inp], _BY_NAME[out]
        kw = dict(request_deserializer=req_cls.FromString,
                  response_serializer=resp_cls.SerializeToString)
        if stream:
            handlers[mname] = grpc.unary_stream_rpc_method_handler(impl[mname], **kw)
        else:
            handlers[mname] = grpc.unary_unary_rpc_method_handler(impl[mname], **kw)
    return grpc.method_handlers_generic_handler(f"{PACKAGE}.{service}", handlers)


class Stub:
    """Client stub for either service over a grpc channel: ``Stub(ch, 'DevicePlugin').Allocate(req)``."""

    def __init__(self, channel, service: str):
        for mname, inp, out, stream in SERVICES[service]:
            req_cls, resp_cls = _BY_NAME[inp], _BY_NAME[out]
            factory = channel.unary_stream if stream else channel.unary_unary
            setattr(self, mname, factory(method_path(service, mname),
                                         request_serializer=req_cls.SerializeToString,
                                         response_deserializer=resp_cls.FromString))


def unix_target(path: str) -> str:
    return "unix://" + path
