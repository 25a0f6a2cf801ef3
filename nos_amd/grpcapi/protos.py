"""Kubelet gRPC APIs built at import time from descriptors (no protoc in
the image): the device-plugin API ``v1beta1`` (Registration + DevicePlugin)
and the PodResources API ``v1`` (PodResourcesLister).

Message and field numbers follow the public Kubernetes protos
(``k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/api.proto``,
``k8s.io/kubelet/pkg/apis/podresources/v1/api.proto``), so the wire format is
what a real kubelet speaks.  The reference consumed PodResources through the
Go client (``pkg/resource/lister.go:26-38``) and relied on NVIDIA's device
plugin; both ends live here.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

F = descriptor_pb2.FieldDescriptorProto
_STR, _BOOL, _I64, _I32, _MSG = F.TYPE_STRING, F.TYPE_BOOL, F.TYPE_INT64, F.TYPE_INT32, F.TYPE_MESSAGE
_OPT, _REP = F.LABEL_OPTIONAL, F.LABEL_REPEATED

_pool = descriptor_pool.DescriptorPool()


def _msg(fdp, name: str, fields: list[tuple], maps: dict[str, int] | None = None) -> None:
    """fields: (name, number, type, label, type_name-or-None)."""
    m = fdp.message_type.add()
    m.name = name
    for fname, num, ftype, label, tname in fields:
        f = m.field.add()
        f.name, f.number, f.type, f.label = fname, num, ftype, label
        f.json_name = fname
        if tname:
            f.type_name = tname
    for fname, num in (maps or {}).items():  # map<string, string>
        entry = m.nested_type.add()
        entry.name = "".join(p.capitalize() for p in fname.split("_")) + "Entry"
        entry.options.map_entry = True
        for kname, knum in (("key", 1), ("value", 2)):
            kf = entry.field.add()
            kf.name, kf.number, kf.type, kf.label = kname, knum, _STR, _OPT
        f = m.field.add()
        f.name, f.number, f.type, f.label = fname, num, _MSG, _REP
        f.type_name = f".{fdp.package}.{name}.{entry.name}"


def _service(fdp, name: str, methods: list[tuple]) -> None:
    s = fdp.service.add()
    s.name = name
    for mname, inp, out, server_streaming in methods:
        m = s.method.add()
        m.name, m.input_type, m.output_type = mname, f".{fdp.package}.{inp}", f".{fdp.package}.{out}"
        m.server_streaming = server_streaming


def _deviceplugin_file() -> descriptor_pb2.FileDescriptorProto:
    fdp = descriptor_pb2.FileDescriptorProto(name="nos_amd/deviceplugin/v1beta1/api.proto", package="v1beta1",
                                             syntax="proto3")
    P = ".v1beta1."
    _msg(fdp, "DevicePluginOptions", [("pre_start_required", 1, _BOOL, _OPT, None),
                                      ("get_preferred_allocation_available", 2, _BOOL, _OPT, None)])
    _msg(fdp, "RegisterRequest", [("version", 1, _STR, _OPT, None), ("endpoint", 2, _STR, _OPT, None),
                                  ("resource_name", 3, _STR, _OPT, None),
                                  ("options", 4, _MSG, _OPT, P + "DevicePluginOptions")])
    _msg(fdp, "Empty", [])
    _msg(fdp, "NUMANode", [("ID", 1, _I64, _OPT, None)])
    _msg(fdp, "TopologyInfo", [("nodes", 1, _MSG, _REP, P + "NUMANode")])
    _msg(fdp, "Device", [("ID", 1, _STR, _OPT, None), ("health", 2, _STR, _OPT, None),
                         ("topology", 3, _MSG, _OPT, P + "TopologyInfo")])
    _msg(fdp, "ListAndWatchResponse", [("devices", 1, _MSG, _REP, P + "Device")])
    _msg(fdp, "PreStartContainerRequest", [("devices_ids", 1, _STR, _REP, None)])
    _msg(fdp, "PreStartContainerResponse", [])
    _msg(fdp, "ContainerPreferredAllocationRequest", [("available_deviceIDs", 1, _STR, _REP, None),
                                                      ("must_include_deviceIDs", 2, _STR, _REP, None),
                                                      ("allocation_size", 3, _I32, _OPT, None)])
    _msg(fdp, "PreferredAllocationRequest",
         [("container_requests", 1, _MSG, _REP, P + "ContainerPreferredAllocationRequest")])
    _msg(fdp, "ContainerPreferredAllocationResponse", [("deviceIDs", 1, _STR, _REP, None)])
    _msg(fdp, "PreferredAllocationResponse",
         [("container_responses", 1, _MSG, _REP, P + "ContainerPreferredAllocationResponse")])
    _msg(fdp, "ContainerAllocateRequest", [("devices_ids", 1, _STR, _REP, None)])
    _msg(fdp, "AllocateRequest", [("container_requests", 1, _MSG, _REP, P + "ContainerAllocateRequest")])
    _msg(fdp, "Mount", [("container_path", 1, _STR, _OPT, None), ("host_path", 2, _STR, _OPT, None),
                        ("read_only", 3, _BOOL, _OPT, None)])
    _msg(fdp, "DeviceSpec", [("container_path", 1, _STR, _OPT, None), ("host_path", 2, _STR, _OPT, None),
                             ("permissions", 3, _STR, _OPT, None)])
    _msg(fdp, "CDIDevice", [("name", 1, _STR, _OPT, None)])
    _msg(fdp, "ContainerAllocateResponse", [("mounts", 2, _MSG, _REP, P + "Mount"),
                                            ("devices", 3, _MSG, _REP, P + "DeviceSpec"),
                                            ("cdi_devices", 5, _MSG, _REP, P + "CDIDevice")],
         maps={"envs": 1, "annotations": 4})
    _msg(fdp, "AllocateResponse", [("container_responses", 1, _MSG, _REP, P + "ContainerAllocateResponse")])
    _service(fdp, "Registration", [("Register", "RegisterRequest", "Empty", False)])
    _service(fdp, "DevicePlugin", [
        ("GetDevicePluginOptions", "Empty", "DevicePluginOptions", False),
        ("ListAndWatch", "Empty", "ListAndWatchResponse", True),
        ("GetPreferredAllocation", "PreferredAllocationRequest", "PreferredAllocationResponse", False),
        ("Allocate", "AllocateRequest", "AllocateResponse", False),
        ("PreStartContainer", "PreStartContainerRequest", "PreStartContainerResponse", False)])
    return fdp


def _podresources_file() -> descriptor_pb2.FileDescriptorProto:
    fdp = descriptor_pb2.FileDescriptorProto(name="nos_amd/podresources/v1/api.proto", package="v1",
                                             syntax="proto3")
    P = ".v1."
    _msg(fdp, "NUMANode", [("ID", 1, _I64, _OPT, None)])
    _msg(fdp, "TopologyInfo", [("nodes", 1, _MSG, _REP, P + "NUMANode")])
    _msg(fdp, "ContainerDevices", [("resource_name", 1, _STR, _OPT, None), ("device_ids", 2, _STR, _REP, None),
                                   ("topology", 3, _MSG, _OPT, P + "TopologyInfo")])
    _msg(fdp, "ContainerMemory", [("memory_type", 1, _STR, _OPT, None), ("size", 2, F.TYPE_UINT64, _OPT, None),
                                  ("topology", 3, _MSG, _OPT, P + "TopologyInfo")])
    _msg(fdp, "ContainerResources", [("name", 1, _STR, _OPT, None),
                                     ("devices", 2, _MSG, _REP, P + "ContainerDevices"),
                                     ("cpu_ids", 3, _I64, _REP, None),
                                     ("memory", 4, _MSG, _REP, P + "ContainerMemory")])
    _msg(fdp, "PodResources", [("name", 1, _STR, _OPT, None), ("namespace", 2, _STR, _OPT, None),
                               ("containers", 3, _MSG, _REP, P + "ContainerResources")])
    _msg(fdp, "ListPodResourcesRequest", [])
    _msg(fdp, "ListPodResourcesResponse", [("pod_resources", 1, _MSG, _REP, P + "PodResources")])
    _msg(fdp, "AllocatableResourcesRequest", [])
    _msg(fdp, "AllocatableResourcesResponse", [("devices", 1, _MSG, _REP, P + "ContainerDevices"),
                                               ("cpu_ids", 2, _I64, _REP, None),
                                               ("memory", 3, _MSG, _REP, P + "ContainerMemory")])
    _service(fdp, "PodResourcesLister", [
        ("List", "ListPodResourcesRequest", "ListPodResourcesResponse", False),
        ("GetAllocatableResources", "AllocatableResourcesRequest", "AllocatableResourcesResponse", False)])
    return fdp


class _Api:
    def __init__(self, fdp: descriptor_pb2.FileDescriptorProto):
        _pool.Add(fdp)
        self.package = fdp.package
        fd = _pool.FindFileByName(fdp.name)
        for m in fdp.message_type:
            setattr(self, m.name, message_factory.GetMessageClass(fd.message_types_by_name[m.name]))
        self.services = {s.name: [(mm.name, mm.input_type.split(".")[-1], mm.output_type.split(".")[-1],
                                   mm.server_streaming) for mm in s.method] for s in fdp.service}

    def method_path(self, service: str, method: str) -> str:
        return f"/{self.package}.{service}/{method}"


deviceplugin = _Api(_deviceplugin_file())
podresources = _Api(_podresources_file())

DEVICE_PLUGIN_VERSION = "v1beta1"
HEALTHY, UNHEALTHY = "Healthy", "Unhealthy"
