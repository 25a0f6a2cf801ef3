"""Kubelet PodResources view: which devices exist and which are in use.

``pkg/resource/client.go:26-87`` + ``lister.go:26-38`` of the reference talk
gRPC to ``/var/lib/kubelet/pod-resources/kubelet.sock``.  Here the lister is
a protocol with two implementations:

* :class:`nos_amd.sim.kubelet.Kubelet` (in-process, used by the simulator and
  the bench);
* :class:`nos_amd.resource.podresources_grpc.GrpcLister` (the real kubelet
  socket, PodResources v1).

Both return plain data (:class:`PodResources` / :class:`ContainerDevices`),
from which :class:`Client` derives the used / allocatable device lists the
agents turn into status annotations.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Protocol

from .device import STATUS_FREE, STATUS_UNKNOWN, STATUS_USED, Device


@dataclass
class ContainerDevices:
    resource_name: str
    device_ids: list[str] = field(default_factory=list)


@dataclass
class ContainerResources:
    name: str
    devices: list[ContainerDevices] = field(default_factory=list)


@dataclass
class PodResources:
    name: str
    namespace: str
    containers: list[ContainerResources] = field(default_factory=list)


class PodResourcesLister(Protocol):
    def list(self) -> list[PodResources]: ...

    def get_allocatable_resources(self) -> list[ContainerDevices]: ...


class Client:
    """``resource.Client``: used devices (status used) and allocatable
    devices (status unknown), optionally restricted to a resource prefix."""

    def __init__(self, lister: PodResourcesLister):
        self.lister = lister

    def get_used_devices(self, prefix: str = "") -> list[Device]:
        out = []
        for pr in self.lister.list():
            for c in pr.containers:
                for cd in c.devices:
                    if cd.resource_name.startswith(prefix):
                        out.extend(Device(cd.resource_name, d, STATUS_USED) for d in cd.device_ids)
        return out

    def get_allocatable_devices(self, prefix: str = "") -> list[Device]:
        out = []
        for cd in self.lister.get_allocatable_resources():
            if cd.resource_name.startswith(prefix):
                out.extend(Device(cd.resource_name, d, STATUS_UNKNOWN) for d in cd.device_ids)
        return out

    def get_devices(self, prefix: str = "") -> list[Device]:
        """Allocatable devices with their used/free status resolved."""
        used = {d.device_id for d in self.get_used_devices(prefix)}
        return [d.with_status(STATUS_USED if d.device_id in used else STATUS_FREE)
                for d in self.get_allocatable_devices(prefix)]
