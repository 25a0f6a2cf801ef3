"""Kubelet PodResources v1 over gRPC (``pkg/resource/lister.go:26-38``).

* :class:`GrpcLister` -- the agents' view of the real kubelet socket
  (``/var/lib/kubelet/pod-resources/kubelet.sock``), with the reference's
  10 s timeout and 16 MiB message cap;
* :func:`serve` -- exposes any in-process lister (e.g. the simulated
  kubelet) on a unix socket, so agents running as separate processes read
  the simulator exactly as they would read a kubelet.
"""
from __future__ import annotations

from pathlib import Path

import grpc

from ..api import constants as C
from ..grpcapi import rpc
from ..grpcapi.protos import podresources as pb
from .client import ContainerDevices, ContainerResources, PodResources, PodResourcesLister


class GrpcLister:
    def __init__(self, socket: str | Path = C.KUBELET_PODRESOURCES_SOCKET,
                 timeout_s: float = C.DEFAULT_PODRESOURCES_TIMEOUT_S,
                 max_msg: int = C.DEFAULT_PODRESOURCES_MAX_MSG):
        self.timeout_s = timeout_s
        self.channel = grpc.insecure_channel(rpc.unix_target(socket),
                                             options=[("grpc.max_receive_message_length", max_msg)])
        self.stub = rpc.Stub(self.channel, pb, "PodResourcesLister")

    def list(self) -> list[PodResources]:
        resp = self.stub.List(pb.ListPodResourcesRequest(), timeout=self.timeout_s)
        return [PodResources(p.name, p.namespace,
                             [ContainerResources(c.name, [ContainerDevices(d.resource_name, list(d.device_ids))
                                                          for d in c.devices]) for c in p.containers])
                for p in resp.pod_resources]

    def get_allocatable_resources(self) -> list[ContainerDevices]:
        resp = self.stub.GetAllocatableResources(pb.AllocatableResourcesRequest(), timeout=self.timeout_s)
        return [ContainerDevices(d.resource_name, list(d.device_ids)) for d in resp.devices]

    def close(self) -> None:
        self.channel.close()


class _Servicer:
    def __init__(self, lister: PodResourcesLister):
        self.lister = lister

    def List(self, request, context):  # noqa: N802
        return pb.ListPodResourcesResponse(pod_resources=[
            pb.PodResources(name=p.name, namespace=p.namespace, containers=[
                pb.ContainerResources(name=c.name, devices=[
                    pb.ContainerDevices(resource_name=d.resource_name, device_ids=d.device_ids) for d in c.devices])
                for c in p.containers]) for p in self.lister.list()])

    def GetAllocatableResources(self, request, context):  # noqa: N802
        return pb.AllocatableResourcesResponse(devices=[
            pb.ContainerDevices(resource_name=d.resource_name, device_ids=d.device_ids)
            for d in self.lister.get_allocatable_resources()])


def serve(lister: PodResourcesLister, socket: str | Path) -> grpc.Server:
    return rpc.serve_unix(socket, [rpc.handler(pb, "PodResourcesLister", _Servicer(lister))])
