"""The kubelet's device-manager side of the device-plugin API, for tests and
the multi-process simulator: a ``Registration`` server on ``kubelet.sock``
that, for every registered plugin endpoint, follows ``ListAndWatch`` and can
allocate devices the way the kubelet does (``GetPreferredAllocation`` then
``Allocate``)."""
from __future__ import annotations

import logging
import threading
from pathlib import Path

import grpc

from ..grpcapi import rpc
from ..grpcapi.protos import HEALTHY
from ..grpcapi.protos import deviceplugin as pb

log = logging.getLogger("nos_amd.sim.kubelet_grpc")


class _Endpoint:
    def __init__(self, mgr: "DeviceManager", resource: str, endpoint: str):
        self.resource = resource
        self.channel = grpc.insecure_channel(rpc.unix_target(mgr.dir / endpoint))
        self.stub = rpc.Stub(self.channel, pb, "DevicePlugin")
        self.devices: dict[str, str] = {}
        self.updates = 0
        self._mgr = mgr
        self._thread = threading.Thread(target=self._watch, daemon=True, name=f"lw-{resource}")
        self._thread.start()

    def _watch(self) -> None:
        try:
            for resp in self.stub.ListAndWatch(pb.Empty()):
                with self._mgr.cond:
                    self.devices = {d.ID: d.health for d in resp.devices}
                    self.updates += 1
                    self._mgr.cond.notify_all()
        except grpc.RpcError as e:
            log.debug("ListAndWatch(%s) ended: %s", self.resource, e.code())
            with self._mgr.cond:
                self.devices = {}
                self._mgr.cond.notify_all()


class DeviceManager:
    def __init__(self, plugin_dir: str | Path):
        self.dir = Path(plugin_dir)
        self.cond = threading.Condition()
        self.endpoints: dict[str, _Endpoint] = {}
        self.allocated: dict[str, set[str]] = {}
        self.server = rpc.serve_unix(self.dir / "kubelet.sock", [rpc.handler(pb, "Registration", self)])

    def Register(self, request, context):  # noqa: N802
        if request.version != "v1beta1":
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"unsupported version {request.version}")
        self.endpoints[request.resource_name] = _Endpoint(self, request.resource_name, request.endpoint)
        return pb.Empty()

    def healthy(self, resource: str) -> list[str]:
        ep = self.endpoints.get(resource)
        return sorted(i for i, h in (ep.devices if ep else {}).items() if h == HEALTHY)

    def wait_for(self, pred, timeout: float = 5.0) -> bool:
        with self.cond:
            return self.cond.wait_for(pred, timeout)

    def allocate(self, resource: str, n: int) -> dict:
        ep = self.endpoints[resource]
        free = [d for d in self.healthy(resource) if d not in self.allocated.get(resource, set())]
        if len(free) < n:
            raise RuntimeError(f"only {len(free)} {resource} free")
        pref = ep.stub.GetPreferredAllocation(pb.PreferredAllocationRequest(container_requests=[
            pb.ContainerPreferredAllocationRequest(available_deviceIDs=free, allocation_size=n)]), timeout=5)
        ids = list(pref.container_responses[0].deviceIDs) or free[:n]
        resp = ep.stub.Allocate(pb.AllocateRequest(container_requests=[pb.ContainerAllocateRequest(
            devices_ids=ids)]), timeout=5)
        self.allocated.setdefault(resource, set()).update(ids)
        c = resp.container_responses[0]
        return {"ids": ids, "envs": dict(c.envs), "devices": [d.host_path for d in c.devices]}

    def stop(self) -> None:
        self.server.stop(grace=0)
        for ep in self.endpoints.values():
            ep.channel.close()
