"""The nos-amd device plugin on the kubelet device-plugin API v1beta1.

One gRPC server per advertised resource (kubelet requires one endpoint per
resource name) under ``/var/lib/kubelet/device-plugins/``, each registered
with the kubelet's ``Registration`` service.  ``ListAndWatch`` streams the
resource's devices again whenever the plugin re-enumerates (mode switch,
new slice table); ``Allocate`` returns the envs / device nodes of
:meth:`NosAmdDevicePlugin.allocate`; ``GetPreferredAllocation`` implements
the pack/spread policy.  When the slice table drops a resource its server is
stopped; when the kubelet restarts (its socket is re-created) every
resource is re-registered -- standard device-plugin lifecycle.
"""
from __future__ import annotations

import logging
import os
import re
import threading
from pathlib import Path

import grpc

from ..api import constants as C
from ..grpcapi import rpc
from ..grpcapi.protos import DEVICE_PLUGIN_VERSION, HEALTHY, UNHEALTHY
from ..grpcapi.protos import deviceplugin as pb
from .plugin import NosAmdDevicePlugin

log = logging.getLogger("nos_amd.deviceplugin.grpc")


def endpoint_name(resource: str) -> str:
    return "nos-amd-" + re.sub(r"[^a-zA-Z0-9.-]+", "_", resource.split("/", 1)[-1]) + ".sock"


class _ResourceServicer:
    def __init__(self, owner: "DevicePluginServers", resource: str):
        self.owner, self.resource = owner, resource
        self.stopped = threading.Event()

    def _devices(self):
        return [pb.Device(ID=d.id, health=HEALTHY if d.healthy else UNHEALTHY)
                for d in sorted(self.owner.plugin.list_devices(self.resource), key=lambda d: d.id)]

    def GetDevicePluginOptions(self, request, context):  # noqa: N802
        return pb.DevicePluginOptions(pre_start_required=False, get_preferred_allocation_available=True)

    def ListAndWatch(self, request, context):  # noqa: N802
        gen = -1
        while not self.stopped.is_set() and context.is_active():
            with self.owner.cond:
                if self.owner.plugin.generation == gen:
                    self.owner.cond.wait(timeout=1.0)
                    continue
                gen = self.owner.plugin.generation
            yield pb.ListAndWatchResponse(devices=self._devices())

    def GetPreferredAllocation(self, request, context):  # noqa: N802
        out = []
        for cr in request.container_requests:
            ids = self.owner.plugin.preferred_allocation(self.resource, list(cr.available_deviceIDs),
                                                         list(cr.must_include_deviceIDs), cr.allocation_size)
            out.append(pb.ContainerPreferredAllocationResponse(deviceIDs=ids))
        return pb.PreferredAllocationResponse(container_responses=out)

    def Allocate(self, request, context):  # noqa: N802
        out = []
        for cr in request.container_requests:
            try:
                a = self.owner.plugin.allocate(self.resource, list(cr.devices_ids), owner="kubelet")
            except (KeyError, RuntimeError) as e:
                context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
            out.append(pb.ContainerAllocateResponse(
                envs=a.envs, devices=[pb.DeviceSpec(container_path=d, host_path=d, permissions="rw")
                                      for d in a.devices],
                mounts=[pb.Mount(container_path=m, host_path=m, read_only=True) for m in a.mounts]))
        return pb.AllocateResponse(container_responses=out)

    def PreStartContainer(self, request, context):  # noqa: N802
        return pb.PreStartContainerResponse()


class DevicePluginServers:
    """Keeps one registered gRPC endpoint per resource of ``plugin``."""

    def __init__(self, plugin: NosAmdDevicePlugin, plugin_dir: str | Path = C.DEVICE_PLUGIN_DIR,
                 kubelet_socket: str | Path | None = None, podresources=None):
        self.plugin = plugin
        self.dir = Path(plugin_dir)
        self.kubelet_socket = Path(kubelet_socket) if kubelet_socket else self.dir / "kubelet.sock"
        self.podresources = podresources
        self.cond = threading.Condition()
        self.servers: dict[str, tuple[grpc.Server, _ResourceServicer]] = {}
        self._kubelet_id: tuple | None = None
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        plugin.listeners.append(lambda _p: self._changed())

    def _changed(self) -> None:
        with self.cond:
            self.cond.notify_all()

    def _register(self, resource: str) -> None:
        with grpc.insecure_channel(rpc.unix_target(self.kubelet_socket)) as ch:
            rpc.Stub(ch, pb, "Registration").Register(pb.RegisterRequest(
                version=DEVICE_PLUGIN_VERSION, endpoint=endpoint_name(resource), resource_name=resource,
                options=pb.DevicePluginOptions(get_preferred_allocation_available=True)), timeout=10)
        log.info("registered %s with the kubelet", resource)

    def sync(self) -> None:
        if self.podresources is not None:
            try:
                used = {d for p in self.podresources.list() for c in p.containers for cd in c.devices
                        for d in cd.device_ids}
                self.plugin.sync_allocated(used)
            except Exception as e:
                log.debug("podresources unavailable: %s", e)
        want = set(self.plugin.resources())
        for res in list(self.servers):
            if res not in want:
                srv, svc = self.servers.pop(res)
                svc.stopped.set()
                srv.stop(grace=1)
                log.info("resource %s withdrawn", res)
        for res in sorted(want - set(self.servers)):
            svc = _ResourceServicer(self, res)
            srv = rpc.serve_unix(self.dir / endpoint_name(res), [rpc.handler(pb, "DevicePlugin", svc)])
            self.servers[res] = (srv, svc)
            try:
                self._register(res)
            except grpc.RpcError as e:
                log.warning("could not register %s: %s", res, e)
        self._changed()

    def _kubelet_changed(self) -> bool:
        try:
            st = os.stat(self.kubelet_socket)
            ident = (st.st_ino, st.st_ctime)
        except FileNotFoundError:
            ident = None
        changed = ident is not None and ident != self._kubelet_id
        self._kubelet_id = ident
        return changed

    def run(self, poll_s: float = 2.0) -> None:
        self._kubelet_changed()
        self.sync()
        while not self._stop.wait(poll_s):
            if self._kubelet_changed():  # kubelet restarted: every endpoint must register again
                log.info("kubelet socket re-created: re-registering")
                for res in list(self.servers):
                    try:
                        self._register(res)
                    except grpc.RpcError as e:
                        log.warning("re-register %s failed: %s", res, e)
            self.sync()

    def start(self) -> "DevicePluginServers":
        self._thread = threading.Thread(target=self.run, daemon=True, name="deviceplugin")
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        for srv, svc in self.servers.values():
            svc.stopped.set()
            srv.stop(grace=1)
        self.servers.clear()
