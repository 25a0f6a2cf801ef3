"""In-process kubelet for the simulator and the bench.

What the reference gets from a real kubelet and that the control plane
depends on:

* node ``status.capacity/allocatable`` tracking the device plugins'
  healthy devices (the partitioner and the scheduler read it);
* device admission: a bound pod's extended-resource requests are served by
  the plugin that owns the resource (``Allocate``); a pod whose devices are
  not available fails with ``UnexpectedAdmissionError`` (kubelet behaviour);
* the PodResources API (``List`` / ``GetAllocatableResources``) the agents
  read device usage from (``pkg/resource/lister.go:26-38``);
* pod lifecycle: Pending -> Running (containers started with the env the
  plugin returned), Succeeded/Failed on completion, devices released when
  the pod terminates or is deleted.

A ``runtime`` hook lets the bench start real GPU tenants with the
``ContainerAllocation`` envs (``ROC_GLOBAL_CU_MASK`` ...); without one the
containers are only recorded.
"""
from __future__ import annotations

import logging
import threading
from dataclasses import dataclass, field
from typing import Callable

from ..deviceplugin.plugin import ContainerAllocation, NosAmdDevicePlugin
from ..kube import objects as ko
from ..resource.client import ContainerDevices, ContainerResources, PodResources
from ..runtime.manager import Controller, Request, Result

log = logging.getLogger("nos_amd.sim.kubelet")

DEFAULT_NODE_RESOURCES = {"cpu": "128", "memory": "2048Gi", "pods": "250", "ephemeral-storage": "2Ti"}


@dataclass
class RunningContainer:
    pod: str                     # namespace/name
    name: str
    allocations: dict[str, ContainerAllocation] = field(default_factory=dict)  # resource -> allocation

    @property
    def envs(self) -> dict[str, str]:
        out: dict[str, str] = {}
        for a in self.allocations.values():
            out.update(a.envs)
        return out


def _extended_requests(c: dict) -> dict[str, int]:
    """Extended resources of a container (requests default to limits)."""
    req = dict(ko.container_limits(c))
    req.update(ko.container_requests(c))
    return {k: int(v) for k, v in req.items() if "/" in k and not k.startswith("nos.nebuly.com/") and v > 0}


class Kubelet:
    """One simulated node agent.  Use :meth:`controller` on a per-node
    :class:`~nos_amd.runtime.manager.Manager`, or call :meth:`sync_pod`
    directly."""

    def __init__(self, api, node_name: str, plugins: list[NosAmdDevicePlugin] | None = None,
                 node_resources: dict[str, str] | None = None,
                 runtime: Callable[[dict, list[RunningContainer]], None] | None = None,
                 on_stop: Callable[[dict, list[RunningContainer]], None] | None = None):
        self.api = api
        self.node_name = node_name
        self.plugins: list[NosAmdDevicePlugin] = list(plugins or [])
        self.node_resources = dict(DEFAULT_NODE_RESOURCES if node_resources is None else node_resources)
        self.runtime = runtime
        self.on_stop = on_stop
        self._lock = threading.RLock()
        self.containers: dict[str, list[RunningContainer]] = {}   # pod key -> containers
        self.pod_devices: dict[str, list[tuple[str, str, list[str]]]] = {}  # key -> (container, res, ids)
        self.admission_failures: dict[str, str] = {}
        for p in self.plugins:
            p.listeners.append(lambda _p: self.sync_node_status())

    # ------------------------------------------------------------ node status
    def register_plugin(self, plugin: NosAmdDevicePlugin) -> None:
        self.plugins.append(plugin)
        plugin.listeners.append(lambda _p: self.sync_node_status())
        self.sync_node_status()

    def device_capacity(self) -> dict[str, int]:
        cap: dict[str, int] = {}
        for p in self.plugins:
            for res, devs in p.resources().items():
                cap[res] = cap.get(res, 0) + sum(1 for d in devs if d.healthy)
        return cap

    def sync_node_status(self) -> None:
        node = self.api.try_get("Node", self.node_name)
        if node is None:
            return
        have = (node.get("status") or {}).get("capacity") or {}
        dev = self.device_capacity()
        want = dict(self.node_resources)
        want.update({k: str(v) for k, v in dev.items()})
        # extended resources of our plugins that vanished go to 0 (kubelet keeps them at 0)
        for k in have:
            if k not in want and any(k.startswith(pre) for pre in ("amd.com/",)):
                want[k] = "0"
        if have == want and ((node.get("status") or {}).get("allocatable") or {}) == want:
            return
        self.api.patch("Node", self.node_name, {"status": {"capacity": want, "allocatable": want}},
                       subresource="status")

    # ------------------------------------------------------------ pods
    def _plugin_for(self, resource: str) -> NosAmdDevicePlugin | None:
        for p in self.plugins:
            if resource in p.resources():
                return p
        return None

    def _free_devices(self, plugin: NosAmdDevicePlugin, resource: str) -> list[str]:
        return sorted(d.id for d in plugin.list_devices(resource) if d.healthy and d.id not in plugin.allocated)

    def admit(self, pod: dict) -> tuple[bool, str, list[RunningContainer]]:
        """Allocate devices for every container; all-or-nothing."""
        key = ko.key(pod)
        granted: list[tuple[NosAmdDevicePlugin, str, list[str]]] = []
        conts: list[RunningContainer] = []
        devs: list[tuple[str, str, list[str]]] = []
        try:
            for c in ko.pod_containers(pod):
                rc = RunningContainer(key, c.get("name", "c"))
                for res, n in sorted(_extended_requests(c).items()):
                    plugin = self._plugin_for(res)
                    if plugin is None:
                        if res.startswith("amd.com/"):
                            raise RuntimeError(f"no device plugin serves {res}")
                        continue
                    free = self._free_devices(plugin, res)
                    if len(free) < n:
                        raise RuntimeError(f"Allocate failed: requested {n} {res}, available {len(free)}")
                    ids = plugin.preferred_allocation(res, free, [], n)
                    rc.allocations[res] = plugin.allocate(res, ids, owner=f"{key}/{rc.name}")
                    granted.append((plugin, res, ids))
                    devs.append((rc.name, res, ids))
                conts.append(rc)
        except Exception as e:  # roll back
            for plugin, _res, ids in granted:
                plugin.release(ids)
            return False, str(e), []
        with self._lock:
            self.containers[key] = conts
            self.pod_devices[key] = devs
        return True, "", conts

    def sync_pod(self, pod: dict) -> None:
        key = ko.key(pod)
        phase = ko.pod_phase(pod)
        if ko.deletion_timestamp(pod) or ko.is_terminated(pod):
            self._teardown(pod)
            return
        if phase == ko.RUNNING:
            return
        if key in self.containers:
            # admitted and started, but the Running status write was lost
            # (e.g. a 409): write it again -- the status is level-triggered
            self._set_running(pod, self.containers[key])
            return
        ok, reason, conts = self.admit(pod)
        if not ok:
            self.admission_failures[key] = reason
            log.info("pod %s rejected on %s: %s", key, self.node_name, reason)
            self.api.patch("Pod", ko.name(pod), {"status": {"phase": ko.FAILED, "reason": "UnexpectedAdmissionError",
                                                            "message": reason}}, ko.namespace(pod),
                           subresource="status")
            return
        if self.runtime is not None:
            self.runtime(pod, conts)
        self._set_running(pod, conts)

    def _set_running(self, pod: dict, conts: list[RunningContainer]) -> None:
        now = ko.now_rfc3339(self.api.clock.now())
        status = {"phase": ko.RUNNING, "startTime": now, "hostIP": "127.0.0.1",
                  "conditions": [c for c in ko.pod_conditions(pod) if c.get("type") != "Ready"]
                  + [{"type": "Ready", "status": "True", "lastTransitionTime": now}],
                  "containerStatuses": [{"name": rc.name, "ready": True, "restartCount": 0,
                                         "state": {"running": {"startedAt": now}}} for rc in conts]}
        self.api.patch("Pod", ko.name(pod), {"status": status}, ko.namespace(pod), subresource="status")

    def _teardown(self, pod: dict) -> None:
        key = ko.key(pod)
        with self._lock:
            conts = self.containers.pop(key, None)
            devs = self.pod_devices.pop(key, None)
        if conts is None:
            return
        if self.on_stop is not None:
            self.on_stop(pod, conts)
        for _c, res, ids in devs or []:
            plugin = self._plugin_for(res)
            if plugin is not None:
                plugin.release(ids)
        self.sync_node_status()

    def complete_pod(self, namespace: str, name: str, succeeded: bool = True) -> None:
        """The pod's containers exited."""
        pod = self.api.get("Pod", name, namespace)
        self.api.patch("Pod", name, {"status": {"phase": ko.SUCCEEDED if succeeded else ko.FAILED}}, namespace,
                       subresource="status")
        self._teardown(pod)

    def reconcile(self, req: Request) -> Result:
        pod = self.api.try_get("Pod", req.name, req.namespace)
        if pod is None:
            key = f"{req.namespace}/{req.name}"
            if key in self.containers:
                self._teardown({"metadata": {"name": req.name, "namespace": req.namespace}})
            return Result()
        if ko.pod_node(pod) != self.node_name:
            return Result()
        self.sync_pod(pod)
        return Result()

    def controller(self) -> Controller:
        from ..runtime.predicates import Funcs

        mine = lambda ev: ko.pod_node(ev.obj) == self.node_name  # noqa: E731
        return Controller(f"kubelet-{self.node_name}", self).for_kind(
            "Pod", Funcs(create=mine, update=mine, delete=mine, generic=mine))

    # ------------------------------------------------------------ PodResources API
    def list(self) -> list[PodResources]:
        with self._lock:
            out = []
            for key, devs in self.pod_devices.items():
                ns, name = key.split("/", 1)
                by_c: dict[str, ContainerResources] = {}
                for cname, res, ids in devs:
                    by_c.setdefault(cname, ContainerResources(cname)).devices.append(ContainerDevices(res, list(ids)))
                out.append(PodResources(name, ns, list(by_c.values())))
            return out

    def get_allocatable_resources(self) -> list[ContainerDevices]:
        out = []
        for p in self.plugins:
            for res, devs in sorted(p.resources().items()):
                ids = [d.id for d in devs if d.healthy]
                if ids:
                    out.append(ContainerDevices(res, ids))
        return out

    def running_containers(self) -> dict[str, list[RunningContainer]]:
        with self._lock:
            return {k: list(v) for k, v in self.containers.items()}
