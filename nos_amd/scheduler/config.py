"""KubeSchedulerConfiguration loading and framework construction.

Accepts the reference's scheduler config (``config/scheduler/deployment/
scheduler_config.yaml``: profile ``nos-scheduler`` with CapacityScheduling at
preFilter/postFilter/reserve and ``pluginConfig`` args) and builds a
:class:`~nos_amd.scheduler.framework.Framework`.  ``CapacitySchedulingArgs``
keeps the reference field as an alias: ``nvidiaGpuResourceMemoryGB`` ->
``amdGpuResourceMemoryGB``; the default is 288 (one MI355X) instead of the
reference's accidental 0 (empty defaulter, ``v1beta3/defaults.go:19-21``).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from pathlib import Path
from typing import Any

import yaml

from ..api import constants as C
from .framework import Framework, Plugin, PodNominator, Snapshot
from .plugins import intree

DEFAULT_PLUGINS = {
    "queue_sort": ["PrioritySort"],
    "pre_filter": ["NodeResourcesFit"],
    "filter": ["NodeUnschedulable", "NodeName", "NodeAffinity", "TaintToleration", "NodeResourcesFit"],
    "post_filter": ["DefaultPreemption"],
    "score": ["NodeResourcesFit"],
    "reserve": [],
    "bind": ["DefaultBinder"],
}

_EP_KEYS = {"queueSort": "queue_sort", "preFilter": "pre_filter", "filter": "filter", "postFilter": "post_filter",
            "preScore": "pre_score", "score": "score", "reserve": "reserve", "permit": "permit",
            "preBind": "pre_bind", "bind": "bind", "postBind": "post_bind"}


@dataclass
class CapacitySchedulingArgs:
    amd_gpu_resource_memory_gb: int = C.DEFAULT_AMD_GPU_RESOURCE_MEMORY_GB

    @classmethod
    def from_dict(cls, d: dict | None) -> "CapacitySchedulingArgs":
        d = d or {}
        v = d.get("amdGpuResourceMemoryGB", d.get("nvidiaGpuResourceMemoryGB"))
        return cls(int(v) if v is not None else C.DEFAULT_AMD_GPU_RESOURCE_MEMORY_GB)

    def to_dict(self) -> dict:
        return {"amdGpuResourceMemoryGB": self.amd_gpu_resource_memory_gb}


@dataclass
class Profile:
    scheduler_name: str = "default-scheduler"
    plugins: dict[str, list[str]] = field(default_factory=lambda: {k: list(v) for k, v in DEFAULT_PLUGINS.items()})
    plugin_config: dict[str, dict] = field(default_factory=dict)


@dataclass
class SchedulerConfiguration:
    profiles: list[Profile] = field(default_factory=lambda: [Profile()])
    leader_elect: bool = False
    resource_name: str = "nos-scheduler"
    resource_namespace: str = "kube-system"


def _apply_plugin_set(base: list[str], spec: dict | None) -> list[str]:
    spec = spec or {}
    out = list(base)
    for d in spec.get("disabled") or []:
        if d.get("name") == "*":
            out = []
        else:
            out = [p for p in out if p != d.get("name")]
    for e in spec.get("enabled") or []:
        if e.get("name") not in out:
            out.append(e["name"])
    return out


def parse(data: dict) -> SchedulerConfiguration:
    le = data.get("leaderElection") or {}
    cfg = SchedulerConfiguration(profiles=[], leader_elect=bool(le.get("leaderElect", False)),
                                 resource_name=le.get("resourceName", "nos-scheduler"),
                                 resource_namespace=le.get("resourceNamespace", "kube-system"))
    for p in data.get("profiles") or [{}]:
        prof = Profile(scheduler_name=p.get("schedulerName", "default-scheduler"))
        for k, ep in _EP_KEYS.items():
            prof.plugins[ep] = _apply_plugin_set(DEFAULT_PLUGINS.get(ep, []), (p.get("plugins") or {}).get(k))
        for pc in p.get("pluginConfig") or []:
            prof.plugin_config[pc["name"]] = pc.get("args") or {}
        cfg.profiles.append(prof)
    return cfg


def load(path: str | Path) -> SchedulerConfiguration:
    return parse(yaml.safe_load(Path(path).read_text()) or {})


def nos_scheduler_config(memory_gb: int = C.DEFAULT_AMD_GPU_RESOURCE_MEMORY_GB) -> SchedulerConfiguration:
    """The ``nos-scheduler`` profile of the reference (CapacityScheduling at
    preFilter / postFilter (all others disabled) / reserve)."""
    return parse({
        "profiles": [{
            "schedulerName": "nos-scheduler",
            "plugins": {"preFilter": {"enabled": [{"name": "CapacityScheduling"}]},
                        "postFilter": {"enabled": [{"name": "CapacityScheduling"}], "disabled": [{"name": "*"}]},
                        "reserve": {"enabled": [{"name": "CapacityScheduling"}]}},
            "pluginConfig": [{"name": "CapacityScheduling", "args": {"amdGpuResourceMemoryGB": memory_gb}}],
        }]})


def registry() -> dict[str, Any]:
    from .plugins.capacity_scheduling import CapacityScheduling

    r: dict[str, Any] = dict(intree.REGISTRY)
    r["CapacityScheduling"] = CapacityScheduling
    return r


def build_framework(profile: Profile, api=None, snapshot: Snapshot | None = None,
                    nominator: PodNominator | None = None, extra_registry: dict | None = None,
                    start_informers: bool = True) -> Framework:
    reg = registry()
    reg.update(extra_registry or {})
    instances: dict[str, Plugin] = {}

    def get(name: str) -> Plugin:
        if name not in instances:
            cls = reg.get(name)
            if cls is None:
                raise ValueError(f"plugin {name!r} not registered")
            args = profile.plugin_config.get(name)
            if name == "CapacityScheduling":
                instances[name] = cls(args, None, api=api, start_informers=start_informers)
            else:
                try:
                    instances[name] = cls(args, None)
                except TypeError:
                    instances[name] = cls()
        return instances[name]

    plugins = {ep: [get(n) for n in names] for ep, names in profile.plugins.items()}
    fw = Framework(plugins, snapshot=snapshot, nominator=nominator, api=api, profile_name=profile.scheduler_name)
    fw.instances = instances  # type: ignore[attr-defined]
    return fw
