"""A whole nos-amd cluster in one process (SURVEY.md 4 "multi-node without a
cluster", 7.2 simulator).

Control plane: the API server, the operator (ElasticQuota /
CompositeElasticQuota reconcilers), the gpupartitioner (node + pod state
controllers, one partitioner controller per strategy) and the nos-scheduler
(CapacityScheduling profile).  Per node: a kubelet, the nos-amd device plugin
(+ its ConfigMap watcher), the node labeler and the agent of the node's
partitioning kind (partition agent reporter/actuator or the CU-mask
gpuagent), each on the node's own controller manager -- the same process
boundaries as the DaemonSets of a real deployment.

``settle()`` drives everything deterministically on a :class:`FakeClock`:
every manager and the scheduler run until idle, then the clock jumps to the
next due requeue / batch deadline.
"""
from __future__ import annotations

import logging
from dataclasses import dataclass, field

from ..agents.devices import NodeLabeler
from ..agents.gpuagent import CuMaskReporter
from ..agents.hybridagent import HybridReporter
from ..agents.partagent import PartitionActuator, PartitionReporter
from ..agents.shared import SharedState
from ..api import constants as C
from ..api import v1alpha1
from ..api.config import GpuPartitionerConfig
from ..controllers.elasticquota import CompositeElasticQuotaReconciler, ElasticQuotaReconciler
from ..controllers.gpupartitioner import NodeController, PartitionerController, PodController
from ..deviceplugin.config_watcher import ConfigWatcher
from ..deviceplugin.plugin import NosAmdDevicePlugin
from ..gpu.fakesmi import FakeSmi
from ..kube import factory as kf
from ..kube import objects as ko
from ..partitioning.state import ClusterState
from ..partitioning.strategies import DevicePluginConfigRef, amdpart_strategy, cumask_strategy, hybrid_strategy
from ..runtime.manager import Manager
from ..scheduler.config import build_framework, nos_scheduler_config
from ..scheduler.scheduler import Scheduler
from ..utils.clock import FakeClock
from .apiserver import ApiServer
from .kubelet import Kubelet

log = logging.getLogger("nos_amd.sim.cluster")


@dataclass
class SimNode:
    name: str
    kind: str | None
    smi: object
    plugin: NosAmdDevicePlugin
    kubelet: Kubelet
    manager: Manager
    agents: dict = field(default_factory=dict)


class SimCluster:
    def __init__(self, clock=None, partitioner_config: GpuPartitionerConfig | None = None,
                 memory_gb: int = C.DEFAULT_AMD_GPU_RESOURCE_MEMORY_GB, scheduler_config=None,
                 resync_s: float | None = None):
        self.resync_s = resync_s  # informer resync period (None: off, event-driven only)
        self.clock = clock or FakeClock()
        self.api = ApiServer(self.clock)
        v1alpha1.register_types(self.api)
        self.cfg = (partitioner_config or GpuPartitionerConfig()).with_defaults()
        self.cm_ref = DevicePluginConfigRef(self.cfg.device_plugin_config_map.name,
                                            self.cfg.device_plugin_config_map.namespace)
        for ns in ("default", C.DEFAULT_DEVICE_PLUGIN_CM_NAMESPACE):
            self.api.create(kf.build_namespace(ns).get())

        # ---- operator
        self.operator = Manager(self.api, "nos-operator", self.clock, resync_s=resync_s)
        self.operator.add(ElasticQuotaReconciler(self.api, memory_gb).controller())
        self.operator.add(CompositeElasticQuotaReconciler(self.api, memory_gb).controller())

        # ---- gpupartitioner
        self.cluster_state = ClusterState()
        self.partitioner = Manager(self.api, "nos-gpupartitioner", self.clock, resync_s=resync_s)
        sched_cfg = scheduler_config or nos_scheduler_config(memory_gb)
        fw = build_framework(sched_cfg.profiles[0], api=self.api)
        amd = amdpart_strategy(self.api, self.clock, self.cfg.reserve_whole_gpus, self.cfg.preferred_memory_mode)
        cum = cumask_strategy(self.api, self.cm_ref, self.cfg.device_plugin_delay_seconds, self.clock,
                              self.cfg.cu_policy, self.cfg.slice_placement,
                              {"isolatedProfiles": self.cfg.isolated_profiles,
                               "isolatedCuSlots": self.cfg.isolated_cu_slots})
        hyb = hybrid_strategy(self.api, self.cm_ref, self.cfg.device_plugin_delay_seconds, self.clock)
        self.partitioner.add(NodeController(self.api, self.cluster_state, amd.initializer).controller())
        self.partitioner.add(PodController(self.api, self.cluster_state).controller())
        self.partitioner_controllers = {}
        for strat in (amd, cum, hyb):
            pc = PartitionerController(self.api, self.cluster_state, strat, fw, self.clock,
                                       self.cfg.batch_window_timeout_seconds, self.cfg.batch_window_idle_seconds,
                                       self.cfg.plan_report_timeout_seconds)
            self.partitioner_controllers[strat.kind] = pc
            self.partitioner.add(pc.controller())

        # ---- scheduler
        self.scheduler = Scheduler(self.api, sched_cfg, self.clock)
        self.scheduler.start_informers()
        self.nodes: dict[str, SimNode] = {}
        self.cu_policy = self.cfg.cu_policy

    # ------------------------------------------------------------ topology
    def add_node(self, name: str, kind: str | None = C.PARTITIONING_CUMASK, gpus: int = 8, compute: str = "SPX",
                 memory: str = "NPS1", smi=None, runtime=None, on_stop=None, probe=None,
                 node_resources: dict | None = None, pod_server_tenants: int = 0,
                 pod_server_dir: str = C.DEFAULT_POD_SERVER_SOCKET_DIR) -> SimNode:
        """``pod_server_tenants`` > 0: the node's cumask slices are served by a
        pod server per GPU (labeler + device plugin as a DaemonSet with
        ``podServerTenants`` / ``podServerSocketDir`` would run them)."""
        smi = smi or FakeSmi(gpus=gpus, compute=compute, memory=memory, node=name)
        labels = {"kubernetes.io/hostname": name}
        if kind:
            labels[C.LABEL_GPU_PARTITIONING] = kind
        self.api.create(kf.build_node(name).with_labels(labels).get())
        plugin = NosAmdDevicePlugin(name, smi, mode=kind, cu_policy=self.cu_policy,
                                    pod_server_dir=pod_server_dir if pod_server_tenants > 0 else "")
        kubelet = Kubelet(self.api, name, [plugin], node_resources=node_resources, runtime=runtime, on_stop=on_stop)
        kubelet.sync_node_status()
        mgr = Manager(self.api, f"node-{name}", self.clock, resync_s=self.resync_s)
        mgr.add(kubelet.controller())
        labeler = NodeLabeler(self.api, name, smi, pod_server_tenants)
        mgr.add(labeler.controller())
        agents: dict = {"labeler": labeler}
        if kind == C.PARTITIONING_AMDPART:
            shared = SharedState()
            agents["reporter"] = PartitionReporter(self.api, name, smi, kubelet, shared)
            agents["actuator"] = PartitionActuator(self.api, name, smi, kubelet, shared, [plugin])
            mgr.add(agents["reporter"].controller())
            mgr.add(agents["actuator"].controller())
        elif kind == C.PARTITIONING_HYBRID:  # partition agent (modes) + slice reporter + slice table watcher
            shared = SharedState()
            agents["config"] = ConfigWatcher(self.api, name, plugin, self.cm_ref)
            agents["reporter"] = HybridReporter(self.api, name, smi, kubelet, shared)
            agents["actuator"] = PartitionActuator(self.api, name, smi, kubelet, shared, [plugin])
            for a in ("config", "reporter", "actuator"):
                mgr.add(agents[a].controller())
        elif kind == C.PARTITIONING_CUMASK:
            agents["config"] = ConfigWatcher(self.api, name, plugin, self.cm_ref)
            agents["reporter"] = CuMaskReporter(self.api, name, smi, kubelet, probe=probe)
            mgr.add(agents["config"].controller())
            mgr.add(agents["reporter"].controller())
        node = SimNode(name, kind, smi, plugin, kubelet, mgr, agents)
        self.nodes[name] = node
        return node

    # ------------------------------------------------------------ workload helpers
    def submit_pod(self, name: str, resources: dict[str, int | str], namespace: str = "default",
                   scheduler: str = "nos-scheduler", priority: int | None = None, cpu_milli: int = 100,
                   labels: dict | None = None) -> dict:
        c = kf.build_container("main").with_cpu_milli_request(cpu_milli).with_requests(resources)
        ext = {k: v for k, v in resources.items() if "/" in k}
        if ext:
            c = c.with_limits(ext)
        b = kf.build_pod(namespace, name).with_container(c.get()).with_scheduler_name(scheduler) \
            .with_phase(ko.PENDING).with_creation_timestamp(self.clock.now())
        if priority is not None:
            b = b.with_priority(priority)
        for k, v in (labels or {}).items():
            b = b.with_label(k, v)
        return self.api.create(b.get())

    def pods(self, namespace: str | None = None) -> list[dict]:
        return self.api.list("Pod", namespace)

    def running_pods(self) -> list[dict]:
        return [p for p in self.pods() if ko.pod_phase(p) == ko.RUNNING]

    def pending_pods(self) -> list[dict]:
        return [p for p in self.pods() if ko.pod_phase(p) == ko.PENDING]

    # ------------------------------------------------------------ driving
    def _managers(self) -> list[Manager]:
        return [self.operator, self.partitioner] + [n.manager for n in self.nodes.values()]

    def step(self) -> int:
        n = 0
        for m in self._managers():
            n += m.step()
        n += self.scheduler.run_until_idle()
        return n

    def next_wakeup(self) -> float | None:
        ds = [d for m in self._managers() if (d := m.next_wakeup()) is not None]
        return min(ds) if ds else None

    def settle(self, max_time: float = 300.0, until=None, max_rounds: int = 100000) -> float:
        """Run to quiescence; jump the fake clock to due requeues up to
        ``max_time`` simulated seconds (or until ``until()`` is true).
        Returns the simulated seconds elapsed."""
        start = self.clock.now()
        for _ in range(max_rounds):
            while self.step():
                if until is not None and until():
                    return self.clock.now() - start
            if until is not None and until():
                break
            d = self.next_wakeup()
            flush = self.scheduler.flush_interval - (self.clock.monotonic() - self.scheduler._last_flush)
            want_flush = self.scheduler.queue.unschedulable_count() or self.resync_s is not None
            cands = [x for x in (d, flush if want_flush else None) if x is not None]
            if not cands:
                break
            dt = max(min(cands), 0) + 1e-3
            if self.clock.now() + dt - start > max_time:
                break
            if not hasattr(self.clock, "advance"):
                break
            self.clock.advance(dt)
        return self.clock.now() - start

    def schedulable_fractional_pods(self, node: str, resource: str) -> int:
        n = self.api.get("Node", node)
        return int(ko.node_allocatable(n).get(resource, 0))
