"""The two partitioning strategies of the gpupartitioner.

``amdpart`` (MIG analogue, ``internal/partitioning/mig/*.go``): nodes labelled
``nos.nebuly.com/gpu-partitioning=partition``; a plan rewrites the node's
``spec-gpu-<i>-<profile>`` annotations (+ ``spec-mode-gpu-<i>`` =
``<COMPUTE>/<NPS>``) and ``spec-partitioning-plan``; the partition agent on the
node applies it with amd-smi and reports back.

``cumask`` (MPS analogue, ``internal/partitioning/mps/*.go``): nodes labelled
``nos.nebuly.com/gpu-partitioning=cumask``; a plan writes the device-plugin
ConfigMap entry ``<node>-<planId>`` with the per-GPU slice table, waits
``devicePluginDelaySeconds``, then points the node label
``nos.nebuly.com/device-plugin.config`` at it.  Unlike the reference it ALSO
writes the spec annotations and ``spec-partitioning-plan`` so the plan
handshake covers this path too (the gpuagent reports
``status-partitioning-plan``; the reference's MPS path had no handshake,
SURVEY.md 3.2).

``hybrid`` (the reference's declared-but-unused kind,
``pkg/gpu/partitioning.go:87-91``): nodes labelled ``hybrid``; a plan picks a
compute/memory mode per GPU AND memory slices (``amd.com/gpu-<N>gb``) that
bin-pack into its partitions (:mod:`nos_amd.gpu.hybrid`).  It writes the
cumask path's device-plugin ConfigMap entry (with each GPU's mode) plus the
amdpart path's ``spec-mode-gpu-<i>`` annotations: the partition agent switches
modes, the device plugin places the slices on the partitions.

Each strategy provides the five pieces of the reference's factory: snapshot
taker, partition calculator, partitioner, slice calculator, slice filter
(+ the node initializer for amdpart).
"""
from __future__ import annotations

import logging
from dataclasses import dataclass

import yaml

from ..api import constants as C
from ..gpu import amdpart as ap
from ..gpu import cumask as cm
from ..gpu import hybrid as hy
from ..gpu.core import SpecAnnotation, is_amdpart_enabled, is_cumask_enabled, partitioning_kind
from ..kube import objects as ko
from ..scheduler.framework import NodeInfo
from .core import ClusterSnapshot, new_plan_id
from . import scoring
from .state import ClusterState, GPUPartitioning, NodePartitioning

log = logging.getLogger("nos_amd.partitioning.strategies")


def _spec_patch(node: dict, specs: list[SpecAnnotation], plan_id: str, extra: dict[str, str] | None = None) -> dict:
    ann: dict[str, str | None] = {}
    for k in ko.annotations(node):
        if k.startswith(C.ANNOTATION_GPU_SPEC_PREFIX) or k.startswith("nos.nebuly.com/spec-mode-gpu"):
            ann[k] = None
    for s in specs:
        ann[s.key()] = s.value()
    ann.update(extra or {})
    ann[C.ANNOTATION_PARTITIONING_PLAN] = plan_id
    return {"metadata": {"annotations": ann}}


# ====================================================================== amdpart
class AmdPartPartitionCalculator:
    def get_partitioning(self, node) -> NodePartitioning:
        if not isinstance(node, ap.PartitionNode):
            return NodePartitioning([])
        out = []
        for g in node.gpus:
            geo = g.geometry()
            mg = g.mode_for(geo)
            out.append(GPUPartitioning.of(g.index, {p.resource_name(): n for p, n in geo.items()},
                                          mg.id() if mg else ""))
        return NodePartitioning(out)


class AmdPartPartitioner:
    def __init__(self, api):
        self.api = api

    def apply_partitioning(self, node: dict, plan_id: str, partitioning: NodePartitioning) -> None:
        specs, modes = [], {}
        for g in partitioning.gpus:
            for r, n in g.resources:
                specs.append(SpecAnnotation(g.gpu_index, ap.profile_of_resource(r).name, n))
            if g.mode:
                modes[C.ANNOTATION_SPEC_MODE_FORMAT.format(index=g.gpu_index)] = g.mode
        self.api.patch("Node", ko.name(node), _spec_patch(node, specs, plan_id, modes))
        log.info("amdpart plan %s applied to node %s: %s", plan_id, ko.name(node), [str(s.key()) for s in specs])


class AmdPartSnapshotTaker:
    def __init__(self, partition_calculator=None, reserve_whole_gpus: int = 0, memory_mode: str = "NPS1"):
        self.pc = partition_calculator or AmdPartPartitionCalculator()
        self.reserve_whole_gpus = reserve_whole_gpus
        self.memory_mode = memory_mode

    def take_snapshot(self, cs: ClusterState) -> ClusterSnapshot:
        nodes = {}
        for name, ni in cs.get_nodes().items():
            n = ni.node()
            if n is None or not is_amdpart_enabled(n):
                continue
            try:
                pn = ap.PartitionNode.from_node_info(ni.clone())
                pn.reserve_whole_gpus = self.reserve_whole_gpus
                pn.set_memory_mode_preference(self.memory_mode)
                nodes[name] = pn
            except Exception as e:  # node not yet labelled by its agent
                log.debug("skipping node %s: %s", name, e)
        return ClusterSnapshot(nodes, self.pc, ap.PartitionSliceCalculator(), ap.PartitionSliceFilter())


class AmdPartNodeInitializer:
    """Give every GPU without a geometry the fewest-slices geometry (SPX),
    ``internal/partitioning/mig/initializer.go:44-83``."""

    def __init__(self, api, partitioner=None, partition_calculator=None, clock=None):
        self.api = api
        self.partitioner = partitioner or AmdPartPartitioner(api)
        self.pc = partition_calculator or AmdPartPartitionCalculator()
        self.clock = clock

    def init_node_partitioning(self, node: dict) -> bool:
        if not is_amdpart_enabled(node):
            raise ValueError(f"partition mode is not enabled on node {ko.name(node)}")
        pn = ap.PartitionNode.from_node_info(NodeInfo(node))
        n_init = 0
        for g in pn.gpus:
            if g.geometry():
                continue
            g.init_geometry()
            n_init += 1
        if not n_init:
            return False
        self.partitioner.apply_partitioning(node, new_plan_id(self.clock), self.pc.get_partitioning(pn))
        return True


# ====================================================================== cumask
class CuMaskPartitionCalculator:
    def get_partitioning(self, node) -> NodePartitioning:
        if not isinstance(node, cm.SliceNode):
            return NodePartitioning([])
        return NodePartitioning([GPUPartitioning.of(g.index, {p.resource_name(): n for p, n in g.geometry().items()})
                                 for g in node.gpus])


@dataclass
class DevicePluginConfigRef:
    name: str = C.DEFAULT_DEVICE_PLUGIN_CM_NAME
    namespace: str = C.DEFAULT_DEVICE_PLUGIN_CM_NAMESPACE


def plugin_config(node_name: str, plan_id: str, partitioning: NodePartitioning, cu_policy: str = "proportional",
                  allocation: str = "pack", gpu_weights: dict[int, float] | None = None,
                  split: dict | None = None) -> dict:
    """Device-plugin configuration for one node (the ``ToPluginConfig`` of
    ``mps/partitioner.go:123-157``, AMD shape).  With ``allocation:
    measured`` it also carries the probe-measured TFLOP/s per GPU
    (``gpuWeights``) that the plugin's GetPreferredAllocation divides among
    the pods of each GPU."""
    gpus = []
    for g in sorted(partitioning.gpus, key=lambda x: x.gpu_index):
        slices = [{"profile": cm.profile_of_resource(r).name, "memoryGB": cm.profile_of_resource(r).memory_gb,
                   "replicas": n} for r, n in g.resources]
        entry = {"index": g.gpu_index, "slices": slices}
        if g.mode:  # hybrid: the compute/memory mode the slices are laid out for
            entry["mode"] = g.mode
        gpus.append(entry)
    out = {"version": "v1", "node": node_name, "planId": plan_id, "cuPolicy": cu_policy, "allocation": allocation,
           "gpus": gpus}
    if gpu_weights:
        out["gpuWeights"] = {int(k): round(float(v), 3) for k, v in sorted(gpu_weights.items())}
    if cu_policy == "split" and split:   # the isolated pool: its profiles and reserved CU slots per XCD
        out["isolatedProfiles"] = list(split.get("isolatedProfiles", []))
        out["isolatedCuSlots"] = int(split.get("isolatedCuSlots", 0))
    return out


class CuMaskPartitioner:
    def __init__(self, api, cm_ref: DevicePluginConfigRef | None = None, delay_s: float = 5.0, clock=None,
                 cu_policy: str = "proportional", allocation: str = "pack", split: dict | None = None):
        self.api = api
        self.split = split
        self.cm_ref = cm_ref or DevicePluginConfigRef()
        self.delay_s = delay_s
        self.clock = clock or api.clock
        self.cu_policy = cu_policy
        self.allocation = allocation

    def apply_partitioning(self, node: dict, plan_id: str, partitioning: NodePartitioning) -> None:
        name = ko.name(node)
        ref = self.cm_ref
        cmap = self.api.try_get("ConfigMap", ref.name, ref.namespace)
        if cmap is None:
            try:
                self.api.create({"kind": "Namespace", "metadata": {"name": ref.namespace}})
            except Exception:
                pass
            cmap = self.api.create({"kind": "ConfigMap", "metadata": {"name": ref.name, "namespace": ref.namespace},
                                    "data": {}})
        data = {k: None for k in (cmap.get("data") or {}) if k.startswith(name + "-")}
        key = f"{name}-{plan_id}"
        weights = None
        if self.allocation == "measured":
            counts = {g.gpu_index: {cm.profile_of_resource(r).name: n for r, n in g.resources}
                      for g in partitioning.gpus}
            weights = scoring.gpu_capacities(scoring.probe_table(ko.annotations(node)), counts) or None
        data[key] = yaml.safe_dump(plugin_config(name, plan_id, partitioning, self.cu_policy, self.allocation,
                                                 weights, self.split), sort_keys=False)
        self.api.patch("ConfigMap", ref.name, {"data": data}, ref.namespace)
        if self.delay_s > 0:
            self.clock.sleep(self.delay_s)  # ConfigMap propagation (kept for fidelity)
        specs = [SpecAnnotation(g.gpu_index, cm.profile_of_resource(r).name, n)
                 for g in partitioning.gpus for r, n in g.resources]
        modes = {C.ANNOTATION_SPEC_MODE_FORMAT.format(index=g.gpu_index): g.mode for g in partitioning.gpus if g.mode}
        patch = _spec_patch(node, specs, plan_id, modes)
        patch["metadata"]["labels"] = {C.LABEL_DEVICE_PLUGIN_CONFIG: key}
        self.api.patch("Node", name, patch)
        log.info("%s plan %s applied to node %s", "hybrid" if modes else "cumask", plan_id, name)


class CuMaskSnapshotTaker:
    def __init__(self, partition_calculator=None, placement: str = "pack"):
        self.pc = partition_calculator or CuMaskPartitionCalculator()
        self.placement = placement

    def take_snapshot(self, cs: ClusterState) -> ClusterSnapshot:
        nodes = {}
        for name, ni in cs.get_nodes().items():
            n = ni.node()
            if n is None or not is_cumask_enabled(n):
                continue
            try:
                sn = cm.SliceNode.from_node_info(ni.clone())
                sn.placement = self.placement
                nodes[name] = sn
            except Exception as e:
                log.debug("skipping node %s: %s", name, e)
        return ClusterSnapshot(nodes, self.pc, cm.SliceCalculator(), cm.SliceFilter())


# ====================================================================== hybrid
class HybridPartitionCalculator:
    def get_partitioning(self, node) -> NodePartitioning:
        if not isinstance(node, hy.HybridNode):
            return NodePartitioning([])
        return NodePartitioning([GPUPartitioning.of(g.index, {p.resource_name(): n for p, n in g.geometry().items()},
                                                    g.mode.id()) for g in node.gpus])


class HybridSnapshotTaker:
    def __init__(self, partition_calculator=None):
        self.pc = partition_calculator or HybridPartitionCalculator()

    def take_snapshot(self, cs: ClusterState) -> ClusterSnapshot:
        nodes = {}
        for name, ni in cs.get_nodes().items():
            n = ni.node()
            if n is None or partitioning_kind(n) != C.PARTITIONING_HYBRID:
                continue
            try:
                nodes[name] = hy.HybridNode.from_node_info(ni.clone())
            except Exception as e:  # node not yet labelled by its agent
                log.debug("skipping node %s: %s", name, e)
        return ClusterSnapshot(nodes, self.pc, hy.HybridSliceCalculator(), hy.HybridSliceFilter())


@dataclass
class Strategy:
    kind: str
    snapshot_taker: object
    partition_calculator: object
    partitioner: object
    slice_calculator: object
    slice_filter: object
    initializer: object | None = None


def amdpart_strategy(api, clock=None, reserve_whole_gpus: int = 0, memory_mode: str = "NPS1") -> Strategy:
    pc = AmdPartPartitionCalculator()
    part = AmdPartPartitioner(api)
    return Strategy(C.PARTITIONING_AMDPART, AmdPartSnapshotTaker(pc, reserve_whole_gpus, memory_mode), pc, part,
                    ap.PartitionSliceCalculator(),
                    ap.PartitionSliceFilter(), AmdPartNodeInitializer(api, part, pc, clock))


def cumask_strategy(api, cm_ref: DevicePluginConfigRef | None = None, delay_s: float = 5.0, clock=None,
                    cu_policy: str = "proportional", placement: str = "pack", split: dict | None = None) -> Strategy:
    pc = CuMaskPartitionCalculator()
    return Strategy(C.PARTITIONING_CUMASK, CuMaskSnapshotTaker(pc, placement), pc,
                    CuMaskPartitioner(api, cm_ref, delay_s, clock, cu_policy, placement, split), cm.SliceCalculator(),
                    cm.SliceFilter())


def hybrid_strategy(api, cm_ref: DevicePluginConfigRef | None = None, delay_s: float = 5.0, clock=None) -> Strategy:
    pc = HybridPartitionCalculator()
    return Strategy(C.PARTITIONING_HYBRID, HybridSnapshotTaker(pc), pc,
                    CuMaskPartitioner(api, cm_ref, delay_s, clock, "shared", "pack"), hy.HybridSliceCalculator(),
                    hy.HybridSliceFilter())
