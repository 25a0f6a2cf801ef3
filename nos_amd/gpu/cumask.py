"""CU-mask slice model -- the MPS analogue (``pkg/gpu/slicing``).

A slice is a memory share of one GPU (``<gb>gb`` profile, resource
``amd.com/gpu-<gb>gb``) plus a set of compute units enforced with a
per-container CU mask (``ROC_GLOBAL_CU_MASK``; see :mod:`nos_amd.gpu.topology`
for why masks are XCD-symmetric).  The memory side follows the reference
exactly (``slicing/gpu.go:67-220``): the sum of the slices' memory must fit the
GPU, slices are created from spare memory smallest-first, free slices may be
dropped to make room and re-created afterwards, used slices are never touched.
The compute side adds two constraints the reference did not have: every
slice needs at least one CU on every XCD, so a GPU holds at most
``cus_per_xcd`` (32 on MI355X) slices, and no more slices than the amdgpu
hardware scheduler runs processes concurrently (node label
``amd.com/gpu.max-concurrent-processes``, 8 by default; :mod:`nos_amd.gpu.kfd`).
On a node whose slices are served by the pod server (label
``nos.nebuly.com/pod-server.tenants``, :mod:`nos_amd.podserver`) the bound is
the server's tenant count instead: all tenants share one GPU process, and
memory bounds the slices as in the reference.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field

from ..api import constants as C
from ..kube import objects as ko
from ..kube import quantity as q
from .core import GenericError, Geometry, get_count, get_memory_gb, get_model, parse_node_annotations
from .topology import MI355X_CUS_PER_XCD, MI355X_XCDS
from ..partitioning import scoring

MIN_SLICE_MEMORY_GB = 1
REPLICA_SEPARATOR = "::"  # device ids of slices: <gpu-uuid>::<replica>
_PROFILE_RE = re.compile(C.REGEX_AMD_SLICE_PROFILE)
_RESOURCE_RE = re.compile(C.REGEX_AMD_SLICE_RESOURCE)


@dataclass(frozen=True, order=True)
class SliceProfile:
    name: str

    def __post_init__(self):
        if not _PROFILE_RE.match(self.name):
            raise ValueError(f"invalid slice profile {self.name!r} (expected <gb>gb)")

    @classmethod
    def of(cls, gb: int) -> "SliceProfile":
        return cls(f"{gb}gb")

    @property
    def memory_gb(self) -> int:
        return int(self.name[:-2])

    def smaller_than(self, other) -> bool:
        return isinstance(other, SliceProfile) and self.memory_gb < other.memory_gb

    def resource_name(self) -> str:
        return C.AMD_SLICE_RESOURCE_PREFIX + self.name

    def __str__(self) -> str:
        return self.name


def is_slice_resource(name: str) -> bool:
    return bool(_RESOURCE_RE.match(name))


def profile_of_resource(name: str) -> SliceProfile:
    m = _RESOURCE_RE.match(name)
    if not m:
        raise ValueError(f"{name!r} is not a CU-mask slice resource")
    return SliceProfile(m.group(1))


def requested_profiles(pod: dict) -> dict[SliceProfile, int]:
    from ..resource.resource import compute_pod_request

    out: dict[SliceProfile, int] = {}
    for name, v in compute_pod_request(pod).items():
        if is_slice_resource(name) and q.value(v) > 0:
            p = profile_of_resource(name)
            out[p] = out.get(p, 0) + q.value(v)
    return out


@dataclass
class SliceGPU:
    model: str
    index: int
    memory_gb: int
    used: dict[SliceProfile, int] = field(default_factory=dict)
    free: dict[SliceProfile, int] = field(default_factory=dict)
    max_slices: int = MI355X_CUS_PER_XCD

    def validate(self) -> None:
        total = 0
        for d in (self.used, self.free):
            for p, n in d.items():
                if p.memory_gb < MIN_SLICE_MEMORY_GB:
                    raise GenericError(f"min allowed slice size is {MIN_SLICE_MEMORY_GB}GB, but profile {p} "
                                       f"has {p.memory_gb}GB")
                total += p.memory_gb * n
        if total > self.memory_gb:
            raise GenericError(f"total memory of profiles ({total}) exceeds GPU memory ({self.memory_gb})")
        if self.num_slices() > self.max_slices:
            raise GenericError(f"{self.num_slices()} slices exceed the {self.max_slices} XCD-symmetric CU masks")

    @classmethod
    def new(cls, model: str, index: int, memory_gb: int, used=None, free=None,
            max_slices: int = MI355X_CUS_PER_XCD) -> "SliceGPU":
        g = cls(model, index, memory_gb, dict(used or {}), dict(free or {}), max_slices)
        g.validate()
        return g

    def clone(self) -> "SliceGPU":
        return SliceGPU(self.model, self.index, self.memory_gb, dict(self.used), dict(self.free), self.max_slices)

    def geometry(self) -> Geometry:
        g = Geometry()
        for d in (self.used, self.free):
            for p, n in d.items():
                if n:
                    g[p] = g.get(p, 0) + n
        return g

    def num_slices(self) -> int:
        return sum(self.used.values()) + sum(self.free.values())

    def tot_slices_memory(self) -> int:
        return sum(p.memory_gb * n for d in (self.used, self.free) for p, n in d.items())

    def can_create_more_slices(self) -> bool:
        return (self.memory_gb - self.tot_slices_memory() >= MIN_SLICE_MEMORY_GB
                and self.num_slices() < self.max_slices)

    def create_slices(self, size_gb: int, num: int = 1) -> None:
        if self.memory_gb - self.tot_slices_memory() < size_gb * num:
            raise GenericError(f"not enough spare memory to create {num} slices of size {size_gb}GB")
        if self.num_slices() + num > self.max_slices:
            raise GenericError(f"cannot create {num} more slices: at most {self.max_slices} per GPU")
        p = SliceProfile.of(size_gb)
        self.free[p] = self.free.get(p, 0) + num

    def has_free_capacity(self) -> bool:
        return any(n > 0 for n in self.free.values()) or self.can_create_more_slices()

    def add_pod(self, pod: dict) -> None:
        req = requested_profiles(pod)
        for p, n in req.items():
            if self.free.get(p, 0) < n:
                raise GenericError(f"not enough free slices (pod requests {n} {p}, but GPU only has "
                                   f"{self.free.get(p, 0)})")
        for p, n in req.items():
            self.free[p] -= n
            if self.free[p] == 0:
                del self.free[p]
            self.used[p] = self.used.get(p, 0) + n

    def missing_slices(self, required: dict) -> dict[SliceProfile, int]:
        out = {}
        for p, n in required.items():
            if isinstance(p, SliceProfile):
                diff = n - self.free.get(p, 0)
                if diff > 0:
                    out[p] = diff
        return out

    def update_geometry_for(self, required: dict) -> bool:
        missing = self.missing_slices(required)
        if not missing:
            return False
        updated = False
        original_free = dict(self.free)
        for p in sorted(missing, key=lambda x: x.memory_gb):
            # 1. create missing slices from spare memory
            if self.can_create_more_slices():
                for _ in range(missing[p]):
                    try:
                        self.create_slices(p.memory_gb)
                    except GenericError:
                        break
                    missing[p] -= 1
                    updated = True
            # 2. drop the original free slices to make room, create the rest
            qty = missing[p]
            for k in original_free:
                self.free.pop(k, None)
            for _ in range(qty):
                if not self.can_create_more_slices():
                    break
                try:
                    self.create_slices(p.memory_gb)
                except GenericError:
                    break
                missing[p] -= 1
                updated = True
            # 3. re-create the original free slices as far as they still fit
            for k, v in original_free.items():
                try:
                    self.create_slices(k.memory_gb, v)
                except GenericError:
                    pass
        return updated


class SliceNode:
    """``slicing.Node`` analogue; implements core.PartitionableNode."""

    def __init__(self, name: str, gpus: list[SliceGPU], node_info, placement: str = "pack"):
        self.name = name
        self.gpus = gpus
        self.node_info = node_info
        # "pack": first-fit over GPUs (the reference, keeps whole GPUs free);
        # "spread": new slices go to the GPU with the most spare memory, so
        # tenants are balanced over the node's GPUs (throughput-first);
        # "measured": new slices go to the GPU where a pod gets the largest
        # share of the probe-measured throughput (partitioning/scoring.py)
        self.placement = placement
        self.capacity: dict[int, float] = {}   # measured TFLOP/s per GPU (probe annotations)
        self.measured = False

    @classmethod
    def from_node_info(cls, ni) -> "SliceNode":
        node = ni.node()
        if node is None:
            raise GenericError("node is nil")
        model = get_model(node)
        count = get_count(node)
        mem = get_memory_gb(node)
        cus = int(ko.labels(node).get(C.LABEL_AMD_CUS, MI355X_XCDS * MI355X_CUS_PER_XCD))
        xcds = int(ko.labels(node).get(C.LABEL_AMD_XCDS, MI355X_XCDS))
        max_slices = max(1, cus // max(1, xcds))
        # more slices than HWS process slots would be time-sliced, not shared (gpu/kfd.py)
        procs = ko.labels(node).get(C.LABEL_AMD_MAX_PROCS)
        if procs and int(procs) > 0:
            max_slices = min(max_slices, int(procs))
        # ... unless the node's pod server hosts the slices: ONE GPU process per
        # GPU whatever the tenant count (nos_amd/podserver, the MPS analogue)
        tenants = ko.labels(node).get(C.LABEL_POD_SERVER_TENANTS, "")
        if tenants.isdigit() and int(tenants) > 0:
            max_slices = int(tenants)
        status, _ = parse_node_annotations(node)
        by_gpu: dict[int, tuple[dict, dict]] = {}
        for a in status:
            try:
                p = SliceProfile(a.profile)
            except ValueError:
                continue
            used, free = by_gpu.setdefault(a.index, ({}, {}))
            (used if a.is_used() else free)[p] = a.quantity
        gpus = [SliceGPU.new(model, i, mem, *by_gpu[i], max_slices=max_slices) for i in sorted(by_gpu)]
        have = {g.index for g in gpus}
        for i in range(count):
            if i not in have:
                gpus.append(SliceGPU(model, i, mem, max_slices=max_slices))
        gpus.sort(key=lambda g: g.index)
        out = cls(ko.name(node), gpus, ni)
        table = scoring.probe_table(ko.annotations(node))
        counts = {g.index: {p.name: g.used.get(p, 0) + g.free.get(p, 0) for p in set(g.used) | set(g.free)}
                  for g in gpus}
        caps = scoring.gpu_capacities(table, counts)
        out.measured = bool(caps)
        out.capacity = scoring.fill_unmeasured(caps, [g.index for g in gpus])
        return out

    def _share(self, g: "SliceGPU") -> float:
        return scoring.expected_share(self.capacity.get(g.index, 1.0), g.num_slices())

    def score(self) -> float | None:
        """Best expected per-pod share of measured throughput on a GPU with
        room for one more slice; ``None`` unless placement is "measured" and
        the node carries probe data (the planner then keeps name order)."""
        if self.placement != "measured" or not self.measured:
            return None
        return scoring.node_score(self.capacity, {g.index: g.num_slices() for g in self.gpus},
                                  lambda gi: any(g.index == gi and g.has_free_capacity() for g in self.gpus))

    def geometry(self) -> dict:
        res: dict = {}
        for g in self.gpus:
            for p, n in g.geometry().items():
                res[p] = res.get(p, 0) + n
        return res

    def has_free_capacity(self) -> bool:
        return any(g.has_free_capacity() for g in self.gpus)

    def update_geometry_for(self, slices: dict) -> bool:
        if not self.gpus or not slices:
            return False
        required = dict(slices)
        if self.placement in ("spread", "measured"):
            updated = self._spread(required)
            self._recompute_allocatable()
            return updated
        updated = False
        for g in self.gpus:
            updated = g.update_geometry_for(required) or updated
            for p, n in g.free.items():
                if p in required:
                    required[p] -= n
                    if required[p] <= 0:
                        del required[p]
        self._recompute_allocatable()
        return updated

    def _spread(self, required: dict) -> bool:
        updated = False
        for p in sorted((x for x in required if isinstance(x, SliceProfile)), key=lambda x: x.memory_gb):
            need = required[p] - sum(g.free.get(p, 0) for g in self.gpus)
            while need > 0:
                cands = [g for g in self.gpus if g.memory_gb - g.tot_slices_memory() >= p.memory_gb
                         and g.num_slices() < g.max_slices]
                if not cands:
                    break
                if self.placement == "measured":
                    g = max(cands, key=lambda g: (self._share(g), g.memory_gb - g.tot_slices_memory(), -g.index))
                else:
                    g = max(cands, key=lambda g: (g.memory_gb - g.tot_slices_memory(), -g.num_slices(), -g.index))
                g.create_slices(p.memory_gb)
                need -= 1
                updated = True
        return updated

    def _recompute_allocatable(self) -> None:
        sc = {k: v for k, v in self.node_info.allocatable.scalar.items() if not is_slice_resource(k)}
        for p, n in self.geometry().items():
            sc[p.resource_name()] = n
        self.node_info.allocatable.scalar = sc

    def add_pod(self, pod: dict) -> None:
        order = self.gpus
        if self.placement == "spread":  # mirror the device plugin's preferred allocation
            order = sorted(self.gpus, key=lambda g: (sum(g.used.values()), g.index))
        elif self.placement == "measured":
            order = sorted(self.gpus, key=lambda g: (-self.capacity.get(g.index, 1.0) / (sum(g.used.values()) + 1),
                                                     g.index))
        for g in order:
            try:
                g.add_pod(pod)
            except GenericError:
                continue
            self.node_info.add_pod(pod)
            return
        raise GenericError("not enough free slices")

    def clone(self) -> "SliceNode":
        c = SliceNode(self.name, [g.clone() for g in self.gpus], self.node_info.clone(), self.placement)
        c.capacity, c.measured = dict(self.capacity), self.measured
        return c


class SliceCalculator:
    def get_requested_slices(self, pod: dict) -> dict:
        return dict(requested_profiles(pod))


class SliceFilter:
    def extract_slices(self, resources: dict[str, int]) -> dict:
        return {profile_of_resource(k): int(v) for k, v in resources.items() if is_slice_resource(k)}
