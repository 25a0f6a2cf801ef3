"""Hybrid partitioning: compute/memory partition modes AND memory slices per
logical partition -- the MI355X way past the 8-process limit of one GPU.

The reference declares ``hybrid`` in its partitioning-kind enum and never uses
it (``pkg/gpu/partitioning.go:87-91``); its MPS slices are bounded only by
memory (``pkg/gpu/slicing/gpu.go:67-97``, 1 GB minimum).  On MI355X a slice
(``amd.com/gpu-<N>gb``) is a process, and the amdgpu hardware scheduler runs
at most ``max-concurrent-processes`` (8) of them per *logical* GPU at once
(:mod:`nos_amd.gpu.kfd`).  Every compute partition is its own logical GPU
(own KFD node, own hardware scheduler and, in CPX, its own XCD and L2), so a
GPU split into ``P`` partitions runs up to ``8 P`` slices concurrently:

==========  =====  ==============  =================================
mode        parts  GB / partition  10 GB slices per GPU (MI355X)
==========  =====  ==============  =================================
SPX/NPS1    1      288             min(28, 8)      = 8
DPX/NPS1    2      144             2 x min(14, 8)  = 16
QPX/NPS1    4      72              4 x min(7, 8)   = 28
CPX/NPS1    8      36              8 x min(3, 8)   = 24
==========  =====  ==============  =================================

A :class:`HybridGPU` is a mode plus a multiset of slices; the slices must
bin-pack into the mode's partitions (memory and process slots per
partition, first-fit decreasing -- the device plugin places replicas the same
way).  Used slices pin the mode (a switch is GPU-wide and needs an idle GPU);
an idle GPU may switch to the mode that hosts the most of the lacking slices.
Inside a partition slices share its CUs (no CU mask: one XCD per CPX
partition cannot be split XCD-symmetrically), memory is the slice's cap.
"""
from __future__ import annotations

from dataclasses import dataclass, field

from ..api import constants as C
from ..kube import objects as ko
from .amdpart import ModeGeometry, get_allowed_geometries
from .core import GenericError, Geometry, get_count, get_model, parse_node_annotations
from .cumask import MIN_SLICE_MEMORY_GB, SliceProfile, is_slice_resource, profile_of_resource, requested_profiles
from .kfd import DEFAULT_MAX_CONCURRENT_PROCESSES


def pack(slices: dict[SliceProfile, int], parts: int, part_memory_gb: int, per_part: int,
         pinned: list[list[SliceProfile]] | None = None) -> list[list[SliceProfile]] | None:
    """First-fit-decreasing of ``slices`` into ``parts`` partitions of
    ``part_memory_gb`` and ``per_part`` process slots, on top of ``pinned``
    (slices already placed per partition).  Returns the placement or None."""
    bins = [list(b) for b in (pinned or [[] for _ in range(parts)])]
    if len(bins) != parts:
        return None
    mem = [sum(p.memory_gb for p in b) for b in bins]
    items = sorted((p for p, n in slices.items() for _ in range(n)), key=lambda p: -p.memory_gb)
    for p in items:
        for k in range(parts):
            if len(bins[k]) < per_part and mem[k] + p.memory_gb <= part_memory_gb:
                bins[k].append(p)
                mem[k] += p.memory_gb
                break
        else:
            return None
    return bins


@dataclass
class HybridGPU:
    model: str
    index: int
    memory_gb: int
    modes: list[ModeGeometry]
    mode: ModeGeometry
    used: dict[SliceProfile, int] = field(default_factory=dict)
    free: dict[SliceProfile, int] = field(default_factory=dict)
    max_procs: int = DEFAULT_MAX_CONCURRENT_PROCESSES

    # ------------------------------------------------------------ geometry of the mode
    @staticmethod
    def parts_of(mode: ModeGeometry) -> int:
        return sum(mode.geometry.values())

    @property
    def parts(self) -> int:
        return self.parts_of(self.mode)

    def part_memory_gb(self, mode: ModeGeometry | None = None) -> int:
        return self.memory_gb // self.parts_of(mode or self.mode)

    def capacity(self, profile: SliceProfile, mode: ModeGeometry | None = None) -> int:
        """Slices of one profile an empty GPU holds in ``mode``."""
        m = mode or self.mode
        return self.parts_of(m) * min(self.max_procs, self.part_memory_gb(m) // max(1, profile.memory_gb))

    def clone(self) -> "HybridGPU":
        return HybridGPU(self.model, self.index, self.memory_gb, self.modes, self.mode, dict(self.used),
                         dict(self.free), self.max_procs)

    def geometry(self) -> Geometry:
        g = Geometry()
        for d in (self.used, self.free):
            for p, n in d.items():
                if n:
                    g[p] = g.get(p, 0) + n
        return g

    def num_slices(self) -> int:
        return sum(self.used.values()) + sum(self.free.values())

    def placement(self, extra: dict[SliceProfile, int] | None = None,
                  mode: ModeGeometry | None = None) -> list[list[SliceProfile]] | None:
        m = mode or self.mode
        every = dict(self.geometry())
        for p, n in (extra or {}).items():
            every[p] = every.get(p, 0) + n
        return pack(every, self.parts_of(m), self.part_memory_gb(m), self.max_procs)

    def fits(self, extra: dict[SliceProfile, int] | None = None, mode: ModeGeometry | None = None) -> bool:
        return self.placement(extra, mode) is not None

    def validate(self) -> None:
        for d in (self.used, self.free):
            for p in d:
                if p.memory_gb < MIN_SLICE_MEMORY_GB:
                    raise GenericError(f"min allowed slice size is {MIN_SLICE_MEMORY_GB}GB")
        if not self.fits():
            raise GenericError(f"gpu {self.index}: slices {dict(self.geometry())} do not fit {self.mode.id()}")

    def can_switch(self) -> bool:
        return not any(self.used.values())

    def has_free_capacity(self) -> bool:
        if any(n > 0 for n in self.free.values()):
            return True
        small = SliceProfile.of(MIN_SLICE_MEMORY_GB)
        if self.fits({small: 1}):
            return True
        return self.can_switch() and any(self.fits({small: 1}, m) for m in self.modes)

    # ------------------------------------------------------------ planning
    def _grow(self, missing: dict[SliceProfile, int], mode: ModeGeometry) -> dict[SliceProfile, int]:
        """Lacking slices (smallest first) that fit next to the current ones in ``mode``."""
        added: dict[SliceProfile, int] = {}
        for p in sorted(missing, key=lambda x: x.memory_gb):
            for _ in range(missing[p]):
                trial = dict(added)
                trial[p] = trial.get(p, 0) + 1
                if not self.fits(trial, mode):
                    break
                added = trial
        return added

    def update_geometry_for(self, required: dict) -> bool:
        """Add lacking slices: in the current mode first; an idle GPU whose
        current mode cannot host all of them may switch to the allowed mode
        hosting the most (ties: fewer partitions, i.e. larger slices stay
        possible).  Free slices survive a switch only as far as they still fit."""
        missing = {p: n - self.free.get(p, 0) for p, n in required.items()
                   if isinstance(p, SliceProfile) and n - self.free.get(p, 0) > 0}
        if not missing:
            return False
        here = self._grow(missing, self.mode)
        best, best_add = self.mode, here
        if self.can_switch() and sum(here.values()) < sum(missing.values()):
            saved_free, self.free = self.free, {}
            for m in self.modes:
                if m.id() == self.mode.id():
                    continue
                add = self._grow(missing, m)
                if sum(add.values()) > sum(best_add.values()) or (
                        sum(add.values()) == sum(best_add.values()) > 0 and best is not self.mode
                        and self.parts_of(m) < self.parts_of(best)):
                    best, best_add = m, add
            if best is not self.mode:
                # keep the original free slices that still fit in the new mode
                kept: dict[SliceProfile, int] = {}
                for p, n in sorted(saved_free.items(), key=lambda kv: kv[0].memory_gb):
                    for _ in range(n):
                        trial = dict(best_add)
                        for q, k in kept.items():
                            trial[q] = trial.get(q, 0) + k
                        trial[p] = trial.get(p, 0) + 1
                        if self.fits(trial, best):
                            kept[p] = kept.get(p, 0) + 1
                self.free = kept
            else:
                self.free = saved_free
        if not best_add:
            return False
        self.mode = best
        for p, n in best_add.items():
            self.free[p] = self.free.get(p, 0) + n
        return True

    def add_pod(self, pod: dict) -> None:
        req = requested_profiles(pod)
        for p, n in req.items():
            if self.free.get(p, 0) < n:
                raise GenericError(f"not enough free slices (pod requests {n} {p}, GPU has {self.free.get(p, 0)})")
        for p, n in req.items():
            self.free[p] -= n
            if self.free[p] == 0:
                del self.free[p]
            self.used[p] = self.used.get(p, 0) + n


def _mode_of(modes: list[ModeGeometry], value: str | None) -> ModeGeometry | None:
    if not value or "/" not in value:
        return None
    c, m = value.split("/", 1)
    for mg in modes:
        if (mg.compute, mg.memory) == (c, m):
            return mg
    return None


class HybridNode:
    """Implements core.PartitionableNode over :class:`HybridGPU`."""

    def __init__(self, name: str, gpus: list[HybridGPU], node_info):
        self.name, self.gpus, self.node_info = name, gpus, node_info

    @classmethod
    def from_node_info(cls, ni) -> "HybridNode":
        node = ni.node()
        if node is None:
            raise GenericError("node is nil")
        model, count = get_model(node), get_count(node)
        labels, ann = ko.labels(node), ko.annotations(node)
        mem_mb = int(labels[C.LABEL_AMD_MEMORY]) if labels.get(C.LABEL_AMD_MEMORY, "").isdigit() else None
        xcds = int(labels[C.LABEL_AMD_XCDS]) if labels.get(C.LABEL_AMD_XCDS, "").isdigit() else None
        procs = labels.get(C.LABEL_AMD_MAX_PROCS, "")
        max_procs = int(procs) if procs.isdigit() and int(procs) > 0 else DEFAULT_MAX_CONCURRENT_PROCESSES
        modes = get_allowed_geometries(model, mem_mb, xcds)
        if modes is None:
            raise GenericError(f"model {model!r} is not associated with any known GPU")
        mem_gb = int(round(mem_mb / 1024)) if mem_mb else 288
        spx = next(m for m in modes if sum(m.geometry.values()) == 1)
        status, _ = parse_node_annotations(node)
        by_gpu: dict[int, tuple[dict, dict]] = {}
        for a in status:
            try:
                p = SliceProfile(a.profile)
            except ValueError:
                continue
            used, free = by_gpu.setdefault(a.index, ({}, {}))
            (used if a.is_used() else free)[p] = a.quantity
        gpus = []
        for i in range(count):
            mode = (_mode_of(modes, ann.get(C.ANNOTATION_STATUS_MODE_FORMAT.format(index=i)))
                    or _mode_of(modes, ann.get(C.ANNOTATION_SPEC_MODE_FORMAT.format(index=i))) or spx)
            used, free = by_gpu.get(i, ({}, {}))
            g = HybridGPU(model, i, mem_gb, modes, mode, dict(used), dict(free), max_procs)
            g.validate()
            gpus.append(g)
        return cls(ko.name(node), gpus, ni)

    def geometry(self) -> dict:
        res: dict = {}
        for g in self.gpus:
            for p, n in g.geometry().items():
                res[p] = res.get(p, 0) + n
        return res

    def has_free_capacity(self) -> bool:
        return any(g.has_free_capacity() for g in self.gpus)

    def _order(self) -> list[HybridGPU]:
        """GPUs that can host slices in their current mode first (no switch),
        then idle GPUs already split, whole idle GPUs last."""
        def key(g):
            return (0 if not g.can_switch() else 1, 0 if g.parts > 1 else 1, g.index)
        return sorted(self.gpus, key=key)

    def update_geometry_for(self, slices: dict) -> bool:
        required = {p: n for p, n in slices.items() if isinstance(p, SliceProfile)}
        if not self.gpus or not required:
            return False
        for g in self.gpus:  # free slices anywhere count first
            for p, n in g.free.items():
                if p in required:
                    required[p] -= n
                    if required[p] <= 0:
                        del required[p]
        updated = False
        for g in self._order():
            if not required:
                break
            before = dict(g.free)
            if g.update_geometry_for(required):
                updated = True
            for p in set(before) | set(g.free):
                if p not in slices:  # free slices of unrequested profiles a switch dropped: nobody waits for them
                    continue
                delta = g.free.get(p, 0) - before.get(p, 0)  # < 0: counted free slices destroyed by a switch
                required[p] = required.get(p, 0) - delta
                if required[p] <= 0:
                    required.pop(p, None)
        self._recompute_allocatable()
        return updated

    def _recompute_allocatable(self) -> None:
        sc = {k: v for k, v in self.node_info.allocatable.scalar.items() if not is_slice_resource(k)}
        for p, n in self.geometry().items():
            sc[p.resource_name()] = n
        self.node_info.allocatable.scalar = sc

    def add_pod(self, pod: dict) -> None:
        for g in self.gpus:
            try:
                g.add_pod(pod)
            except GenericError:
                continue
            self.node_info.add_pod(pod)
            return
        raise GenericError("not enough free slices")

    def clone(self) -> "HybridNode":
        return HybridNode(self.name, [g.clone() for g in self.gpus], self.node_info.clone())


class HybridSliceCalculator:
    def get_requested_slices(self, pod: dict) -> dict:
        return dict(requested_profiles(pod))


class HybridSliceFilter:
    def extract_slices(self, resources: dict[str, int]) -> dict:
        return {profile_of_resource(k): int(v) for k, v in resources.items() if is_slice_resource(k)}


__all__ = ["HybridGPU", "HybridNode", "pack", "HybridSliceCalculator", "HybridSliceFilter"]
