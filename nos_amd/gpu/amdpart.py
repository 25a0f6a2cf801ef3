"""AMD compute/memory partition model -- the MIG analogue (``pkg/gpu/mig``).

An MI355X is split GPU-wide: the compute partition mode decides how many
logical GPUs its 8 XCDs form (SPX 1x8, DPX 2x4, QPX 4x2, CPX 8x1) and the
memory partition mode (NPS1 / NPS2 / NPS4) how HBM is interleaved.  A
*profile* names one logical GPU: ``<xcds>xcd.<gb>gb`` (no ``-``, because the
annotation keys are split on ``-``).  A *geometry* maps profiles to counts;
unlike MIG, every allowed geometry is homogeneous (one profile) because the
mode is GPU-wide.

The algorithms are the reference's:

* ``can_apply_geometry``: the geometry is allowed for the model and keeps at
  least as many devices of every used profile (``mig/gpu.go:97-110``) -- for
  homogeneous modes this means a GPU with any partition in use can only keep
  its current mode ("repartition only idle GPUs");
* ``init_geometry``: fewest-slices geometry (SPX) (``:118-127``);
* ``update_geometry_for``: pick the allowed geometry that provides the most
  lacking profiles (``:158-212``);
* node: parse labels + status annotations, greedy per-GPU geometry update,
  recompute allocatable partition resources, first-fit ``add_pod``
  (``mig/node.go``).
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from pathlib import Path

import yaml

from ..api import constants as C
from ..kube import objects as ko
from ..kube import quantity as q
from .core import GenericError, Geometry, fewest_slices_geometry, get_count, get_model, parse_node_annotations

_PROFILE_RE = re.compile(C.REGEX_AMD_PARTITION_PROFILE)
_RESOURCE_RE = re.compile(C.REGEX_AMD_PARTITION_RESOURCE)


@dataclass(frozen=True, order=True)
class PartitionProfile:
    name: str

    def __post_init__(self):
        if not _PROFILE_RE.match(self.name):
            raise ValueError(f"invalid partition profile {self.name!r} (expected <n>xcd.<gb>gb)")

    @property
    def xcds(self) -> int:
        return int(_PROFILE_RE.match(self.name).group(1))

    @property
    def memory_gb(self) -> int:
        return int(_PROFILE_RE.match(self.name).group(2))

    def smaller_than(self, other) -> bool:
        """Memory first, then XCDs (``mig/profile.go`` SmallerThan)."""
        if not isinstance(other, PartitionProfile):
            return False
        if self.memory_gb != other.memory_gb:
            return self.memory_gb < other.memory_gb
        return self.xcds < other.xcds

    def resource_name(self) -> str:
        return C.AMD_PARTITION_RESOURCE_PREFIX + self.name

    def __str__(self) -> str:
        return self.name


def profile(name: str) -> PartitionProfile:
    return PartitionProfile(name)


def is_partition_resource(resource_name: str) -> bool:
    return bool(_RESOURCE_RE.match(resource_name))


def profile_of_resource(resource_name: str) -> PartitionProfile:
    m = _RESOURCE_RE.match(resource_name)
    if not m:
        raise ValueError(f"{resource_name!r} is not an AMD partition resource")
    return PartitionProfile(m.group(1))


def requested_profiles(pod: dict) -> dict[PartitionProfile, int]:
    from ..resource.resource import compute_pod_request

    out: dict[PartitionProfile, int] = {}
    for name, v in compute_pod_request(pod).items():
        if is_partition_resource(name) and q.value(v) > 0:
            p = profile_of_resource(name)
            out[p] = out.get(p, 0) + q.value(v)
    return out


# ----------------------------------------------------------------- known geometries
@dataclass(frozen=True)
class ModeGeometry:
    """One allowed (compute mode, memory mode) pair and the devices it yields."""

    compute: str
    memory: str
    geometry: Geometry

    def id(self) -> str:
        return f"{self.compute}/{self.memory}"


def partition_profile(memory_gb: int, xcds: int, parts: int) -> PartitionProfile:
    """The profile of one of ``parts`` logical devices of a GPU with
    ``memory_gb`` / ``xcds`` (as amd-smi reports them).  The planner (from the
    node labels) and the device plugin (from amd-smi) both name partitions
    through this one function, so their profiles always agree."""
    return PartitionProfile(f"{max(1, xcds // parts)}xcd.{memory_gb // parts}gb")


def mi355x_geometries(memory_gb: int = 288, xcds: int = 8) -> list[ModeGeometry]:
    out = []
    for compute, parts in (("SPX", 1), ("DPX", 2), ("QPX", 4), ("CPX", 8)):
        prof = partition_profile(memory_gb, xcds, parts)
        for memory in ("NPS1", "NPS2") if parts in (2, 8) else ("NPS1",):
            out.append(ModeGeometry(compute, memory, Geometry({prof: parts})))
    return out


_DEFAULT_MODELS = ["AMD Instinct MI355X", "AMD-Instinct-MI355X", "MI355X",
                   "AMD Instinct MI350X", "AMD-Instinct-MI350X", "MI350X"]
# explicitly configured tables (knownPartitionGeometriesFile) win; otherwise the
# geometries of a known model are derived from the memory / XCDs amd-smi reports
_known: dict[str, list[ModeGeometry]] = {}


def set_known_geometries(table: dict[str, list[ModeGeometry]]) -> None:
    validate_known(table)
    _known.clear()
    _known.update(table)


def get_allowed_geometries(model: str, memory_mb: int | None = None, xcds: int | None = None
                           ) -> list[ModeGeometry] | None:
    """Configured table of ``model``, else (MI350-series models) the mode
    geometries of the GPU's measured memory (``amd.com/gpu.memory``, MB) and
    XCD count -- never a hard-coded 288 GB when the node reports its size."""
    if model in _known:
        return _known[model]
    if model in _DEFAULT_MODELS:
        gb = int(round(memory_mb / 1024)) if memory_mb else 288
        return mi355x_geometries(gb, xcds or 8)
    return None


def validate_known(table: dict[str, list[ModeGeometry]]) -> None:
    for model, gs in table.items():
        if not gs:
            raise ValueError(f"model {model!r} has no allowed geometries")
        for g in gs:
            if len(g.geometry) != 1:
                raise ValueError(f"{model}: partition geometries must be homogeneous, got {g.geometry}")
            if g.compute not in ("SPX", "DPX", "TPX", "QPX", "CPX"):
                raise ValueError(f"{model}: unknown compute mode {g.compute}")
            if g.memory not in ("NPS1", "NPS2", "NPS4", "NPS8"):
                raise ValueError(f"{model}: unknown memory mode {g.memory}")


def load_known_geometries(path: str | Path) -> dict[str, list[ModeGeometry]]:
    """YAML: ``[{models: [...], allowedGeometries: [{compute: CPX, memory: NPS2,
    profiles: {1xcd.36gb: 8}}]}]`` (the reference's known_mig_geometries.yaml
    shape, with the mode pair added)."""
    data = yaml.safe_load(Path(path).read_text()) or []
    table: dict[str, list[ModeGeometry]] = {}
    for entry in data:
        if "models" not in entry:
            raise ValueError("missing field 'models'")
        if "allowedGeometries" not in entry:
            raise ValueError("missing field 'allowedGeometries'")
        gs = [ModeGeometry(g["compute"], g["memory"],
                           Geometry({PartitionProfile(p): int(n) for p, n in g["profiles"].items()}))
              for g in entry["allowedGeometries"]]
        for m in entry["models"]:
            table[m] = gs
    validate_known(table)
    return table


# ----------------------------------------------------------------- GPU
@dataclass
class PartitionGPU:
    model: str
    index: int
    allowed: list[ModeGeometry]
    used: dict[PartitionProfile, int] = field(default_factory=dict)
    free: dict[PartitionProfile, int] = field(default_factory=dict)
    memory_mode_preference: str = "NPS1"

    @classmethod
    def new(cls, model: str, index: int, used=None, free=None, memory_mb: int | None = None,
            xcds: int | None = None) -> "PartitionGPU":
        allowed = get_allowed_geometries(model, memory_mb, xcds)
        if allowed is None:
            raise GenericError(f"model {model!r} is not associated with any known GPU")
        return cls(model, index, allowed, dict(used or {}), dict(free or {}))

    def clone(self) -> "PartitionGPU":
        return PartitionGPU(self.model, self.index, self.allowed, dict(self.used), dict(self.free),
                            self.memory_mode_preference)

    def geometry(self) -> Geometry:
        g = Geometry()
        for d in (self.used, self.free):
            for p, n in d.items():
                if n:
                    g[p] = g.get(p, 0) + n
        return g

    def allowed_geometries(self) -> list[Geometry]:
        seen, out = set(), []
        for mg in self.allowed:
            if mg.geometry.id() not in seen:
                seen.add(mg.geometry.id())
                out.append(mg.geometry)
        return out

    def allows_geometry(self, g: Geometry) -> bool:
        return any(dict(g) == dict(a) for a in self.allowed_geometries())

    def can_apply_geometry(self, g: Geometry) -> tuple[bool, str]:
        if not self.allows_geometry(g):
            return False, f"GPU model {self.model} does not allow the provided partition geometry"
        for p, n in self.used.items():
            if g.get(p, 0) < n:
                return False, "cannot apply partition geometry: cannot delete partitions being used"
        return True, ""

    def apply_geometry(self, g: Geometry) -> None:
        ok, reason = self.can_apply_geometry(g)
        if not ok:
            raise GenericError(reason)
        for p, n in g.items():
            self.free[p] = n - self.used.get(p, 0)
        for p in list(self.free):
            if p not in g:
                del self.free[p]

    def init_geometry(self) -> None:
        g = fewest_slices_geometry(self.allowed_geometries())
        self.apply_geometry(g)

    def update_geometry_for(self, required: dict) -> bool:
        provided: dict[str, int] = {}
        lookup: dict[str, Geometry] = {}
        order: list[str] = []
        for cand in self.allowed_geometries():
            for prof, qty in required.items():
                if not isinstance(prof, PartitionProfile):
                    continue
                if self.free.get(prof, 0) >= qty:
                    continue
                n = min(cand.get(prof, 0) - self.used.get(prof, 0), qty)
                if n <= 0:
                    continue
                if not self.can_apply_geometry(cand)[0]:
                    continue
                gid = cand.id()
                if gid not in provided:
                    order.append(gid)
                provided[gid] = provided.get(gid, 0) + n
                lookup[gid] = cand
        best, best_n = None, 0
        for gid in order:
            if provided[gid] > best_n:
                best, best_n = lookup[gid], provided[gid]
        if best is None:
            return False
        self.apply_geometry(best)
        return True

    def add_pod(self, pod: dict) -> None:
        req = requested_profiles(pod)
        for p, n in req.items():
            if self.free.get(p, 0) < n:
                raise GenericError(f"not enough free partitions (pod requests {n} {p}, GPU has {self.free.get(p, 0)})")
        for p, n in req.items():
            self.free[p] -= n
            self.used[p] = self.used.get(p, 0) + n

    def has_free_partitions(self) -> bool:
        return any(n > 0 for n in self.free.values())

    def mode_for(self, g: Geometry | None = None) -> ModeGeometry | None:
        """The (compute, memory) pair realising geometry g, preferring the configured NPS mode."""
        g = g if g is not None else self.geometry()
        cands = [mg for mg in self.allowed if dict(mg.geometry) == dict(g)]
        if not cands:
            return None
        for mg in cands:
            if mg.memory == self.memory_mode_preference:
                return mg
        return cands[0]


# ----------------------------------------------------------------- node
class PartitionNode:
    """``mig.Node`` analogue; implements core.PartitionableNode."""

    def __init__(self, name: str, gpus: list[PartitionGPU], node_info, reserve_whole_gpus: int = 0):
        self.name = name
        self.gpus = gpus
        self.node_info = node_info
        # anti-starvation packing policy: a mode switch is GPU-wide
        # and needs an idle GPU, so fractional requests are steered onto GPUs that are
        # already partitioned, and the last ``reserve_whole_gpus`` whole (SPX) GPUs of
        # the node are never split for them -- whole-GPU pods cannot starve behind
        # a stream of small ones
        self.reserve_whole_gpus = reserve_whole_gpus

    def set_memory_mode_preference(self, nps: str) -> None:
        for g in self.gpus:
            g.memory_mode_preference = nps

    @classmethod
    def from_node_info(cls, ni) -> "PartitionNode":
        node = ni.node()
        if node is None:
            raise GenericError("node is nil")
        model = get_model(node)
        count = get_count(node)
        labels = ko.labels(node)
        mem = int(labels[C.LABEL_AMD_MEMORY]) if labels.get(C.LABEL_AMD_MEMORY, "").isdigit() else None
        xcds = int(labels[C.LABEL_AMD_XCDS]) if labels.get(C.LABEL_AMD_XCDS, "").isdigit() else None
        status, _ = parse_node_annotations(node)
        by_gpu: dict[int, list] = {}
        for a in status:
            by_gpu.setdefault(a.index, []).append(a)
        gpus = []
        for idx in sorted(by_gpu):
            used, free = {}, {}
            for a in by_gpu[idx]:
                try:
                    p = PartitionProfile(a.profile)
                except ValueError:
                    continue
                (used if a.is_used() else free)[p] = a.quantity
            gpus.append(PartitionGPU.new(model, idx, used, free, mem, xcds))
        have = {g.index for g in gpus}
        for i in range(count):
            if i not in have:
                gpus.append(PartitionGPU.new(model, i, memory_mb=mem, xcds=xcds))
        gpus.sort(key=lambda g: g.index)
        return cls(ko.name(node), gpus, ni)

    def geometry(self) -> dict:
        res: dict = {}
        for g in self.gpus:
            for p, n in g.geometry().items():
                res[p] = res.get(p, 0) + n
        return res

    def has_free_capacity(self) -> bool:
        if not self.gpus:
            return False
        for g in self.gpus:
            if g.has_free_partitions():
                return True
            if not g.allows_geometry(g.geometry()):
                return True
        return False

    def _is_whole(self, g: PartitionGPU) -> bool:
        geo = g.geometry()
        return len(geo) == 1 and next(iter(geo.values())) == 1

    def _order(self) -> list[PartitionGPU]:
        """Free partitions first (no switch), then GPUs already split (a switch
        between split modes), whole GPUs last."""
        def key(g):
            has_free = any(n > 0 for n in g.free.values())
            return (0 if has_free else 1, 1 if self._is_whole(g) else 0, g.index)
        return sorted(self.gpus, key=key)

    def update_geometry_for(self, slices: dict) -> bool:
        if not self.gpus or not slices:
            return False
        required = dict(slices)
        # already-free partitions count first: no GPU is switched for demand they
        # cover.  covered[gpu][p] remembers how much demand each GPU's free
        # partitions absorbed, so that a later switch of that GPU (which destroys
        # its free partitions: modes are GPU-wide) puts that demand back
        # (mig/node.go:145-177 counts free devices after each GPU's update)
        covered: dict[int, dict] = {}
        for g in self.gpus:
            for p, n in g.free.items():
                if p in required and n > 0:
                    take = min(n, required[p])
                    covered.setdefault(g.index, {})[p] = take
                    required[p] -= take
                    if required[p] <= 0:
                        del required[p]
        updated = False
        whole_idle = sum(1 for g in self.gpus if self._is_whole(g) and not any(g.used.values()))
        for g in self._order():
            if not required:
                break
            whole = self._is_whole(g)
            if whole and not any(g.used.values()) and whole_idle <= self.reserve_whole_gpus:
                continue  # keep the reserve of whole GPUs
            before = dict(g.free)
            if g.update_geometry_for(required):
                updated = True
                if whole and not self._is_whole(g):
                    whole_idle -= 1
                # demand the destroyed free partitions covered is lacking again
                for p, n in covered.pop(g.index, {}).items():
                    lost = min(n, max(0, before.get(p, 0) - g.free.get(p, 0)))
                    if lost > 0:
                        required[p] = required.get(p, 0) + lost
                for p, n in g.free.items():
                    gained = n - before.get(p, 0)
                    if p in required and gained > 0:
                        required[p] -= gained
                        if required[p] <= 0:
                            del required[p]
        self._recompute_allocatable()
        return updated

    def _recompute_allocatable(self) -> None:
        sc = {k: v for k, v in self.node_info.allocatable.scalar.items() if not is_partition_resource(k)}
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
        raise GenericError("not enough free partitions")

    def clone(self) -> "PartitionNode":
        return PartitionNode(self.name, [g.clone() for g in self.gpus], self.node_info.clone(),
                             self.reserve_whole_gpus)


class PartitionSliceCalculator:
    def get_requested_slices(self, pod: dict) -> dict:
        return dict(requested_profiles(pod))


class PartitionSliceFilter:
    def extract_slices(self, resources: dict[str, int]) -> dict:
        out = {}
        for name, n in resources.items():
            if is_partition_resource(name):
                out[profile_of_resource(name)] = int(n)
        return out
