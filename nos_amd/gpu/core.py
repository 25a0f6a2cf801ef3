"""GPU domain model shared by both partitioning strategies.

Behavioural equivalent of the reference's ``pkg/gpu`` package:

* :class:`GpuDevice` / device-list group-bys (``device.go:26-137``);
* spec / status annotation codec (``annotation.go:29-224``): keys
  ``nos.nebuly.com/spec-gpu-<i>-<profile>`` and
  ``nos.nebuly.com/status-gpu-<i>-<profile>-<free|used>``.  The key is split on
  ``-`` so profile names must not contain ``-`` (validated here);
* :class:`Slice` protocol, :class:`Geometry` and
  :func:`fewest_slices_geometry` (``partitioning.go:28-79``);
* partitioning kind of a node (``partitioning.go:87-130``) with AMD kinds;
* node GPU facts from the agent-written ``amd.com/gpu.*`` labels
  (``util.go:30-73``) and ``compute_free_devices_and_update_status``;
* typed errors (``errors.go:24-99``).
"""
from __future__ import annotations

import json
from collections import defaultdict
from dataclasses import dataclass
from typing import Callable, Iterable, Protocol, runtime_checkable

from ..api import constants as C
from ..kube import objects as ko
from ..resource.device import STATUS_FREE, STATUS_USED, Device, parse_status


# ----------------------------------------------------------------- errors
class GpuError(Exception):
    pass


class NotFoundError(GpuError):
    """A device / GPU index was not found (triggers a device-plugin refresh)."""


class GenericError(GpuError):
    pass


def is_not_found(e: BaseException) -> bool:
    return isinstance(e, NotFoundError)


# ----------------------------------------------------------------- devices
@dataclass(frozen=True)
class GpuDevice:
    device: Device
    gpu_index: int

    @property
    def resource_name(self) -> str:
        return self.device.resource_name

    @property
    def device_id(self) -> str:
        return self.device.device_id

    @property
    def status(self) -> str:
        return self.device.status

    def is_used(self) -> bool:
        return self.device.is_used()

    def is_free(self) -> bool:
        return self.device.is_free()

    def full_resource_name(self) -> str:
        return f"{self.gpu_index}/{self.resource_name}"

    def __str__(self) -> str:
        return f"{self.gpu_index}/{self.resource_name}/{self.device_id}/{self.status}"


def group_by(devs: Iterable, key: Callable) -> dict:
    out: dict = defaultdict(list)
    for d in devs:
        out[key(d)].append(d)
    return dict(out)


def group_by_gpu(devs: Iterable[GpuDevice]) -> dict[int, list[GpuDevice]]:
    return group_by(devs, lambda d: d.gpu_index)


def sort_by_device_id(devs: Iterable[GpuDevice]) -> list[GpuDevice]:
    return sorted(devs, key=lambda d: d.device_id)


def free(devs: Iterable[GpuDevice]) -> list[GpuDevice]:
    return [d for d in devs if d.is_free()]


def used(devs: Iterable[GpuDevice]) -> list[GpuDevice]:
    return [d for d in devs if d.is_used()]


def compute_free_devices_and_update_status(used_devs: list[GpuDevice], allocatable: list[GpuDevice]) -> list[GpuDevice]:
    used_ids = {u.device_id for u in used_devs}
    return [GpuDevice(a.device.with_status(STATUS_FREE), a.gpu_index) for a in allocatable
            if a.device_id not in used_ids]


# ----------------------------------------------------------------- annotations
@dataclass(frozen=True)
class SpecAnnotation:
    index: int
    profile: str
    quantity: int

    def key(self) -> str:
        return C.ANNOTATION_GPU_SPEC_FORMAT.format(index=self.index, profile=self.profile)

    def value(self) -> str:
        return str(self.quantity)

    def index_with_profile(self) -> str:
        return f"{self.index}-{self.profile}"


@dataclass(frozen=True)
class StatusAnnotation:
    index: int
    profile: str
    status: str
    quantity: int

    def key(self) -> str:
        return C.ANNOTATION_GPU_STATUS_FORMAT.format(index=self.index, profile=self.profile, status=self.status)

    def value(self) -> str:
        return str(self.quantity)

    def is_used(self) -> bool:
        return self.status == STATUS_USED

    def is_free(self) -> bool:
        return self.status == STATUS_FREE

    def index_with_profile(self) -> str:
        return f"{self.index}-{self.profile}"


def validate_profile_name(profile: str) -> str:
    if not profile or "-" in profile:
        raise ValueError(f"invalid profile name {profile!r}: must be non-empty and contain no '-'")
    return profile


def parse_spec_annotation(key: str, value: str) -> SpecAnnotation:
    if not key.startswith(C.ANNOTATION_GPU_SPEC_PREFIX):
        raise ValueError(f"expected spec annotation prefix {C.ANNOTATION_GPU_SPEC_PREFIX!r}, got {key!r}")
    parts = key.split("-")
    if len(parts) != 4:
        raise ValueError(f"invalid spec annotation key {key!r}")
    return SpecAnnotation(int(parts[2]), parts[3], int(value))


def parse_status_annotation(key: str, value: str) -> StatusAnnotation:
    if not key.startswith(C.ANNOTATION_GPU_STATUS_PREFIX):
        raise ValueError(f"expected status prefix {C.ANNOTATION_GPU_STATUS_PREFIX!r}, got {key!r}")
    parts = key.split("-")
    if len(parts) != 5:
        raise ValueError(f"invalid status annotation key {key!r}")
    return StatusAnnotation(int(parts[2]), parts[3], parse_status(parts[4]), int(value))


def parse_node_annotations(node: dict) -> tuple[list[StatusAnnotation], list[SpecAnnotation]]:
    status, spec = [], []
    for k, v in ko.annotations(node).items():
        try:
            spec.append(parse_spec_annotation(k, v))
            continue
        except ValueError:
            pass
        try:
            status.append(parse_status_annotation(k, v))
        except ValueError:
            pass
    status.sort(key=lambda a: (a.index, a.profile, a.status))
    spec.sort(key=lambda a: (a.index, a.profile))
    return status, spec


def devices_as_status_annotations(devs: Iterable[GpuDevice], get_profile: Callable[[str], str]) -> list[StatusAnnotation]:
    """``DeviceList.AsStatusAnnotation``: one annotation per (gpu, profile, status) with the count."""
    counts: dict[tuple[int, str, str], int] = defaultdict(int)
    for d in devs:
        try:
            prof = get_profile(d.resource_name)
        except ValueError:
            continue
        counts[(d.gpu_index, prof, d.status)] += 1
    return sorted((StatusAnnotation(i, p, s, n) for (i, p, s), n in counts.items()),
                  key=lambda a: (a.index, a.profile, a.status))


def status_equal(a: list[StatusAnnotation], b: list[StatusAnnotation]) -> bool:
    return sorted(a, key=repr) == sorted(b, key=repr)


def spec_matches_status(spec: list[SpecAnnotation], status: list[StatusAnnotation]) -> bool:
    """Per (gpu, profile), spec quantity == free + used quantity (``mig/annotation.go:24-35``)."""
    want: dict[tuple[int, str], int] = defaultdict(int)
    have: dict[tuple[int, str], int] = defaultdict(int)
    for s in spec:
        if s.quantity:
            want[(s.index, s.profile)] += s.quantity
    for s in status:
        if s.quantity:
            have[(s.index, s.profile)] += s.quantity
    return dict(want) == dict(have)


# ----------------------------------------------------------------- slices
@runtime_checkable
class Slice(Protocol):
    def smaller_than(self, other: "Slice") -> bool: ...

    def __str__(self) -> str: ...


class Geometry(dict):
    """Mapping Slice -> quantity with a stable string id."""

    def id(self) -> str:
        return str(self)

    def __str__(self) -> str:  # "profile:qty, " pairs ordered by profile name
        return "".join(f"{p}:{self[p]}, " for p in sorted(self, key=str))

    def to_json(self) -> str:
        return json.dumps({str(k): v for k, v in self.items()}, sort_keys=True)

    def __hash__(self):  # geometries are used as set members in tests
        return hash(tuple(sorted((str(k), v) for k, v in self.items())))


def fewest_slices_geometry(geometries: list[Geometry]) -> Geometry | None:
    best = None
    for g in geometries:
        if best is None or len(g) < len(best):
            best = g
    return best


class SliceCalculator(Protocol):
    def get_requested_slices(self, pod: dict) -> dict: ...


class SliceFilter(Protocol):
    def extract_slices(self, resources: dict[str, int]) -> dict: ...


# ----------------------------------------------------------------- partitioning kind
def partitioning_kind(node: dict) -> str | None:
    v = ko.labels(node).get(C.LABEL_GPU_PARTITIONING)
    return v if v in (C.PARTITIONING_AMDPART, C.PARTITIONING_CUMASK, C.PARTITIONING_HYBRID) else None


def is_amdpart_enabled(node: dict) -> bool:
    return ko.labels(node).get(C.LABEL_GPU_PARTITIONING) == C.PARTITIONING_AMDPART


def is_cumask_enabled(node: dict) -> bool:
    return ko.labels(node).get(C.LABEL_GPU_PARTITIONING) == C.PARTITIONING_CUMASK


# ----------------------------------------------------------------- node facts
def get_model(node: dict) -> str:
    v = ko.labels(node).get(C.LABEL_AMD_PRODUCT)
    if v is None:
        raise GenericError(f"cannot get GPU model from node {ko.name(node)} labels: missing {C.LABEL_AMD_PRODUCT}")
    return v


def get_count(node: dict) -> int:
    v = ko.labels(node).get(C.LABEL_AMD_COUNT)
    if v is None:
        raise GenericError(f"cannot get GPU count from node labels, missing label {C.LABEL_AMD_COUNT}")
    return int(v)


def get_memory_gb(node: dict) -> int:
    """Label holds MB (as the NVIDIA label did); GB = ceil(MB / 1000) like the reference
    (``pkg/gpu/util.go:59-73``) -- but MI355X labels are written in MiB, so 294912 MiB
    is reported as 288 GB by dividing by 1024 when the value is a whole number of GiB."""
    v = ko.labels(node).get(C.LABEL_AMD_MEMORY)
    if v is None:
        raise GenericError(f"cannot get GPU memory from node labels, missing label {C.LABEL_AMD_MEMORY}")
    mb = int(v)
    if mb % 1024 == 0:
        return mb // 1024
    return -(-mb // 1000)
