"""Kubelet-visible devices (``pkg/resource/device.go:26-68``)."""
from __future__ import annotations

from dataclasses import dataclass

STATUS_USED, STATUS_FREE, STATUS_UNKNOWN = "used", "free", "unknown"
_STATUSES = (STATUS_USED, STATUS_FREE, STATUS_UNKNOWN)


def parse_status(s: str) -> str:
    if s not in _STATUSES:
        raise ValueError(f"invalid device status {s!r}")
    return s


@dataclass(frozen=True)
class Device:
    resource_name: str
    device_id: str
    status: str = STATUS_UNKNOWN

    def is_used(self) -> bool:
        return self.status == STATUS_USED

    def is_free(self) -> bool:
        return self.status == STATUS_FREE

    def with_status(self, status: str) -> "Device":
        return Device(self.resource_name, self.device_id, status)
