"""Allocation records: what ties a pod-server tenant to its device-plugin slice.

The reference's MPS slices are fixed by the device plugin -- each replica's
memory and device (``/root/reference/internal/partitioning/mps/partitioner.go:123-157``)
-- and MPS enforces the limit per client.  Here the device plugin's
``Allocate`` (deviceplugin/plugin.py) mints a random per-allocation token,
hands it to the pod in ``NOS_AMD_POD_TOKEN`` and writes the allocation's
record -- GPU, slice memory, CU mask, device ids, owner -- under the SHA-256
of the token into a directory that only the node's pod servers read (it is
never mounted into pods; a pod gets only its own GPU's socket directory).
The server admits a ``register`` only with a token whose record exists,
takes the slice from the record (never from the client), holds at most one
tenant per token, and evicts a tenant whose record disappears: the plugin
deletes records when it releases their devices (kubelet teardown, or a
PodResources sync showing the pod gone), and the server can also check
PodResources itself (``pkg/resource/client.go:39-87``).

Layout under the pod-server root directory::

    <root>/gpu-<i>/server.sock                 # mounted into GPU i's slice pods
    <root>/.allocations/gpu-<i>/<sha256>.json  # records, mode 0600
"""
from __future__ import annotations

import hashlib
import json
import os
import secrets
from pathlib import Path

RECORDS = ".allocations"


def socket_dir(root: str | os.PathLike, gpu: int) -> Path:
    return Path(root) / f"gpu-{gpu}"


def socket_path(root: str | os.PathLike, gpu: int) -> Path:
    return socket_dir(root, gpu) / "server.sock"


def records_dir(root: str | os.PathLike, gpu: int) -> Path:
    return Path(root) / RECORDS / f"gpu-{gpu}"


def token_hash(token: str) -> str:
    return hashlib.sha256(token.encode()).hexdigest()


def new_token() -> str:
    return secrets.token_urlsafe(24)


class AllocationStore:
    """The device plugin's side: write and delete records.

    The device -> record index is rebuilt from the files at construction
    (:meth:`load`), so a restarted plugin still finds -- and on release
    deletes -- the records it wrote before the restart; their tenants keep
    running until then (reference: the MIG agent re-reads the devices it
    created from the driver and kubelet at start-up,
    ``/root/reference/internal/controllers/migagent/actuator.go:134-138``,
    ``pkg/resource/client.go:39-87``)."""

    def __init__(self, root: str | os.PathLike):
        self.root = Path(root)
        self._by_device: dict[str, set[Path]] = {}
        self.load()

    def load(self) -> list[tuple[Path, dict]]:
        """(path, record) of every record on disk (all GPUs), re-indexed by
        device id; half-written (``.tmp``) or unreadable files are skipped."""
        out = []
        self._by_device = {}
        base = self.root / RECORDS
        if not base.is_dir():
            return out
        for path in sorted(base.glob("gpu-*/*")):
            if path.suffix != ".json":
                continue
            try:
                rec = json.loads(path.read_text())
                if not isinstance(rec, dict):
                    raise ValueError("not an object")
            except (OSError, ValueError):
                continue
            for did in rec.get("device_ids", []):
                self._by_device.setdefault(did, set()).add(path)
            out.append((path, rec))
        return out

    def devices(self) -> set[str]:
        """Device ids that hold a record."""
        return {d for d, ps in self._by_device.items() if ps}

    def write(self, gpu: int, token: str, record: dict) -> Path:
        d = records_dir(self.root, gpu)
        d.mkdir(parents=True, exist_ok=True)
        os.chmod(self.root / RECORDS, 0o700)
        path = d / f"{token_hash(token)}.json"
        tmp = path.with_suffix(".tmp")
        fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
        with os.fdopen(fd, "w") as f:
            json.dump({**record, "gpu": gpu}, f)
        os.replace(tmp, path)
        for did in record.get("device_ids", []):
            self._by_device.setdefault(did, set()).add(path)
        return path

    def remove_devices(self, device_ids) -> int:
        """Delete every record holding one of ``device_ids`` (their tenants are
        evicted by the server's reaper)."""
        gone: set[Path] = set()
        for did in device_ids:
            gone |= self._by_device.pop(did, set())
        for p in gone:
            try:
                p.unlink()
            except FileNotFoundError:
                pass
        for paths in self._by_device.values():
            paths -= gone
        return len(gone)


def lookup(records: str | os.PathLike, token: str) -> tuple[dict, Path] | None:
    """The server's side: the record of ``token`` in this GPU's records dir."""
    if not token or len(token) > 256:
        return None
    path = Path(records) / f"{token_hash(token)}.json"
    try:
        with open(path) as f:
            return json.load(f), path
    except (FileNotFoundError, json.JSONDecodeError):
        return None


__all__ = ["AllocationStore", "lookup", "new_token", "token_hash", "socket_path", "socket_dir", "records_dir",
           "RECORDS"]
