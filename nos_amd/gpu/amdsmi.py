"""Python binding of ``libnos_amdsmi.so`` (csrc/amdsmi/nos_amdsmi.cpp).

This is the node-local device layer of the partition agent and gpuagent --
the MI355X replacement for the reference's NVML client
(``pkg/gpu/nvml/interface.go:23-35``).  Two backends share one interface:

* ``AmdSmi.real()``  -- amd-smi (read-only unless ``allow_set=True``);
  indices are PHYSICAL GPUs; :meth:`AmdSmi.partitions` lists the logical
  devices (one amd-smi processor handle each) of a GPU in DPX/QPX/CPX;
* ``AmdSmi.fake(...)`` -- an in-memory MI355X node (C++), with programmable
  processes, activity and fault injection, for the simulator and tests.
"""
from __future__ import annotations

import ctypes
import dataclasses
import threading
from dataclasses import dataclass
from pathlib import Path

_LIB = Path(__file__).resolve().parent.parent / "_native" / "libnos_amdsmi.so"

COMPUTE_MODES = {1: "SPX", 2: "DPX", 3: "TPX", 4: "QPX", 5: "CPX"}
COMPUTE_IDS = {v: k for k, v in COMPUTE_MODES.items()}
MEMORY_MODES = {1: "NPS1", 2: "NPS2", 4: "NPS4", 8: "NPS8"}
MEMORY_IDS = {v: k for k, v in MEMORY_MODES.items()}
PARTITIONS_PER_MODE = {"SPX": 1, "DPX": 2, "TPX": 3, "QPX": 4, "CPX": 8}
LINK_TYPES = {0: "internal", 1: "pcie", 2: "xgmi", 3: "n/a", 4: "unknown"}

ERRORS = {0: "ok", -1: "not open", -2: "bad index", -3: "backend error", -4: "unsupported",
          -5: "busy (processes on GPU)", -6: "injected fault", -7: "invalid argument", -8: "timeout",
          -9: "mode switch in progress"}
ERR_SWITCHING = -9


class AmdSmiError(RuntimeError):
    def __init__(self, rc: int, what: str):
        super().__init__(f"{what}: {ERRORS.get(rc, rc)}")
        self.rc = rc


class _GpuInfo(ctypes.Structure):
    _fields_ = [("index", ctypes.c_int), ("num_cus", ctypes.c_int), ("num_xcds", ctypes.c_int),
                ("compute_mode", ctypes.c_int), ("memory_mode", ctypes.c_int),
                ("num_partitions", ctypes.c_int), ("hip_id", ctypes.c_int), ("drm_render", ctypes.c_int),
                ("vram_mb", ctypes.c_longlong), ("bdf", ctypes.c_char * 32), ("uuid", ctypes.c_char * 64),
                ("market_name", ctypes.c_char * 128)]


class _PartInfo(ctypes.Structure):
    _fields_ = [("gpu_index", ctypes.c_int), ("partition", ctypes.c_int), ("hip_id", ctypes.c_int),
                ("drm_render", ctypes.c_int), ("kfd_node", ctypes.c_int), ("num_cus", ctypes.c_int),
                ("num_xcds", ctypes.c_int), ("memory_shared", ctypes.c_int), ("vram_mb", ctypes.c_longlong),
                ("bdf", ctypes.c_char * 32), ("uuid", ctypes.c_char * 64)]


class _ProcInfo(ctypes.Structure):
    _fields_ = [("pid", ctypes.c_uint), ("cu_occupancy", ctypes.c_uint), ("vram_bytes", ctypes.c_longlong),
                ("name", ctypes.c_char * 64)]


@dataclass(frozen=True)
class GpuInfo:
    index: int
    num_cus: int
    num_xcds: int
    compute_mode: str
    memory_mode: str
    num_partitions: int
    hip_id: int
    drm_render: int
    vram_mb: int
    bdf: str
    uuid: str
    market_name: str
    switching: bool = False  # a mode switch is in flight: the fields are the last known state

    @property
    def memory_gb(self) -> int:
        return int(round(self.vram_mb / 1024))


@dataclass(frozen=True)
class PartitionInfo:
    """One logical device (compute partition) of a physical GPU.  In SPX a GPU
    has exactly one, equal to the GPU itself."""

    gpu_index: int
    partition: int
    hip_id: int
    drm_render: int
    kfd_node: int
    num_cus: int
    num_xcds: int
    memory_shared: bool   # NPS1 with several partitions: vram_mb is a 1/n share of one pool
    vram_mb: int
    bdf: str
    uuid: str

    @property
    def memory_gb(self) -> int:
        return int(round(self.vram_mb / 1024))


@dataclass(frozen=True)
class ProcInfo:
    pid: int
    cu_occupancy: int
    vram_bytes: int
    name: str


_load_lock = threading.Lock()
_lib = None


def _L():
    global _lib
    with _load_lock:
        if _lib is None:
            if not _LIB.exists():
                raise RuntimeError(f"{_LIB} missing: run `python -m nos_amd._native.build --only amdsmi`")
            L = ctypes.CDLL(str(_LIB))
            L.nos_smi_open.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
            L.nos_smi_gpu_info.argtypes = [ctypes.c_int, ctypes.POINTER(_GpuInfo)]
            L.nos_smi_set_compute_partition.argtypes = [ctypes.c_int, ctypes.c_int]
            L.nos_smi_set_memory_partition.argtypes = [ctypes.c_int, ctypes.c_int]
            L.nos_smi_activity.argtypes = [ctypes.c_int] + [ctypes.POINTER(ctypes.c_int)] * 3
            L.nos_smi_processes.argtypes = [ctypes.c_int, ctypes.POINTER(_ProcInfo), ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_int)]
            L.nos_smi_link.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                       ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_longlong)]
            L.nos_smi_fake_inject.argtypes = [ctypes.c_char_p]
            L.nos_smi_fake_add_process.argtypes = [ctypes.c_int, ctypes.c_uint, ctypes.c_longlong, ctypes.c_uint]
            L.nos_smi_fake_remove_process.argtypes = [ctypes.c_int, ctypes.c_uint]
            L.nos_smi_fake_set_activity.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
            L.nos_smi_partition_count.argtypes = [ctypes.c_int]
            L.nos_smi_clock.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
            L.nos_smi_partition_info.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(_PartInfo)]
            L.nos_smi_struct_sizes.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
            a, b = ctypes.c_int(), ctypes.c_int()
            L.nos_smi_struct_sizes(ctypes.byref(a), ctypes.byref(b))
            if (a.value != ctypes.sizeof(_GpuInfo) or b.value != ctypes.sizeof(_ProcInfo)
                    or L.nos_smi_part_struct_size() != ctypes.sizeof(_PartInfo)):
                raise RuntimeError("libnos_amdsmi ABI mismatch")
            _lib = L
    return _lib


class AmdSmi:
    """Process-wide amd-smi session (the C library keeps one backend)."""

    _active: "AmdSmi | None" = None

    def __init__(self, backend: str, spec: str = "", allow_set: bool = False):
        self.backend = backend
        rc = _L().nos_smi_open(backend.encode(), spec.encode(), int(allow_set))
        if rc != 0:
            raise AmdSmiError(rc, f"amdsmi open ({backend})")
        AmdSmi._active = self
        self._last: dict[int, GpuInfo] = {}

    @classmethod
    def real(cls, allow_set: bool = False) -> "AmdSmi":
        return cls("amdsmi", "", allow_set)

    @classmethod
    def fake(cls, gpus: int = 8, compute: str = "SPX", memory: str = "NPS1", cus: int = 256, xcds: int = 8,
             vram_mb: int = 294912, model: str = "AMD Instinct MI355X") -> "AmdSmi":
        spec = f"gpus={gpus};cus={cus};xcds={xcds};vram_mb={vram_mb};compute={compute};memory={memory};model={model}"
        return cls("fake", spec)

    def close(self) -> None:
        _L().nos_smi_close()

    def rescan(self) -> None:
        """Re-enumerate the devices.  The session enumerates at open and after
        its own mode switches; a mode another process switched (the partition
        agent, the amd-smi CLI) is only visible after this call.  Raises with
        ``rc == ERR_SWITCHING`` while one of this session's switches runs."""
        rc = _L().nos_smi_rescan()
        if rc != 0:
            raise AmdSmiError(rc, "rescan")

    # ------------------------------------------------------------- queries
    def count(self) -> int:
        n = _L().nos_smi_count()
        if n < 0:
            raise AmdSmiError(n, "count")
        return n

    def gpu(self, i: int) -> GpuInfo:
        g = _GpuInfo()
        rc = _L().nos_smi_gpu_info(i, ctypes.byref(g))
        if rc != 0:
            raise AmdSmiError(rc, f"gpu_info({i})")
        info = GpuInfo(g.index, g.num_cus, g.num_xcds, COMPUTE_MODES.get(g.compute_mode, "UNKNOWN"),
                       MEMORY_MODES.get(g.memory_mode, "UNKNOWN"), g.num_partitions, g.hip_id, g.drm_render,
                       g.vram_mb, g.bdf.decode(), g.uuid.decode(), g.market_name.decode())
        self._last[i] = info
        return info

    def gpus(self) -> list[GpuInfo]:
        """Every GPU; one whose mode switch is in flight (in another thread) is
        reported from its last known state with ``switching=True``."""
        out = []
        for i in range(self.count()):
            try:
                out.append(self.gpu(i))
            except AmdSmiError as e:
                if e.rc != ERR_SWITCHING or i not in self._last:
                    raise
                out.append(dataclasses.replace(self._last[i], switching=True))
        return out

    def partitions(self, i: int) -> list[PartitionInfo]:
        """Logical devices of physical GPU ``i`` in enumeration order (amd-smi
        lists one processor handle per partition; the library groups them)."""
        n = _L().nos_smi_partition_count(i)
        if n < 0:
            raise AmdSmiError(n, f"partition_count({i})")
        out = []
        for p in range(n):
            x = _PartInfo()
            rc = _L().nos_smi_partition_info(i, p, ctypes.byref(x))
            if rc != 0:
                raise AmdSmiError(rc, f"partition_info({i}, {p})")
            out.append(PartitionInfo(x.gpu_index, x.partition, x.hip_id, x.drm_render, x.kfd_node, x.num_cus,
                                     x.num_xcds, bool(x.memory_shared), x.vram_mb, x.bdf.decode(), x.uuid.decode()))
        return out

    def activity(self, i: int) -> dict[str, int]:
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        rc = _L().nos_smi_activity(i, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        if rc != 0:
            raise AmdSmiError(rc, f"activity({i})")
        return {"gfx": a.value, "umc": b.value, "mm": c.value}

    def clock(self, i: int) -> dict[str, int]:
        """Current and maximum GFX clock (MHz) -- tells DVFS apart from a kernel limit."""
        a, b = ctypes.c_int(), ctypes.c_int()
        rc = _L().nos_smi_clock(i, ctypes.byref(a), ctypes.byref(b))
        if rc != 0:
            raise AmdSmiError(rc, f"clock({i})")
        return {"sclk_mhz": a.value, "max_sclk_mhz": b.value}

    def processes(self, i: int, max_procs: int = 256) -> list[ProcInfo]:
        arr = (_ProcInfo * max_procs)()
        n = ctypes.c_int()
        rc = _L().nos_smi_processes(i, arr, max_procs, ctypes.byref(n))
        if rc != 0:
            raise AmdSmiError(rc, f"processes({i})")
        return [ProcInfo(p.pid, p.cu_occupancy, p.vram_bytes, p.name.decode()) for p in arr[: min(n.value, max_procs)]]

    def link(self, i: int, j: int) -> dict:
        t, h, w = ctypes.c_int(), ctypes.c_longlong(), ctypes.c_longlong()
        rc = _L().nos_smi_link(i, j, ctypes.byref(t), ctypes.byref(h), ctypes.byref(w))
        if rc != 0:
            raise AmdSmiError(rc, f"link({i},{j})")
        return {"type": LINK_TYPES.get(t.value, "unknown"), "hops": h.value, "weight": w.value}

    # ------------------------------------------------------------- setters
    def set_compute_partition(self, i: int, mode: str) -> None:
        rc = _L().nos_smi_set_compute_partition(i, COMPUTE_IDS[mode])
        if rc != 0:
            raise AmdSmiError(rc, f"set_compute_partition({i}, {mode})")

    def set_memory_partition(self, i: int, mode: str) -> None:
        rc = _L().nos_smi_set_memory_partition(i, MEMORY_IDS[mode])
        if rc != 0:
            raise AmdSmiError(rc, f"set_memory_partition({i}, {mode})")

    # ------------------------------------------------------- fake controls
    def inject(self, fault: str) -> None:
        rc = _L().nos_smi_fake_inject(fault.encode())
        if rc != 0:
            raise AmdSmiError(rc, f"inject({fault})")

    def fake_add_process(self, i: int, pid: int, vram: int = 1 << 30, cus: int = 0) -> None:
        rc = _L().nos_smi_fake_add_process(i, pid, vram, cus)
        if rc != 0:
            raise AmdSmiError(rc, "fake_add_process")

    def fake_remove_process(self, i: int, pid: int) -> None:
        rc = _L().nos_smi_fake_remove_process(i, pid)
        if rc != 0:
            raise AmdSmiError(rc, "fake_remove_process")

    def fake_set_activity(self, i: int, gfx: int, umc: int = 0) -> None:
        rc = _L().nos_smi_fake_set_activity(i, gfx, umc)
        if rc != 0:
            raise AmdSmiError(rc, "fake_set_activity")


class ActivitySampler:
    """Background sampler of gfx activity (%) for a set of GPUs (bench / metrics)."""

    def __init__(self, smi: AmdSmi | None, gpus: list[int], period_s: float = 0.05):
        self.smi, self.gpus, self.period = smi, gpus, period_s
        self.samples: list[dict[int, int]] = []
        self._stop = threading.Event()
        self._t: threading.Thread | None = None

    def _run(self) -> None:
        while not self._stop.is_set():
            try:
                self.samples.append({g: self.smi.activity(g)["gfx"] for g in self.gpus})
            except Exception:
                pass
            self._stop.wait(self.period)

    def __enter__(self) -> "ActivitySampler":
        if self.smi is not None:
            self._t = threading.Thread(target=self._run, daemon=True)
            self._t.start()
        return self

    def __exit__(self, *exc) -> None:
        self._stop.set()
        if self._t:
            self._t.join(timeout=2)

    def mean(self) -> float | None:
        if not self.samples:
            return None
        vals = [v for s in self.samples for v in s.values()]
        return sum(vals) / len(vals) if vals else None
