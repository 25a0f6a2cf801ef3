"""Per-node, pure-Python GPU inventory with the :class:`~nos_amd.gpu.amdsmi.AmdSmi`
interface, for multi-node simulations.

The native ``libnos_amdsmi`` keeps ONE backend per process (like the real
amd-smi library), so a simulator with many nodes in one process gives each
node a :class:`FakeSmi` instead.  Semantics match the C++ fake backend
(``csrc/amdsmi/nos_amdsmi.cpp``): a compute-partition switch is refused while
the GPU has processes, the partition count follows the mode, and faults can
be injected.

Like a real amd-smi session it distinguishes the hardware from what the
session enumerated: ``external_switch=<gpu>:<mode>`` changes the hardware
only (another process switched the mode) and :meth:`rescan` makes it
visible.  ``switch_delay_ms=<n>`` makes every switch take that long in real
time WITHOUT holding the inventory lock; queries about a GPU whose switch is
in flight raise ``AmdSmiError(ERR_SWITCHING)`` and :meth:`gpus` reports it
from the last known state with ``switching=True`` (native library semantics).
"""
from __future__ import annotations

import dataclasses
import threading
import time

from .amdsmi import ERR_SWITCHING, PARTITIONS_PER_MODE, AmdSmiError, GpuInfo, PartitionInfo, ProcInfo

_MEMORY_MODES = ("NPS1", "NPS2", "NPS4", "NPS8")


class FakeSmi:
    backend = "pyfake"

    def __init__(self, gpus: int = 8, compute: str = "SPX", memory: str = "NPS1", cus: int = 256, xcds: int = 8,
                 vram_mb: int = 294912, model: str = "AMD Instinct MI355X", node: str = "node",
                 max_procs: int = 8, hip_order: list[int] | None = None):
        """``hip_order``: HIP id of each GPU (SPX), a permutation -- HIP's
        enumeration need not follow amd-smi's index order."""
        self._lock = threading.RLock()
        self.hip_order = list(hip_order) if hip_order is not None else None
        self.max_concurrent_processes = max_procs  # KFD HWS concurrent processes per logical GPU
        self.node = node
        self.model = model
        self.cus, self.xcds, self.vram_mb = cus, xcds, vram_mb
        self.compute = [compute] * gpus      # the session's view
        self.memory = [memory] * gpus
        self.hw_compute = [compute] * gpus   # the hardware
        self.hw_memory = [memory] * gpus
        self.switching: set[int] = set()
        self.switch_delay_s = 0.0
        self._last: dict[int, GpuInfo] = {}
        self.procs: list[dict[int, ProcInfo]] = [dict() for _ in range(gpus)]
        self.activity_gfx = [0] * gpus
        self.activity_umc = [0] * gpus
        self.faults: set[str] = set()
        self.lost: set[int] = set()
        self.switches = 0

    # ------------------------------------------------------------ queries
    def count(self) -> int:
        return len(self.compute) - len(self.lost)

    def _check(self, i: int, what: str) -> None:
        if i < 0 or i >= len(self.compute) or i in self.lost:
            raise AmdSmiError(-2, f"{what}({i})")
        if i in self.switching:
            raise AmdSmiError(ERR_SWITCHING, f"{what}({i})")

    def gpu(self, i: int) -> GpuInfo:
        with self._lock:
            self._check(i, "gpu")
            base = sum(PARTITIONS_PER_MODE[self.compute[j]] for j in range(i) if j not in self.lost)
            if self.hip_order is not None:
                base = self.hip_order[i]
            g = GpuInfo(index=i, num_cus=self.cus, num_xcds=self.xcds, compute_mode=self.compute[i],
                        memory_mode=self.memory[i], num_partitions=PARTITIONS_PER_MODE[self.compute[i]],
                        hip_id=base, drm_render=128 + base, vram_mb=self.vram_mb, bdf=f"0000:{0x11 + i:02x}:00.0",
                        uuid=f"GPU-{self.node}-{i:04d}", market_name=self.model)
            self._last[i] = g
            return g

    def gpus(self) -> list[GpuInfo]:
        """Every GPU; one whose mode switch is in flight is reported from its
        last known state with ``switching=True`` (it cannot be queried now)."""
        out = []
        for i in range(len(self.compute)):
            if i in self.lost:
                continue
            try:
                out.append(self.gpu(i))
            except AmdSmiError as e:
                if e.rc != ERR_SWITCHING or i not in self._last:
                    raise
                out.append(dataclasses.replace(self._last[i], switching=True))
        return out

    def rescan(self) -> None:
        with self._lock:
            if self.switching:
                raise AmdSmiError(ERR_SWITCHING, "rescan")
            self.compute, self.memory = list(self.hw_compute), list(self.hw_memory)

    def partitions(self, i: int) -> list[PartitionInfo]:
        """Logical devices of GPU ``i``, numbered GPU-major like the driver
        enumerates them (same model as the C++ fake backend)."""
        with self._lock:
            self._check(i, "partitions")
            base = sum(PARTITIONS_PER_MODE[self.compute[j]] for j in range(i) if j not in self.lost)
            n = PARTITIONS_PER_MODE[self.compute[i]]
            shared = self.memory[i] == "NPS1" and n > 1
            return [PartitionInfo(gpu_index=i, partition=p, hip_id=base + p, drm_render=128 + base + p,
                                  kfd_node=1 + base + p, num_cus=self.cus // n, num_xcds=max(1, self.xcds // n),
                                  memory_shared=shared, vram_mb=self.vram_mb // n,
                                  bdf=f"0000:{0x11 + i:02x}:00.{p}", uuid=f"GPU-{self.node}-{i:04d}-p{p}")
                    for p in range(n)]

    def clock(self, i: int) -> dict[str, int]:
        self._check(i, "clock")
        return {"sclk_mhz": 2400 if self.activity_gfx[i] > 0 else 500, "max_sclk_mhz": 2400}

    def activity(self, i: int) -> dict[str, int]:
        self._check(i, "activity")
        return {"gfx": self.activity_gfx[i], "umc": self.activity_umc[i], "mm": 0}

    def processes(self, i: int, max_procs: int = 256) -> list[ProcInfo]:
        with self._lock:
            self._check(i, "processes")
            return list(self.procs[i].values())[:max_procs]

    def link(self, i: int, j: int) -> dict:
        if i == j:
            return {"type": "internal", "hops": 0, "weight": 0}
        return {"type": "xgmi", "hops": 1, "weight": 15}

    # ------------------------------------------------------------ setters
    def _switch(self, i: int, mode: str, compute: bool) -> None:
        what = "set_compute_partition" if compute else "set_memory_partition"
        with self._lock:
            self._check(i, what)
            if ("fail_set_compute" if compute else "fail_set_memory") in self.faults:
                raise AmdSmiError(-3, f"{what}({i}, {mode})")
            if mode not in (PARTITIONS_PER_MODE if compute else _MEMORY_MODES):
                raise AmdSmiError(-4, f"unsupported {'compute' if compute else 'memory'} mode {mode}")
            if self.procs[i]:
                raise AmdSmiError(-5, f"gpu {i} busy")
            self.switching.add(i)
            delay = self.switch_delay_s
        try:
            if delay > 0:  # the driver at work: the inventory lock is NOT held
                time.sleep(delay)
        finally:
            with self._lock:
                self.switching.discard(i)
                hw = self.hw_compute if compute else self.hw_memory
                if hw[i] != mode and "stale_mode" not in self.faults:  # stale: silently no effect
                    hw[i] = mode
                    if compute:
                        self.switches += 1
                    if "lose_after_switch" in self.faults:
                        self.lost.add(i)
                # the session re-enumerates after its own switch (GPUs still switching keep their view)
                for j in range(len(self.compute)):
                    if j not in self.switching:
                        self.compute[j], self.memory[j] = self.hw_compute[j], self.hw_memory[j]

    def set_compute_partition(self, i: int, mode: str) -> None:
        self._switch(i, mode, True)

    def set_memory_partition(self, i: int, mode: str) -> None:
        self._switch(i, mode, False)

    # ------------------------------------------------------------ fake controls
    def inject(self, fault: str) -> None:
        with self._lock:
            if fault == "clear":
                self.faults.clear()
                self.lost.clear()
                self.switch_delay_s = 0.0
            elif fault.startswith("lose_gpu="):
                self.lost.add(int(fault.split("=", 1)[1]))
            elif fault.startswith("switch_delay_ms="):
                self.switch_delay_s = int(fault.split("=", 1)[1]) / 1000.0
            elif fault.startswith("external_switch="):
                gi, mode = fault.split("=", 1)[1].split(":", 1)
                if mode in PARTITIONS_PER_MODE:
                    self.hw_compute[int(gi)] = mode
                elif mode in _MEMORY_MODES:
                    self.hw_memory[int(gi)] = mode
                else:
                    raise AmdSmiError(-7, f"inject({fault})")
            else:
                self.faults.add(fault)

    def fake_add_process(self, i: int, pid: int, vram: int = 1 << 30, cus: int = 0) -> None:
        with self._lock:
            self.procs[i][pid] = ProcInfo(pid, cus, vram, f"proc{pid}")

    def fake_remove_process(self, i: int, pid: int) -> None:
        with self._lock:
            self.procs[i].pop(pid, None)

    def fake_set_activity(self, i: int, gfx: int, umc: int = 0) -> None:
        self.activity_gfx[i], self.activity_umc[i] = gfx, umc

    def close(self) -> None:
        pass
