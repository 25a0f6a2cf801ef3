"""KFD (amdgpu compute driver) limits that shape how many pods a GPU can run.

The amdgpu hardware scheduler (HWS) maps at most ``hws_max_conc_proc``
processes onto the GPU at once (one VMID each; the driver default is 8 -- the
VMIDs KFD owns).  A GPU with more GPU-using processes than that is
*time-sliced* between them: measured on MI355X (SPX) with fp32 YOLOS pods,
aggregate throughput peaks at 8 processes (256 inf/s) and falls with more
(10: 225, 14: 189 inf/s) while per-pod latency quantises to the ~50 ms
runlist quantum (profiles/r02_pods_vs_throughput_hwqueues.json).  The reference
never meets this limit (MPS serves up to 48 clients through one server
process); on MI355X it is the real bound on concurrently running fractional
pods per logical GPU, so the node labeler publishes it and the cumask
partitioner never creates more slices per GPU than it allows.
"""
from __future__ import annotations

from pathlib import Path

DEFAULT_MAX_CONCURRENT_PROCESSES = 8
_PARAM = Path("/sys/module/amdgpu/parameters/hws_max_conc_proc")


def hws_max_concurrent_processes(param: Path = _PARAM) -> int:
    """The amdgpu ``hws_max_conc_proc`` module parameter (readable without
    privileges); values <= 0 (driver default) and unreadable files mean 8."""
    try:
        v = int(param.read_text().strip())
    except (OSError, ValueError):
        return DEFAULT_MAX_CONCURRENT_PROCESSES
    return v if v > 0 else DEFAULT_MAX_CONCURRENT_PROCESSES


def max_concurrent_processes(smi) -> int:
    """Per logical GPU: the backend's own value (fake backends) or the driver's."""
    v = getattr(smi, "max_concurrent_processes", None)
    if callable(v):
        v = v()
    return int(v) if v else hws_max_concurrent_processes()
