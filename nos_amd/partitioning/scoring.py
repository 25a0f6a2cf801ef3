"""Measured-throughput and xGMI-topology scoring for placement decisions.

The reference places slices by first fit and walks candidate nodes in name
order (``internal/partitioning/core/snapshot.go:93-103``,
``pkg/gpu/slicing/gpu.go:162-220``): every GPU is assumed to deliver the same
throughput.  On a shared MI355X that is not true -- a GPU can be held down by
DVFS, by a co-resident tenant or by a degraded device -- so the north star
(BASELINE.json) asks that the partitioner "sees real per-slice throughput".

The CU-mask gpuagent publishes what its gfx950 probe kernels measured on each
slice (``nos.nebuly.com/probe-gpu-<i>-<profile>-tflops``, see
:mod:`nos_amd.agents.gpuagent`).  This module turns those annotations into:

* a per-GPU **capacity** (measured TFLOP/s of the whole GPU = Σ over its slices
  of the slice's measured TFLOP/s; slices of an even split partition the CUs);
* the **expected share** a new pod would get on that GPU,
  ``capacity / (slices + 1)`` -- shared-policy pods co-run on the GPU's CUs,
  even-policy pods get ``1/n`` of them, and both divide the measured capacity;
* a **node score** (the best expected share on any GPU that still has room),
  used to order the planner's candidate nodes and, with ``placement:
  measured``, to choose the GPU that receives new slices;
* an **xGMI-aware** device choice for multi-device requests
  (:func:`choose_devices_xgmi`): one device per GPU first, GPUs whose xGMI
  links carry the fewest multi-device tenants next (a ring all-reduce is
  bounded per link, SURVEY.md 5.8 / 7.4 hard part 6), lowest amd-smi link
  weight to the GPUs already chosen last.

GPUs without probe data fall back to the mean measured capacity of the node
(or a nominal 1.0 when nothing is measured), which reproduces the
reference's behaviour exactly when no probe runs.
"""
from __future__ import annotations

import re
from typing import Callable, Iterable

from ..api import constants as C

_PROBE_RE = re.compile(re.escape(C.ANNOTATION_PROBE_PREFIX) +
                       r"-(\d+)-([^-]+)-(tflops|gbps|gemmtflops|sclkmhz|loadedgbps|loadedgemmtflops)$")


def _rate(p: dict[str, float]) -> float:
    """A slice's measured compute rate: the realistic GEMM probe when published,
    else the MFMA peak (older agents)."""
    return p.get("gemmtflops", p.get("tflops", 0.0))


def probe_table(annotations: dict[str, str]) -> dict[int, dict[str, dict[str, float]]]:
    """``{gpu index: {profile: {"tflops": x, "gbps": y}}}`` from node annotations."""
    out: dict[int, dict[str, dict[str, float]]] = {}
    for k, v in (annotations or {}).items():
        m = _PROBE_RE.match(k)
        if not m:
            continue
        try:
            val = float(v)
        except (TypeError, ValueError):
            continue
        out.setdefault(int(m.group(1)), {}).setdefault(m.group(2), {})[m.group(3)] = val
    return out


def gpu_capacities(table: dict[int, dict[str, dict[str, float]]],
                   slice_counts: dict[int, dict[str, int]]) -> dict[int, float]:
    """Measured whole-GPU TFLOP/s per GPU: Σ_profile tflops(profile) × slices of it.

    A GPU whose slices were probed but whose current slice table is empty
    (e.g. right after the slices were drained) keeps the best per-slice number
    scaled by how many such slices it held when probed: we only know the
    per-slice rate, so take the maximum over profiles as a lower bound.
    """
    caps: dict[int, float] = {}
    for gi, profs in table.items():
        counts = slice_counts.get(gi, {})
        tot = sum(_rate(p) * counts.get(name, 0) for name, p in profs.items())
        if tot <= 0:
            tot = max((_rate(p) for p in profs.values()), default=0.0)
        if tot > 0:
            caps[gi] = tot
    return caps


def fill_unmeasured(caps: dict[int, float], gpu_indices: Iterable[int]) -> dict[int, float]:
    """Every GPU gets a capacity: its measured one, else the node mean, else 1.0."""
    idx = list(gpu_indices)
    default = (sum(caps.values()) / len(caps)) if caps else 1.0
    return {i: caps.get(i, default) for i in idx}


def expected_share(capacity: float, slices: int) -> float:
    return capacity / (slices + 1)


def node_score(caps: dict[int, float], slices: dict[int, int], has_room: Callable[[int], bool]) -> float | None:
    """Best expected per-pod share over the GPUs that can take another slice;
    ``None`` when nothing on the node is measured (name order then decides)."""
    best = None
    for gi, cap in caps.items():
        if not has_room(gi):
            continue
        s = expected_share(cap, slices.get(gi, 0))
        best = s if best is None or s > best else best
    return best


def choose_devices_xgmi(candidates: list[str], size: int, must_include: list[str],
                        gpu_of: Callable[[str], int], link_weight: Callable[[int, int], float],
                        collective_load: dict[int, int], load: dict[int, int]) -> list[str]:
    """Pick ``size`` devices for one container that spans several devices.

    Order of preference for each next device:
    1. a GPU not used by this container yet (every rank its own HBM stack and
       its own xGMI links),
    2. fewest multi-device tenants already on that GPU (they share its links),
    3. lowest Σ link weight (amd-smi ``topo_get_link_weight``; lower = closer)
       to the GPUs chosen so far,
    4. fewest devices allocated on that GPU, then the GPU index, then the id.
    """
    out = list(must_include)[:size]
    chosen_gpus = [gpu_of(d) for d in out]
    cand = [d for d in candidates if d not in out]
    while len(out) < size and cand:
        def key(d: str):
            g = gpu_of(d)
            return (g in chosen_gpus, collective_load.get(g, 0),
                    sum(link_weight(g, c) for c in chosen_gpus if c != g), load.get(g, 0), g, d)

        best = min(cand, key=key)
        out.append(best)
        cand.remove(best)
        chosen_gpus.append(gpu_of(best))
    return out


__all__ = ["probe_table", "gpu_capacities", "fill_unmeasured", "expected_share", "node_score",
           "choose_devices_xgmi"]
