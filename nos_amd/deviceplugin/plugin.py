"""nos-amd device plugin: the devices the kubelet hands to pods.

Replaces the NVIDIA device plugin + MPS daemon the reference depends on
(SURVEY.md 2.8).  It advertises three kinds of extended resources:

* ``amd.com/gpu`` -- whole GPUs (nodes without a partitioning label, or
  ``exposePartitionsAsGpu`` in static CPX mode: every logical partition is an
  ``amd.com/gpu``, BASELINE config 2);
* ``amd.com/partition-<n>xcd.<gb>gb`` -- the logical GPUs of the current
  compute/memory partition mode (amdpart nodes), read from amd-smi;
* ``amd.com/gpu-<gb>gb`` -- CU-mask slices (cumask nodes), replicas of each
  GPU as listed by the gpupartitioner's plugin ConfigMap entry; on hybrid
  nodes the same memory slices placed on the GPU's logical partitions (first
  fit decreasing over partition memory and HWS process slots, allocated
  replicas never move; no CU mask inside a partition).

``allocate`` returns what a real ``ContainerAllocateResponse`` carries:
``HIP_VISIBLE_DEVICES`` (``device_env="container"``, the DaemonSet default:
0..k-1 over the allocated render nodes in host order, because the container
runtime mounts only those nodes and HIP numbers what it sees from 0;
``"host"``: host HIP ids, for tenants that see every GPU -- simulator, bare
metal), ``ROC_GLOBAL_CU_MASK``
for slices (XCD-symmetric, see :mod:`nos_amd.gpu.topology`),
``NOS_AMD_MEMORY_LIMIT_GB`` (cooperative memory cap; AMD has no MPS-style hard
limit, SURVEY.md 7.4 hard part 3) and the ``/dev/kfd`` + ``/dev/dri/renderD*``
device nodes.  CU masks of allocated replicas never move: when the slice
table changes, new replicas are laid out in the CU slots left free.

The slice table is re-read on change (no plugin restart, unlike the
reference's NVIDIA plugin).  Partition modes are a different matter: an
amd-smi session only sees the devices it enumerated, so a mode switched by
the partition agent (another process) becomes visible when :meth:`rescan`
re-enumerates (``nos_smi_rescan``); the plugin binary calls it every poll,
and it follows the node's partitioning label (:meth:`set_mode`).  The agent
still restarts the plugin pod after a switch (``agents/dpclient.py``), the
reference-compatible path.  :mod:`nos_amd.deviceplugin.grpc_server` exposes
this object over the kubelet device-plugin v1beta1 gRPC API.
"""
from __future__ import annotations

import logging
import threading
from dataclasses import dataclass, field

import yaml

from ..api import constants as C
from ..gpu.amdpart import partition_profile
from ..gpu.amdsmi import AmdSmi, GpuInfo
from ..gpu.kfd import max_concurrent_processes
from ..gpu.topology import MI355X_CUS_PER_XCD, MI355X_MEMORY_GB, MI355X_XCDS, CUSlotSet, layout_slots, layout_split, logical_cu
from ..ops.streams import mask_hex
from ..partitioning import scoring

log = logging.getLogger("nos_amd.deviceplugin")


@dataclass
class Device:
    id: str
    resource: str
    gpu_index: int
    healthy: bool = True
    partition: int = 0          # logical partition index (amdpart)
    profile: str = ""           # partition / slice profile
    memory_gb: int = 0
    hip_id: int = -1            # logical device's HIP ordinal (amdpart; -1: the GPU's)
    drm_render: int = -1


@dataclass
class ContainerAllocation:
    envs: dict[str, str] = field(default_factory=dict)
    devices: list[str] = field(default_factory=list)
    device_ids: list[str] = field(default_factory=list)
    # host directories mounted at the same path, always READ-ONLY: the pod-server
    # socket directory -- connect() on a unix socket needs no write access to the
    # mount, and a writable one would let a tenant unlink server.sock (cutting off
    # every co-tenant) or bind a listener there that collects other pods' tokens
    mounts: list[str] = field(default_factory=list)


class NosAmdDevicePlugin:
    def __init__(self, node_name: str, smi: AmdSmi, mode: str | None = None, expose_partitions_as_gpu: bool = False,
                 cu_policy: str = "proportional", device_env: str = "host", pod_server_dir: str = "",
                 adopt_records: bool = False):
        """``adopt_records``: the node's only plugin process (the deployed
        binary) adopts the pod-server allocation records a previous process
        wrote and deletes orphans (:meth:`_restore_records`); simulations that
        run several plugins over one records directory leave them alone."""
        if device_env not in ("host", "container"):
            raise ValueError(f"device_env must be 'host' or 'container', not {device_env!r}")
        self.node_name = node_name
        # cumask slices served by the node's pod server (nos_amd/podserver): the
        # pod gets the socket of its GPU's server, never a device node
        self.pod_server_dir = pod_server_dir
        self.pod_server_allocations = None
        if pod_server_dir:
            from ..podserver.allocations import AllocationStore

            self.pod_server_allocations = AllocationStore(pod_server_dir)
        # records a previous plugin process wrote: device id -> (owner, CU slots),
        # adopted at the first refresh that has the slice table (_restore_records)
        self._restored: dict[str, tuple[str, frozenset]] = {}
        if self.pod_server_allocations is not None and adopt_records:
            for _path, rec in self.pod_server_allocations.load():
                slots = rec.get("cu_slots") or {}
                for did in rec.get("device_ids", []):
                    self._restored[did] = (str(rec.get("owner") or "restored"), frozenset(slots.get(did, ())))
        # "container": the runtime mounts only the allocated render nodes, so
        # HIP inside the container numbers them 0..k-1 in host order;
        # "host": tenants run on the host and see every GPU (simulator, bare metal)
        self.device_env = device_env
        self.smi = smi
        self.mode = mode              # None | "partition" | "cumask"
        self.expose_partitions_as_gpu = expose_partitions_as_gpu
        self.cu_policy = cu_policy
        self._lock = threading.RLock()
        self.config: dict | None = None
        self.config_key: str | None = None
        self.devices: dict[str, Device] = {}
        self.allocated: dict[str, str] = {}      # device id -> owner (pod uid / container)
        self.cu_slots: dict[str, CUSlotSet] = {}   # slice device id -> CU slots
        self.listeners: list = []
        self.generation = 0
        self._links: dict[tuple[int, int], float] = {}
        self.refresh()

    # ------------------------------------------------------------ inventory
    def _gpus(self) -> list[GpuInfo]:
        return self.smi.gpus()

    def rescan(self) -> None:
        """Re-enumerate amd-smi (modes another process switched become visible),
        then recompute the devices.  A GPU whose switch is in flight keeps its
        current devices until the next poll."""
        rs = getattr(self.smi, "rescan", None)
        if rs is not None:
            try:
                rs()
            except Exception as e:  # e.g. a switch of this session in flight: retry next poll
                log.info("amd-smi rescan deferred: %s", e)
        self.refresh()

    def set_mode(self, mode: str | None) -> bool:
        """Follow the node's ``nos.nebuly.com/gpu-partitioning`` label (read
        once at start-up before).  Returns True when the mode changed."""
        with self._lock:
            if mode == self.mode:
                return False
            log.info("node %s: partitioning mode %s -> %s", self.node_name, self.mode, mode)
            self.mode = mode
            if mode not in SLICE_MODES:
                self.config, self.config_key = None, None
        self.refresh()
        return True

    def set_config(self, key: str | None, cfg_yaml: str | dict | None) -> None:
        with self._lock:
            self.config_key = key
            self.config = yaml.safe_load(cfg_yaml) if isinstance(cfg_yaml, str) else cfg_yaml
            if self.config and self.config.get("cuPolicy"):
                self.cu_policy = self.config["cuPolicy"]
        self.refresh()

    def refresh(self) -> None:
        """Recompute the advertised devices (after a mode switch or config change)."""
        with self._lock:
            devs: dict[str, Device] = {}
            gpus = self._gpus()
            if self.mode == C.PARTITIONING_CUMASK:
                table = {g["index"]: g for g in (self.config or {}).get("gpus", [])}
                for gi in gpus:
                    for s in table.get(gi.index, {}).get("slices", []):
                        prof = s["profile"]
                        for r in range(int(s.get("replicas", 0))):
                            did = f"{gi.uuid}::{prof}::{r}"
                            devs[did] = Device(did, C.AMD_SLICE_RESOURCE_PREFIX + prof, gi.index, profile=prof,
                                               memory_gb=int(s.get("memoryGB", prof[:-2])))
            elif self.mode == C.PARTITIONING_HYBRID:
                self._hybrid_devices(gpus, devs)
            elif self.mode == C.PARTITIONING_AMDPART:
                # one device per logical partition amd-smi enumerates for the GPU, named
                # from the GPU's reported memory / XCDs (same function as the planner)
                for gi in gpus:
                    if getattr(gi, "switching", False):  # cannot be enumerated now: keep what it had
                        devs.update({k: d for k, d in self.devices.items() if d.gpu_index == gi.index})
                        continue
                    parts = self.smi.partitions(gi.index)
                    prof = str(partition_profile(gi.memory_gb, gi.num_xcds or MI355X_XCDS, len(parts)))
                    res = C.RESOURCE_AMD_GPU if self.expose_partitions_as_gpu else C.AMD_PARTITION_RESOURCE_PREFIX + prof
                    for pi in parts:
                        did = f"{gi.uuid}::p{pi.partition}"
                        devs[did] = Device(did, res, gi.index, partition=pi.partition, profile=prof,
                                           memory_gb=pi.memory_gb, hip_id=pi.hip_id, drm_render=pi.drm_render)
            else:
                for gi in gpus:
                    devs[gi.uuid] = Device(gi.uuid, C.RESOURCE_AMD_GPU, gi.index, profile="", memory_gb=gi.memory_gb)
            # devices that disappeared but are still allocated stay (unhealthy) until released
            for did, owner in self.allocated.items():
                if did not in devs and did in self.devices:
                    d = self.devices[did]
                    devs[did] = Device(d.id, d.resource, d.gpu_index, False, d.partition, d.profile, d.memory_gb,
                                       d.hip_id, d.drm_render)
            before = {k: (d.resource, d.healthy) for k, d in self.devices.items()}
            self.devices = devs
            self._restore_records()
            self._layout_cu_slots()
            changed = {k: (d.resource, d.healthy) for k, d in self.devices.items()} != before or self.generation == 0
            if not changed:
                return
            self.generation += 1
        for cb in list(self.listeners):
            try:
                cb(self)
            except Exception:
                log.exception("device plugin listener failed")

    def _hybrid_devices(self, gpus: list[GpuInfo], devs: dict[str, "Device"]) -> None:
        """Slice replicas of the table placed on each GPU's CURRENT logical
        partitions: allocated replicas keep their partition, the others go
        first-fit (largest first) where partition memory and the HWS process
        slots allow; what does not fit (e.g. the table is laid out for CPX
        while the agent has not switched the GPU yet) is advertised unhealthy
        until a refresh after the switch."""
        table = {g["index"]: g for g in (self.config or {}).get("gpus", [])}
        per_part = max_concurrent_processes(self.smi)
        for gi in gpus:
            if getattr(gi, "switching", False):  # cannot be enumerated now: keep what it had
                devs.update({k: d for k, d in self.devices.items() if d.gpu_index == gi.index})
                continue
            parts = self.smi.partitions(gi.index)
            if not parts:
                continue
            entry = table.get(gi.index, {})
            reps = [(f"{gi.uuid}::{s['profile']}::{r}", s["profile"], int(s.get("memoryGB", s["profile"][:-2])))
                    for s in entry.get("slices", []) for r in range(int(s.get("replicas", 0)))]
            # the table is laid out for entry["mode"]: until the partition agent has
            # switched the GPU, only already-allocated replicas stay advertised --
            # a pod bound to a slice of the OLD mode would block the switch forever
            ready = entry.get("mode") in (None, "", f"{gi.compute_mode}/{gi.memory_mode}")
            room = {p.partition: [p.memory_gb, per_part] for p in parts}
            where: dict[str, int] = {}
            for did, _, mem in reps:  # allocated replicas never move
                old = self.devices.get(did)
                if did in self.allocated and old is not None and old.partition in room:
                    where[did] = old.partition
                    room[old.partition][0] -= mem
                    room[old.partition][1] -= 1
            for did, _, mem in sorted(reps, key=lambda x: (-x[2], x[0])):
                if did in where or not ready:
                    continue
                for p in parts:
                    left = room[p.partition]
                    if left[1] >= 1 and left[0] >= mem:
                        where[did] = p.partition
                        left[0] -= mem
                        left[1] -= 1
                        break
            by_part = {p.partition: p for p in parts}
            for did, prof, mem in reps:
                pi = by_part.get(where.get(did, -1))
                devs[did] = Device(did, C.AMD_SLICE_RESOURCE_PREFIX + prof, gi.index, healthy=pi is not None,
                                   partition=pi.partition if pi else -1, profile=prof, memory_gb=mem,
                                   hip_id=pi.hip_id if pi else -1, drm_render=pi.drm_render if pi else -1)

    def _restore_records(self) -> None:
        """After a plugin restart: adopt the pod-server allocations whose
        records survived -- their devices stay allocated to the same owner and
        keep their CU slots, so new replicas are laid out around live tenants'
        masks -- and delete orphan records (devices the current slice table no
        longer has).  Waits until the slice table is loaded (the devices of a
        cumask node are unknown before).  A later PodResources sync
        (:meth:`sync_allocated`) releases the adopted devices no pod holds,
        which deletes their records and evicts their tenants."""
        if not self._restored or self.mode != C.PARTITIONING_CUMASK or self.config is None:
            return
        info = {g.index: g for g in self._gpus()}
        orphans = []
        for did, (owner, slots) in self._restored.items():
            d = self.devices.get(did)
            if d is None:
                orphans.append(did)
                continue
            self.allocated.setdefault(did, owner)
            if slots and did not in self.cu_slots:
                self.cu_slots[did] = CUSlotSet(slots, _cu_geometry(info.get(d.gpu_index))[0])
        self._restored.clear()
        if orphans:
            n = self.pod_server_allocations.remove_devices(orphans)
            log.warning("deleted %d orphan pod-server allocation record(s): devices %s are gone", n, orphans)

    def _layout_cu_slots(self) -> None:
        """XCD-symmetric CU slots for every slice replica (:func:`layout_slots`):
        allocated replicas keep theirs, the others get exactly their policy
        share of the free slots, and a replica that cannot get it is advertised
        unhealthy (never a smaller or overlapping mask)."""
        slots: dict[str, CUSlotSet] = {}
        if self.mode != C.PARTITIONING_CUMASK:  # hybrid slices share their partition's CUs
            self.cu_slots = slots
            return
        by_gpu: dict[int, list[Device]] = {}
        for d in self.devices.values():
            if d.resource.startswith(C.AMD_SLICE_RESOURCE_PREFIX):
                by_gpu.setdefault(d.gpu_index, []).append(d)
        info = {g.index: g for g in self._gpus()}
        for gi, devs in by_gpu.items():
            g = info.get(gi)
            xcds, per_xcd = _cu_geometry(g)
            keep = {d.id: self.cu_slots[d.id].slots for d in devs if d.id in self.allocated and d.id in self.cu_slots}
            live = [d for d in devs if d.healthy or d.id in keep]
            cfg = self.config or {}
            if self.cu_policy == "split":   # an isolated pool for some profiles, a shared pool for the rest
                iso = {int(str(p).rstrip("gb")) for p in cfg.get("isolatedProfiles", []) if str(p).rstrip("gb").isdigit()}
                got, bad = layout_split([(d.id, d.memory_gb) for d in live], keep, iso,
                                        int(cfg.get("isolatedCuSlots", 0)) * per_xcd // 32,
                                        g.memory_gb if g else MI355X_MEMORY_GB, per_xcd)
            else:
                got, bad = layout_slots([(d.id, d.memory_gb) for d in live], keep, self.cu_policy,
                                        g.memory_gb if g else MI355X_MEMORY_GB, per_xcd)
            for did, sl in got.items():
                slots[did] = CUSlotSet(sl, xcds)
            for did in bad:
                d = self.devices[did]
                self.devices[did] = Device(d.id, d.resource, d.gpu_index, False, d.partition, d.profile, d.memory_gb,
                                           d.hip_id, d.drm_render)
                log.warning("slice %s gets no CU slots (%s policy, %d allocated replicas hold the rest): unhealthy",
                            did, self.cu_policy, len(keep))
        self.cu_slots = slots

    # ------------------------------------------------------------ device-plugin API
    def resources(self) -> dict[str, list[Device]]:
        with self._lock:
            out: dict[str, list[Device]] = {}
            for d in self.devices.values():
                out.setdefault(d.resource, []).append(d)
            return out

    def list_devices(self, resource: str) -> list[Device]:
        return self.resources().get(resource, [])

    def preferred_allocation(self, resource: str, available: list[str], must_include: list[str], size: int) -> list[str]:
        """``GetPreferredAllocation`` (config ``allocation``):

        * "pack" fills GPUs in index order; "spread" picks the GPU with the
          fewest allocated devices; "measured" the GPU where the pod gets the
          largest share of the probe-measured TFLOP/s (``gpuWeights`` written
          by the partitioner, partitioning/scoring.py);
        * a request for several devices (one container spanning GPUs, e.g. an
          RCCL tenant) is placed xGMI-aware whatever the policy: one device
          per GPU first, then GPUs whose links carry the fewest multi-device
          tenants, then the lowest amd-smi link weight to the GPUs already
          chosen (``scoring.choose_devices_xgmi``).
        """
        with self._lock:
            out = list(must_include)[:size]
            cand = [d for d in available if d not in out and d in self.devices]
            cfg = self.config or {}
            policy = cfg.get("allocation", "pack")
            weights = {int(k): float(v) for k, v in (cfg.get("gpuWeights") or {}).items()}
            load: dict[int, int] = {}
            owners: dict[str, set[int]] = {}
            for did, owner in self.allocated.items():
                d = self.devices.get(did)
                if d is not None:
                    load[d.gpu_index] = load.get(d.gpu_index, 0) + 1
                    owners.setdefault(owner, set()).add(d.gpu_index)
            if size > 1:
                coll: dict[int, int] = {}
                for gpus in owners.values():
                    if len(gpus) > 1:
                        for g in gpus:
                            coll[g] = coll.get(g, 0) + 1
                return scoring.choose_devices_xgmi(cand + out, size, out, lambda x: self.devices[x].gpu_index,
                                                   self._link_weight, coll, load)
            default_w = (sum(weights.values()) / len(weights)) if weights else 1.0
            while len(out) < size and cand:
                if policy == "spread":
                    best = min(cand, key=lambda x: (load.get(self.devices[x].gpu_index, 0),
                                                    self.devices[x].gpu_index, x))
                elif policy == "measured":
                    best = min(cand, key=lambda x: (-weights.get(self.devices[x].gpu_index, default_w) /
                                                    (load.get(self.devices[x].gpu_index, 0) + 1),
                                                    self.devices[x].gpu_index, x))
                else:
                    best = min(cand, key=lambda x: (self.devices[x].gpu_index, x))
                out.append(best)
                cand.remove(best)
                gi = self.devices[best].gpu_index
                load[gi] = load.get(gi, 0) + 1
            return out

    def _link_weight(self, i: int, j: int) -> float:
        key = (min(i, j), max(i, j))
        w = self._links.get(key)
        if w is None:
            try:
                w = float(self.smi.link(i, j).get("weight", 0))
            except Exception:  # topology unreadable: every pair equal
                w = 0.0
            self._links[key] = w
        return w

    def allocate(self, resource: str, device_ids: list[str], owner: str = "") -> ContainerAllocation:
        if (self.pod_server_dir and self.mode == C.PARTITIONING_CUMASK
                and resource.startswith(C.AMD_SLICE_RESOURCE_PREFIX)):
            return self._allocate_pod_server(resource, device_ids, owner)
        with self._lock:
            alloc = ContainerAllocation(device_ids=list(device_ids))
            gpus = {g.index: g for g in self._gpus()}
            visible: list[tuple[int, str]] = []   # (render minor, host HIP id)
            mask_cus: set[int] = set()
            n_cus = 0
            mem = 0
            for did in device_ids:
                d = self.devices.get(did)
                if d is None or d.resource != resource:
                    raise KeyError(f"unknown device {did} for {resource}")
                if not d.healthy:
                    raise RuntimeError(f"device {did} is unhealthy")
                gi = gpus.get(d.gpu_index)
                # logical partitions carry their own HIP id (amd-smi enumeration info)
                hip = str(d.hip_id if d.hip_id >= 0 else (gi.hip_id if gi and gi.hip_id >= 0 else d.gpu_index))
                render = (d.drm_render if d.drm_render >= 0 else
                          gi.drm_render if gi and gi.drm_render >= 0 else 128 + d.gpu_index)
                if all(h != hip for _, h in visible):
                    visible.append((render, hip))
                if resource.startswith(C.AMD_SLICE_RESOURCE_PREFIX):
                    s = self.cu_slots.get(did)
                    if s is not None:
                        mask_cus.update(s.cus())
                    xcds, per_xcd = _cu_geometry(gi)
                    n_cus = max(n_cus, xcds * per_xcd)
                mem += d.memory_gb
                self.allocated[did] = owner or "unknown"
                dev = f"/dev/dri/renderD{render}"
                if dev not in alloc.devices:
                    alloc.devices.append(dev)
            alloc.devices.insert(0, "/dev/kfd")
            if self.device_env == "container":
                # the runtime mounts only the allocated render nodes; HIP numbers
                # them 0..k-1 in host (render minor) order
                alloc.envs[C.ENV_VISIBLE_DEVICES] = ",".join(str(k) for k in range(len(visible)))
            else:
                alloc.envs[C.ENV_VISIBLE_DEVICES] = ",".join(h for _, h in visible)
            if mask_cus and len(mask_cus) < n_cus:  # a full mask would only cost a dedicated HW queue
                alloc.envs[C.ENV_CU_MASK] = mask_hex(sorted(mask_cus), n_cus)
            if mem:
                alloc.envs[C.ENV_MEMORY_LIMIT_GB] = str(mem)
            return alloc

    def _allocate_pod_server(self, resource: str, device_ids: list[str], owner: str) -> ContainerAllocation:
        """A slice served by the GPU's pod server (the MPS-client analogue).

        The pod gets its GPU's server socket (only that GPU's socket
        directory is mounted), a fresh allocation token, and no ``/dev/kfd``
        or render node: it must not open the GPU (that would take an HWS
        process slot, which is what the server saves).  The slice -- memory
        and, unless the CU policy is "shared", the CU mask -- goes into an
        allocation record keyed by the token's hash that only the server
        reads (podserver/allocations.py): the server takes the slice from
        the record, never from the pod, and evicts the tenant when
        :meth:`release` deletes the record (reference: the MPS replica's
        memory fixed by the plugin, ``internal/partitioning/mps/partitioner.go:123-157``)."""
        from ..podserver.allocations import new_token, socket_dir, socket_path

        with self._lock:
            alloc = ContainerAllocation(device_ids=list(device_ids))
            gpus = {g.index: g for g in self._gpus()}
            per_gpu: dict[int, dict] = {}
            for did in device_ids:
                d = self.devices.get(did)
                if d is None or d.resource != resource:
                    raise KeyError(f"unknown device {did} for {resource}")
                if not d.healthy:
                    raise RuntimeError(f"device {did} is unhealthy")
                g = per_gpu.setdefault(d.gpu_index, {"memory_gb": 0, "cus": set(), "device_ids": [], "n_cus": 0})
                s = self.cu_slots.get(did)
                if s is not None:
                    g["cus"].update(s.cus())
                xcds, per_xcd = _cu_geometry(gpus.get(d.gpu_index))
                g["n_cus"] = xcds * per_xcd
                g["memory_gb"] += d.memory_gb
                g["device_ids"].append(did)
            token = new_token()
            socks, masks = [], []
            for gi, g in sorted(per_gpu.items()):
                mask = mask_hex(sorted(g["cus"]), g["n_cus"]) if g["cus"] and len(g["cus"]) < g["n_cus"] else None
                self.pod_server_allocations.write(gi, token, {
                    "memory_gb": g["memory_gb"], "cu_mask": mask, "device_ids": g["device_ids"],
                    "owner": owner or "unknown", "resource": resource,
                    # per-device CU slots: a restarted plugin keeps them (_restore_records)
                    "cu_slots": {did: sorted(self.cu_slots[did].slots) for did in g["device_ids"]
                                 if did in self.cu_slots}})
                socks.append(str(socket_path(self.pod_server_dir, gi)))
                alloc.mounts.append(str(socket_dir(self.pod_server_dir, gi)))
                if mask:
                    masks.append(mask)
            for did in device_ids:
                self.allocated[did] = owner or "unknown"
            mem = sum(g["memory_gb"] for g in per_gpu.values())
            alloc.envs[C.ENV_POD_SERVER] = ",".join(socks)
            alloc.envs[C.ENV_POD_TOKEN] = token
            if masks:
                alloc.envs[C.ENV_POD_CU_MASK] = ",".join(masks)
            if mem:
                alloc.envs[C.ENV_MEMORY_LIMIT_GB] = str(mem)
            return alloc

    def release(self, device_ids: list[str]) -> None:
        """Free devices; freed CU slots are laid out again at once (a replica
        that was unhealthy for lack of slots may become healthy)."""
        with self._lock:
            released = [did for did in device_ids if self.allocated.pop(did, None) is not None]
            stale = [did for did in device_ids if did in self.devices and not self.devices[did].healthy]
            for did in stale:
                self.devices.pop(did, None)
            if released and self.pod_server_allocations is not None:
                # the pod server evicts the tenants of these records
                self.pod_server_allocations.remove_devices(released)
        if released and self.mode in SLICE_MODES:
            self.refresh()

    def sync_allocated(self, used_device_ids: set[str]) -> None:
        """The device-plugin API has no Deallocate: a deployed plugin learns
        which devices are still in use from kubelet PodResources."""
        with self._lock:
            for did in list(self.allocated):
                if did not in used_device_ids:
                    self.release([did])
            for did in used_device_ids:
                self.allocated.setdefault(did, "podresources")

    def cu_slice_of(self, device_id: str) -> CUSlotSet | None:
        return self.cu_slots.get(device_id)

    def cus_of(self, device_id: str) -> list[int]:
        s = self.cu_slots.get(device_id)
        return s.cus() if s else []


SLICE_MODES = (C.PARTITIONING_CUMASK, C.PARTITIONING_HYBRID)  # modes whose slice table comes from the ConfigMap


def _cu_geometry(g: GpuInfo | None) -> tuple[int, int]:
    """(XCDs, CUs per XCD) of a GPU as amd-smi reports it (MI355X when unknown)."""
    if g is None or not g.num_xcds or not g.num_cus or g.num_cus % g.num_xcds:
        return MI355X_XCDS, MI355X_CUS_PER_XCD
    return g.num_xcds, g.num_cus // g.num_xcds


__all__ = ["NosAmdDevicePlugin", "Device", "ContainerAllocation", "logical_cu"]
