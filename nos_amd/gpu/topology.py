"""MI355X compute topology: XCDs, CU numbering, XCD-symmetric CU-mask slices.

Measured on MI355X (profiles/r01_explore_first_contact.json, probe_placement):

* a queue's CU-mask bit ``i`` is logical CU ``i`` and lives on XCD ``i % 8``
  (bits 0-7 -> one CU on each of the 8 XCDs; bits 0-31 -> 4 CUs per XCD);
* workgroups are dealt round-robin over the 8 XCDs regardless of the mask --
  a mask only restricts which CUs *inside* each XCD may run them;
* a mask that leaves an XCD with no CU leaves that XCD UNRESTRICTED (bit 0
  alone ran on 225 CUs: 1 on XCD 0 + 32 on each other XCD).

So in SPX mode a CU-mask slice must be XCD-symmetric: ``n`` CUs on every XCD
(``8n`` CUs), ``1 <= n <= 32``.  XCD isolation (private L2 per tenant) is what
compute partitions (CPX) are for.
"""
from __future__ import annotations

from dataclasses import dataclass

MI355X_XCDS = 8
MI355X_CUS_PER_XCD = 32
MI355X_CUS = MI355X_XCDS * MI355X_CUS_PER_XCD
MI355X_MEMORY_GB = 288


def xcd_of(cu: int, num_xcds: int = MI355X_XCDS) -> int:
    return cu % num_xcds


def logical_cu(xcd: int, local: int, num_xcds: int = MI355X_XCDS) -> int:
    return local * num_xcds + xcd


@dataclass(frozen=True)
class CUSlice:
    """``per_xcd`` consecutive local CU slots starting at ``start`` on every XCD."""

    start: int
    per_xcd: int
    num_xcds: int = MI355X_XCDS

    @property
    def num_cus(self) -> int:
        return self.per_xcd * self.num_xcds

    def cus(self) -> list[int]:
        return sorted(logical_cu(x, self.start + j, self.num_xcds)
                      for x in range(self.num_xcds) for j in range(self.per_xcd))

    def overlaps(self, other: "CUSlice") -> bool:
        return not (self.start + self.per_xcd <= other.start or other.start + other.per_xcd <= self.start)


def split_even(n_slices: int, cus_per_xcd: int = MI355X_CUS_PER_XCD,
               num_xcds: int = MI355X_XCDS) -> list[CUSlice]:
    """Split a GPU into ``n_slices`` XCD-symmetric slices; leftover CU slots go
    to the first slices (every CU is owned by exactly one slice)."""
    if not 1 <= n_slices <= cus_per_xcd:
        raise ValueError(f"1 <= slices <= {cus_per_xcd} required for XCD-symmetric masks")
    base, extra = divmod(cus_per_xcd, n_slices)
    out, s = [], 0
    for i in range(n_slices):
        k = base + (1 if i < extra else 0)
        out.append(CUSlice(s, k, num_xcds))
        s += k
    return out


def pack_slices(sizes_per_xcd: list[int], cus_per_xcd: int = MI355X_CUS_PER_XCD,
                num_xcds: int = MI355X_XCDS) -> list[CUSlice]:
    """First-fit placement of slices given in CUs-per-XCD; raises if they do not fit."""
    if sum(sizes_per_xcd) > cus_per_xcd:
        raise ValueError("slices exceed the GPU's CUs")
    out, s = [], 0
    for k in sizes_per_xcd:
        if k < 1:
            raise ValueError("a slice needs at least one CU per XCD")
        out.append(CUSlice(s, k, num_xcds))
        s += k
    return out


@dataclass(frozen=True)
class CUSlotSet:
    """An arbitrary set of local CU slots, the same on every XCD (XCD-symmetric,
    not necessarily contiguous: slices keep their slots while neighbours come
    and go, so free slots fragment)."""

    slots: frozenset
    num_xcds: int = MI355X_XCDS

    @property
    def per_xcd(self) -> int:
        return len(self.slots)

    @property
    def num_cus(self) -> int:
        return self.per_xcd * self.num_xcds

    def cus(self) -> list[int]:
        return sorted(logical_cu(x, j, self.num_xcds) for x in range(self.num_xcds) for j in self.slots)

    def overlaps(self, other: "CUSlotSet") -> bool:
        return bool(self.slots & other.slots)


SLOT_POLICIES = ("shared", "proportional", "even")


def slot_wants(replicas: list[tuple[str, int]], policy: str, gpu_memory_gb: int,
               cus_per_xcd: int = MI355X_CUS_PER_XCD) -> dict[str, int]:
    """CU slots per XCD each replica is entitled to.

    * ``proportional``: its memory share of the GPU (a 36 GB slice of a 288 GB
      MI355X gets 4 of 32 slots per XCD), at least 1 -- stable as slices come
      and go, so the default for exclusive slices;
    * ``even``: an equal split among the replicas that exist now (leftover
      slots to the first ones) -- for static slice tables;
    * ``shared``: every slot (no mask, the MPS-like behaviour)."""
    if policy == "shared":
        return {rid: cus_per_xcd for rid, _ in replicas}
    if policy == "proportional":
        return {rid: max(1, cus_per_xcd * mem // max(1, gpu_memory_gb)) for rid, mem in replicas}
    if policy == "even":
        if not replicas:
            return {}
        base, extra = divmod(cus_per_xcd, len(replicas))
        return {rid: max(1, base + (1 if i < extra else 0)) for i, (rid, _) in enumerate(sorted(replicas))}
    raise ValueError(f"unknown CU slot policy {policy!r} (one of {SLOT_POLICIES})")


def layout_split(replicas: list[tuple[str, int]], keep: dict[str, frozenset], isolated_gb: set[int],
                 reserved: int, gpu_memory_gb: int, cus_per_xcd: int = MI355X_CUS_PER_XCD
                 ) -> tuple[dict[str, frozenset], set[str]]:
    """The ``split`` policy: the top ``reserved`` slots of every XCD form an
    isolated pool in which each replica of an isolated profile (memory GB in
    ``isolated_gb``) gets its proportional share, disjoint from every other
    mask; all other replicas share the remaining slots (one mask, the MPS-like
    pool), so the isolated tenants' CUs never run a shared tenant's waves.
    Allocated replicas keep their slots; an isolated replica the pool cannot
    hold is unhealthy."""
    shared = frozenset(range(cus_per_xcd - reserved))
    pool = list(range(cus_per_xcd - reserved, cus_per_xcd))
    out: dict[str, frozenset] = {}
    iso = [(rid, mem) for rid, mem in replicas if mem in isolated_gb]
    for rid, mem in replicas:
        if mem not in isolated_gb:
            out[rid] = keep.get(rid, shared)
        elif rid in keep:
            out[rid] = frozenset(keep[rid])
    taken = {s for rid, _ in iso if rid in out for s in out[rid]}
    free = [s for s in pool if s not in taken]
    wants = slot_wants(iso, "proportional", gpu_memory_gb, cus_per_xcd)
    bad: set[str] = set()
    for rid, _ in sorted(iso):
        if rid in out:
            continue
        w = wants[rid]
        if w > len(free):
            bad.add(rid)
            continue
        out[rid] = frozenset(free[:w])
        free = free[w:]
    return out, bad


def layout_slots(replicas: list[tuple[str, int]], keep: dict[str, frozenset], policy: str, gpu_memory_gb: int,
                 cus_per_xcd: int = MI355X_CUS_PER_XCD) -> tuple[dict[str, frozenset], set[str]]:
    """Lay out the CU slots of one GPU's slice replicas.

    ``replicas``: (id, memory GB) of every replica, ``keep``: the slots of
    replicas that are allocated to running pods (they never move).  Every other
    replica gets exactly its :func:`slot_wants` share out of the slots no kept
    replica holds (lowest free slots first, in replica-id order); a replica for
    which not enough free slots remain is returned as *unhealthy* instead of
    being given a smaller or overlapping mask.  Returns (slots per replica id,
    unhealthy ids)."""
    full = frozenset(range(cus_per_xcd))
    if policy == "shared":
        return {rid: full for rid, _ in replicas}, set()
    wants = slot_wants(replicas, policy, gpu_memory_gb, cus_per_xcd)
    out: dict[str, frozenset] = {}
    taken: set[int] = set()
    for rid, _ in replicas:
        if rid in keep:
            out[rid] = frozenset(keep[rid])
            taken |= keep[rid]
    free = [s for s in range(cus_per_xcd) if s not in taken]
    bad: set[str] = set()
    for rid, _ in sorted(replicas):
        if rid in out:
            continue
        w = wants[rid]
        if w > len(free):
            bad.add(rid)
            continue
        out[rid] = frozenset(free[:w])
        free = free[w:]
    return out, bad
