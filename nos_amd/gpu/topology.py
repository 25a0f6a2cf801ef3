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
