"""CU-slot layout of the device plugin's slice replicas under fragmentation
(nos_amd/gpu/topology.py:layout_slots, deviceplugin/plugin.py)."""
from __future__ import annotations

from collections import Counter

import yaml
from hypothesis import given, settings
from hypothesis import strategies as st

from nos_amd.api import constants as C
from nos_amd.deviceplugin.plugin import NosAmdDevicePlugin
from nos_amd.gpu.fakesmi import FakeSmi
from nos_amd.gpu.topology import layout_slots, slot_wants, xcd_of


def _cfg(slices: list[tuple[int, int]], policy: str) -> str:
    return yaml.safe_dump({"cuPolicy": policy, "gpus": [
        {"index": 0, "slices": [{"profile": f"{gb}gb", "memoryGB": gb, "replicas": n} for gb, n in slices]}]})


def _plugin(policy: str) -> NosAmdDevicePlugin:
    return NosAmdDevicePlugin("n", FakeSmi(gpus=1, node="n"), mode=C.PARTITIONING_CUMASK, cu_policy=policy)


def test_fragmented_free_slots_are_used_as_sets():
    """The round-1 failure: 10gb::0 and ::2 allocated, a 20 GB slice added -> a
    replica was silently cut to 1 CU/XCD.  Now every replica gets its full share."""
    p = _plugin("even")
    p.set_config("a", _cfg([(10, 4)], "even"))
    ids = sorted(d.id for d in p.list_devices("amd.com/gpu-10gb"))
    for i in (0, 2):
        p.allocate("amd.com/gpu-10gb", [ids[i]], owner=f"pod{i}")
    held = {i: set(p.cus_of(ids[i])) for i in (0, 2)}
    p.set_config("b", _cfg([(10, 4), (20, 1)], "even"))
    assert {i: set(p.cus_of(ids[i])) for i in (0, 2)} == held  # allocated replicas never move
    healthy = [d for d in p.devices.values() if d.healthy]
    sizes = {d.id: len(p.cus_of(d.id)) // 8 for d in healthy}
    # 32 slots: 0 and 2 keep 8 each; the 16 free slots (two non-contiguous runs) hold 2 more even shares
    # (32 / 5 -> 7 or 6); the replica that does not fit is unhealthy, not squeezed onto 1 CU/XCD
    assert all(v >= 6 for v in sizes.values()), sizes
    assert sum(1 for d in p.devices.values() if not d.healthy) == 1
    seen: set[int] = set()
    for did in sizes:
        cus = set(p.cus_of(did))
        assert not (seen & cus)
        seen |= cus


def test_proportional_sizes_by_memory():
    p = _plugin("proportional")
    p.set_config("a", _cfg([(36, 2), (72, 1), (144, 1)], "proportional"))
    per = {d.id.split("::")[1]: len(p.cus_of(d.id)) // 8 for d in p.devices.values()}
    assert per == {"36gb": 4, "72gb": 8, "144gb": 16}
    assert all(d.healthy for d in p.devices.values())
    assert len(set().union(*(set(p.cus_of(d)) for d in p.devices))) == 256


def test_shared_policy_has_no_mask():
    p = _plugin("shared")
    p.set_config("a", _cfg([(36, 8)], "shared"))
    d = sorted(p.devices)[0]
    alloc = p.allocate("amd.com/gpu-36gb", [d], owner="x")
    assert C.ENV_CU_MASK not in alloc.envs and alloc.envs[C.ENV_MEMORY_LIMIT_GB] == "36"


ops = st.lists(st.one_of(
    st.tuples(st.just("config"), st.lists(st.tuples(st.sampled_from([9, 10, 20, 36, 72]), st.integers(0, 6)),
                                          min_size=0, max_size=3)),
    st.tuples(st.just("alloc"), st.integers(0, 50)),
    st.tuples(st.just("release"), st.integers(0, 50)),
), min_size=1, max_size=25)


@settings(max_examples=120, deadline=None)
@given(policy=st.sampled_from(["even", "proportional"]), seq=ops)
def test_random_allocate_release_reconfigure(policy, seq):
    p = _plugin(policy)
    held: dict[str, frozenset] = {}
    for op, arg in seq:
        if op == "config":
            slices: dict[int, int] = {}
            for gb, n in arg:  # merge duplicates, keep the table within the GPU's memory
                slices[gb] = slices.get(gb, 0) + n
            while sum(gb * n for gb, n in slices.items()) > 288:
                gb = max(g for g, n in slices.items() if n)
                slices[gb] -= 1
            p.set_config(f"c{len(seq)}", _cfg(sorted(slices.items()), policy))
        elif op == "alloc":
            free = sorted(d.id for d in p.devices.values() if d.healthy and d.id not in p.allocated)
            if free:
                did = free[arg % len(free)]
                res = p.devices[did].resource
                alloc = p.allocate(res, [did], owner=did)
                cus = set(p.cus_of(did))
                held[did] = frozenset(cus)
                assert alloc.envs.get(C.ENV_CU_MASK) or len(cus) == 256
        else:
            if p.allocated:
                did = sorted(p.allocated)[arg % len(p.allocated)]
                p.release([did])
                held.pop(did, None)
        # allocated replicas never move
        for did, cus in held.items():
            assert frozenset(p.cus_of(did)) == cus
        # exclusive policies: masks of healthy/allocated replicas are disjoint and XCD-symmetric
        seen: set[int] = set()
        for did, d in p.devices.items():
            if not (d.healthy or did in p.allocated):
                continue
            cus = set(p.cus_of(did))
            assert cus, did
            counts = Counter(xcd_of(c) for c in cus)
            assert len(counts) == 8 and len(set(counts.values())) == 1
            assert not (seen & cus), did
            seen |= cus
        # every healthy unallocated replica holds exactly its policy share
        reps = [(did, d.memory_gb) for did, d in sorted(p.devices.items())]
        want = slot_wants(reps, policy, 288)
        for did, d in p.devices.items():
            if d.healthy and did not in p.allocated and did not in held:
                assert len(p.cus_of(did)) // 8 == want[did], (did, policy)


def test_layout_slots_unit():
    got, bad = layout_slots([("a", 36), ("b", 36), ("c", 36)], {"b": frozenset({0, 1, 2, 3})}, "proportional", 288)
    assert got["b"] == frozenset({0, 1, 2, 3}) and got["a"] == frozenset({4, 5, 6, 7})
    assert got["c"] == frozenset({8, 9, 10, 11}) and not bad
    got, bad = layout_slots([("a", 10), ("b", 10)], {"a": frozenset(range(32))}, "even", 288)
    assert bad == {"b"} and "b" not in got
