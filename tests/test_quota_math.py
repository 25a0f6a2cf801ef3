"""Elastic-quota math: golden vectors + property tests.

The table cases carry the input/expected numbers of the reference's
``pkg/scheduler/plugins/capacityscheduling/elasticquotainfo_test.go``
(TestReserveResource :30, TestUnReserveResource :95, UsedOverMaxWith :160,
GetGuaranteedOverquotas :196-385, getGuaranteedOverquotasPercentage
:387-580, getAggregatedOverquotas :582-720, usedLteWith :722-790,
AggregatedUsedOverMinWith :792-881) with ``nvidia.com/gpu`` replaced by
``amd.com/gpu``.  The hypothesis properties check the invariants those
tables only sample (percentages sum to 1, guaranteed over-quotas never
exceed the aggregate, reserve/unreserve are inverse, ...).
"""
from __future__ import annotations

import math

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from nos_amd.api.constants import RESOURCE_AMD_GPU as GPU, RESOURCE_GPU_MEMORY as GPU_MEM
from nos_amd.resource.resource import Resource
from nos_amd.scheduler.plugins.elasticquotainfo import ElasticQuotaInfo, ElasticQuotaInfos

NEW = "nebuly.com/new-resource"
MAXI64 = 2**63 - 1


def R(cpu=0, mem=0, eph=0, pods=0, **scalar) -> Resource:
    sc = {}
    for k, v in scalar.items():
        sc[{"gpu": GPU, "gpu_mem": GPU_MEM, "new": NEW}.get(k, k)] = v
    return Resource(cpu, mem, eph, pods, sc)


def EQ(ns="ns-1", mn=None, mx=None, used=None, enforced=False, name=None) -> ElasticQuotaInfo:
    return ElasticQuotaInfo(name or ns, ns, {ns}, mn, mx, used if used is not None else Resource(), enforced)


def infos(**kv) -> ElasticQuotaInfos:
    out = ElasticQuotaInfos()
    for k, v in kv.items():
        out[k.replace("_", "-")] = v
    return out


def same(a: Resource, b: Resource) -> bool:
    """Value equality, ignoring scalar keys that are zero on one side only."""
    keys = set(a.scalar) | set(b.scalar)
    return ((a.milli_cpu, a.memory, a.ephemeral_storage, a.allowed_pod_number) ==
            (b.milli_cpu, b.memory, b.ephemeral_storage, b.allowed_pod_number) and
            all(a.scalar.get(k, 0) == b.scalar.get(k, 0) for k in keys))


# --------------------------------------------------------------- golden cases
GPU_GB = 32  # the reference's DefaultNvidiaGPUResourceMemory; the values only scale


def test_reserve_and_unreserve():
    reqs = [R(1000, 50, gpu=1, gpu_mem=GPU_GB), R(2000, 100, gpu=0, gpu_mem=0), R(0, 0, gpu=2, gpu_mem=2 * GPU_GB)]
    eq = EQ(used=R(1000, 200, gpu=2, gpu_mem=2 * GPU_GB))
    for r in reqs:
        eq.reserve(r)
    assert same(eq.used, R(4000, 350, gpu=5, gpu_mem=5 * GPU_GB))
    eq = EQ(used=R(4000, 200, gpu=5, gpu_mem=5 * GPU_GB))
    for r in reqs:
        eq.unreserve(r)
    assert same(eq.used, R(1000, 50, gpu=2, gpu_mem=2 * GPU_GB))


@pytest.mark.parametrize("eq,req,want", [
    (EQ(enforced=False), R(100), False),
    (EQ(used=R(100), mx=R(100), enforced=True), R(100), True),
    (EQ(used=R(50), mx=R(100), enforced=True), R(50), False),
], ids=["max-not-enforced", "used-over-max", "used-equals-max"])
def test_used_over_max_with(eq, req, want):
    assert eq.used_over_max_with(req) is want


def test_guaranteed_overquotas_missing_quota_raises():
    with pytest.raises(KeyError):
        ElasticQuotaInfos().get_guaranteed_overquotas("not-present")


def test_guaranteed_overquotas_empty_quota():
    q = infos(eq_1=EQ("eq-1", R(), R(), R()),
              eq_2=EQ("eq-2", R(100, 1000, 0, 10), R(200, 2000, 0, 20), R(50, 50, 0, 5)))
    assert same(q.get_guaranteed_overquotas("eq-1"), R())
    q = infos(eq_1=EQ("eq-1", R(), R(), R()), eq_2=EQ("eq-2", R(), R(), R()))
    assert same(q.get_guaranteed_overquotas("eq-1"), R())


def test_guaranteed_overquotas_proportional_to_min():
    q = infos(
        eq_1=EQ("ns-1", R(10, 10, 0, 10, gpu=5, gpu_mem=64, new=3), used=R(5, 5, 0, 5, gpu=0, gpu_mem=10, new=1)),
        eq_2=EQ("ns-2", R(30, 30, 30, 30, gpu=3, gpu_mem=24), used=R(35, 35, 0, 5, gpu=0, gpu_mem=10)),
        eq_3=EQ("ns-3", R(20, 20, 20, 0), used=R(10, 10, 10, 0)),
    )
    got = q.get_guaranteed_overquotas("eq-1")
    # floor(10/60 * (5+0+10)) = 2 ; pods floor(10/40 * (5+25+0)) = 7 ;
    # gpu floor(5/8 * (5+3)) = 5 ; gpu-mem floor(64/88 * (54+14)) = 49 ; new-resource only in eq-1 -> all 2
    assert same(got, R(2, 2, 0, 7, gpu=5, gpu_mem=49, new=2))


def _pct_cases():
    full = dict(cpu=1.0, memory=1.0, pods=1.0, **{"ephemeral-storage": 1.0, GPU_MEM: 1.0, GPU: 1.0})
    m30 = R(30, 30, 30, 30, gpu=3, gpu_mem=24)
    yield "single-empty", infos(eq_1=EQ("ns-1")), "eq-1", {}
    yield "one-empty", infos(eq_1=EQ("ns-1", m30.clone()), eq_2=EQ("ns-2")), "eq-1", full
    yield "single", infos(eq_1=EQ("ns-1", m30.clone())), "eq-1", full
    yield "max-values", infos(eq_1=EQ("ns-1", R(MAXI64, MAXI64, MAXI64, MAXI64, gpu=MAXI64, gpu_mem=MAXI64))), \
        "eq-1", full
    yield "partial-min", infos(eq_1=EQ("ns-1", R(10, 10, gpu=10)), eq_2=EQ("ns-2", R(10, 0, 0, 10, gpu_mem=10))), \
        "eq-1", {"cpu": 0.5, "memory": 1.0, "pods": 0.0, "ephemeral-storage": 0.0, GPU: 1.0}
    yield "proportional", infos(
        eq_1=EQ("ns-1", R(50, 10, 0, 10, gpu=5, gpu_mem=64, new=3)),
        eq_2=EQ("ns-2", R(30, 30, 30, 30, gpu=3, gpu_mem=24)),
        eq_3=EQ("ns-3", R(20, 60, 20, 0))), "eq-1", \
        {"cpu": 0.5, "memory": 0.1, "pods": 0.25, "ephemeral-storage": 0.0, NEW: 1.0,
         GPU_MEM: 64 / (64 + 24), GPU: 5 / (5 + 3)}


@pytest.mark.parametrize("name,q,key,want", list(_pct_cases()), ids=[c[0] for c in _pct_cases()])
def test_guaranteed_overquota_percentages(name, q, key, want):
    got = q.guaranteed_overquotas_percentages(q[key])
    assert got.keys() == want.keys()
    for k in want:
        assert got[k] == pytest.approx(want[k], rel=1e-12)
    # across all quotas the percentages of a resource sum to 1 (or are all 0)
    tot: dict[str, float] = {}
    for info in q._unique():
        for r, p in q.guaranteed_overquotas_percentages(info).items():
            tot[r] = tot.get(r, 0.0) + p
    for r, p in tot.items():
        assert p == 0 or abs(p - 1.0) < 1e-4, (r, p)


@pytest.mark.parametrize("q,want", [
    (infos(), R()),
    (infos(eq=EQ("ns", R(100, 200, 5, 10, gpu=5, gpu_mem=5), used=R(0, 100, 0, 0, gpu=5, gpu_mem=0))),
     R(100, 100, 5, 10, gpu=0, gpu_mem=5)),
    (infos(eq_1=EQ("ns-1", R(100, 200, 5, 5, gpu=5, gpu_mem=5), used=R(150, 250, 10, 10, gpu=10, gpu_mem=10)),
           eq_2=EQ("ns-2", R(200, 200, 5, 5, gpu=5, gpu_mem=5), used=R(200, 0, 0, 0, gpu=0, gpu_mem=0)),
           eq_3=EQ("ns-3", R(200, 200, 5, 5, gpu=5), used=R(0, 10, 0, 0, gpu=1))),
     R(200, 390, 10, 10, gpu=9, gpu_mem=5)),
], ids=["empty", "single", "multiple"])
def test_aggregated_overquotas(q, want):
    got = q.aggregated_overquotas()
    assert same(got, want)
    mn = q.aggregated_min()
    for r in got.names():
        assert got.get(r) <= mn.get(r)


@pytest.mark.parametrize("used,req,limit,want", [
    (R(gpu_mem=20, **{"amd.com/partition-1xcd.36gb": 2}), R(**{"amd.com/partition-1xcd.36gb": 1}),
     R(gpu_mem=40), True),
    (R(gpu_mem=20, **{"amd.com/partition-1xcd.36gb": 2}), R(gpu_mem=20, **{"amd.com/partition-1xcd.36gb": 1}),
     R(gpu_mem=25, **{"amd.com/partition-1xcd.36gb": 0}), False),
], ids=["resources-not-in-limit-ignored", "over-limit"])
def test_used_lte_with(used, req, limit, want):
    assert EQ(used=used).used_lte_with(limit, req) is want


def test_aggregated_used_over_min_with():
    q = infos(eq_1=EQ("ns-1", R(20), used=R(gpu_mem=0)), eq_2=EQ("ns-2", R(10), used=R(40, gpu_mem=0)),
              eq_3=EQ("ns-3", R(10), used=R(gpu_mem=0)))
    assert q.aggregated_used_over_min_with(R(10, gpu_mem=0)) is True
    q = infos(eq_1=EQ("ns-1", R(20), used=R()), eq_2=EQ("ns-2", R(10), used=R(10)))
    assert q.aggregated_used_over_min_with(R(10)) is False  # 20 <= 30


# ----------------------------------------------------------------- properties
small = st.integers(min_value=0, max_value=10_000)
SC = [GPU, GPU_MEM, NEW]


@st.composite
def resources(draw, scalars=True):
    r = Resource(draw(small), draw(small), draw(small), draw(small))
    if scalars:
        for k in draw(st.sets(st.sampled_from(SC))):
            r.scalar[k] = draw(small)
    return r


@st.composite
def quota_sets(draw):
    n = draw(st.integers(1, 5))
    q = ElasticQuotaInfos()
    for i in range(n):
        q[f"ns-{i}"] = EQ(f"ns-{i}", draw(resources()), None, draw(resources()))
    return q


@settings(max_examples=150, deadline=None)
@given(quota_sets())
def test_prop_percentages_sum_to_one(q):
    tot: dict[str, float] = {}
    for info in q._unique():
        for r, p in q.guaranteed_overquotas_percentages(info).items():
            assert 0.0 <= p <= 1.0
            tot[r] = tot.get(r, 0.0) + p
    for r, p in tot.items():
        assert p == 0 or math.isclose(p, 1.0, abs_tol=1e-9), (r, p)


@settings(max_examples=150, deadline=None)
@given(quota_sets())
def test_prop_guaranteed_overquotas_bounded_by_aggregate(q):
    agg = q.aggregated_overquotas()
    mn = q.aggregated_min()
    total = Resource()
    for ns in q:
        g = q.get_guaranteed_overquotas(ns)
        for r in g.names():
            assert 0 <= g.get(r) <= agg.get(r)
        total = total + g
    for r in total.names():
        assert total.get(r) <= agg.get(r) <= mn.get(r)


@settings(max_examples=150, deadline=None)
@given(resources(), st.lists(resources(), max_size=6))
def test_prop_reserve_unreserve_inverse(start, reqs):
    eq = EQ(used=start.clone())
    for r in reqs:
        eq.reserve(r)
    for r in reversed(reqs):
        eq.unreserve(r)
    assert same(eq.used, start)


@settings(max_examples=150, deadline=None)
@given(resources(), resources(), resources())
def test_prop_lte_is_negation_of_over_for_present_resources(used, req, limit):
    eq = EQ(mn=limit, mx=limit, used=used, enforced=True)
    # sum_less_than_equal and sum_greater_than are exact complements
    assert eq.used_lte_with(limit, req) is (not eq.used_over_max_with(req))
    assert eq.used_over_min_with(req) is eq.used_over_max_with(req)


@settings(max_examples=100, deadline=None)
@given(resources(), resources())
def test_prop_resource_algebra(a, b):
    assert same((a + b) - b, a)
    assert same(a.subtract_non_negative(a), Resource())
    d = a.subtract_non_negative(b)
    for r in d.names():
        assert d.get(r) >= 0
    assert same((a - b).abs(), (b - a).abs())
    c = a.clone()
    c.iadd(b)
    assert same(c, a + b)
    c.isub(b)
    assert same(c, a)
