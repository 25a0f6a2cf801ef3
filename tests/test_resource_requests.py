"""Pod resource requests (nos_amd/resource/resource.py): the effective request
is max(sum of containers + overhead, max of init containers) per resource, the
rule the reference's ComputePodRequest follows (/root/reference/pkg/resource/
resource.go) with the pod overhead applied (the reference drops it).  Also the
per-plan memo and the Resource conversions the scheduler and the quota math
rely on (reference: pkg/resource/resource_test.go Sum / Subtract /
SubtractNonNegative)."""
from __future__ import annotations

from fractions import Fraction

from nos_amd.kube import factory as F
from nos_amd.resource.resource import (DefaultCalculator, Resource, compute_pod_request, pod_request_resource,
                                       request_memo)

GPU10 = "amd.com/gpu-10gb"


def _pod(containers=(), init=(), overhead=None) -> dict:
    b = F.build_pod("ns", "p")
    for c in containers:
        b = b.with_container(c)
    for c in init:
        b = b.with_init_container(c)
    if overhead:
        b = b.with_overhead(overhead)
    return b.get()


def _c(cpu_m=0, mem=None, gpu=0):
    b = F.build_container()
    if cpu_m:
        b = b.with_cpu_milli_request(cpu_m)
    if mem:
        b = b.with_memory_request(mem)
    if gpu:
        b = b.with_scalar_resource_request(GPU10, gpu)
    return b.get()


def test_containers_are_summed():
    r = compute_pod_request(_pod([_c(500, "1Gi", 1), _c(250, "512Mi", 2)]))
    assert r["cpu"] == Fraction(3, 4) and r["memory"] == 1536 * 2 ** 20 and r[GPU10] == 3


def test_init_containers_take_the_max_not_the_sum():
    pod = _pod([_c(500, "1Gi")], init=[_c(2000, "256Mi"), _c(1000, "4Gi")])
    r = compute_pod_request(pod)
    assert r["cpu"] == 2 and r["memory"] == 4 * 2 ** 30  # per resource: max(containers, max init)


def test_an_init_container_smaller_than_the_containers_changes_nothing():
    assert compute_pod_request(_pod([_c(1000, "2Gi")], init=[_c(100, "1Gi")])) == \
        compute_pod_request(_pod([_c(1000, "2Gi")]))


def test_overhead_is_added_to_the_containers():
    r = compute_pod_request(_pod([_c(1000, "1Gi")], overhead={"cpu": "250m", "memory": "128Mi"}))
    assert r["cpu"] == Fraction(5, 4) and r["memory"] == (1024 + 128) * 2 ** 20


def test_scalar_resources_survive_the_max_rule():
    pod = _pod([_c(100, gpu=1)], init=[_c(5000)])
    r = compute_pod_request(pod)
    assert r[GPU10] == 1 and r["cpu"] == 5


def test_empty_pod_requests_nothing():
    assert all(v == 0 for v in compute_pod_request(_pod()).values())


def test_memo_returns_equal_copies_and_scopes_to_the_block():
    pod = _pod([_c(1000, "1Gi", 1)])
    with request_memo():
        a = compute_pod_request(pod)
        a["cpu"] = Fraction(99)  # a caller mutating its copy does not poison the memo
        b = compute_pod_request(pod)
        assert b["cpu"] == 1
        with request_memo():  # nested blocks share the outer memo
            assert compute_pod_request(pod)["cpu"] == 1
    pod["spec"]["containers"][0]["resources"]["requests"]["cpu"] = "2"
    assert compute_pod_request(pod)["cpu"] == 2  # outside the block: recomputed


def test_pod_request_resource_and_calculator_agree():
    pod = _pod([_c(1500, "3Gi", 2)])
    r = pod_request_resource(pod)
    assert r.milli_cpu == 1500 and r.memory == 3 * 2 ** 30 and r.scalar[GPU10] == 2
    assert DefaultCalculator().compute_pod_request(pod) == compute_pod_request(pod)


def test_sum_subtract_and_subtract_non_negative():
    a = Resource.from_list({"cpu": 2, "memory": "4Gi", GPU10: 3})
    b = Resource.from_list({"cpu": "500m", "memory": "8Gi", "amd.com/gpu-20gb": 1})
    s = a + b
    assert s.milli_cpu == 2500 and s.memory == 12 * 2 ** 30 and s.scalar == {GPU10: 3, "amd.com/gpu-20gb": 1}
    d = a - b
    assert d.milli_cpu == 1500 and d.memory == -4 * 2 ** 30 and d.scalar["amd.com/gpu-20gb"] == -1
    n = a.subtract_non_negative(b)
    assert n.milli_cpu == 1500 and n.memory == 0 and n.scalar.get("amd.com/gpu-20gb", 0) == 0 and n.scalar[GPU10] == 3
    assert (a - a).is_zero() and not a.is_zero()
    assert d.abs().memory == 4 * 2 ** 30


def test_in_place_add_and_sub_round_trip():
    a = Resource.from_list({"cpu": 1, "memory": "1Gi", "pods": 3, GPU10: 1})
    b = Resource.from_list({"cpu": "250m", GPU10: 2})
    c = Resource.from_list({"cpu": 1, "memory": "1Gi", "pods": 3, GPU10: 1})
    c.iadd(b)
    c.isub(b)
    assert c.milli_cpu == a.milli_cpu and c.memory == a.memory and c.allowed_pod_number == 3
    assert c.scalar[GPU10] == 1
    assert Resource.from_list(a.to_list()).milli_cpu == 1000
