"""Annotation codec, profile names, quantities and the batcher.

Golden cases mirror the reference's ``pkg/gpu/annotation_test.go:319-449``
(ParseStatusAnnotation / ParseSpecAnnotation error and success tables) and
``pkg/util/batcher_test.go:35-290`` (ready/idle/timeout/restart semantics),
re-expressed against a fake clock so no case depends on sleeps.  Hypothesis
properties cover what the tables only sample: format/parse round trips,
"profile names contain no '-'" (the key parser splits on '-'),
spec-matches-status symmetry, and quantity parse/format round trips.
"""
from __future__ import annotations

import threading
import time
from fractions import Fraction

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from nos_amd.api import constants as C
from nos_amd.gpu import amdpart, cumask
from nos_amd.gpu.core import (SpecAnnotation, StatusAnnotation, parse_node_annotations, parse_spec_annotation,
                              parse_status_annotation, spec_matches_status, validate_profile_name)
from nos_amd.kube import quantity as q
from nos_amd.utils.batcher import Batcher
from nos_amd.utils.clock import FakeClock, RealClock


# ------------------------------------------------------------------ annotation golden cases
@pytest.mark.parametrize("key,value", [
    ("", ""),
    ("nos.nebuly.com/foo", "1"),
    (C.ANNOTATION_GPU_STATUS_PREFIX + "foo", "1"),
    (C.ANNOTATION_GPU_STATUS_FORMAT.format(index=0, profile="1xcd.36gb", status="free"), "foo"),
    ("nos.nebuly.com/status-gpu-foo-1xcd.36gb-free", "1"),
    ("nos.nebuly.com/status-gpu-0-1xcd.36gb-foo", "1"),
], ids=["empty", "no-prefix", "no-status", "qty-not-int", "index-not-int", "invalid-status"])
def test_parse_status_annotation_errors(key, value):
    with pytest.raises(ValueError):
        parse_status_annotation(key, value)


def test_parse_status_annotation_valid():
    a = parse_status_annotation("nos.nebuly.com/status-gpu-1-1xcd.36gb-used", "2")
    assert a == StatusAnnotation(1, "1xcd.36gb", "used", 2) and a.is_used() and not a.is_free()
    assert a.index_with_profile() == "1-1xcd.36gb"


@pytest.mark.parametrize("key,value", [
    ("", ""), ("nos.nebuly.com/foo", "1"), (C.ANNOTATION_GPU_SPEC_PREFIX + "foo", "1"),
    (C.ANNOTATION_GPU_SPEC_FORMAT.format(index=0, profile="10gb"), "foo"),
], ids=["empty", "no-prefix", "no-spec", "qty-not-int"])
def test_parse_spec_annotation_errors(key, value):
    with pytest.raises(ValueError):
        parse_spec_annotation(key, value)


def test_parse_spec_annotation_valid_and_node_parse():
    a = parse_spec_annotation(C.ANNOTATION_GPU_SPEC_FORMAT.format(index=1, profile="10gb"), "3")
    assert a == SpecAnnotation(1, "10gb", 3)
    node = {"metadata": {"name": "n", "annotations": {
        a.key(): a.value(),
        "nos.nebuly.com/status-gpu-0-10gb-free": "1", "nos.nebuly.com/status-gpu-0-10gb-used": "2",
        "unrelated/annotation": "x", "nos.nebuly.com/spec-partitioning-plan": "42"}}}
    status, spec = parse_node_annotations(node)
    assert spec == [a]
    assert [(s.index, s.status, s.quantity) for s in status] == [(0, "free", 1), (0, "used", 2)]


# ------------------------------------------------------------------ annotation properties
amd_profiles = st.one_of(
    st.builds(lambda g: f"{g}gb", st.integers(1, 288)),
    st.builds(lambda x, g: f"{x}xcd.{g}gb", st.sampled_from([1, 2, 4, 8]), st.integers(1, 288)),
)


@settings(max_examples=200, deadline=None)
@given(st.integers(0, 63), amd_profiles, st.sampled_from(["free", "used"]), st.integers(0, 10_000))
def test_prop_status_annotation_roundtrip(idx, prof, status, qty):
    a = StatusAnnotation(idx, prof, status, qty)
    assert parse_status_annotation(a.key(), a.value()) == a


@settings(max_examples=200, deadline=None)
@given(st.integers(0, 63), amd_profiles, st.integers(0, 10_000))
def test_prop_spec_annotation_roundtrip(idx, prof, qty):
    a = SpecAnnotation(idx, prof, qty)
    assert parse_spec_annotation(a.key(), a.value()) == a
    assert validate_profile_name(prof) == prof


@settings(max_examples=100, deadline=None)
@given(st.text(alphabet="abcxyz0123456789.-", min_size=1, max_size=12))
def test_prop_profile_names_with_dash_rejected(name):
    if "-" in name:
        with pytest.raises(ValueError):
            validate_profile_name(name)
    else:
        assert validate_profile_name(name) == name


@settings(max_examples=100, deadline=None)
@given(st.integers(1, 288), st.sampled_from([1, 2, 4, 8]))
def test_prop_resource_profile_roundtrip(gb, xcds):
    s = cumask.SliceProfile.of(gb)
    assert cumask.profile_of_resource(s.resource_name()) == s and s.memory_gb == gb
    p = amdpart.profile(f"{xcds}xcd.{gb}gb")
    assert amdpart.profile_of_resource(p.resource_name()) == p
    assert (p.xcds, p.memory_gb) == (xcds, gb)
    assert not cumask.is_slice_resource(p.resource_name())
    assert not amdpart.is_partition_resource(s.resource_name())


@st.composite
def spec_and_status(draw):
    spec, status = [], []
    for gpu in range(draw(st.integers(0, 3))):
        for prof in draw(st.sets(st.sampled_from(["10gb", "20gb", "1xcd.36gb"]), max_size=3)):
            used, free = draw(st.integers(0, 4)), draw(st.integers(0, 4))
            spec.append(SpecAnnotation(gpu, prof, used + free))
            if used:
                status.append(StatusAnnotation(gpu, prof, "used", used))
            if free:
                status.append(StatusAnnotation(gpu, prof, "free", free))
    return spec, status


@settings(max_examples=150, deadline=None)
@given(spec_and_status(), st.data())
def test_prop_spec_matches_status(pair, data):
    spec, status = pair
    assert spec_matches_status(spec, status)
    # zero-quantity spec entries do not matter
    assert spec_matches_status(spec + [SpecAnnotation(9, "10gb", 0)], status)
    if status:
        i = data.draw(st.integers(0, len(status) - 1))
        s = status[i]
        bumped = status[:i] + [StatusAnnotation(s.index, s.profile, s.status, s.quantity + 1)] + status[i + 1:]
        assert not spec_matches_status(spec, bumped)


# ------------------------------------------------------------------ quantities
@pytest.mark.parametrize("s,val,milli", [
    ("100m", 1, 100), ("1", 1, 1000), ("0.5", 1, 500), ("1.2", 2, 1200), ("1Gi", 2**30, 2**30 * 1000),
    ("2k", 2000, 2_000_000), ("1e3", 1000, 1_000_000), ("250u", 1, 1),
])
def test_quantity_golden(s, val, milli):
    assert q.value(s) == val and q.milli_value(s) == milli


@settings(max_examples=200, deadline=None)
@given(st.integers(0, 10**12), st.booleans())
def test_prop_quantity_int_roundtrip(v, binary):
    assert q.parse(q.fmt(v, binary=binary)) == v


@settings(max_examples=200, deadline=None)
@given(st.integers(0, 10**9))
def test_prop_quantity_milli_roundtrip(m):
    assert q.milli_value(q.fmt(q.from_milli(m))) == m
    assert q.parse(q.fmt(Fraction(m, 1000))) == Fraction(m, 1000)


# ------------------------------------------------------------------ batcher (fake clock)
# times in the fake-clock cases are the reference's milliseconds, used as seconds so
# that float rounding of the clock cannot move a window edge
def _started(timeout_s, idle_s, buffer_size=0):
    clk = FakeClock()
    b = Batcher(timeout_s=timeout_s, idle_s=idle_s, clock=clk, buffer_size=buffer_size)
    b.start()
    return b, clk


def test_batcher_items_before_start_ignored():
    b = Batcher(timeout_s=10, idle_s=10, clock=FakeClock())
    assert not b.add("a") and not b.add("b")
    b.start()
    b.add("c")
    b.clock.advance(20)
    assert b.ready() == ["c"]


def test_batcher_ready_after_idle():
    b, clk = _started(200, 10)
    b.add(1)
    clk.advance(9)
    assert b.ready() is None
    clk.advance(1)
    assert b.ready() == [1]
    assert b.ready() is None  # a ready batch is delivered once


def test_batcher_add_resets_idle_but_not_timeout():
    b, clk = _started(500, 50)
    for _ in range(3):
        b.add(0)
        clk.advance(25)
        assert b.ready() is None
    clk.advance(25)
    assert len(b.ready()) == 3  # ready after > 2x idle, < timeout
    b2, clk2 = _started(40, 20)
    got = None
    for i in range(10):
        b2.add(i)
        clk2.advance(5)
        got = got or b2.ready()
    assert got is not None and len(got) == 8  # the timeout closed the window at t=40ms


def test_batcher_start_twice_errors_and_restart_after_stop():
    b, _ = _started(20, 10)
    with pytest.raises(RuntimeError):
        b.start()
    b.stop()
    b.start()  # restartable
    assert b.add(1)


def test_batcher_single_ready_buffer_and_reset():
    b, clk = _started(1000, 100)
    b.add(1)
    clk.advance(200)
    b.poll()
    b.add(2)
    clk.advance(200)
    b.poll()  # second ready batch dropped while the first is unconsumed
    assert b.ready() == [1]
    assert b.ready() is None
    b.add(3)
    assert b.next_deadline() == pytest.approx(100)
    b.reset()
    assert len(b) == 0 and b.next_deadline() is None


def test_batcher_buffer_size_bounds_batch():
    b, clk = _started(10, 10, buffer_size=2)
    assert b.add(1) and b.add(2) and not b.add(3)
    assert len(b) == 2


def test_batcher_includes_all_items_threaded_real_clock():
    b = Batcher(timeout_s=0.3, idle_s=0.1, clock=RealClock())
    b.start(threaded=True, period=0.005)
    try:
        threads = [threading.Thread(target=lambda i=i: b.add(i)) for i in range(20)]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        deadline = time.monotonic() + 5
        got = None
        while got is None and time.monotonic() < deadline:
            time.sleep(0.01)
            got = b.ready()
        assert sorted(got) == list(range(20))
        b.stop()
        b.start(threaded=True, period=0.005)  # restart after stop polls again
        b.add("x")
        deadline = time.monotonic() + 5
        got = None
        while got is None and time.monotonic() < deadline:
            time.sleep(0.01)
            got = b._ready
        assert got == ["x"]
    finally:
        b.stop()
