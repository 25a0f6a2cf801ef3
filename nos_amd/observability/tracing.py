"""Lightweight span tracer writing JSON lines (SURVEY.md 5.1 [NEW]).

``with span("partitioner.plan", kind="cumask") as s: ...; s.set(plan_id=...)``
records start/end/duration + attributes.  Spans go to an in-memory ring (for
tests and the simulator) and, if ``NOS_AMD_TRACE_FILE`` is set, to that file,
so batch -> plan -> apply -> report latency per plan id can be reconstructed.
"""
from __future__ import annotations

import collections
import contextlib
import json
import os
import threading
import time

_lock = threading.Lock()
_ring: collections.deque = collections.deque(maxlen=10000)
_local = threading.local()


class Span:
    def __init__(self, name: str, attrs: dict):
        self.name = name
        self.attrs = dict(attrs)
        self.start = time.time()
        self.end: float | None = None
        self.parent = getattr(_local, "current", None)

    def set(self, **kw) -> None:
        self.attrs.update(kw)

    def record(self) -> dict:
        return {"name": self.name, "start": self.start, "end": self.end,
                "duration_s": (self.end or time.time()) - self.start,
                "parent": self.parent.name if self.parent else None, **self.attrs}


@contextlib.contextmanager
def span(name: str, **attrs):
    s = Span(name, attrs)
    prev = getattr(_local, "current", None)
    _local.current = s
    try:
        yield s
    except Exception as e:
        s.set(error=f"{type(e).__name__}: {e}")
        raise
    finally:
        s.end = time.time()
        _local.current = prev
        rec = s.record()
        with _lock:
            _ring.append(rec)
            path = os.environ.get("NOS_AMD_TRACE_FILE")
            if path:
                with open(path, "a") as f:
                    f.write(json.dumps(rec, default=str) + "\n")


def event(name: str, **attrs) -> None:
    with span(name, **attrs):
        pass


def spans(name: str | None = None) -> list[dict]:
    with _lock:
        return [s for s in _ring if name is None or s["name"] == name]


def clear() -> None:
    with _lock:
        _ring.clear()


def plan_report_latencies() -> dict[str, float]:
    """Seconds from each ``partitioner.plan`` span (plan applied) to the first
    ``agent.plan_reported`` event of that plan id -- the batch -> plan ->
    apply -> report latency of SURVEY.md 5.1."""
    with _lock:
        recs = list(_ring)
    planned = {r["plan_id"]: r["end"] for r in recs if r["name"] == "partitioner.plan" and r.get("plan_id")}
    out: dict[str, float] = {}
    for r in recs:
        if r["name"] == "agent.plan_reported" and r.get("plan_id") in planned and r["plan_id"] not in out:
            out[r["plan_id"]] = max(0.0, r["end"] - planned[r["plan_id"]])
    return out
