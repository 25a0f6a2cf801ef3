"""Clocks: real wall clock and a fake, manually-advanced clock for deterministic
tests of timing-based components (batcher windows, requeue-after, leases)."""
from __future__ import annotations

import threading
import time


class RealClock:
    def now(self) -> float:
        return time.time()

    def monotonic(self) -> float:
        return time.monotonic()

    def sleep(self, s: float) -> None:
        if s > 0:
            time.sleep(s)


class FakeClock:
    def __init__(self, start: float = 1_700_000_000.0):
        self._t = start
        self._lock = threading.Lock()
        self._cond = threading.Condition(self._lock)

    def now(self) -> float:
        with self._lock:
            return self._t

    def monotonic(self) -> float:
        return self.now()

    def advance(self, s: float) -> None:
        with self._cond:
            self._t += s
            self._cond.notify_all()

    def sleep(self, s: float) -> None:
        # a fake sleep just advances time (single-threaded deterministic use)
        self.advance(s)

    def set(self, t: float) -> None:
        with self._cond:
            self._t = t
            self._cond.notify_all()
