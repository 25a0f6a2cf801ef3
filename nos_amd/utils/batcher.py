"""Time-windowed batcher (``pkg/util/batcher.go:25-130``).

Items are collected into a batch; the batch becomes *ready* when either the
idle timer (reset on every added item) or the timeout timer (started by the
first item of the batch) fires.  Semantics kept from the reference:

* ``add`` is non-blocking; items added before ``start`` are dropped;
* only one ready batch is buffered (a second ready batch is dropped);
* ``reset`` clears the current batch and any ready batch.

Clock-driven instead of goroutine + timers: ``poll()`` evaluates the timers
against the (real or fake) clock, so tests need no sleeps (the reference's
timing-based batcher tests were flaky-prone).  A background
thread (``start(threaded=True)``) polls for real-time use.
"""
from __future__ import annotations

import threading
from typing import Generic, TypeVar

T = TypeVar("T")


class Batcher(Generic[T]):
    def __init__(self, timeout_s: float, idle_s: float, clock, buffer_size: int = 0):
        self.timeout_s, self.idle_s, self.clock = timeout_s, idle_s, clock
        self.buffer_size = buffer_size
        self._lock = threading.Lock()
        self._batch: list[T] = []
        self._ready: list[T] | None = None
        self._first_t: float | None = None
        self._last_t: float | None = None
        self.running = False
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None

    def start(self, threaded: bool = False, period: float = 0.05) -> None:
        if self.running:
            raise RuntimeError("batcher already started")
        self.running = True
        self._stop.clear()  # a stopped batcher can be started again
        self.reset()
        if threaded:
            def loop():
                while not self._stop.wait(period):
                    self.poll()
            self._thread = threading.Thread(target=loop, daemon=True, name="batcher")
            self._thread.start()

    def stop(self) -> None:
        self._stop.set()
        self.running = False
        if self._thread:
            self._thread.join(timeout=1)

    def add(self, item: T) -> bool:
        with self._lock:
            if not self.running:
                return False
            if self.buffer_size and len(self._batch) >= self.buffer_size:
                return False
            now = self.clock.monotonic()
            if not self._batch:
                self._first_t = now
            self._batch.append(item)
            self._last_t = now
            return True

    def poll(self) -> None:
        with self._lock:
            if not self._batch:
                return
            now = self.clock.monotonic()
            if now - self._last_t >= self.idle_s or now - self._first_t >= self.timeout_s:
                if self._ready is None:
                    self._ready = self._batch
                self._batch = []
                self._first_t = self._last_t = None

    def ready(self) -> list[T] | None:
        """Non-blocking receive from the ready channel."""
        self.poll()
        with self._lock:
            b, self._ready = self._ready, None
            return b

    def next_deadline(self) -> float | None:
        with self._lock:
            if not self._batch:
                return None
            return min(self._last_t + self.idle_s, self._first_t + self.timeout_s) - self.clock.monotonic()

    def reset(self) -> None:
        with self._lock:
            self._batch = []
            self._ready = None
            self._first_t = self._last_t = None

    def __len__(self) -> int:
        with self._lock:
            return len(self._batch)
