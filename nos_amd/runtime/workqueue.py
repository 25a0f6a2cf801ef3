"""Rate-limited, de-duplicating, delaying work queue (client-go workqueue semantics).

* an item is queued at most once; re-adding an item that is being processed
  marks it dirty and it is queued again when ``done`` is called;
* ``add_after`` schedules an item on the queue's clock (real or fake);
* ``add_rate_limited`` backs off exponentially per item until ``forget``.
"""
from __future__ import annotations

import heapq
import itertools
import threading
from typing import Any, Hashable


class WorkQueue:
    def __init__(self, clock, base_delay: float = 0.005, max_delay: float = 60.0):
        self.clock = clock
        self._cond = threading.Condition()
        self._queue: list[Hashable] = []
        self._dirty: set[Hashable] = set()
        self._processing: set[Hashable] = set()
        self._delayed: list[tuple[float, int, Hashable]] = []
        self._seq = itertools.count()
        self._failures: dict[Hashable, int] = {}
        self._shutdown = False
        self.base_delay, self.max_delay = base_delay, max_delay
        self.adds = 0

    # ------------------------------------------------------------------ add
    def add(self, item: Hashable) -> None:
        with self._cond:
            if self._shutdown or item in self._dirty:
                return
            self.adds += 1
            self._dirty.add(item)
            if item not in self._processing:
                self._queue.append(item)
                self._cond.notify()

    def add_after(self, item: Hashable, delay: float) -> None:
        if delay <= 0:
            self.add(item)
            return
        with self._cond:
            if self._shutdown:
                return
            heapq.heappush(self._delayed, (self.clock.monotonic() + delay, next(self._seq), item))
            self._cond.notify()

    def add_rate_limited(self, item: Hashable) -> None:
        n = self._failures.get(item, 0)
        self._failures[item] = n + 1
        self.add_after(item, min(self.max_delay, self.base_delay * (2 ** n)))

    def forget(self, item: Hashable) -> None:
        self._failures.pop(item, None)

    def num_requeues(self, item: Hashable) -> int:
        return self._failures.get(item, 0)

    # ------------------------------------------------------------------ get
    def _promote_due(self) -> None:
        now = self.clock.monotonic()
        while self._delayed and self._delayed[0][0] <= now:
            _, _, item = heapq.heappop(self._delayed)
            if item not in self._dirty:
                self._dirty.add(item)
                self.adds += 1
                if item not in self._processing:
                    self._queue.append(item)

    def get_nowait(self) -> Any | None:
        with self._cond:
            self._promote_due()
            if not self._queue:
                return None
            item = self._queue.pop(0)
            self._processing.add(item)
            self._dirty.discard(item)
            return item

    def get(self, timeout: float | None = None) -> Any | None:
        """Blocking get (real-clock mode). Returns None on timeout/shutdown."""
        import time

        deadline = None if timeout is None else time.monotonic() + timeout
        with self._cond:
            while True:
                self._promote_due()
                if self._queue:
                    item = self._queue.pop(0)
                    self._processing.add(item)
                    self._dirty.discard(item)
                    return item
                if self._shutdown:
                    return None
                wait = 0.05
                if self._delayed:
                    wait = max(0.0, min(wait, self._delayed[0][0] - self.clock.monotonic()))
                if deadline is not None:
                    rem = deadline - time.monotonic()
                    if rem <= 0:
                        return None
                    wait = min(wait, rem)
                self._cond.wait(wait)

    def done(self, item: Hashable) -> None:
        with self._cond:
            self._processing.discard(item)
            if item in self._dirty:
                self._queue.append(item)
                self._cond.notify()

    # ------------------------------------------------------------------ state
    def __len__(self) -> int:
        with self._cond:
            return len(self._queue)

    def next_delay(self) -> float | None:
        with self._cond:
            if not self._delayed:
                return None
            return self._delayed[0][0] - self.clock.monotonic()

    def pending(self) -> int:
        with self._cond:
            return len(self._queue) + len(self._delayed) + len(self._processing)

    def shutdown(self) -> None:
        with self._cond:
            self._shutdown = True
            self._cond.notify_all()
