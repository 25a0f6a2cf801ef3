"""State shared by a node's reporter and actuator (``internal/controllers/migagent/shared.go:24-57``).

Guarantees at least one report between two consecutive applies: the
actuator waits until :meth:`at_least_one_report_since_last_apply` before
planning again, so it never plans from stale status annotations.
"""
from __future__ import annotations

import threading


class SharedState:
    def __init__(self):
        self.lock = threading.RLock()
        self._reported_since_apply = True
        self.last_parsed_plan_id = ""

    def on_report_done(self) -> None:
        with self.lock:
            self._reported_since_apply = True

    def on_apply_done(self) -> None:
        with self.lock:
            self._reported_since_apply = False

    def at_least_one_report_since_last_apply(self) -> bool:
        with self.lock:
            return self._reported_since_apply
