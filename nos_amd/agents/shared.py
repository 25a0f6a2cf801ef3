"""State shared by a node's reporter and actuator (``internal/controllers/migagent/shared.go:24-57``).

Guarantees at least one report between two consecutive applies: the
actuator waits until :meth:`at_least_one_report_since_last_apply` before
planning again, so it never plans from stale status annotations.

``failed_gpus`` carries the actuator's per-GPU switch failures (a switch that
failed, did not take effect, or is still running past its deadline) to the
reporter, which publishes them as ``status-error-gpu-<i>`` annotations.  The
lock is held for planning and reporting only, never across a mode switch.
"""
from __future__ import annotations

import threading


class SharedState:
    def __init__(self):
        self.lock = threading.RLock()
        self._reported_since_apply = True
        self.last_parsed_plan_id = ""
        self.failed_gpus: dict[int, str] = {}

    def mark_failed(self, gpu: int, reason: str) -> None:
        with self.lock:
            self.failed_gpus[gpu] = reason

    def clear_failed(self, gpu: int) -> None:
        with self.lock:
            self.failed_gpus.pop(gpu, None)

    def failures(self) -> dict[int, str]:
        with self.lock:
            return dict(self.failed_gpus)

    def on_report_done(self) -> None:
        with self.lock:
            self._reported_since_apply = True

    def on_apply_done(self) -> None:
        with self.lock:
            self._reported_since_apply = False

    def at_least_one_report_since_last_apply(self) -> bool:
        with self.lock:
            return self._reported_since_apply
