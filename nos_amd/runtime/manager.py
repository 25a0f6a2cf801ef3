"""Controller runtime: controllers, watches, manager, leader election, health.

The controller-runtime pattern of the reference (``Reconcile(ctx, req)`` +
``SetupWithManager``) on top of :mod:`nos_amd.sim.apiserver`:

* a :class:`Controller` owns a de-duplicating work queue, a reconciler, its
  watches (``for_kind`` = enqueue the object itself; ``watches`` = map
  function) and predicates;
* the :class:`Manager` registers one API watch per (controller, kind) and runs
  the controllers either with worker threads (``start()``; ``max_concurrent``
  workers per controller like ``MaxConcurrentReconciles``) or deterministically
  (``run_until_idle()`` / ``run_for()``, which also advance a fake clock to the
  next requeue) -- the latter replaces envtest's ``Eventually`` polling;
* optional Lease-based leader election (``leaderElect: true`` in the
  reference's component configs) and healthz/readyz checks.
"""
from __future__ import annotations

import logging
import threading
import time
import traceback
from dataclasses import dataclass, field
from typing import Any, Callable, Protocol

from ..kube import objects as ko
from ..observability import metrics
from ..sim.apiserver import ADDED, DELETED, MODIFIED, AlreadyExists, ApiServer, Conflict, NotFound, WatchEvent
from .predicates import Event, Predicate
from .workqueue import WorkQueue

log = logging.getLogger("nos_amd.runtime")


@dataclass(frozen=True)
class Request:
    name: str
    namespace: str = ""

    def __str__(self) -> str:
        return f"{self.namespace}/{self.name}" if self.namespace else self.name


@dataclass
class Result:
    requeue: bool = False
    requeue_after: float = 0.0


class Reconciler(Protocol):
    def reconcile(self, req: Request) -> Result | None: ...


MapFunc = Callable[[dict], list[Request]]


def request_for(obj: dict) -> Request:
    return Request(ko.name(obj), ko.namespace(obj))


@dataclass
class _WatchSpec:
    kind: str
    mapper: MapFunc
    predicates: list[Predicate] = field(default_factory=list)
    namespace: str | None = None
    label_selector: Any = None


_EV_TYPE = {ADDED: "create", MODIFIED: "update", DELETED: "delete"}


class Controller:
    def __init__(self, name: str, reconciler: Reconciler, max_concurrent: int = 1):
        self.name = name
        self.reconciler = reconciler
        self.max_concurrent = max_concurrent
        self.watch_specs: list[_WatchSpec] = []
        self.queue: WorkQueue | None = None
        self.reconcile_count = 0
        self.error_count = 0
        self.last_error: str | None = None

    def for_kind(self, kind: str, *predicates: Predicate, namespace: str | None = None,
                 label_selector: Any = None) -> "Controller":
        self.watch_specs.append(_WatchSpec(kind, lambda o: [request_for(o)], list(predicates), namespace,
                                           label_selector))
        return self

    def watches(self, kind: str, mapper: MapFunc, *predicates: Predicate, namespace: str | None = None,
                label_selector: Any = None) -> "Controller":
        self.watch_specs.append(_WatchSpec(kind, mapper, list(predicates), namespace, label_selector))
        return self

    def _handle(self, spec: _WatchSpec, wev: WatchEvent) -> None:
        ev = Event(_EV_TYPE[wev.type], wev.object, wev.old)
        if not all(p(ev) for p in spec.predicates):
            return
        try:
            reqs = spec.mapper(wev.object)
        except Exception:  # a mapper must never kill the watch
            log.exception("mapper failed in %s", self.name)
            return
        for r in reqs:
            self.queue.add(r)

    def process_one(self, item: Request) -> None:
        try:
            res = self.reconciler.reconcile(item) or Result()
            self.reconcile_count += 1
            if res.requeue_after > 0:
                self.queue.forget(item)
                self.queue.add_after(item, res.requeue_after)
                metrics.RECONCILES.labels(self.name, "requeue_after").inc()
            elif res.requeue:
                self.queue.add_rate_limited(item)
                metrics.RECONCILES.labels(self.name, "requeue").inc()
            else:
                self.queue.forget(item)
                metrics.RECONCILES.labels(self.name, "success").inc()
        except Exception as e:
            metrics.RECONCILES.labels(self.name, "error").inc()
            self.error_count += 1
            self.last_error = f"{type(e).__name__}: {e}"
            if not isinstance(e, (Conflict, NotFound)):
                log.debug("reconcile %s %s failed: %s", self.name, item, traceback.format_exc())
            self.queue.add_rate_limited(item)
        finally:
            self.queue.done(item)


class LeaderElector:
    """coordination.k8s.io/v1 Lease based leader election."""

    def __init__(self, api: ApiServer, lease_name: str, namespace: str, identity: str,
                 lease_duration: float = 15.0, clock=None):
        self.api, self.name, self.ns, self.identity = api, lease_name, namespace, identity
        self.duration = lease_duration
        self.clock = clock or api.clock

    def try_acquire_or_renew(self) -> bool:
        now = self.clock.now()
        lease = self.api.try_get("Lease", self.name, self.ns)
        spec = {"holderIdentity": self.identity, "leaseDurationSeconds": int(self.duration),
                "renewTime": ko.now_rfc3339(now)}
        if lease is None:
            try:
                self.api.create({"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                                 "metadata": {"name": self.name, "namespace": self.ns},
                                 "spec": {**spec, "acquireTime": ko.now_rfc3339(now)}})
                return True
            except AlreadyExists:
                return False
        s = lease.get("spec", {})
        holder = s.get("holderIdentity")
        expired = ko.parse_time(s.get("renewTime")) + float(s.get("leaseDurationSeconds", self.duration)) < now
        if holder not in (None, "", self.identity) and not expired:
            return False
        if holder != self.identity:
            spec["acquireTime"] = ko.now_rfc3339(now)
            spec["leaseTransitions"] = int(s.get("leaseTransitions", 0)) + 1
        lease["spec"] = {**s, **spec}
        try:
            self.api.update(lease)
            return True
        except Conflict:
            return False

    def release(self) -> None:
        lease = self.api.try_get("Lease", self.name, self.ns)
        if lease and lease.get("spec", {}).get("holderIdentity") == self.identity:
            lease["spec"]["holderIdentity"] = ""
            try:
                self.api.update(lease)
            except Conflict:
                pass


class LeaseKeeper:
    """Keeps a Lease the way client-go's leader elector does: renew every
    ``retry_period``; when no renewal has succeeded for ``renew_deadline``
    (renewals refused because another identity holds an unexpired lease, or
    the API server unreachable), leadership is LOST: ``on_lost`` runs once
    and the keeper stops.  controller-runtime then exits the process
    (``leaderelection lost``); our binaries do the same via ``on_lost``, so a
    process that lost the lease never acts as leader again (no split brain).

    Deterministic use (fake clocks): call :meth:`tick` from the driving loop."""

    def __init__(self, elector: LeaderElector, renew_deadline: float | None = None,
                 retry_period: float | None = None, on_lost: Callable[[], None] | None = None):
        self.elector = elector
        self.clock = elector.clock
        self.renew_deadline = renew_deadline if renew_deadline is not None else elector.duration * 2 / 3
        self.retry_period = retry_period if retry_period is not None else max(0.2, elector.duration / 7.5)
        self.on_lost = on_lost
        self.leading = False
        self.lost = threading.Event()
        self._last_ok: float | None = None
        self._last_try: float | None = None
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None

    def _try(self) -> bool:
        try:
            return self.elector.try_acquire_or_renew()
        except Exception as e:  # API blip: counts as a failed renewal, never kills the keeper
            log.warning("lease %s/%s renew error: %s", self.elector.ns, self.elector.name, e)
            return False

    def acquire(self, stop: threading.Event | None = None, poll_s: float | None = None) -> bool:
        """Block until the lease is ours (False if ``stop`` fires first)."""
        stop = stop or self._stop
        while not stop.is_set():
            if self._try():
                self.leading = True
                self._last_ok = self._last_try = self.clock.monotonic()
                return True
            stop.wait(poll_s if poll_s is not None else self.retry_period)
        return False

    def tick(self) -> bool:
        """One renewal step when due; returns whether we still lead."""
        if not self.leading or self.lost.is_set():
            return False
        now = self.clock.monotonic()
        if self._last_try is not None and now - self._last_try < self.retry_period:
            return True
        self._last_try = now
        if self._try():
            self._last_ok = now
            return True
        if self._last_ok is None or now - self._last_ok >= self.renew_deadline or self._held_by_other():
            self._lose()
            return False
        return True

    def _held_by_other(self) -> bool:
        try:
            lease = self.elector.api.try_get("Lease", self.elector.name, self.elector.ns)
        except Exception:
            return False
        holder = (lease or {}).get("spec", {}).get("holderIdentity")
        return bool(holder) and holder != self.elector.identity

    def _lose(self) -> None:
        self.leading = False
        if not self.lost.is_set():
            self.lost.set()
            log.error("leader election lost: lease %s/%s (identity %s)", self.elector.ns, self.elector.name,
                      self.elector.identity)
            if self.on_lost:
                self.on_lost()

    def start(self) -> None:
        def loop():
            while not self._stop.wait(self.retry_period / 2):
                if not self.tick():
                    return

        self._thread = threading.Thread(target=loop, daemon=True, name=f"lease-{self.elector.name}")
        self._thread.start()

    def stop(self, release: bool = True) -> None:
        self._stop.set()
        if self._thread and self._thread is not threading.current_thread():
            self._thread.join(timeout=2)
        if release and self.leading:
            self.leading = False
            try:
                self.elector.release()
            except Exception:
                pass


class Manager:
    def __init__(self, api: ApiServer, name: str = "manager", clock=None, leader_election: bool = False,
                 leader_election_id: str | None = None, leader_election_namespace: str = "nos-system",
                 identity: str | None = None, resync_s: float | None = None):
        self.api = api
        # informer resync: re-deliver every watched object periodically, so a
        # lost watch event (fault injection, broken stream) cannot strand an
        # object forever (controller-runtime SyncPeriod)
        self.resync_s = resync_s
        self._next_resync: float | None = None
        self.name = name
        self.clock = clock or api.clock
        self.controllers: list[Controller] = []
        self.runnables: list[Any] = []
        self._watches = []
        self._threads: list[threading.Thread] = []
        self._stop = threading.Event()
        self.started = False
        self.health_checks: dict[str, Callable[[], bool]] = {"ping": lambda: True}
        self.ready_checks: dict[str, Callable[[], bool]] = {"ping": lambda: True}
        self.elector = (LeaderElector(api, leader_election_id or f"{name}-leader", leader_election_namespace,
                                      identity or f"{name}-{id(self):x}", clock=self.clock)
                        if leader_election else None)
        self.lease = LeaseKeeper(self.elector, on_lost=self._on_lease_lost) if self.elector else None
        self.is_leader = not leader_election
        # set when the lease was lost: the workers have stopped and the binary must
        # exit non-zero (cmd/common.py), like controller-runtime -- never re-acquire
        self.lost_leadership = threading.Event()
        self.health_checks["leader"] = lambda: not self.lost_leadership.is_set()

    def add(self, controller: Controller) -> Controller:
        controller.queue = WorkQueue(self.clock)
        self.controllers.append(controller)
        if self.started:
            self._bind(controller)
        return controller

    def add_runnable(self, r: Any) -> None:
        """r has start(manager) and optionally stop()."""
        self.runnables.append(r)

    def _bind(self, c: Controller) -> None:
        for spec in c.watch_specs:
            w = self.api.watch(spec.kind, namespace=spec.namespace, label_selector=spec.label_selector,
                               callback=lambda ev, c=c, spec=spec: c._handle(spec, ev))
            self._watches.append(w)

    # ------------------------------------------------------------ lifecycle
    def _elect(self) -> bool:
        """Acquire (not yet leading) or renew when due (leading).  A manager that
        lost its lease stays stopped."""
        if self.elector is None:
            return True
        if self.lost_leadership.is_set():
            return False
        if not self.lease.leading:
            if self.lease._try():
                self.lease.leading = True
                self.lease._last_ok = self.lease._last_try = self.clock.monotonic()
        else:
            self.lease.tick()
        self.is_leader = self.lease.leading
        return self.is_leader

    def _on_lease_lost(self) -> None:
        self.is_leader = False
        self.lost_leadership.set()
        self._stop.set()  # workers, resync and renew loops end; watches are closed by stop()

    def setup(self) -> None:
        """Bind watches (initial lists enqueue every existing object)."""
        if self.started:
            return
        self.started = True
        for c in self.controllers:
            self._bind(c)
        for r in self.runnables:
            if hasattr(r, "start"):
                r.start(self)

    def start(self) -> None:
        """Threaded mode.  With leader election this blocks until the lease is
        acquired; losing it later stops every worker (``lost_leadership``)."""
        if self.elector is not None:
            if not self.lease.acquire(self._stop, poll_s=1.0):
                return
            self.is_leader = True
            self.lease.start()
        self.setup()
        for c in self.controllers:
            for i in range(c.max_concurrent):
                t = threading.Thread(target=self._worker, args=(c,), daemon=True, name=f"{c.name}-{i}")
                t.start()
                self._threads.append(t)
        if self.resync_s:
            t = threading.Thread(target=self._resync_loop, daemon=True, name=f"{self.name}-resync")
            t.start()
            self._threads.append(t)

    def _resync_loop(self) -> None:
        while not self._stop.wait(self.resync_s):
            if self.is_leader:
                self.resync()

    def _worker(self, c: Controller) -> None:
        while not self._stop.is_set():
            item = c.queue.get(timeout=0.1)
            if item is None:
                continue
            if not self.is_leader:  # lease lost between get() and here: leave the item unprocessed
                return
            c.process_one(item)

    def stop(self) -> None:
        self._stop.set()
        for c in self.controllers:
            c.queue.shutdown()
        for w in self._watches:
            w.stop()
        for r in self.runnables:
            if hasattr(r, "stop"):
                r.stop()
        for t in self._threads:
            if t is not threading.current_thread():
                t.join(timeout=2)
        if self.lease is not None:
            self.lease.stop(release=not self.lost_leadership.is_set())

    # ------------------------------------------------------------ deterministic mode
    def resync(self) -> int:
        """Re-enqueue every object of every watch (as update events old == new)."""
        n = 0
        for c in self.controllers:
            for spec in c.watch_specs:
                try:
                    objs = self.api.list(spec.kind, spec.namespace, spec.label_selector)
                except Exception as e:  # an unreachable API server must not kill the loop
                    log.debug("resync list %s failed: %s", spec.kind, e)
                    continue
                for o in objs:
                    c._handle(spec, WatchEvent(MODIFIED, o, o))
                    n += 1
        return n

    def _maybe_resync(self) -> None:
        if self.resync_s is None:
            return
        now = self.clock.monotonic()
        if self._next_resync is None:
            self._next_resync = now + self.resync_s
        elif now >= self._next_resync:
            self._next_resync = now + self.resync_s
            self.resync()

    def step(self) -> int:
        """Process every item ready now once; returns the number processed."""
        if not self.started:
            self.setup()
        if not self._elect():
            return 0
        self._maybe_resync()
        n = 0
        for c in self.controllers:
            while True:
                item = c.queue.get_nowait()
                if item is None:
                    break
                c.process_one(item)
                n += 1
                if n > 100000:
                    raise RuntimeError("runaway reconcile loop")
        return n

    def next_wakeup(self) -> float | None:
        ds = [d for c in self.controllers if (d := c.queue.next_delay()) is not None]
        if self.resync_s is not None and self._next_resync is not None:
            ds.append(max(0.0, self._next_resync - self.clock.monotonic()))
        return min(ds) if ds else None

    def run_until_idle(self, max_time: float = 0.0, max_steps: int = 10000) -> int:
        """Run ready work; with a fake clock, advance time to due requeues up to `max_time` seconds."""
        total = 0
        start = self.clock.now()
        for _ in range(max_steps):
            n = self.step()
            total += n
            if n:
                continue
            d = self.next_wakeup()
            if d is None or max_time <= 0:
                break
            if self.clock.now() + max(d, 0) - start > max_time:
                break
            if hasattr(self.clock, "advance"):
                self.clock.advance(max(d, 0) + 1e-6)
            else:
                time.sleep(max(d, 0))
        return total

    def run_for(self, seconds: float, tick: float = 1.0) -> int:
        """Advance a fake clock by `seconds` in `tick` increments, processing work."""
        total = 0
        end = self.clock.now() + seconds
        while self.clock.now() < end:
            total += self.run_until_idle()
            if hasattr(self.clock, "advance"):
                self.clock.advance(min(tick, end - self.clock.now()))
            else:
                time.sleep(min(tick, end - self.clock.now()))
        total += self.run_until_idle()
        return total

    # ------------------------------------------------------------ health
    def healthz(self) -> bool:
        return all(f() for f in self.health_checks.values())

    def readyz(self) -> bool:
        return all(f() for f in self.ready_checks.values())
