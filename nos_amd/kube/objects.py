"""Kubernetes objects as plain JSON-compatible dicts, plus typed accessors.

The in-process API server (:mod:`nos_amd.sim.apiserver`) stores exactly what a
real kube-apiserver would (``apiVersion``/``kind``/``metadata``/``spec``/
``status`` dicts), so manifests, merge-patches and CRD YAML work unchanged.
These helpers are the "client-go / apimachinery" accessors the controllers use.
"""
from __future__ import annotations

import copy
import datetime as _dt
import uuid as _uuid
from fractions import Fraction
from typing import Any

from . import quantity as q

Obj = dict[str, Any]

# ------------------------------------------------------------------ time
_EPOCH = _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc)


def now_rfc3339(t: float | None = None) -> str:
    if t is None:
        d = _dt.datetime.now(_dt.timezone.utc)
    else:
        d = _EPOCH + _dt.timedelta(seconds=t)
    return d.strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def parse_time(s: str | None) -> float:
    """RFC3339 (with or without fractional seconds) -> unix seconds (0 if absent)."""
    if not s:
        return 0.0
    s = s.replace("Z", "+00:00")
    return _dt.datetime.fromisoformat(s).timestamp()


# ------------------------------------------------------------------ meta
def meta(o: Obj) -> dict:
    return o.setdefault("metadata", {})


def name(o: Obj) -> str:
    return o.get("metadata", {}).get("name", "")


def namespace(o: Obj) -> str:
    return o.get("metadata", {}).get("namespace", "") or ""


def key(o: Obj) -> str:
    ns = namespace(o)
    return f"{ns}/{name(o)}" if ns else name(o)


def uid(o: Obj) -> str:
    return o.get("metadata", {}).get("uid", "")


def labels(o: Obj) -> dict[str, str]:
    return o.get("metadata", {}).get("labels") or {}


def annotations(o: Obj) -> dict[str, str]:
    return o.get("metadata", {}).get("annotations") or {}


def set_label(o: Obj, k: str, v: str) -> None:
    meta(o).setdefault("labels", {})[k] = v


def set_annotation(o: Obj, k: str, v: str) -> None:
    meta(o).setdefault("annotations", {})[k] = v


def creation_time(o: Obj) -> float:
    return parse_time(o.get("metadata", {}).get("creationTimestamp"))


def resource_version(o: Obj) -> str:
    return o.get("metadata", {}).get("resourceVersion", "")


def deletion_timestamp(o: Obj) -> str | None:
    return o.get("metadata", {}).get("deletionTimestamp")


def owner_kinds(o: Obj) -> list[str]:
    return [r.get("kind", "") for r in o.get("metadata", {}).get("ownerReferences") or []]


def deep_copy(o: Obj) -> Obj:
    return copy.deepcopy(o)


def new_uid() -> str:
    return str(_uuid.uuid4())


# ------------------------------------------------------------------ pods
PENDING, RUNNING, SUCCEEDED, FAILED, UNKNOWN = "Pending", "Running", "Succeeded", "Failed", "Unknown"


def pod_phase(p: Obj) -> str:
    return (p.get("status") or {}).get("phase", "")


def pod_node(p: Obj) -> str:
    return (p.get("spec") or {}).get("nodeName", "") or ""


def pod_nominated_node(p: Obj) -> str:
    return (p.get("status") or {}).get("nominatedNodeName", "") or ""


def pod_priority(p: Obj) -> int:
    v = (p.get("spec") or {}).get("priority")
    return int(v) if v is not None else 0


def pod_priority_or_none(p: Obj) -> int | None:
    v = (p.get("spec") or {}).get("priority")
    return None if v is None else int(v)


def pod_containers(p: Obj) -> list[dict]:
    return (p.get("spec") or {}).get("containers") or []


def pod_init_containers(p: Obj) -> list[dict]:
    return (p.get("spec") or {}).get("initContainers") or []


def pod_conditions(p: Obj) -> list[dict]:
    return (p.get("status") or {}).get("conditions") or []


def get_condition(p: Obj, ctype: str) -> dict | None:
    for c in pod_conditions(p):
        if c.get("type") == ctype:
            return c
    return None


def set_condition(p: Obj, ctype: str, status: str, reason: str = "", message: str = "") -> None:
    st = p.setdefault("status", {})
    conds = st.setdefault("conditions", [])
    for c in conds:
        if c.get("type") == ctype:
            c.update({"status": status, "reason": reason, "message": message})
            return
    conds.append({"type": ctype, "status": status, "reason": reason, "message": message,
                  "lastTransitionTime": now_rfc3339()})


def container_requests(c: dict) -> dict[str, Fraction]:
    return q.rl_parse(((c.get("resources") or {}).get("requests")) or {})


def container_limits(c: dict) -> dict[str, Fraction]:
    return q.rl_parse(((c.get("resources") or {}).get("limits")) or {})


def pod_overhead(p: Obj) -> dict[str, Fraction]:
    return q.rl_parse((p.get("spec") or {}).get("overhead") or {})


def is_terminated(p: Obj) -> bool:
    return pod_phase(p) in (SUCCEEDED, FAILED)


def node_allocatable(n: Obj) -> dict[str, Fraction]:
    return q.rl_parse((n.get("status") or {}).get("allocatable") or {})


def node_capacity(n: Obj) -> dict[str, Fraction]:
    return q.rl_parse((n.get("status") or {}).get("capacity") or {})


def gvk(o: Obj) -> tuple[str, str]:
    return o.get("apiVersion", ""), o.get("kind", "")
