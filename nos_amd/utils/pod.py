"""Pod predicates (``pkg/util/pod/pod.go:31-101``)."""
from __future__ import annotations

from ..api import constants as C
from ..kube import objects as ko


def is_over_quota(pod: dict) -> bool:
    return ko.labels(pod).get(C.LABEL_CAPACITY_INFO) == C.CAPACITY_OVER_QUOTA


def is_unschedulable(pod: dict) -> bool:
    c = ko.get_condition(pod, "PodScheduled")
    return c is not None and c.get("status") == "False" and c.get("reason") == "Unschedulable"


def extra_resources_could_help_scheduling(pod: dict) -> bool:
    """True when the pod is pending, not scheduled, marked Unschedulable by
    the scheduler, not preempting (no nominated node) and not owned by a
    DaemonSet or a Node -- i.e. re-partitioning GPUs could let it schedule."""
    if ko.pod_node(pod):
        return False
    if ko.pod_phase(pod) != ko.PENDING:
        return False
    if not is_unschedulable(pod):
        return False
    if ko.pod_nominated_node(pod):
        return False
    if any(k in ("DaemonSet", "Node") for k in ko.owner_kinds(pod)):
        return False
    return True


def get_namespaced_name(obj: dict) -> str:
    return ko.key(obj)
