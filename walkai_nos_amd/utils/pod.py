"""Pod-state predicates (reference ``pkg/util/pod/pod.go:28-88``)."""
from __future__ import annotations

from typing import Any, Dict

Obj = Dict[str, Any]


def is_pending(pod: Obj) -> bool:
    return pod.get("status", {}).get("phase") == "Pending"


def is_running(pod: Obj) -> bool:
    return pod.get("status", {}).get("phase") == "Running"


def is_terminated(pod: Obj) -> bool:
    return pod.get("status", {}).get("phase") in ("Succeeded", "Failed")


def is_terminating(pod: Obj) -> bool:
    """Deleted with a grace period and not gone yet (``metadata.deletionTimestamp`` set)."""
    return bool(pod.get("metadata", {}).get("deletionTimestamp"))


def is_scheduled(pod: Obj) -> bool:
    return bool(pod.get("spec", {}).get("nodeName"))


def is_preempting(pod: Obj) -> bool:
    return bool(pod.get("status", {}).get("nominatedNodeName"))


def is_unschedulable(pod: Obj) -> bool:
    for c in pod.get("status", {}).get("conditions") or []:
        if c.get("type") == "PodScheduled" and c.get("reason") == "Unschedulable":
            return True
    return False


# nos-scheduler's PreFilter messages (quota/scheduler.py): the pod waits for quota, not for devices
QUOTA_UNSCHEDULABLE_PREFIX = "quota "


def is_blocked_by_quota(pod: Obj) -> bool:
    for c in pod.get("status", {}).get("conditions") or []:
        if c.get("type") == "PodScheduled" and c.get("reason") == "Unschedulable":
            return (c.get("message") or "").startswith(QUOTA_UNSCHEDULABLE_PREFIX)
    return False


def is_owned_by(pod: Obj, api_version: str, kind: str) -> bool:
    for ref in pod.get("metadata", {}).get("ownerReferences") or []:
        if ref.get("apiVersion") == api_version and ref.get("kind") == kind:
            return True
    return False


def is_owned_by_daemonset(pod: Obj) -> bool:
    return is_owned_by(pod, "apps/v1", "DaemonSet")


def is_owned_by_node(pod: Obj) -> bool:
    return is_owned_by(pod, "v1", "Node")


def extra_resources_could_help_scheduling(pod: Obj) -> bool:
    return (not is_scheduled(pod) and is_pending(pod) and is_unschedulable(pod) and not is_preempting(pod)
            and not is_owned_by_daemonset(pod) and not is_owned_by_node(pod))


def priority(pod: Obj) -> int:
    return int(pod.get("spec", {}).get("priority") or 0)


def is_more_important(p1: Obj, p2: Obj) -> bool:
    return priority(p1) > priority(p2)
