"""Node-side plan: actual partitions + desired spec -> per-GPU mode changes.

Reference: ``internal/controllers/migagent/plan/{plan,mig_state,operation}.go`` (SURVEY Appendix
B.4/B.5).  The MIG plan is a list of instance deletes/creates (free devices first, "re-create the
free ones for a clean slate", then an n!-permutation create search).  On MI355X a GPU's geometry is
one homogeneous mode, so the plan collapses to one :class:`ModeChange` per GPU whose mode differs
from the spec, plus an optional node-wide NPS change.  The invariants carry over:

* only GPUs named in the spec are touched;
* a GPU with *used* partitions is never flipped (a flip destroys every partition) — it is
  reported as ``blocked`` instead (the MIG plan's "delete used candidates last" case);
* ``matches`` compares per (GPU, profile) device counts with the spec (``MigState.Matches``).
"""
from __future__ import annotations

from collections import defaultdict
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Mapping, Optional, Tuple

from ...models.annotation import SpecAnnotation
from ...models.device import DeviceList
from ...models.xcp.profile import extract_profile_name, is_valid_profile, parse_profile


@dataclass(frozen=True)
class ModeChange:
    gpu_index: int
    from_profile: Optional[str]
    to_profile: str


@dataclass
class XcpConfigPlan:
    changes: List[ModeChange] = field(default_factory=list)
    memory_partition: Optional[str] = None           # target NPS when a node-wide change is needed
    blocked: List[Tuple[int, str]] = field(default_factory=list)
    invalid: List[Tuple[int, str]] = field(default_factory=list)

    def is_empty(self) -> bool:
        return not self.changes and self.memory_partition is None

    def equal(self, other: Optional["XcpConfigPlan"]) -> bool:
        if other is None:
            return False
        return (sorted(self.changes, key=lambda c: c.gpu_index) == sorted(other.changes, key=lambda c: c.gpu_index)
                and self.memory_partition == other.memory_partition)


class XcpState:
    """Actual partition devices grouped by physical GPU (``MigState``)."""

    def __init__(self, devices: Iterable):
        self.by_gpu: Dict[int, DeviceList] = DeviceList(devices).group_by_gpu_index()

    def counts(self) -> Dict[Tuple[int, str], int]:
        out: Dict[Tuple[int, str], int] = defaultdict(int)
        for g, devs in self.by_gpu.items():
            for d in devs:
                p = extract_profile_name(d.resource_name)
                if p is not None:
                    out[(g, p)] += 1
        return dict(out)

    def matches(self, spec: Iterable[SpecAnnotation]) -> bool:
        want: Dict[Tuple[int, str], int] = defaultdict(int)
        for a in spec:
            want[(a.index, a.profile)] += a.quantity
        return dict(want) == self.counts()

    def used_on(self, gpu: int) -> int:
        return sum(1 for d in self.by_gpu.get(gpu, []) if d.is_used())


def desired_profiles(spec: Iterable[SpecAnnotation]) -> Tuple[Dict[int, str], List[Tuple[int, str]]]:
    per_gpu: Dict[int, Dict[str, int]] = defaultdict(lambda: defaultdict(int))
    for a in spec:
        per_gpu[a.index][a.profile] += a.quantity
    desired: Dict[int, str] = {}
    invalid: List[Tuple[int, str]] = []
    for g, profs in per_gpu.items():
        profs = {p: q for p, q in profs.items() if q > 0}
        if len(profs) != 1:
            invalid.append((g, f"spec for GPU {g} must name exactly one compute-partition profile, got {dict(profs)}"))
            continue
        (p, q), = profs.items()
        if not is_valid_profile(p):
            invalid.append((g, f"invalid profile {p!r}"))
            continue
        if q != parse_profile(p).partitions:
            invalid.append((g, f"profile {p} yields {parse_profile(p).partitions} partitions, spec asks {q}"))
            continue
        desired[g] = p
    return desired, invalid


def new_xcp_config_plan(state: XcpState, current: Mapping[int, str], spec: Iterable[SpecAnnotation],
                        spec_nps: Optional[str] = None, current_nps: Optional[str] = None) -> XcpConfigPlan:
    spec = list(spec)
    plan = XcpConfigPlan()
    desired, plan.invalid = desired_profiles(spec)
    target_nps = spec_nps.lower() if spec_nps else None
    if target_nps is None and desired:
        # all desired profiles must agree on the NPS mode; infer it from the spec
        modes = {parse_profile(p).nps for p in desired.values()}
        target_nps = modes.pop() if len(modes) == 1 else None
    if target_nps and current_nps and target_nps != current_nps.lower():
        busy = [g for g in current if state.used_on(g) > 0]
        if busy:
            # nothing moves until the whole node is idle: flipping the idle GPUs' compute modes now
            # would only give them partitions of the old memory mode to be flipped again
            plan.blocked.extend((g, f"memory partition change to {target_nps} needs the whole node idle")
                                for g in sorted(current))
            return plan
        plan.memory_partition = target_nps
    for g, p in sorted(desired.items()):
        cur = current.get(g)
        if cur == p:
            continue  # mode already right; the device count converges after re-enumeration
        if state.used_on(g) > 0:
            plan.blocked.append((g, f"GPU {g} has {state.used_on(g)} partition(s) in use"))
            continue
        plan.changes.append(ModeChange(g, cur, p))
    return plan
