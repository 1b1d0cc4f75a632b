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

GPUs the spec wants *sliced* (``spec-sliced-gpus``, ``models/xcp/slices.py``) are planned the MIG
way instead: the GPU must be in SPX (a flip there needs it idle, like any flip), and then its
slices are re-carved around the used ones (:func:`~walkai_nos_amd.models.xcp.slices.recarve`):
free slices not in the spec are deleted, missing ones created when they fit — no flip, no drain.
A GPU leaving the sliced layout drops its slices once none is in use.
"""
from __future__ import annotations

from collections import defaultdict
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Mapping, Optional, Tuple

from ...models.annotation import SpecAnnotation
from ...models.device import DeviceList
from ...models.slicing.cumask import Slice
from ...models.xcp.profile import extract_profile_name, is_valid_profile, parse_profile
from ...models.xcp.slices import SLICE_NPS, SLICED_MODE, apply_recarve, recarve, spec_by_gpu


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
    #: GPU -> its new CU-mask slice layout ([] = no longer sliced), for the GPUs whose slices change
    slices: Dict[int, List[Slice]] = field(default_factory=dict)

    def is_empty(self) -> bool:
        return not self.changes and self.memory_partition is None and not self.slices

    def equal(self, other: Optional["XcpConfigPlan"]) -> bool:
        if other is None:
            return False
        ids = lambda p: {g: [(s.id, s.profile) for s in ss] for g, ss in p.slices.items()}  # noqa: E731
        return (sorted(self.changes, key=lambda c: c.gpu_index) == sorted(other.changes, key=lambda c: c.gpu_index)
                and self.memory_partition == other.memory_partition and ids(self) == ids(other))


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
                        spec_nps: Optional[str] = None, current_nps: Optional[str] = None,
                        sliced: Iterable[int] = (), slices: Optional[Mapping[int, List[Slice]]] = None,
                        used_ids: Iterable[str] = (), gpu_ids: Optional[Mapping[int, str]] = None,
                        vram_bytes: Optional[Mapping[int, int]] = None) -> XcpConfigPlan:
    """``sliced``: GPUs the spec wants as CU-mask slices; ``slices``: the current slice layout;
    ``gpu_ids`` / ``vram_bytes``: per GPU the id slice ids are built from (its BDF) and its HBM."""
    spec = list(spec)
    plan = XcpConfigPlan()
    sliced = set(sliced)
    slices = dict(slices or {})
    used = set(used_ids)
    sliced_spec = [a for a in spec if a.index in sliced]
    spec = [a for a in spec if a.index not in sliced]
    _plan_slices(plan, state, current, sliced, sliced_spec, slices, used, gpu_ids or {}, vram_bytes or {})
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
        if slices.get(g):
            # leaving the sliced layout: only once no slice is in use
            if any(s.id in used for s in slices[g]):
                plan.blocked.append((g, f"GPU {g} has slices in use"))
                continue
            plan.slices[g] = []
        if cur == p:
            continue  # mode already right; the device count converges after re-enumeration
        if state.used_on(g) > 0:
            plan.blocked.append((g, f"GPU {g} has {state.used_on(g)} partition(s) in use"))
            continue
        plan.changes.append(ModeChange(g, cur, p))
    return plan


def _plan_slices(plan: XcpConfigPlan, state: XcpState, current: Mapping[int, str], sliced: Iterable[int],
                 spec: List[SpecAnnotation], slices: Dict[int, List[Slice]], used: set,
                 gpu_ids: Mapping[int, str], vram_bytes: Mapping[int, int]) -> None:
    want = spec_by_gpu(spec)
    spx = f"{SLICED_MODE}_{SLICE_NPS}"
    for g in sorted(sliced):
        w = want.get(g, {})
        bad = [p for p in w if not is_valid_profile(p) or parse_profile(p).nps != SLICE_NPS]
        if bad:
            plan.invalid.append((g, f"sliced GPU {g}: profiles {bad} are not NPS1 compute-partition sizes"))
            continue
        have = list(slices.get(g, []))
        cur = current.get(g)
        if cur != spx:
            if state.used_on(g) > 0:
                plan.blocked.append((g, f"GPU {g} has {state.used_on(g)} partition(s) in use: not sliced yet"))
                continue
            plan.changes.append(ModeChange(g, cur, spx))
            have = []
        rc = recarve(have, used, w)
        if not rc.achievable:
            plan.blocked.append((g, f"GPU {g}: the slices in use leave no room for {w} yet (draining)"))
        if g not in gpu_ids:
            plan.invalid.append((g, f"GPU {g} is not in the device map"))
            continue
        new = apply_recarve(have, rc, gpu_ids[g], vram_bytes.get(g, 288 * 10**9))
        if [s.id for s in new] != [s.id for s in slices.get(g, [])] or cur != spx:
            plan.slices[g] = new
