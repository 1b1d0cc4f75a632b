"""Spec/status GPU annotations (exact reference grammar).

Behaviour reproduced from ``pkg/gpu/annotation.go:29-224``:

* a key must start with the prefix; ``key.split("-")`` must give exactly 4 parts (spec) or
  5 parts (status) — hence profile names never contain ``-``;
* GPU index = ``parts[2]``; profile = last part (spec) / ``parts[3]`` (status); status =
  ``parts[4]``, case-insensitive ``free|used|unknown``; the value is an int;
* ``parse_node_annotations`` silently ignores unparsable keys;
* list equality is order-insensitive.
"""
from __future__ import annotations

from collections import defaultdict
from dataclasses import dataclass
from typing import Dict, Iterable, List, Mapping, Tuple

from ..api import v1alpha1 as api
from ..utils.util import unordered_equal
from .device import STATUS_FREE, STATUS_USED, parse_status


def _atoi(s: str) -> int:
    s2 = s.strip()
    if not s2 or not (s2.lstrip("+-").isdigit()):
        raise ValueError(f"invalid integer {s!r}")
    return int(s2)


@dataclass(frozen=True)
class SpecAnnotation:
    profile: str
    index: int
    quantity: int

    @property
    def key(self) -> str:
        return api.ANNOTATION_GPU_SPEC_FORMAT.format(index=self.index, profile=self.profile)

    def value(self) -> str:
        return str(self.quantity)

    def index_with_profile(self) -> str:
        return f"{self.index}-{self.profile}"

    def __str__(self) -> str:
        return self.key


@dataclass(frozen=True)
class StatusAnnotation:
    profile: str
    index: int
    status: str
    quantity: int

    @property
    def key(self) -> str:
        return api.ANNOTATION_GPU_STATUS_FORMAT.format(index=self.index, profile=self.profile, status=self.status)

    def value(self) -> str:
        return str(self.quantity)

    def is_used(self) -> bool:
        return self.status == STATUS_USED

    def is_free(self) -> bool:
        return self.status == STATUS_FREE

    def index_with_profile(self) -> str:
        return f"{self.index}-{self.profile}"

    def __str__(self) -> str:
        return self.key


def parse_spec_annotation(key: str, value: str) -> SpecAnnotation:
    if not key.startswith(api.ANNOTATION_GPU_SPEC_PREFIX):
        raise ValueError(f"expected spec annotation prefix is {api.ANNOTATION_GPU_SPEC_PREFIX!r}, but got {key!r}")
    parts = key.split("-")
    if len(parts) != 4:
        raise ValueError(f"invalid spec annotation key {key!r}")
    quantity = _atoi(value)
    try:
        index = _atoi(parts[2])
    except ValueError as e:
        raise ValueError(f"invalid GPU index: {e}") from e
    return SpecAnnotation(profile=parts[-1], index=index, quantity=quantity)


def parse_status_annotation(key: str, value: str) -> StatusAnnotation:
    if not key.startswith(api.ANNOTATION_GPU_STATUS_PREFIX):
        raise ValueError(f"expected status prefix is {api.ANNOTATION_GPU_STATUS_PREFIX!r}, but got {key!r}")
    parts = key.split("-")
    if len(parts) != 5:
        raise ValueError(f"invalid status annotation key {key!r}")
    quantity = _atoi(value)
    try:
        index = _atoi(parts[2])
    except ValueError as e:
        raise ValueError(f"invalid GPU index: {e}") from e
    try:
        status = parse_status(parts[-1])
    except ValueError as e:
        raise ValueError(f"invalid GPU status: {e}") from e
    return StatusAnnotation(profile=parts[3], index=index, status=status, quantity=quantity)


def parse_node_annotations(annotations: Mapping[str, str]) -> Tuple[List[StatusAnnotation], List[SpecAnnotation]]:
    status: List[StatusAnnotation] = []
    spec: List[SpecAnnotation] = []
    for k, v in (annotations or {}).items():
        try:
            spec.append(parse_spec_annotation(k, v))
            continue
        except ValueError:
            pass
        try:
            status.append(parse_status_annotation(k, v))
        except ValueError:
            pass
    spec.sort(key=lambda a: (a.index, a.profile))
    status.sort(key=lambda a: (a.index, a.profile, a.status))
    return status, spec


def group_by_gpu_index(items: Iterable) -> Dict[int, list]:
    out: Dict[int, list] = defaultdict(list)
    for a in items:
        out[a.index].append(a)
    return dict(out)


def get_used(items: Iterable[StatusAnnotation]) -> List[StatusAnnotation]:
    return [a for a in items if a.is_used()]


def get_free(items: Iterable[StatusAnnotation]) -> List[StatusAnnotation]:
    return [a for a in items if a.is_free()]


def annotations_equal(a: Iterable, b: Iterable) -> bool:
    return unordered_equal(list(a), list(b))


def spec_matches_status(spec: Iterable[SpecAnnotation], status: Iterable[StatusAnnotation]) -> bool:
    """Appendix B.5: map "<idx>-<profile>" -> sum(quantity) over spec vs over status (free+used)."""
    s: Dict[str, int] = defaultdict(int)
    for a in spec:
        s[a.index_with_profile()] += a.quantity
    t: Dict[str, int] = defaultdict(int)
    for a in status:
        t[a.index_with_profile()] += a.quantity
    return dict(s) == dict(t)


def group_spec_by_profile(spec: Iterable[SpecAnnotation]) -> Dict[str, List[SpecAnnotation]]:
    out: Dict[str, List[SpecAnnotation]] = defaultdict(list)
    for a in spec:
        out[a.profile].append(a)
    return dict(out)
