"""Slices and geometries (reference ``pkg/gpu/partitioning.go:28-127``).

A *slice* is a profile name (``str``); a *geometry* is ``{profile: quantity}``.  ``geometry_id``
is the sorted, deterministic ``"p:q, "`` rendering the reference uses both as identity and as
the last tie-breaker of the geometry selection score (Appendix B.1).
"""
from __future__ import annotations

import json
from typing import Dict, Iterable, List, Mapping, Optional

from ..api import v1alpha1 as api

Geometry = Dict[str, int]


def geometry_id(g: Mapping[str, int]) -> str:
    return "".join(f"{p}:{g[p]}, " for p in sorted(g))


def geometry_json(g: Mapping[str, int]) -> str:
    return json.dumps(dict(sorted(g.items())))


def total_slices(g: Mapping[str, int]) -> int:
    return sum(g.values())


def geometry_distance(current: Mapping[str, int], candidate: Mapping[str, int]) -> int:
    keys = set(current) | set(candidate)
    return sum(abs(candidate.get(k, 0) - current.get(k, 0)) for k in keys)


def geometries_equal(a: Mapping[str, int], b: Mapping[str, int]) -> bool:
    return dict(a) == dict(b)


def get_fewest_slices_geometry(geometries: Iterable[Mapping[str, int]]) -> Optional[Geometry]:
    """Geometry with the fewest *distinct* slices; first in list order wins ties (B.3)."""
    best: Optional[Geometry] = None
    for g in geometries:
        if best is None or len(g) < len(best):
            best = dict(g)
    return best


def get_partitioning_kind(node_labels: Mapping[str, str]) -> Optional[str]:
    kind = (node_labels or {}).get(api.LABEL_GPU_PARTITIONING)
    return kind if kind in api.PARTITIONING_KINDS else None


def is_xcp_partitioning_enabled(node_labels: Mapping[str, str]) -> bool:
    return get_partitioning_kind(node_labels) == api.PARTITIONING_KIND_XCP


def is_cumask_partitioning_enabled(node_labels: Mapping[str, str]) -> bool:
    return get_partitioning_kind(node_labels) == api.PARTITIONING_KIND_CUMASK


def sorted_profiles(g: Mapping[str, int]) -> List[str]:
    return sorted(g)
