"""Reference-compatible MIG profile tables (parity harness only, no NVIDIA runtime path).

The MI355X partitioner never drives MIG; these tables exist so the generic scored geometry search
(:class:`~walkai_nos_amd.models.partitioned.PartitionedGPU`) can be checked against the
reference's own MIG test vectors (``pkg/gpu/mig/gpu_test.go:297-596``), and so the GPU-memory
calculator can price ``nvidia.com/mig-<g>g.<m>gb`` requests in mixed clusters (reference
``pkg/gpu/util/resource.go:28-86``). Allowed geometries are NVIDIA's published MIG layouts for the
three models the reference knows (``pkg/gpu/model.go:25-29``).
"""
from __future__ import annotations

import re
from typing import Dict, List, Optional

from ..partitioned import PartitionedGPU

PROFILE_RE = re.compile(r"^(\d+)g\.(\d+)gb$")
RESOURCE_RE = re.compile(r"^nvidia\.com/mig-(\d+g\.\d+gb)$")

A30 = "A30"
A100_SXM4_40GB = "NVIDIA-A100-40GB-SXM4"
A100_PCIE_80GB = "NVIDIA-A100-80GB-PCIe"

# the reference's tables entry for entry (``pkg/gpu/mig/known_configs.go:26-140``), including its
# A100-80GB rows that mix 20 GB and 40 GB profiles: they are parity data, not a statement about
# what an A100 accepts
KNOWN_GEOMETRIES: Dict[str, List[Dict[str, int]]] = {
    A30: [{"4g.24gb": 1}, {"2g.12gb": 2}, {"2g.12gb": 1, "1g.6gb": 2}, {"1g.6gb": 4}],
    A100_SXM4_40GB: [
        {"7g.40gb": 1}, {"4g.20gb": 1, "2g.10gb": 1, "1g.5gb": 1}, {"4g.20gb": 1, "1g.5gb": 3},
        {"3g.20gb": 2}, {"3g.20gb": 1, "2g.10gb": 1, "1g.5gb": 1}, {"3g.20gb": 1, "1g.5gb": 3},
        {"2g.10gb": 2, "3g.20gb": 1}, {"2g.10gb": 1, "1g.5gb": 2, "3g.20gb": 1}, {"2g.10gb": 3, "1g.5gb": 1},
        {"2g.10gb": 2, "1g.5gb": 3}, {"2g.10gb": 1, "1g.5gb": 5}, {"1g.5gb": 7},
    ],
    A100_PCIE_80GB: [
        {"7g.79gb": 1}, {"4g.40gb": 1, "2g.20gb": 1, "1g.10gb": 1}, {"4g.40gb": 1, "1g.10gb": 3},
        {"3g.40gb": 2}, {"3g.40gb": 1, "2g.20gb": 1, "1g.10gb": 1}, {"3g.40gb": 1, "1g.10gb": 3},
        {"2g.20gb": 2, "3g.20gb": 1}, {"2g.10gb": 1, "1g.10gb": 2, "3g.40gb": 1}, {"2g.20gb": 3, "1g.10gb": 1},
        {"2g.20gb": 2, "1g.10gb": 3}, {"2g.20gb": 1, "1g.10gb": 5}, {"1g.10gb": 7},
    ],
}


def parse_profile(name: str) -> Optional[tuple]:
    m = PROFILE_RE.match(name)
    return (int(m.group(1)), int(m.group(2))) if m else None


def memory_gb(profile: str) -> int:
    p = parse_profile(profile)
    if p is None:
        raise ValueError(f"invalid MIG profile {profile!r}")
    return p[1]


def extract_profile_name(resource: str) -> Optional[str]:
    m = RESOURCE_RE.match(resource)
    return m.group(1) if m else None


def new_gpu(model: str, index: int = 0, used: Optional[Dict[str, int]] = None,
            free: Optional[Dict[str, int]] = None) -> PartitionedGPU:
    """A MIG GPU on the generic partition model (same scored search as the MI355X planner)."""
    if model not in KNOWN_GEOMETRIES:
        raise ValueError(f"unknown MIG model {model!r}")
    return PartitionedGPU(model, index, [dict(g) for g in KNOWN_GEOMETRIES[model]], dict(used or {}),
                          dict(free or {}))
