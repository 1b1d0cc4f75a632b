"""Desired partitioning state (reference ``internal/partitioning/state/partitioning.go:24-56``)."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..utils.util import unordered_equal


@dataclass
class GPUPartitioning:
    gpu_index: int
    resources: Dict[str, int] = field(default_factory=dict)  # resource name -> quantity
    #: MI355X: served as CU-mask slices of an SPX GPU (models/xcp/slices.py)
    sliced: bool = False

    def canonical(self) -> str:
        return f"{self.gpu_index}|" + ",".join(f"{k}={v}" for k, v in sorted(self.resources.items())) + \
            ("|sliced" if self.sliced else "")


@dataclass
class NodePartitioning:
    gpus: List[GPUPartitioning] = field(default_factory=list)
    #: MI355X: desired node-wide memory partition mode (None = leave unchanged)
    memory_partition: Optional[str] = None

    def equal(self, other: "NodePartitioning") -> bool:
        return self.memory_partition == other.memory_partition and unordered_equal(self.gpus, other.gpus)


PartitioningState = Dict[str, NodePartitioning]


def states_equal(a: PartitioningState, b: PartitioningState) -> bool:
    if set(a) != set(b):
        return False
    return all(a[k].equal(b[k]) for k in a)
