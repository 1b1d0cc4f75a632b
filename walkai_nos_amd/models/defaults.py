"""Planner-wide model defaults, passed explicitly to every node model a planner builds.

Two partitioner settings change how a node's GPUs are modelled: ``defaultXcpLayout`` (the layout of
an ``xcp`` node without the ``nos.nebuly.com/xcp-layout`` label) and ``sharedSliceSkipCounts`` (the
memory-only slice counts a ``cumask`` GPU is never left at). They used to be module globals set once
by ``cmd/gpupartitioner.py``; any other entry point that built node models silently got the import-
time values. A :class:`ModelDefaults` is now handed to ``new_node`` / ``new_node_model`` by the
planner that owns it (``PodController``, ``NodeInitializer``, ``setup_partitioner``), so two
planners in one process — a test, the simulator, the bench — each see their own.

The library default (``ModelDefaults()``) is the reference's behaviour, hardware compute partitions
for an unlabeled node; the partitioner's config default (``GpuPartitionerConfig.defaultXcpLayout``,
``slices``) reaches the models through :meth:`ModelDefaults.from_config`.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Iterable, Tuple

#: the layouts a node may take (``models/xcp/slices.py`` LAYOUTS)
_LAYOUTS = ("partitions", "slices", "auto")


@dataclass(frozen=True)
class ModelDefaults:
    #: layout of an ``xcp`` node without the ``nos.nebuly.com/xcp-layout`` label
    xcp_layout: str = "partitions"
    #: memory-only slice counts never left on a ``cumask`` GPU (``models/slicing/profile.py``)
    shared_skip_counts: Tuple[int, ...] = (5, 7)

    def __post_init__(self) -> None:
        if self.xcp_layout not in _LAYOUTS:
            raise ValueError(f"unknown xcp layout {self.xcp_layout!r}")
        object.__setattr__(self, "shared_skip_counts", _counts(self.shared_skip_counts))

    @classmethod
    def from_config(cls, cfg: Any) -> "ModelDefaults":
        """From a ``GpuPartitionerConfig`` (``defaultXcpLayout``, ``sharedSliceSkipCounts``)."""
        return cls(xcp_layout=cfg.defaultXcpLayout, shared_skip_counts=tuple(cfg.sharedSliceSkipCounts))


def _counts(counts: Iterable[int]) -> Tuple[int, ...]:
    return tuple(sorted({int(c) for c in counts}))


LIBRARY_DEFAULTS = ModelDefaults()
