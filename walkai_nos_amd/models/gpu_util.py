"""Node-label helpers (reference ``pkg/gpu/util.go:30-89``), AMD node-labeller flavoured.

``GetMemoryGB`` in the reference divides the NVIDIA MB label by 1000 with ceil; the
AMD labeller publishes VRAM with a unit suffix (``288G``), parsed here with its own units.
"""
from __future__ import annotations

import math
import re
from typing import Any, Dict, Optional

from .. import constant
from ..api import v1alpha1 as api
from ..kube import objects as ko
from .xcp.known_configs import get_model_spec


def get_model(node: Dict[str, Any]) -> str:
    v = ko.labels(node).get(constant.LABEL_AMD_GPU_PRODUCT)
    if not v:
        raise ValueError(f"cannot get GPU model: missing label {constant.LABEL_AMD_GPU_PRODUCT}")
    return v


def get_count(node: Dict[str, Any]) -> int:
    v = ko.labels(node).get(constant.LABEL_AMD_GPU_COUNT)
    if v is None:
        raise ValueError(f"cannot get GPU count: missing label {constant.LABEL_AMD_GPU_COUNT}")
    try:
        n = int(v)
    except ValueError as e:
        raise ValueError(f"cannot get GPU count: invalid label value {v!r}") from e
    if n < 0:
        raise ValueError("GPU count cannot be negative")
    return n


_VRAM_RE = re.compile(r"^\s*(\d+(?:\.\d+)?)\s*([KMGT]i?B?|[KMGT])?\s*$", re.I)


def parse_vram_gb(v: str) -> int:
    m = _VRAM_RE.match(v)
    if not m:
        raise ValueError(f"invalid VRAM label {v!r}")
    num = float(m.group(1))
    unit = (m.group(2) or "M").upper().rstrip("B")
    scale = {"K": 1e-6, "M": 1e-3, "G": 1.0, "T": 1e3, "KI": 1e-6, "MI": 1e-3, "GI": 1.0, "TI": 1e3}[unit]
    return int(math.ceil(num * scale - 1e-9))


def get_memory_gb(node: Dict[str, Any]) -> int:
    v = ko.labels(node).get(constant.LABEL_AMD_GPU_VRAM)
    if v:
        return parse_vram_gb(v)
    spec = get_model_spec(get_model(node))
    if spec is None:
        raise ValueError(f"cannot get GPU memory: missing label {constant.LABEL_AMD_GPU_VRAM} and unknown model")
    return spec.memory_gb


def get_cu_count(node: Dict[str, Any]) -> int:
    v = ko.labels(node).get(constant.LABEL_AMD_GPU_CU_COUNT)
    if v:
        return int(v)
    spec = get_model_spec(get_model(node))
    if spec is None:
        raise ValueError(f"cannot get CU count: missing label {constant.LABEL_AMD_GPU_CU_COUNT} and unknown model")
    return spec.compute_units


def get_memory_partition(node: Dict[str, Any]) -> str:
    """Observed NPS mode: agent status annotation, then labeller label, else ``nps1``."""
    ann = ko.annotations(node).get(api.ANNOTATION_MEMORY_PARTITION_STATUS)
    if ann:
        return ann.lower()
    lbl = ko.labels(node).get(constant.LABEL_AMD_MEMORY_PARTITION)
    if lbl:
        return lbl.lower()
    return "nps1"


def get_spec_memory_partition(node: Dict[str, Any]) -> Optional[str]:
    v = ko.annotations(node).get(api.ANNOTATION_MEMORY_PARTITION_SPEC)
    return v.lower() if v else None
