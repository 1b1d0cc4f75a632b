"""Install-time telemetry exporter (reference ``cmd/metricsexporter/{metricsexporter.go,metrics/metrics.go}``).

A Helm post-install/upgrade job reads a YAML metrics file (rendered by the chart from a ``lookup``
of every Node, keeping only ``amd.com*`` and ``node.kubernetes.io/instance-type`` labels) and POSTs
it as JSON.  Every failure exits 0 so telemetry can never fail an installation.

Payload: ``{"installationUUID", "nodes": [{"name", "capacity", "labels", "nodeInfo"}],
"chartValues", "components": {"nosGpuPartitioner", "nosScheduler", "nosOperator"}}`` (Appendix A.6).
"""
from __future__ import annotations

import json
import logging
import sys
from dataclasses import asdict, dataclass, field
from typing import Any, Callable, Dict, List, Optional

import yaml

log = logging.getLogger("nos.telemetry")


@dataclass
class NodeMetrics:
    name: str = ""
    capacity: Dict[str, Any] = field(default_factory=dict)
    labels: Dict[str, str] = field(default_factory=dict)
    nodeInfo: Dict[str, Any] = field(default_factory=dict)
    #: MI355X: the node's probe-on-commit summary (bf16 TFLOP/s per CU of each partition or slice,
    #: degraded targets) from the agent's ``status-probe`` annotation
    probe: Dict[str, Any] = field(default_factory=dict)


def probe_digest(raw: Any) -> Dict[str, Any]:
    """``status-probe`` JSON -> {targets, bf16_tflops, bf16_tflops_per_cu (min/max), degraded}."""
    try:
        doc = json.loads(raw) if isinstance(raw, str) else (raw or {})
    except ValueError:
        return {}
    rows = [r for r in (doc.get("slices") or {}).values() if isinstance(r, dict) and "bf16_tflops" in r]
    if not rows:
        return {}
    per_cu = [r["bf16_tflops"] / max(1, int(r.get("n_cus", 1))) for r in rows]
    return {"targets": len(rows), "bf16_tflops": round(sum(r["bf16_tflops"] for r in rows), 1),
            "bf16_tflops_per_cu_min": round(min(per_cu), 3), "bf16_tflops_per_cu_max": round(max(per_cu), 3),
            "degraded": sorted(str(r["degraded"]) for r in rows if r.get("degraded"))}


@dataclass
class Components:
    nosGpuPartitioner: bool = False
    nosScheduler: bool = False
    nosOperator: bool = False


@dataclass
class Metrics:
    installationUUID: str = ""
    nodes: List[NodeMetrics] = field(default_factory=list)
    chartValues: Any = None
    components: Components = field(default_factory=Components)

    @staticmethod
    def from_yaml(text: str) -> "Metrics":
        doc = yaml.safe_load(text) or {}
        nodes = []
        for n in doc.get("nodes") or []:
            n = dict(n or {})
            if "probe" in n:
                n["probe"] = probe_digest(n["probe"])
            nodes.append(NodeMetrics(**{k: v for k, v in n.items() if k in NodeMetrics.__dataclass_fields__}))
        comps = Components(**{k: bool(v) for k, v in (doc.get("components") or {}).items()
                              if k in Components.__dataclass_fields__})
        return Metrics(str(doc.get("installationUUID", "")), nodes, doc.get("chartValues"), comps)

    def to_json(self) -> str:
        return json.dumps(asdict(self))


def filter_labels(labels: Dict[str, str]) -> Dict[str, str]:
    return {k: v for k, v in (labels or {}).items()
            if k.startswith("amd.com") or k == "node.kubernetes.io/instance-type"}


def run(metrics_file: str, endpoint: str, post: Optional[Callable[[str, bytes], int]] = None) -> int:
    """Returns the process exit code — always 0."""
    try:
        with open(metrics_file) as f:
            m = Metrics.from_yaml(f.read())
    except Exception as e:  # noqa: BLE001
        log.error("unable to read metrics file %s: %s", metrics_file, e)
        return 0
    try:
        if post is None:
            from .clusterinfo import _http_post
            code = _http_post(endpoint, m.to_json().encode(), {"Content-Type": "application/json"}, 10.0)
        else:
            code = post(endpoint, m.to_json().encode())
        if code >= 300:
            log.error("telemetry endpoint returned %d", code)
    except Exception as e:  # noqa: BLE001
        log.error("unable to send telemetry: %s", e)
    return 0


if __name__ == "__main__":
    sys.exit(run(sys.argv[1], sys.argv[2]))
