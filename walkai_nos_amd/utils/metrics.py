"""Prometheus metrics.

The reference registers **no** custom metrics (only controller-runtime's
defaults on ``127.0.0.1:8080``).  The north star asks for first-class utilisation and density
gauges, per-phase timings and probe-kernel FLOP/s per CU; they are all defined here on one
registry so every component exports the same names.
"""
from __future__ import annotations

import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Callable, Dict, Optional, Tuple

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest
from prometheus_client.exposition import CONTENT_TYPE_LATEST

_PHASE_BUCKETS = (0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30, 60)


class Metrics:
    def __init__(self, registry: Optional[CollectorRegistry] = None):
        self.registry = registry or CollectorRegistry()
        r = self.registry
        self.reconcile_total = Counter("nos_controller_reconcile_total", "Reconciles by controller and result",
                                       ["controller", "result"], registry=r)
        self.reconcile_seconds = Histogram("nos_controller_reconcile_seconds", "Reconcile latency",
                                           ["controller"], buckets=_PHASE_BUCKETS, registry=r)
        self.phase_seconds = Histogram("nos_partitioning_phase_seconds",
                                       "Per-phase partitioning latency (plan, patch, amdsmi_apply, commit_barrier, "
                                       "device_plugin_reregister)", ["phase"], buckets=_PHASE_BUCKETS, registry=r)
        self.gpu_utilization = Gauge("nos_gpu_allocated_fraction",
                                     "Fraction of each GPU's capacity allocated to running pods",
                                     ["node", "gpu"], registry=r)
        self.node_utilization = Gauge("nos_node_gpu_utilization_percent",
                                      "Aggregate allocated GPU capacity of the node in percent", ["node"], registry=r)
        self.pods_scheduled = Gauge("nos_node_fractional_pods", "Pods holding a GPU fraction on the node",
                                    ["node"], registry=r)
        self.pending_pods = Gauge("nos_pending_gpu_pods", "Unschedulable pods requesting GPU fractions", registry=r)
        self.repartitions = Counter("nos_repartitions_total", "Geometry changes written by the partitioner",
                                    ["node", "kind"], registry=r)
        self.apply_errors = Counter("nos_agent_apply_errors_total", "Failed partition apply operations",
                                    ["node", "op"], registry=r)
        self.probe_tflops_per_cu = Gauge("nos_probe_tflops_per_cu",
                                         "Achievable TFLOP/s per CU measured by the MFMA probe kernel in a slice",
                                         ["node", "gpu", "slice", "dtype"], registry=r)
        self.probe_slice_tflops = Gauge("nos_probe_slice_tflops", "Achievable TFLOP/s of a whole slice",
                                        ["node", "gpu", "slice", "dtype"], registry=r)
        self.probe_hbm_gbps = Gauge("nos_probe_hbm_gbps", "Achievable HBM GB/s measured in a slice",
                                    ["node", "gpu", "slice"], registry=r)
        self.gpu_activity = Gauge("nos_amdsmi_gfx_activity_percent", "amd-smi GFX activity", ["node", "gpu"],
                                  registry=r)
        self.gpu_vram_used = Gauge("nos_amdsmi_vram_used_bytes", "amd-smi VRAM used", ["node", "gpu"], registry=r)
        self.quota_used = Gauge("nos_elastic_quota_used", "ElasticQuota used resources",
                                ["namespace", "quota", "resource"], registry=r)
        self.preemptions = Counter("nos_scheduler_preemptions_total", "Pods preempted by capacity scheduling",
                                   registry=r)

    def render(self) -> bytes:
        return generate_latest(self.registry)


REGISTRY = Metrics()


class _Handler(BaseHTTPRequestHandler):
    routes: Dict[str, Callable[[], Tuple[int, str, bytes]]] = {}

    def do_GET(self) -> None:  # noqa: N802
        fn = self.routes.get(self.path.split("?")[0])
        if fn is None:
            code, ctype, body = 404, "text/plain", b"not found"
        else:
            code, ctype, body = fn()
        self.send_response(code)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def log_message(self, *args: object) -> None:  # silence
        return


def serve(bind: str, routes: Dict[str, Callable[[], Tuple[int, str, bytes]]]) -> ThreadingHTTPServer:
    """Serve ``routes`` on ``host:port`` in a daemon thread (health probes and /metrics)."""
    host, _, port = bind.rpartition(":")
    handler = type("H", (_Handler,), {"routes": routes})
    srv = ThreadingHTTPServer((host or "0.0.0.0", int(port)), handler)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv


def metrics_route(m: Metrics) -> Callable[[], Tuple[int, str, bytes]]:
    return lambda: (200, CONTENT_TYPE_LATEST, m.render())


def check_route(fn: Callable[[], bool]) -> Callable[[], Tuple[int, str, bytes]]:
    return lambda: (200, "text/plain", b"ok") if fn() else (500, "text/plain", b"unhealthy")
