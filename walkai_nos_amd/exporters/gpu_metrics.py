"""amd-smi telemetry → Prometheus (the DCGM-exporter role for nos nodes).

The reference leaves GPU telemetry to NVIDIA's DCGM exporter; on MI355X the node agent samples
amd-smi itself (``csrc/amdsmi_backend.cpp``: GFX/UMC activity, VRAM) every ``interval`` seconds
and publishes per-GPU gauges next to the agent's own metrics:

* ``nos_amdsmi_gfx_activity_percent{node,gpu}``
* ``nos_amdsmi_vram_used_bytes{node,gpu}``
* ``nos_amdsmi_partition_info{node,gpu,compute,memory}`` = number of logical devices in that mode
  (1 for SPX ... 8 for CPX), so dashboards can join utilisation with the current partitioning;
* ``nos_amdsmi_power_watts`` / ``nos_amdsmi_power_limit_watts`` / ``nos_amdsmi_gfx_clock_mhz``: a
  fully busy MI355X is power-capped and clocks its matrix pipes down, so aggregate partition
  throughput is read against these (``profiles/kbench_r2_modes_power.json``).
"""
from __future__ import annotations

import logging
from typing import Any, Dict

from prometheus_client import Gauge

from ..models.xcp.profile import COMPUTE_MODES
from ..utils.metrics import REGISTRY

log = logging.getLogger("nos.exporters.gpu")

_partition_info = Gauge("nos_amdsmi_partition_info", "Logical devices of the GPU in its current compute mode",
                        ["node", "gpu", "compute", "memory"], registry=REGISTRY.registry)
_power = Gauge("nos_amdsmi_power_watts", "amd-smi socket power", ["node", "gpu"], registry=REGISTRY.registry)
_power_limit = Gauge("nos_amdsmi_power_limit_watts", "amd-smi socket power limit", ["node", "gpu"],
                     registry=REGISTRY.registry)
_gfx_clock = Gauge("nos_amdsmi_gfx_clock_mhz", "amd-smi current GFX clock", ["node", "gpu"], registry=REGISTRY.registry)


class GpuMetricsPoller:
    def __init__(self, smi: Any, node: str):
        self.smi, self.node = smi, node
        self._last_mode: Dict[int, tuple] = {}
        self.samples = 0

    def poll(self) -> None:
        for g in self.smi.list_gpus():
            idx = str(g.index)
            try:
                act = self.smi.activity(g.index)
                vram = self.smi.vram_usage(g.index)
                compute = self.smi.get_compute_partition(g.index)
                memory = self.smi.get_memory_partition(g.index)
            except Exception as e:  # noqa: BLE001 - a GPU mid-flip must not stop the exporter
                log.debug("amd-smi sample of GPU %s failed: %s", idx, e)
                continue
            REGISTRY.gpu_activity.labels(self.node, idx).set(float(act.get("gfx", 0.0)))
            try:
                pc = self.smi.power_clock(g.index)
            except Exception:  # noqa: BLE001 - optional telemetry
                pc = {}
            if pc:
                _power.labels(self.node, idx).set(pc.get("power_w", 0.0))
                _power_limit.labels(self.node, idx).set(pc.get("power_limit_w", 0.0))
                _gfx_clock.labels(self.node, idx).set(pc.get("gfx_mhz", 0.0))
            REGISTRY.gpu_vram_used.labels(self.node, idx).set(float(vram.get("used", 0)))
            prev = self._last_mode.get(g.index)
            if prev is not None and prev != (compute, memory):
                try:
                    _partition_info.remove(self.node, idx, *prev)
                except KeyError:
                    pass
            _partition_info.labels(self.node, idx, compute, memory).set(COMPUTE_MODES.get(compute.lower(), 1))
            self._last_mode[g.index] = (compute, memory)
        self.samples += 1

    def register(self, mgr: Any, interval: float = 15.0) -> None:
        """Run on the agent's manager (node-local: no leader election needed)."""
        mgr.add_runnable("amdsmi-metrics", self.poll, interval, needs_leader=False)
