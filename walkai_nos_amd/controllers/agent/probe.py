"""Probe-on-commit: measure what every new partition can actually deliver.

After each successful node commit (``SharedState.commit_seq`` advances) the agent runs the HIP
probe kernels (``csrc/probe.hip``) on every logical device the node now exposes — bf16 and fp32
MFMA throughput and HBM copy bandwidth — in a spawned helper process (``cmd/gpuhelper.py``: the
agent itself never initialises HIP, and the helper is stopped before the next flip), from a
background thread, and publishes the result as the
``nos.nebuly.com/status-probe`` node annotation (through the reporter's extra-annotation hook) and
as Prometheus gauges (``nos_probe_slice_tflops``, ``nos_probe_tflops_per_cu``,
``nos_probe_hbm_gbps``). This is the MI355X addition to the reference's status protocol
(SURVEY §2.M item 1): a scheduler or an operator can see that a CPX partition really delivers
1/8 of the chip, and a degraded partition shows up as an outlier instead of a silent slowdown.

For CU-mask slices the runner probes each slice's CU set on a CU-masked stream of the physical GPU.
"""
from __future__ import annotations

import logging
import threading
import time
from typing import Any, Callable, Dict, List, Optional

from ...utils.metrics import REGISTRY
from .reporter import probe_annotation
from .shared import SharedState

log = logging.getLogger("nos.agent.probe")

#: (device index, optional CU list, label) -> {"bf16": tflops, "fp32": tflops, "hbm_gbps": ..., "n_cus": ...}
ProbeFn = Callable[[int, Optional[List[int]], str], Dict[str, float]]
TargetsFn = Callable[[], List[tuple]]


def hip_probe(device: int, cus: Optional[List[int]], label: str) -> Dict[str, float]:
    """Real probe on the GPU: short MFMA runs (bf16, fp32) and a 256 MiB HBM copy."""
    from ...ops import probe as P
    with P.Stream(device, cus) as s:
        bf = P.probe_mfma("bf16", device, s, iters=1024, reps=2)
        f32 = P.probe_mfma("fp32", device, s, iters=512, reps=2)
        hbm = P.probe_hbm(device, s, nbytes=1 << 28, reps=2)
    return {"n_cus": bf.n_cus, "bf16_tflops": round(bf.tflops, 1), "fp32_tflops": round(f32.tflops, 2),
            "hbm_gbps": round(float(hbm.get("gbps", 0.0)), 0)}


def device_map_targets(smi: Any) -> TargetsFn:
    """Every logical device of the node's current device map, labelled ``gpu<i>.p<k>``; the
    device index is the HIP ordinal a freshly spawned helper sees for it."""
    def targets() -> List[tuple]:
        return [(d.hip_id, None, f"gpu{d.gpu_index}.p{d.partition_index}")
                for d in sorted(smi.logical_devices(), key=lambda d: d.hip_id) if d.hip_id >= 0]
    return targets


#: targets -> {label: result}; the default runs them all in one spawned helper process
RoundFn = Callable[[List[tuple]], Dict[str, Any]]


def spawned_round(registry: Any = None, backend: str = "hip") -> RoundFn:
    from ...parallel.spawned import spawned_probe_round
    return lambda targets: spawned_probe_round(targets, backend=backend, registry=registry)


class ProbeRunner:
    """``round_fn`` (default for agents: a spawned helper, so the agent never holds a GPU context)
    probes all targets of one commit; ``probe_fn`` is the in-process per-target alternative used
    by the GPU tests."""

    def __init__(self, shared: SharedState, node_name: str, probe_fn: Optional[ProbeFn] = None,
                 targets: Optional[TargetsFn] = None, asynchronous: bool = True,
                 round_fn: Optional[RoundFn] = None):
        self.shared, self.node = shared, node_name
        if probe_fn is None and round_fn is None:
            round_fn = spawned_round(shared.helpers)
        if targets is None:
            raise ValueError("ProbeRunner needs a targets function (e.g. device_map_targets(smi))")
        self.probe_fn, self.round_fn, self.targets = probe_fn, round_fn, targets
        self.asynchronous = asynchronous
        self._seen = -1
        self._lock = threading.Lock()
        self._running = False
        self.results: Dict[str, Any] = {}

    def poll(self) -> None:
        """Start a probe round if a new commit happened since the last one."""
        with self._lock:
            seq = self.shared.commit_seq
            if seq == self._seen or self._running:
                return
            self._seen, self._running = seq, True
        if self.asynchronous:
            threading.Thread(target=self._run, args=(seq,), name="nos-probe", daemon=True).start()
        else:
            self._run(seq)

    def _run(self, seq: int) -> None:
        t0 = time.time()
        out: Dict[str, Any] = {}
        try:
            targets = list(self.targets())
            batch: Dict[str, Any] = {}
            if self.round_fn is not None:
                try:
                    batch = self.round_fn(targets)
                except Exception as e:  # noqa: BLE001 - a failed helper is reported, not raised
                    log.warning("probe round failed: %s", e)
                    batch = {label: {"error": str(e)[:200]} for _, _, label in targets}
            for dev, cus, label in targets:
                if self.round_fn is not None:
                    r = batch.get(label, {"error": "no result"})
                else:
                    try:
                        r = self.probe_fn(dev, cus, label)
                    except Exception as e:  # noqa: BLE001 - one bad partition must not hide the others
                        r = {"error": str(e)[:200]}
                out[label] = r
                if "error" in r:
                    log.warning("probe of %s failed: %s", label, r["error"])
                    continue
                n = max(1, int(r.get("n_cus", 1)))
                for dt in ("bf16", "fp32"):
                    if f"{dt}_tflops" in r:
                        REGISTRY.probe_slice_tflops.labels(self.node, str(dev), label, dt).set(r[f"{dt}_tflops"])
                        REGISTRY.probe_tflops_per_cu.labels(self.node, str(dev), label, dt).set(r[f"{dt}_tflops"] / n)
                if "hbm_gbps" in r:
                    REGISTRY.probe_hbm_gbps.labels(self.node, str(dev), label).set(r["hbm_gbps"])
        finally:
            with self._lock:
                self.results = {"commit": seq, "at": int(t0), "slices": out}
                self._running = False
        log.info("probe after commit %d: %s", seq, out)

    def annotations(self) -> Dict[str, str]:
        """Reporter extra-annotation hook: kick a probe round if needed, publish the latest."""
        self.poll()
        with self._lock:
            return probe_annotation(self.results) if self.results else {}
