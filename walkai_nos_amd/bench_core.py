"""Fractional-GPU serving benchmark: the control plane and the GPU data plane in one loop.

Headline metric (BASELINE.json): *aggregate GPU utilization % + schedulable pods/node under a
mixed fractional-GPU load*, on the workload the reference publishes numbers for (YOLOS-small
batch-1 inference pods, ``demos/gpu-sharing-comparison``).  ``value`` is the aggregate inference
rate the node sustains; allocation %, pods/node and per-profile service are reported next to it.

**Time model: a compressed replay of cluster time.**  One *quantum* = ``cluster_s`` (60) seconds
of cluster time, replayed in ``quantum_s`` (0.5) wall seconds of GPU serving; one driver step =
``quanta_per_step`` (2) quanta, so the driver's 20 timed steps span 40 quanta = 10 mean pod
lifetimes (a 20-quantum window's allocation varies with the churn seed by sd 5.9 points, a
40-quantum one by 3.2: ``profiles/window_length_r5.json``).  Every cluster-time duration is
compressed by the same factor — pod lifetimes (2-6 quanta), the planner's thresholds and every
compute-partition flip's outage — while the GPU serves at its real rate, so inferences per wall
second of the replay equal inferences per second of the cluster.  Per quantum:

1. churn: pods whose served lifetime is over finish, new pods arrive (seeded Poisson arrivals at
   ``offered_load`` GPUs of demand per GPU; profiles 1/8, 1/2 and 1/1 GPU = ``amd.com/cpx_nps1``,
   ``dpx_nps1``, ``spx_nps1`` drawn 50/30/20 in seeded stratified blocks);
2. the *real* control plane runs for ``cluster_s`` on the virtual clock against the in-memory API
   server: the partitioner (flip-aware ``pack`` policy), per node the partition agent (reporter,
   actuator, commit barrier — RCCL across the bench's ranks) and the **nos partition device
   plugin** whose health rule enforces drains (every partition of a GPU being re-partitioned is
   Unhealthy, ``deviceplugin/partitions.py``), a kubelet that admits pods onto healthy devices
   only, and a scheduler with kube-scheduler semantics (node allocatable minus requests; it knows
   nothing about GPUs);
3. **every flip is charged**: the flipped GPU serves nothing for ``flip_cost_s`` of cluster time
   (the measured commit barrier + the amd-smi mode switch + the plugin's pushed update + the
   probe round: :data:`FLIP_COST_COMPONENTS`); the dark part of a quantum is idle wall time in the
   replay, pods on the GPU neither serve nor age meanwhile;
4. for the rest of the quantum every running pod on this rank's GPU runs the reference demo's
   loop: one YOLOS-small inference (fp32-accurate, batch 1, 800x1066; a HIP graph replay on a
   stream whose CU mask is the partition's CU set) after another.

Because the box is not root, compute-partition modes cannot be flipped on the real device; a
CPX/QPX/DPX partition is emulated by an XCD-symmetric CU mask of the same CU count (32/64/128
CUs; mask bit i -> XCD i mod 8, and an XCD whose mask bits are all zero is NOT disabled, so every
slice must span all eight XCDs). An XCD-pinned emulation (``--emulation pinned``, ``csrc/pin.h``)
gives each partition its own XCDs like real hardware, but its exit-only workgroups on the other
XCDs couple the partitions (see EMULATION). Mode changes go through the fake amd-smi backend
(whose device map re-enumerates like the real one); everything else — kernels, streams,
collectives — is real.

After the timed window a **density** phase saturates the node through the same control plane and
data plane: 8 CPX pods per GPU (the reference's MIG maximum is 7 per A100), then a CU-mask node
with dedicated-CU and memory-only slices beyond 8 per GPU.  It is reported, never timed.
"""
from __future__ import annotations

import collections
import json
import math
import os
import random
import threading
import time
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

from .kube import objects as ko
from .models.xcp.profile import COMPUTE_MODES, extract_profile_name
from .models.xcp.slices import slice_groups

# reference numbers: 1x A100-80GB PCIe, 7 pods, MPS 10 GB slices
BASELINE_INFER_PER_S_PER_GPU = 21.89
BASELINE_LABEL = "MPS 7-pod aggregate throughput on 1x A100-80GB (BASELINE.md), scaled by n_gpus"

MIX = (("cpx_nps1", 0.5), ("dpx_nps1", 0.3), ("spx_nps1", 0.2))

#: CU-mask density phases: dedicated-CU slices plus memory-only slices on the shared rows, and
#: memory-only slices alone (the reference's MPS semantics: HBM budgets, compute shared by all) —
#: name -> (per-GPU mix, the node's nos.nebuly.com/max-slices-per-gpu or None for the chart default
#: of 8). The default-cap rows are what a default-configured node schedules; the *_threads_cap_lifted
#: rows lift the cap to 16 by label and serve the pods as threads of the bench process — as
#: processes, past eight per GPU the hardware scheduler time-slices them (profiles/procs_cap_r4.json:
#: 12 memory-only pods 292 inf/s against 383 at 8), so they are never a saturation figure
CUMASK_DENSITY = {"cumask": ((("32cu.24gb", 4), ("8gb", 4)), None),
                  "cumask_shared": ((("16gb", 8),), None),
                  "cumask_threads_cap_lifted": ((("32cu.24gb", 6), ("8gb", 10)), 16),
                  "cumask_shared_threads_cap_lifted": ((("16gb", 16),), 16)}


#: How a compute partition is emulated on the SPX device (the box is not root, so modes cannot be
#: flipped): "spread" — an XCD-symmetric CU mask of the partition's CU count over all eight XCDs;
#: "pinned" — the partition's kernels run only on its own XCDs (CPX partition k = XCD k, QPX k = XCDs
#: 2k..2k+1, DPX k = XCDs 4k..4k+3; ``csrc/pin.h``), the layout a real partition has. Pinned is
#: correct (tests/test_gpu_pin.py) but cannot stand in for real partitions: every pinned launch also
#: dispatches exit-only workgroups to the other XCDs, which need a free slot there, so a partition's
#: kernel waits on its neighbours' workgroups — 8 busy CPX partitions run at 253 inf/s pinned vs 375
#: spread, while one partition alone runs 16.1 vs 14.8 ms per inference
#: (profiles/partition_emulation_r2.json). ``NOS_PARTITION_EMULATION`` overrides.
EMULATION = os.environ.get("NOS_PARTITION_EMULATION", "spread")
#: why a GPU's capacity went unallocated in a quantum (``NodeBench._account_idle``)
IDLE_CAUSES = ("flip_outage", "drain", "fragmentation", "placement_lag", "no_demand")
XCDS = 8
#: emulations whose partitions run on their own XCDs (kernels pinned with ``csrc/pin.h``). "landing":
#: pinned, and the CU mask gives a partition its own XCDs minus one CU per XCD plus that reserved
#: "landing" CU on every other XCD, so the launch's exit-only workgroups never wait for a slot behind
#: the other partitions' real work (the coupling that made "pinned" slow); 31 of 32 CUs per XCD work.
PINNED_EMULATIONS = ("pinned", "landing")


def working_cus(cus: Optional[List[int]], pin: int, total_cus: int = 256) -> int:
    """CUs that run a slice's real work: every masked CU, or under a pin only those on its XCDs."""
    if cus is None:
        return total_cus
    if not pin:
        return len(cus)
    return sum(1 for c in cus if (pin >> (c % XCDS)) & 1)


#: One compute-partition flip, in cluster seconds, from its measured parts.  The GPU serves nothing
#: from the amd-smi switch until the agent has committed and its pods can start:
#:
#: * ``commit_barrier_s`` — the node-atomic commit: the native helper's wall time (spawn, hipInit,
#:   the xGMI P2P token ring, exit), warm median 0.33 s (profiles/operator_gpu_report_r3.json; the
#:   RCCL communicator variant takes 2.9-3.4 s, almost all of it ncclCommInitAll + destroy);
#: * ``probe_s`` — the probe-on-commit round after the flip (profiles/operator_gpu_report_r2.json);
#: * ``plugin_push_s`` — the nos partition plugin's ListAndWatch push + allocatable patch (no plugin
#:   restart; the reference waits up to 60 s for the NVIDIA plugin pod, ref pkg/gpu/client.go:86-135);
#: * ``amdsmi_switch_s`` — the amd-smi compute-partition switch itself: NOT measurable here (the box
#:   is not root, so the setter returns AMDSMI_STATUS_PERMISSION); 10 s is an estimate covering the
#:   driver re-creating the partitions and the re-enumeration, flagged as such in BENCH.
#:
#: ``--flip-cost`` overrides the total; BENCH also reports the control plane's sensitivity to it.
FLIP_COST_COMPONENTS = {"commit_barrier_s": 0.33, "probe_s": 0.39, "plugin_push_s": 0.05, "amdsmi_switch_s": 10.0}
FLIP_COST_MEASURED = ("commit_barrier_s", "probe_s", "plugin_push_s")

#: A new pod's start-up: from its process starting (kubelet has admitted it and holds its slice) to
#: its first inference — interpreter + torch import, model load, warm-up and HIP-graph capture of the
#: reference demo's client (``dataplane/client.py``), spawned with ``Allocate``'s environment. The
#: slice is allocated but serves nothing meanwhile: every pod bound in the window spends this much of
#: its lifetime (cluster time) starting before it serves (``bench.py`` measures it on the box before
#: the window, :func:`measure_pod_start`; this is the fallback).
POD_START_S = 8.0


def default_flip_cost(commit_barrier_s: Optional[float] = None) -> float:
    """The flip outage from its components, with this run's measured commit barrier if given."""
    parts = dict(FLIP_COST_COMPONENTS)
    if commit_barrier_s is not None and commit_barrier_s >= 0:
        parts["commit_barrier_s"] = commit_barrier_s
    return round(sum(parts.values()), 3)


@dataclass
class BenchConfig:
    gpus: int = 1
    steps: int = 20
    warmup: int = 5
    seed: int = 1234
    offered_load: float = 1.0            # offered GPU-equivalents per GPU (= capacity)
    quantum_s: float = 0.5               # wall seconds of serving per quantum
    cluster_s: float = 60.0              # cluster seconds one quantum stands for (the replay's compression)
    quanta_per_step: int = 2             # quanta per driver step (window = steps x this many quanta)
    flip_cost_s: float = -1.0            # cluster seconds a GPU is dark per flip (<0: FLIP_COST_COMPONENTS)
    lifetime: Tuple[int, int] = (2, 6)   # served quanta per pod (uniform, stratified): mean 4 = 10 in 20 steps
    hw: Tuple[int, int] = (800, 1066)
    backend: str = "hip"
    graphs: bool = True
    depth: int = 1                       # inferences in flight per pod stream (1 = the reference's loop)
    pod_streams: int = 1                 # concurrent request streams per pod (1 = the reference demo's loop)
    lane_cus: int = 0                    # >0: a partition pod wider than this serves on disjoint CU runs of
                                         # this many CUs, one batch-1 request loop per run (0 = one loop)
    preroll: int = 60                    # control-plane-only steps before warmup (steady state)
    rank: int = 0
    world: int = 1
    policy: str = "pack"                 # planner policy (pack | fifo | batch | simulate)
    density: bool = True
    emulation: str = EMULATION           # compute-partition emulation: pinned | spread
    nodes: int = 1                       # cluster nodes of `gpus` GPUs (control-plane simulation only)
    device_plugin: str = "nos"           # nos (drain enforced by device health) | amd (no drain enforcement)
    pack: Optional[Dict[str, float]] = None  # PackParams overrides (field name -> value)
    arrivals: str = "steady"             # steady (constant rate, seeded phase) | poisson
    layout: str = "partitions"           # node label nos.nebuly.com/xcp-layout: partitions | slices | auto
    data_plane: bool = True              # False: a rehearsal of the launch path without a GPU (inferences
                                         # priced with MODE_RATES, never a measurement)
    commit_barrier_s: float = -1.0       # this run's measured node commit barrier (<0: the component constant)
    partitions_window: bool = True       # also time the same window on hardware partitions (config 4)
    pod_start_s: float = -1.0            # cluster seconds a newly bound pod holds its slice before it serves
                                         # (<0: POD_START_S; bench.py measures it on the box before the window)
    declared_bound_quanta: float = 0.0   # >0: every pod declares spec.activeDeadlineSeconds = this many quanta
                                         # (plus its start-up), no tighter than the churn's longest lifetime

    def __post_init__(self) -> None:
        #: the flip cost is the components' sum (so a measured commit barrier replaces its constant)
        self.flip_cost_default = self.flip_cost_s < 0
        if self.flip_cost_s < 0:
            self.flip_cost_s = default_flip_cost(self.commit_barrier_s)
        self.pod_start_default = self.pod_start_s < 0
        if self.pod_start_s < 0:
            self.pod_start_s = POD_START_S

    @property
    def pod_start_quanta(self) -> float:
        """A new pod's start-up (process start to first inference) in quanta."""
        return self.pod_start_s / self.cluster_s

    @property
    def flip_quanta(self) -> float:
        """A flip's outage in quanta (fractional)."""
        return self.flip_cost_s / self.cluster_s

    @property
    def warmup_quanta(self) -> int:
        return self.warmup * self.quanta_per_step

    @property
    def window_quanta(self) -> int:
        return self.steps * self.quanta_per_step

    @property
    def mean_lifetime_quanta(self) -> float:
        return (self.lifetime[0] + self.lifetime[1]) / 2


class ChurnProcess:
    """Deterministic pod arrival process (identical on every rank): Poisson arrivals at the offered
    load; profiles and lifetimes drawn from seeded shuffles of stratified blocks (every block of 10
    arrivals holds the 50/30/20 mix exactly, every block of lifetimes each value once), so a short
    window sees the mix it is configured with."""

    def __init__(self, cfg: BenchConfig):
        self.cfg = cfg
        self.rng = random.Random(cfg.seed)
        self.seq = 0
        mean_frac = sum((1.0 / COMPUTE_MODES[p.split("_")[0]]) * w for p, w in MIX)
        self.rate = cfg.offered_load * cfg.gpus * cfg.nodes / (mean_frac * cfg.mean_lifetime_quanta)
        self._profiles: List[str] = []
        self._lifetimes: List[int] = []
        self._acc: Optional[float] = None

    def _next_profile(self) -> str:
        if not self._profiles:
            block = [p for p, w in MIX for _ in range(int(round(10 * w)))]
            self.rng.shuffle(block)
            self._profiles = block
        return self._profiles.pop()

    def arrivals(self) -> List[str]:
        if self.cfg.arrivals == "poisson":
            # Poisson(rate) via inversion, seeded
            n, p, L = 0, 1.0, math.exp(-self.rate)
            while True:
                p *= self.rng.random()
                if p <= L:
                    break
                n += 1
        else:
            # constant rate (a load generator submitting pods at a steady pace), seeded phase
            if self._acc is None:
                self._acc = self.rng.random()
            self._acc += self.rate
            n = int(self._acc)
            self._acc -= n
        return [self._next_profile() for _ in range(n)]

    def lifetime(self) -> int:
        if not self._lifetimes:
            block = list(range(self.cfg.lifetime[0], self.cfg.lifetime[1] + 1))
            self.rng.shuffle(block)
            self._lifetimes = block
        return self._lifetimes.pop()


def partition_xcds(profile: str, partition: int) -> Optional[List[int]]:
    """The XCDs of compute partition ``partition`` of ``profile`` (None = the whole GPU)."""
    n = COMPUTE_MODES[profile.split("_")[0]]
    if n == 1:
        return None
    per = XCDS // n
    return list(range(partition * per, (partition + 1) * per))


def slice_pin(profile: str, partition: int, emulation: Optional[str] = None) -> int:
    """XCD mask the partition's kernels are pinned to (0 = unpinned: SPX, or the spread emulation)."""
    xcds = partition_xcds(profile, partition)
    if xcds is None or (emulation or EMULATION) not in PINNED_EMULATIONS:
        return 0
    return sum(1 << x for x in xcds)


def slice_cus(profile: str, partition: int, total_cus: int = 256,
              emulation: Optional[str] = None) -> Optional[List[int]]:
    """CU-mask bits (bit i -> XCD i mod 8) of compute partition ``partition`` of ``profile``.
    pinned: every CU of the partition's XCDs; spread: a contiguous run of total/partitions bits, i.e.
    that many CUs spread evenly over all XCDs."""
    n = COMPUTE_MODES[profile.split("_")[0]]
    if n == 1:
        return None
    emulation = emulation or EMULATION
    if emulation == "pinned":
        xcds = set(partition_xcds(profile, partition))
        return [i for i in range(total_cus) if i % XCDS in xcds]
    if emulation == "landing":
        # own XCDs minus their landing CU, plus the landing CU of every other XCD: a pinned launch's
        # exit-only workgroups on a foreign XCD can only be placed on that XCD's landing CU, which
        # no partition runs real work on (an all-zero XCD in a CU mask would enable the whole XCD)
        xcds = set(partition_xcds(profile, partition))
        land = total_cus // XCDS - 1
        return [i for i in range(total_cus)
                if (i % XCDS in xcds and i // XCDS != land) or (i % XCDS not in xcds and i // XCDS == land)]
    per = total_cus // n
    return list(range(partition * per, (partition + 1) * per))


def lane_cu_runs(cus: Optional[List[int]], lane_cus: int, total_cus: int = 256) -> List[Optional[List[int]]]:
    """Split a partition's CUs into request lanes of ``lane_cus`` CUs each (disjoint, contiguous runs
    of the partition's CU bits; bit i sits on XCD i mod 8, so a run of a multiple of 8 bits is
    XCD-balanced).  A batch-1 YOLOS inference does not fill a whole MI355X — its attention tail,
    LayerNorms and heads leave CUs idle — while inferences on disjoint quarters keep every CU busy
    (profiles/kbench_r2_modes_tiles256.json: one loop on the whole GPU 358, four 64-CU partitions
    440 inf/s per GPU; profiles/bench_r2_lane_width_ab.json: 64- vs 128-CU lanes).  ``lane_cus``
    <= 0, or a partition not wider than it, gives one lane on the whole partition."""
    all_cus = list(range(total_cus)) if cus is None else list(cus)
    if lane_cus <= 0 or len(all_cus) <= lane_cus or len(all_cus) % lane_cus or lane_cus % XCDS:
        return [cus]
    return [all_cus[i:i + lane_cus] for i in range(0, len(all_cus), lane_cus)]


class _Lane:
    """One stream of a pod: a CU-masked HIP stream, an input, and the inference graph captured on it."""

    def __init__(self, cus: Optional[List[int]], device: int, cfg: "BenchConfig", seed: int, pin: int = 0):
        import torch

        from .models.workload.yolos import demo_input
        from .ops.probe import Stream
        self.n_cus = working_cus(cus, pin)
        self.hip_stream = Stream(device, cus)
        self.stream = self.hip_stream.torch_stream()
        with torch.cuda.stream(self.stream):
            self.x = demo_input(1, cfg.hw, f"cuda:{device}", seed=seed)
        self.graph = None
        self.out = None
        self.inflight: collections.deque = collections.deque()

    def close(self) -> None:
        self.inflight.clear()
        self.graph = None
        self.x = None
        self.out = None
        self.stream = None
        if self.hip_stream is not None:
            self.hip_stream.close()
            self.hip_stream = None


class Slot:
    """One partition (or CU-mask slice) of this rank's GPU: a model replica serving
    ``cfg.pod_streams`` concurrent request streams (lanes) per CU run (``lane_cu_runs``; one run
    unless ``split`` and ``cfg.lane_cus``), each a CU-masked stream with its own input and captured
    graph; an inference is one HIP graph replay on the least-loaded lane."""

    def __init__(self, cus: Optional[List[int]], device: int, cfg: BenchConfig, template: Any, seed: int = 0,
                 pin: int = 0, split: bool = False):
        import copy

        import torch

        self.cus = cus
        self.pin = pin
        self.cfg = cfg
        runs = lane_cu_runs(cus, cfg.lane_cus) if split and not pin else [cus]
        self.lanes = [_Lane(run, device, cfg, seed + 1000 * i + 100 * j, pin)
                      for j, run in enumerate(runs) for i in range(max(1, cfg.pod_streams))]
        self.latency_ms: List[float] = []  # GPU time of each completed inference (its lane's events)
        with torch.cuda.stream(self.lanes[0].stream):
            self.model = copy.deepcopy(template).to(f"cuda:{device}").eval()
        torch.cuda.synchronize()

    @property
    def n_cus(self) -> int:
        return working_cus(self.cus, self.pin)

    @property
    def stream(self):
        return self.lanes[0].stream if self.lanes else None

    @property
    def in_flight(self) -> int:
        return sum(len(l.inflight) for l in self.lanes)

    @property
    def capacity(self) -> int:
        """Inferences this pod keeps in flight: ``depth`` per lane."""
        return self.cfg.depth * len(self.lanes)

    def warm(self) -> None:
        import torch

        from .ops import kernels as K
        K.set_slice_pin(self.pin)
        for lane in self.lanes:
            K.set_slice_cus(lane.n_cus)
            with torch.no_grad(), torch.cuda.stream(lane.stream):
                for _ in range(2):
                    lane.out = self.model(lane.x)
            lane.stream.synchronize()
            if self.cfg.graphs:
                g = torch.cuda.CUDAGraph()
                with torch.no_grad():
                    with torch.cuda.graph(g, stream=lane.stream):
                        lane.out = self.model(lane.x)
                lane.stream.synchronize()
                lane.graph = g

    def submit(self) -> None:
        """Enqueue one inference on the lane with the fewest in flight, and an event marking its end."""
        import torch

        from .ops import kernels as K
        lane = min(self.lanes, key=lambda l: len(l.inflight))
        K.set_slice_cus(lane.n_cus)
        K.set_slice_pin(self.pin)
        with torch.no_grad(), torch.cuda.stream(lane.stream):
            st = torch.cuda.Event(enable_timing=True)
            st.record(lane.stream)  # runs when the lane's previous inference has finished
            if lane.graph is not None:
                lane.graph.replay()
            else:
                lane.out = self.model(lane.x)
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(lane.stream)
        lane.inflight.append((st, ev))

    def _done(self, st, ev) -> None:
        self.latency_ms.append(st.elapsed_time(ev))

    def reap(self) -> None:
        for lane in self.lanes:
            while lane.inflight and lane.inflight[0][1].query():
                self._done(*lane.inflight.popleft())

    def drain(self) -> None:
        for lane in self.lanes:
            while lane.inflight:
                st, ev = lane.inflight.popleft()
                ev.synchronize()
                self._done(st, ev)

    def close(self) -> None:
        for lane in self.lanes:
            lane.close()
        self.lanes = []
        self.model = None


class DataPlane:
    """This rank's GPU: one slot per partition of every compute mode (15 model replicas)."""

    def __init__(self, cfg: BenchConfig):
        import torch

        from .models.workload.yolos import YolosSmall
        from .ops import kernels as K
        K.set_backend(cfg.backend)
        self.cfg = cfg
        self.device = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
        torch.cuda.set_device(self.device)
        self.template = YolosSmall()
        self.slots: Dict[Any, Slot] = {}
        for prof, n in (("spx_nps1", 1), ("dpx_nps1", 2), ("qpx_nps1", 4), ("cpx_nps1", 8)):
            for k in range(n):
                self.slots[(prof, k)] = Slot(slice_cus(prof, k, emulation=cfg.emulation), self.device, cfg,
                                             self.template, seed=k, pin=slice_pin(prof, k, cfg.emulation),
                                             split=True)
        for s in self.slots.values():
            s.warm()
        torch.cuda.synchronize()
        self._layout: frozenset = frozenset()
        self.drains = 0
        self._mask_streams: Dict[Tuple[int, ...], Tuple[Any, Any]] = {}  # row groups -> CU-masked stream

    def add_slots(self, slots: Dict[Any, List[int]]) -> None:
        import torch
        for key, cus in slots.items():
            if key not in self.slots:
                s = Slot(cus, self.device, self.cfg, self.template, seed=len(self.slots))
                s.warm()
                self.slots[key] = s
        torch.cuda.synchronize()

    def drain_all(self) -> None:
        for s in self.slots.values():
            s.drain()

    def serve(self, keys: List[Any], deadline: float, start_at: Optional[Dict[Any, float]] = None) -> Dict[Any, int]:
        """Keep every listed slot busy until ``deadline``; returns the inferences enqueued per slot.
        ``start_at``: key -> wall time its pod starts serving (a pod still starting up).

        A different set of compute modes than in the last quantum means the GPU was re-partitioned:
        every queued inference of the old layout finishes first (the agent only flips an idle GPU),
        so slots of two layouts never overlap."""
        remap: Dict[Any, Tuple[Any, Any]] = {}
        if any(k not in self.slots for k in keys):
            remap = self._unaligned(keys)
        layout = frozenset(k[0] for k in keys)
        if layout != self._layout:
            if any(s.in_flight for s in self.slots.values()):
                self.drains += 1
            self.drain_all()
            self._layout = layout
        active = [(k, self.slots[remap[k][0]] if k in remap else self.slots[k]) for k in keys]
        if self.cfg.depth <= 1 and active:
            return self._serve_loops(active, deadline, {k: v[1] for k, v in remap.items()}, start_at)
        n: Dict[Any, int] = {k: 0 for k in keys}
        while True:
            now = time.perf_counter()
            if now >= deadline:
                break
            if not active:
                time.sleep(deadline - now)
                break
            progressed = False
            for k, s in active:
                s.reap()
                if s.in_flight < s.capacity:
                    s.submit()
                    n[k] += 1
                    progressed = True
            if not progressed:
                time.sleep(0.0002)
        return n

    def _unaligned(self, keys: List[Any]) -> Dict[Any, Tuple[Any, Any]]:
        """A CU-mask slice on row groups no pre-warmed slot covers (("slice", profile, groups)):
        served by an idle slot of its profile — same CU count, so the same captured graph — replayed
        on a stream masked to the slice's own CUs (a HIP graph runs on the stream it is replayed on,
        profiles/graph_cu_mask_probe_r3.json). At most ``partitions`` slices of a profile exist at
        once, so a slot is always free; only a stream is created, never a replica in the window."""
        from .ops.probe import Stream
        taken = {k for k in keys if k in self.slots}
        out: Dict[Any, Tuple[Any, Any]] = {}
        for k in keys:
            if k in self.slots:
                continue
            prof, groups = k[1], k[2]
            slot = next((sk for sk in sorted(self.slots, key=str) if sk[0] == prof and sk not in taken
                         and len(self.slots[sk].lanes) == 1), None)
            if slot is None:  # more slices of a profile than its partitions: a replica of its own
                self.add_slots({k: [32 * g + i for g in groups for i in range(32)]})
                taken.add(k)
                continue
            taken.add(slot)
            if groups not in self._mask_streams:
                st = Stream(self.device, [32 * g + i for g in groups for i in range(32)])
                self._mask_streams[groups] = (st, st.torch_stream())
            out[k] = (slot, self._mask_streams[groups][1])
        return out

    def _serve_loops(self, active: List[Tuple[Any, "Slot"]], deadline: float,
                     streams: Optional[Dict[Any, Any]] = None,
                     start_at: Optional[Dict[Any, float]] = None) -> Dict[Any, int]:
        """The reference demo's loop (``client/main.py:23-25``), one per pod lane, each on its own
        thread: start one inference, wait for it (a blocking event wait, the GIL released), record
        its GPU time, start the next — until ``deadline``. A polling loop over every pod would leave
        each GPU idle for a poll interval after every inference; a thread per loop resubmits as
        soon as its inference is done, as a pod's own process would."""
        import torch

        from .ops import kernels as K
        counts: Dict[Any, List[int]] = {k: [] for k, _ in active}

        def run(key: Any, slot: "Slot", lane: "_Lane") -> None:
            K.set_slice_cus(lane.n_cus)
            K.set_slice_pin(slot.pin)
            done = 0
            stream = (streams or {}).get(key) or lane.stream
            wait = (start_at or {}).get(key, 0.0) - time.perf_counter()
            if wait > 0:
                time.sleep(min(wait, max(0.0, deadline - time.perf_counter())))
            with torch.no_grad(), torch.cuda.stream(stream):
                while time.perf_counter() < deadline:
                    st = torch.cuda.Event(enable_timing=True)
                    st.record(stream)
                    if lane.graph is not None:
                        lane.graph.replay()
                    else:
                        lane.out = slot.model(lane.x)
                    ev = torch.cuda.Event(enable_timing=True)
                    ev.record(stream)
                    ev.synchronize()
                    slot.latency_ms.append(st.elapsed_time(ev))
                    done += 1
            counts[key].append(done)

        threads = [threading.Thread(target=run, args=(k, s, lane), daemon=True, name=f"pod-{k}")
                   for k, s in active for lane in s.lanes]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        return {k: sum(v) for k, v in counts.items()}

    def close(self) -> None:
        """Release graphs, model replicas and CU-masked streams before interpreter teardown (a
        graph destroyed after the HIP runtime has been finalised crashes the process at exit)."""
        import gc

        import torch
        self.drain_all()
        torch.cuda.synchronize()
        for s in self.slots.values():
            for lane in s.lanes:
                lane.graph = None
        gc.collect()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        for s in self.slots.values():
            s.close()
        self.slots.clear()
        for st, _ in self._mask_streams.values():
            st.close()
        self._mask_streams.clear()
        gc.collect()


class HwBusySampler:
    """amd-smi gfx activity of this rank's GPU, sampled on a thread during the timed window (the
    bench process may use amd-smi; only the partition agent must stay HIP-free)."""

    def __init__(self, hip_device: int, period: float = 0.1):
        self.samples: List[float] = []
        self.power: List[Dict[str, float]] = []
        self.period = period
        self._stop = threading.Event()
        self._t: Optional[threading.Thread] = None
        self.error = ""
        try:
            from .device.amdsmi import NativeAmdSmi
            self.smi = NativeAmdSmi()
            devs = [d for d in self.smi.logical_devices() if d.hip_id == hip_device]
            self.gpu = devs[0].gpu_index if devs else 0
        except Exception as e:  # noqa: BLE001 - the figure is reported as unavailable
            self.smi, self.error = None, str(e)[:200]

    def _run(self) -> None:
        while not self._stop.wait(self.period):
            try:
                self.samples.append(self.smi.activity(self.gpu)["gfx"])
                self.power.append(self.smi.power_clock(self.gpu))
            except Exception as e:  # noqa: BLE001
                self.error = str(e)[:200]
                return

    def start(self) -> None:
        if self.smi is not None:
            self._t = threading.Thread(target=self._run, name="nos-hw-busy", daemon=True)
            self._t.start()

    def stop(self) -> Optional[float]:
        self._stop.set()
        if self._t is not None:
            self._t.join()
        return round(sum(self.samples) / len(self.samples), 1) if self.samples else None

    def power_summary(self) -> Dict[str, float]:
        if not self.power:
            return {}
        keys = self.power[0].keys()
        return {f"mean_{k}": round(sum(p[k] for p in self.power) / len(self.power), 1) for k in keys}


class NodeBench:
    """The simulated node (real control plane, nos partition device plugin, kube-scheduler
    semantics) + the outage model + this rank's data plane. With ``cfg.nodes > 1`` (control plane
    only, ``nos-simulate --nodes``) the cluster has that many nodes and the outage model tracks
    every (node, GPU); the data plane serves the first node."""

    def __init__(self, cfg: BenchConfig, barrier_factory=None, gpu_data_plane: bool = True,
                 verify=None):
        from .sim.cluster import SimCluster

        self.cfg = cfg
        from .controllers.partitioner.pod_controller import PackParams
        self.cluster = SimCluster(n_nodes=cfg.nodes, gpus_per_node=cfg.gpus, refresh_interval=5.0, policy=cfg.policy,
                                  device_plugin=cfg.device_plugin, pack=PackParams(**(cfg.pack or {})),
                                  xcp_layout=cfg.layout)
        self.sn = next(iter(self.cluster.nodes.values()))  # the node this rank's data plane serves
        if barrier_factory is not None or verify is not None:
            self._set_commit(barrier_factory, verify)
        self.churn = ChurnProcess(cfg)
        self.cluster.run(30)  # node initialisation (SPX everywhere)
        self.live: Dict[str, float] = {}              # running pod -> served quanta left
        self.profile_of: Dict[str, str] = {}          # pod -> requested profile
        self.created: Dict[str, float] = {}           # pod -> cluster time it was created
        self.bound_at: Dict[str, float] = {}          # pod -> cluster time it was bound
        self.outage: Dict[Tuple[str, int], float] = {}  # (node, GPU) -> quanta of outage left
        self.starting: Dict[str, float] = {}          # pod -> quanta of start-up left (serves nothing)
        self._flips_seen = {n: len(sn.smi.set_calls) for n, sn in self.cluster.nodes.items()}
        self._binds_seen = 0
        self.reset_stats()
        self.data: Optional[DataPlane] = DataPlane(cfg) if gpu_data_plane else None

    def reset_stats(self) -> None:
        self.inferences = 0
        self.flips = 0
        self.outage_gpu_quanta = 0.0
        self.gpu_quanta = 0
        self.util_samples: List[float] = []
        self.raw_util_samples: List[float] = []
        self.pods_samples: List[int] = []
        self.pending_samples: List[int] = []
        self.host_s = {"control": 0.0, "serve": 0.0}
        self.empty_steps = 0
        self.profile_inferences: Dict[str, int] = collections.defaultdict(int)
        self.profile_pods: Dict[str, set] = collections.defaultdict(set)        # pods that served in the window
        self.tts: Dict[str, List[float]] = collections.defaultdict(list)        # bound in the window: wait (s)
        self.dark_wall_s = 0.0
        self.start_gpu_quanta = 0.0      # allocated GPU-quanta spent in pods' start-up
        self.idle_acct: Dict[str, float] = collections.defaultdict(float)  # cause -> GPU-quanta
        self.offered_gpu_quanta = 0.0    # GPU-quanta of work that arrived (expected lifetime x size)

    def dark(self, gpu: int, node: Optional[str] = None) -> float:
        """Fraction of this quantum ``gpu`` of ``node`` (default: this rank's node) is dark (flip outage)."""
        return min(1.0, max(0.0, self.outage.get((node or self.sn.name, gpu), 0.0)))

    def _set_commit(self, factory: Any, verify: Any) -> None:
        for c in self.sn.manager.controllers:
            actuator = getattr(c.reconciler, "__self__", None)
            if actuator is not None and hasattr(actuator, "barrier_factory"):
                if factory is not None:
                    actuator.barrier_factory = factory
                if verify is not None:
                    actuator.verify = verify

    # -- control plane + outage model ------------------------------------------------------
    def pod_gpus(self) -> Dict[str, set]:
        out: Dict[str, set] = {}
        for sn in self.cluster.nodes.values():
            for (_, name), devs in sn.kubelet.allocations.items():
                out[name] = {(sn.name, sn.smi.resolve(d).gpu_index) for _, d in devs}
        return out

    def control_step(self) -> None:
        t0 = time.perf_counter()
        c = self.cluster
        for name in [n for n, left in self.live.items() if left <= 1e-9]:
            del self.live[name]
            c.complete(name)
            c.delete_pod(name)  # the owning controller garbage-collects finished pods
        now = c.clock()
        for prof in self.churn.arrivals():
            name = f"p{self.churn.seq}"
            bound = (self.cfg.declared_bound_quanta * self.cfg.cluster_s + self.cfg.pod_start_s
                     if self.cfg.declared_bound_quanta > 0 else None)
            c.submit({f"amd.com/{prof}": 1}, name=name, deadline_s=bound)
            self.profile_of[name] = prof
            self.offered_gpu_quanta += self.cfg.mean_lifetime_quanta / COMPUTE_MODES[prof.split("_")[0]]
            self.created[name] = now
            self.churn.seq += 1
        c.run(self.cfg.cluster_s)
        c.clock.set(now + self.cfg.cluster_s)  # a quantum is cluster_s of cluster time, idle or not
        for nname, sn in c.nodes.items():
            calls = sn.smi.set_calls
            for kind, gpu, _ in calls[self._flips_seen[nname]:]:
                self.flips += 1
                for g in (range(self.cfg.gpus) if gpu is None else (gpu,)):
                    self.outage[(nname, g)] = max(self.outage.get((nname, g), 0.0), self.cfg.flip_quanta)
            self._flips_seen[nname] = len(calls)
        for t, name, _ in c.binds[self._binds_seen:]:
            self.bound_at[name] = t
            if self.cfg.pod_start_quanta > 0:
                self.starting[name] = self.cfg.pod_start_quanta
            if name in self.created:
                self.tts[self.profile_of.get(name, "?")].append(t - self.created[name])
        self._binds_seen = len(c.binds)
        for p in c.running_pods():
            n = ko.name(p)
            if n not in self.live:
                self.live[n] = float(self.churn.lifetime())
        frac = c.gpu_allocated_fraction()
        self._account_idle(frac)
        self.raw_util_samples.append(100.0 * sum(frac.values()) / max(1, len(frac)))
        self.util_samples.append(100.0 * sum(v * (1.0 - self.dark(g, n)) for (n, g), v in frac.items())
                                 / max(1, len(frac)))
        self.pods_samples.append(len(c.running_pods()))
        self.pending_samples.append(len(c.pending_pods()))
        self.gpu_quanta += self.cfg.gpus * self.cfg.nodes
        self.outage_gpu_quanta += sum(self.dark(g, n) for (n, g) in frac)
        self.host_s["control"] += time.perf_counter() - t0

    def _account_idle(self, frac: Dict[Tuple[str, int], float]) -> None:
        """Charge every GPU's unallocated share of this quantum to one cause (:data:`IDLE_CAUSES`),
        in GPU-quanta: ``flip_outage`` (dark), ``drain`` (the GPU's spec asks for what it cannot
        host yet: no new pod is placed on it until enough leave), ``fragmentation`` (pods wait, but
        every one of them is bigger than the GPU's unused room — on a hardware-partitioned GPU: no
        waiting pod asks for its free partitions' profile), ``placement_lag`` (a waiting pod would
        fit: the control plane has not placed it yet) and ``no_demand`` (nothing waits)."""
        from .models.xcp import node as xnode
        waiting = [self.profile_of.get(ko.name(p), "") for p in self.cluster.pending_pods()]
        waiting = [p for p in waiting if p]
        for nname, sn in self.cluster.nodes.items():
            try:
                model = xnode.new_node(self.cluster.api.get("Node", nname))
            except (ValueError, KeyError, NotImplementedError):
                model = None
            gpus = {g.index: g for g in model.gpus} if model is not None else {}
            for idx in range(self.cfg.gpus):
                v = frac.get((nname, idx))
                if v is None:
                    continue
                dark = self.dark(idx, nname)
                self.idle_acct["flip_outage"] += dark
                idle = max(0.0, 1.0 - v) * (1.0 - dark)
                if idle <= 1e-9:
                    continue
                g = gpus.get(idx)
                if g is not None and g.target is not None:
                    cause = "drain"
                elif not waiting:
                    cause = "no_demand"
                elif g is not None and getattr(g, "sliced", False):
                    need = min(1.0 / COMPUTE_MODES[p.split("_")[0]] for p in waiting)
                    cause = "placement_lag" if need <= idle + 1e-9 else "fragmentation"
                elif g is not None:
                    cause = "placement_lag" if any(g.free.get(p, 0) > 0 for p in waiting) else "fragmentation"
                else:
                    cause = "fragmentation"
                self.idle_acct[cause] += idle

    def idle_report(self) -> Dict[str, Any]:
        """Unallocated GPU-quanta of the window by cause, and each cause's share of GPU time (%);
        ``offered_pct``: the work that arrived in the window, in % of the window's GPU time (below 100
        allocation is bounded by it, plus what the queue held when the window began)."""
        total = max(1, self.gpu_quanta)
        return {"gpu_quanta": self.gpu_quanta,
                "offered_pct": round(100.0 * self.offered_gpu_quanta / total, 2),
                "by_cause_gpu_quanta": {k: round(self.idle_acct.get(k, 0.0), 3) for k in IDLE_CAUSES},
                "by_cause_pct": {k: round(100.0 * self.idle_acct.get(k, 0.0) / total, 2) for k in IDLE_CAUSES}}

    def start_dark(self, name: str) -> float:
        """Fraction of this quantum pod ``name`` spends starting up (allocated, not serving)."""
        return min(1.0, max(0.0, self.starting.get(name, 0.0)))

    def end_step(self) -> None:
        """Age every running pod by the part of the quantum its GPU was lit (a pod's lifetime
        includes its start-up, during which it holds its slice and serves nothing), then let outages
        and start-ups run."""
        gpus_of = self.pod_gpus()
        for name in list(self.live):
            lit = min((1.0 - self.dark(g, n) for (n, g) in gpus_of.get(name, ())), default=1.0)
            sd = self.start_dark(name)
            if sd > 0 and lit > 0:
                prof = self.profile_of.get(name, "")
                self.start_gpu_quanta += min(sd, lit) / COMPUTE_MODES.get(prof.split("_")[0], 1)
            if lit > sd:
                self.profile_pods[self.profile_of.get(name, "?")].add(name)
            self.live[name] -= lit
        for name in list(self.starting):
            self.starting[name] -= 1.0
            if self.starting[name] <= 1e-9 or name not in self.live:
                del self.starting[name]
        for g in list(self.outage):
            self.outage[g] -= 1.0
            if self.outage[g] <= 1e-9:
                del self.outage[g]

    def my_pods(self) -> List[Tuple[Any, ...]]:
        """Data-plane keys of the pods served on this rank's GPU this quantum (:func:`pod_keys`)."""
        return list(pod_keys(self.sn, self.cfg.rank).values())

    def step(self, deadline: Optional[float] = None) -> int:
        """One quantum: control plane, then the dark part of the quantum idle (a flip in progress),
        then every pod of this rank's GPU served until ``deadline``."""
        t0 = time.perf_counter()
        deadline = deadline if deadline is not None else t0 + self.cfg.quantum_s
        self.control_step()
        by_pod = pod_keys(self.sn, self.cfg.rank)
        keys = list(by_pod.values())
        dark = self.dark(self.cfg.rank)
        if not keys:
            self.empty_steps += 1
        t1 = time.perf_counter()
        n: Dict[Any, int] = {}
        if self.data is not None:
            lit_from = deadline - (1.0 - dark) * self.cfg.quantum_s
            if dark > 0:
                self.data.drain_all()  # the flipped GPU ran nothing of the old layout past the flip
                wait = lit_from - time.perf_counter()
                if wait > 0:
                    time.sleep(wait)
                    self.dark_wall_s += wait
            # a pod still starting up holds its slice and serves from the end of its start-up on
            start_at = {key: lit_from + self.start_dark(name) * self.cfg.quantum_s
                        for (_, name), key in by_pod.items() if self.start_dark(name) > 0}
            n = self.data.serve(keys if dark < 1.0 else [], deadline, start_at)
        elif self.cfg.world > 1 or not self.cfg.data_plane:
            # a rehearsal without a GPU: this rank's pods priced with the measured mode rates
            for (_, name), key in by_pod.items():
                lit = max(0.0, 1.0 - dark - self.start_dark(name))
                m = str(key[1] if key[0] == "slice" else key[0]).split("_")[0]
                n[key] = int(MODE_RATES[m] / COMPUTE_MODES[m] * self.cfg.quantum_s * lit)
            wait = deadline - time.perf_counter()
            if wait > 0:
                time.sleep(wait)
        self.host_s["serve"] += time.perf_counter() - t1
        total = sum(n.values())
        self.inferences += total
        for k, v in n.items():
            self.profile_inferences[str(k[1] if k[0] == "slice" else k[0])] += v
        self.end_step()
        return total

    def profile_report(self, window_s: float) -> Dict[str, Dict[str, Any]]:
        """Per profile: inferences served in the window, pods that served, time-to-schedule of the
        pods bound in the window (cluster seconds and mean pod lifetimes), waits of pods still
        pending at the end."""
        life_s = self.cfg.mean_lifetime_quanta * self.cfg.cluster_s
        now = self.cluster.clock()
        pending_age: Dict[str, List[float]] = collections.defaultdict(list)
        for p in self.cluster.pending_pods():
            n = ko.name(p)
            if n in self.created:
                pending_age[self.profile_of.get(n, "?")].append(now - self.created[n])
        out: Dict[str, Dict[str, Any]] = {}
        for prof, _ in MIX:
            tts = sorted(self.tts.get(prof, []))
            waits = sorted(pending_age.get(prof, []))
            row: Dict[str, Any] = {"inferences": int(self.profile_inferences.get(prof, 0)),
                                   "inf_per_s": round(self.profile_inferences.get(prof, 0) / max(1e-9, window_s), 2),
                                   "pods_served": len(self.profile_pods.get(prof, ())),
                                   "pods_bound": len(tts)}
            if tts:
                row["tts_s"] = {"p50": round(tts[len(tts) // 2], 1),
                                "p99": round(tts[min(len(tts) - 1, int(0.99 * len(tts)))], 1),
                                "max": round(tts[-1], 1)}
                row["tts_lifetimes_p99"] = round(row["tts_s"]["p99"] / life_s, 2)
            row["pending_at_end"] = len(waits)
            if waits:
                row["pending_wait_s_max"] = round(waits[-1], 1)
            out[prof] = row
        return out

    def close(self) -> None:
        if self.data is not None:
            self.data.close()


def pod_keys(sn: Any, gpu: int) -> Dict[Tuple[str, str], Tuple[Any, ...]]:
    """(namespace, pod) -> data-plane key of every pod on GPU ``gpu`` of simulated node ``sn``:
    (profile, partition index) of a partition, and of a CU-mask slice whose row groups are that
    partition's CU set (slices are placed buddy-aligned, so they usually are); ("slice", profile,
    groups) of any other slice."""
    out: Dict[Tuple[str, str], Tuple[Any, ...]] = {}
    slices = {s.id: s for ss in (sn.xcp_slices.load() if sn.xcp_slices is not None else {}).values() for s in ss}
    for pod, devs in sn.kubelet.allocations.items():
        for r, dev_id in devs:
            prof = extract_profile_name(r)
            if prof is None:
                continue
            d = sn.smi.resolve(dev_id)
            if d.gpu_index != gpu:
                continue
            s = slices.get(dev_id)
            if s is None:
                out[pod] = (prof, d.partition_index)
                continue
            groups = slice_groups(s)
            n = len(groups)
            if groups == list(range(groups[0], groups[0] + n)) and groups[0] % n == 0:
                out[pod] = (prof, groups[0] // n)
            else:
                out[pod] = ("slice", prof, tuple(groups))
    return out


# -- density --------------------------------------------------------------------------------
def _per_pod_spread(got: Dict[Any, int], keys: List[Any], dt: float) -> Dict[str, Any]:
    """Per-pod inferences/s of one density serve: min, max, max/min (how evenly the pods shared)."""
    rates = sorted(got.get(k, 0) / max(dt, 1e-9) for k in keys)
    if not rates:
        return {}
    return {"min": round(rates[0], 1), "max": round(rates[-1], 1),
            "max_over_min": round(rates[-1] / rates[0], 2) if rates[0] > 0 else None}


def density_phase(cfg: BenchConfig, data: Optional[DataPlane], serve_s: float = 1.0) -> Dict[str, Any]:
    """Saturate a fresh node through the control plane, then serve every pod on this rank's GPU
    at once: 8 CPX pods per GPU (as partitions, then on sliced GPUs), then a CU-mask node with
    dedicated-CU + memory-only slices."""
    import torch

    from .api import v1alpha1 as api
    from .models.slicing.cumask import cus_of
    from .sim.cluster import SimCluster
    out: Dict[str, Any] = {}
    # 8 x 1/8-GPU pods per GPU: as CPX compute partitions (a flip) and on sliced GPUs (no flip)
    for name, layout in (("xcp", "partitions"), ("xcp_slices", "slices")):
        c = SimCluster(n_nodes=1, gpus_per_node=cfg.gpus, refresh_interval=5.0, policy=cfg.policy, xcp_layout=layout)
        c.run(30)
        for i in range(8 * cfg.gpus):
            c.submit({"amd.com/cpx_nps1": 1}, name=f"d{i}")
        c.run(120)
        sn = next(iter(c.nodes.values()))
        per_gpu = collections.Counter(sn.smi.resolve(d).gpu_index for devs in sn.kubelet.allocations.values()
                                      for _, d in devs)
        out[name] = {"pods_per_gpu": round(sum(per_gpu.values()) / cfg.gpus, 2),
                     "pods_per_gpu_min": min(per_gpu.get(g, 0) for g in range(cfg.gpus)),
                     "pods_per_node": sum(per_gpu.values()), "pending": len(c.pending_pods()),
                     "flips": len(sn.smi.set_calls)}
        if data is not None:
            keys = sorted(set(pod_keys(sn, cfg.rank).values()), key=str)
            t0 = time.perf_counter()
            got = data.serve(keys, t0 + serve_s)
            data.drain_all()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            out[name]["inf_per_s_per_gpu"] = round(sum(got.values()) / dt, 1)
            out[name]["per_pod"] = _per_pod_spread(got, keys, dt)
    # CU-mask slices at the chart's cap (8 per GPU), then beyond it with the cap lifted by label —
    # the bench serves these pods as threads of one process; as processes, past 8 the hardware
    # scheduler time-slices them (profiles/procs_cap_r4.json), which CUMASK_DENSITY's names say
    for variant, (mix, cap) in CUMASK_DENSITY.items():
        c2 = SimCluster(n_nodes=1, gpus_per_node=cfg.gpus, refresh_interval=5.0, kind=api.PARTITIONING_KIND_CUMASK,
                        policy="fifo")
        if cap is not None:
            for n in c2.nodes:
                c2.api.patch("Node", n, {"metadata": {"labels": {api.LABEL_MAX_SLICES_PER_GPU: str(cap)}}})
        c2.run(30)
        k = 0
        for _ in range(cfg.gpus):
            for prof, n_pods in mix:
                for _ in range(n_pods):
                    c2.submit({f"amd.com/gpu-{prof}": 1}, name=f"s{k}")
                    k += 1
        c2.run(240)
        sn2 = next(iter(c2.nodes.values()))
        per_gpu2 = collections.Counter(sn2.smi.gpu_index_of(d) for devs in sn2.kubelet.allocations.values()
                                       for _, d in devs)
        # first-fit packing may fill some GPUs beyond the per-GPU mix and leave the last one
        # lighter: the mean over GPUs is the density, the minimum is reported beside it
        out[variant] = {"pods_per_gpu": round(sum(per_gpu2.values()) / cfg.gpus, 2),
                        "pods_per_gpu_min": min(per_gpu2.get(g, 0) for g in range(cfg.gpus)),
                        "pods_per_node": sum(per_gpu2.values()), "pending": len(c2.pending_pods()),
                        "profiles": {p: n for p, n in mix},
                        "max_slices_per_gpu": cap or 8,
                        "served_as": "threads of the bench process" + (
                            ": beyond the default cap of 8, not what a default node schedules; as processes "
                            "the hardware time-slices past 8 (profiles/procs_cap_r4.json)" if cap else "")}
        if data is not None:
            slices = sn2.plugin.store.load().get(cfg.rank, [])
            mine = {d for devs in sn2.kubelet.allocations.values() for _, d in devs
                    if sn2.smi.gpu_index_of(d) == cfg.rank}
            wanted = {(variant, s.id): cus_of(s, slices, 256) for s in slices if s.id in mine}
            data.add_slots(wanted)
            t0 = time.perf_counter()
            got = data.serve(list(wanted), t0 + serve_s)
            data.drain_all()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            out[variant]["inf_per_s_per_gpu"] = round(sum(got.values()) / dt, 1)
            out[variant]["per_pod"] = _per_pod_spread(got, list(wanted), dt)
    return out


# -- driver ---------------------------------------------------------------------------------
def inference_latency(data: Optional[DataPlane]) -> Dict[str, Dict[str, float]]:
    """GPU time of the inferences completed on this rank since the slots' lists were cleared, per
    compute mode: each inference is timed between events around its graph replay on its lane, so
    under concurrency (other partitions, the pod's other lane) it is the latency a request sees
    once the lane starts it."""
    out: Dict[str, Dict[str, float]] = {}
    if data is None:
        return out
    by_mode: Dict[str, List[float]] = collections.defaultdict(list)
    for key, s in data.slots.items():
        prof = key[1] if key[0] == "slice" else key[0]
        by_mode[str(prof).split("_")[0]] += s.latency_ms
    for mode, v in sorted(by_mode.items()):
        if v:
            v = sorted(v)
            out[mode] = {"n": len(v), "mean": round(sum(v) / len(v), 3), "p50": round(v[len(v) // 2], 3),
                         "p99": round(v[min(len(v) - 1, int(0.99 * len(v)))], 3)}
    return out


def _mean(v: List[float]) -> float:
    return sum(v) / max(1, len(v))


def flip_cost_report(cfg: BenchConfig) -> Dict[str, Any]:
    out: Dict[str, Any] = {"total_s": cfg.flip_cost_s, "per_quantum": round(cfg.flip_quanta, 4)}
    if abs(cfg.flip_cost_s - default_flip_cost(cfg.commit_barrier_s)) < 1e-9:
        out["components_s"] = dict(FLIP_COST_COMPONENTS)
        if cfg.commit_barrier_s >= 0:
            out["components_s"]["commit_barrier_s"] = round(cfg.commit_barrier_s, 3)
            out["commit_barrier_source"] = "measured in this run before the window (xgmi helper over every device)"
        out["measured"] = list(FLIP_COST_MEASURED)
        out["estimated"] = [k for k in FLIP_COST_COMPONENTS if k not in FLIP_COST_MEASURED]
    else:
        out["components_s"] = "overridden by --flip-cost"
    return out


def flip_sensitivity(cfg: BenchConfig, costs=(2.0, 5.0, 10.0, 30.0), steps: Optional[int] = None) -> Dict[str, Any]:
    """The control plane alone (no GPU) over the same seeded window for several flip costs: how much
    allocation the cost of a flip takes (``control_only``, priced with the measured mode rates)."""
    import dataclasses
    out: Dict[str, Any] = {}
    for fc in costs:
        c = dataclasses.replace(cfg, flip_cost_s=fc, rank=0, world=1)
        r = control_only(c, steps if steps is not None else cfg.warmup_quanta + cfg.window_quanta,
                         skip=cfg.warmup_quanta)
        out[f"{fc:g}s"] = {k: r[k] for k in ("util_pct", "flips", "time_in_flip_pct", "inf_per_s_model")}
    return out


def pod_start_sensitivity(cfg: BenchConfig, factors=(0.0, 1.0, 2.0, 4.0)) -> Dict[str, Any]:
    """The control plane alone over the same seeded window with pods' start-up at these multiples
    of the charged one (what start-up costs in allocation and modelled inferences; replaces the
    flip-cost sensitivity on layouts that never flip)."""
    import dataclasses
    out: Dict[str, Any] = {}
    for f in factors:
        c = dataclasses.replace(cfg, pod_start_s=f * cfg.pod_start_s, rank=0, world=1)
        r = control_only(c, cfg.warmup_quanta + cfg.window_quanta, skip=cfg.warmup_quanta)
        out[f"{round(f * cfg.pod_start_s, 1):g}s"] = {k: r[k] for k in ("util_pct", "inf_per_s_model")}
    return out


def seed_model(cfg: BenchConfig, seeds=tuple(range(1, 11))) -> Dict[str, Any]:
    """The control plane alone over the same window for other churn seeds (no GPU): how much the
    default seed's window is representative. ``inf_per_s_model`` prices served partition-time with
    :data:`MODE_RATES`; ``cpx_served_windows``: windows in which some 1/8-GPU pod was served."""
    import dataclasses
    rows = {}
    for sd in seeds:
        c = dataclasses.replace(cfg, seed=sd, rank=0, world=1)
        r = control_only(c, cfg.warmup_quanta + cfg.window_quanta, skip=cfg.warmup_quanta)
        rows[str(sd)] = {"inf_per_s_model": r["inf_per_s_model"], "util_pct": r["util_pct"],
                         "pending_mean": r["pending_mean"],
                         "served": {p: v["inferences"] > 0 for p, v in r["per_profile"].items()}}
    v = [x["inf_per_s_model"] for x in rows.values()]
    u = sorted(x["util_pct"] for x in rows.values())
    c = dataclasses.replace(cfg, rank=0, world=1)
    own = control_only(c, cfg.warmup_quanta + cfg.window_quanta, skip=cfg.warmup_quanta)
    return {"seeds": list(seeds), "mean": round(sum(v) / len(v), 1), "min": min(v), "max": max(v),
            "util_pct_mean": round(sum(u) / len(u), 2), "util_pct_min": u[0],
            "this_seed_model": own["inf_per_s_model"], "this_seed_util_pct": own["util_pct"],
            "cpx_served_windows": sum(1 for x in rows.values() if x["served"]["cpx_nps1"]),
            "per_seed": rows}


def sustainable_load_row(cfg: BenchConfig, load: float = 0.85, seeds=(1, 2, 3, 4), steps: int = 120) -> Dict[str, Any]:
    """The control plane alone at the load the planner keeps up with (no GPU): allocation, queue and
    the worst seed's p99 time-to-schedule per profile, in mean pod lifetimes."""
    import dataclasses
    util, pend, p99 = [], [], {}
    for sd in seeds:
        c = dataclasses.replace(cfg, seed=sd, offered_load=load, rank=0, world=1)
        r = control_only(c, steps)
        util.append(r["util_pct"])
        pend.append(r["pending_mean"])
        for prof, row in r["per_profile"].items():
            if row.get("tts_lifetimes_p99") is not None:
                p99[prof] = max(p99.get(prof, 0.0), row["tts_lifetimes_p99"])
    return {"offered_load": load, "seeds": list(seeds), "steps": steps, "util_pct_mean": round(_mean(util), 2),
            "pending_mean": round(_mean(pend), 2), "tts_p99_lifetimes_worst_seed": p99}


def _timed_window(cfg: BenchConfig, bf: Any, gpu: bool, distributed: bool) -> Tuple[Any, float, float, Any, Any]:
    """Preroll, warm-up and the timed window of ``cfg``'s layout on a fresh simulated node: returns
    (the NodeBench, window seconds (max over ranks), inferences (sum over ranks), hardware busy %,
    the busy sampler). Every rank runs it in lock-step (barriers around the window)."""
    import torch
    import torch.distributed as dist
    nb = NodeBench(cfg, barrier_factory=bf, gpu_data_plane=gpu)

    def sync() -> None:
        if nb.data is not None:
            nb.data.drain_all()
            torch.cuda.synchronize()
    for _ in range(cfg.preroll):
        nb.control_step()
        nb.end_step()
    for _ in range(cfg.warmup_quanta):
        nb.step()
    sync()
    if distributed:
        dist.barrier()
    nb.reset_stats()
    for s in (nb.data.slots.values() if nb.data is not None else ()):
        s.latency_ms.clear()
    busy = HwBusySampler(nb.data.device) if nb.data is not None else None
    if busy is not None:
        busy.start()
    t0 = time.perf_counter()
    deadline = t0
    for _ in range(cfg.window_quanta):
        deadline += cfg.quantum_s
        nb.step(deadline)
    sync()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    hw_busy = busy.stop() if busy is not None else None
    on_gpu = (dist.get_backend() == "nccl" if distributed else True) and gpu
    profs = [p for p, _ in MIX]
    stats = torch.tensor([elapsed, float(nb.inferences), hw_busy if hw_busy is not None else -1.0]
                         + [float(nb.profile_inferences.get(p, 0)) for p in profs],
                         dtype=torch.float64, device=f"cuda:{nb.data.device}" if on_gpu and nb.data else "cpu")
    if distributed:
        t = stats[:1].clone()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        s = stats[1:].clone()
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        elapsed, total_inf = float(t.item()), float(s[0].item())
        hw_busy = round(float(s[1].item()) / cfg.world, 1) if hw_busy is not None else None
        for i, p in enumerate(profs):
            nb.profile_inferences[p] = int(s[2 + i].item())
    else:
        total_inf = float(nb.inferences)
    return nb, elapsed, total_inf, hw_busy, busy


def partitions_window(cfg: BenchConfig, gpu: bool, distributed: bool) -> Dict[str, Any]:
    """BASELINE config 4 beside the headline: the same seed's window on hardware compute partitions
    (``--layout partitions``: SPX/DPX/QPX/CPX flips under churn, drains enforced by the partition
    plugin, every flip through the node commit barrier and dark for the flip cost), on a fresh
    node, timed by its own clock. The amd-smi setter needs root, which the box does not give, so the
    flip's outage is the components' cost (``flip_cost.estimated`` names the estimated ones); the
    flips, the drains and the commit barriers are the control plane's own."""
    import dataclasses

    from .parallel.barrier import LocalBarrier, RankCommitBarrier
    c = dataclasses.replace(cfg, layout="partitions", density=False)
    commits = [0]

    def bf(n):
        commits[0] += 1
        return RankCommitBarrier(rank=c.rank, world=c.world) if distributed else LocalBarrier(n)
    t0 = time.perf_counter()
    nb, elapsed, total_inf, hw_busy, _ = _timed_window(c, bf, gpu, distributed)
    try:
        return {"layout": "partitions", "value": round(total_inf / elapsed, 3), "unit": "inferences/s",
                "window_s": round(elapsed, 3), "wall_s_incl_setup": round(time.perf_counter() - t0, 1),
                "gpu_utilization_pct": round(_mean(nb.util_samples), 2),
                "allocation_pct_incl_outage": round(_mean(nb.raw_util_samples), 2),
                "hw_busy_pct": hw_busy, "flips": nb.flips,
                "time_in_flip_pct": round(100.0 * nb.outage_gpu_quanta / max(1, nb.gpu_quanta), 2),
                "commit_barriers": commits[0], "flip_cost": flip_cost_report(c),
                "pending_pods_mean": round(_mean(nb.pending_samples), 2),
                "pods_per_node": round(_mean(nb.pods_samples), 2),
                "per_profile": nb.profile_report(elapsed), "idle": nb.idle_report(),
                "layout_drains": nb.data.drains if nb.data is not None else 0}
    finally:
        nb.close()


def dist_report(cfg: BenchConfig, barrier_node: Optional[Dict[str, Any]]) -> Dict[str, Any]:
    """Who ran: the process group's backend and size, each rank's LOCAL_RANK, the devices it sees
    and the one it serves (gathered over the group), and the devices of the node commit barrier."""
    import torch
    import torch.distributed as dist
    me = {"rank": cfg.rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
          "visible_devices": torch.cuda.device_count() if torch.cuda.is_available() else 0,
          "device": torch.cuda.current_device() if torch.cuda.is_available() and cfg.data_plane else None,
          "hip_visible_devices": os.environ.get("HIP_VISIBLE_DEVICES")}
    ranks = [me]
    backend = None
    if cfg.world > 1 and dist.is_initialized():
        backend = dist.get_backend()
        ranks = [None] * cfg.world
        dist.all_gather_object(ranks, me)
    return {"backend": backend, "world_size": cfg.world, "ranks": ranks,
            "commit_barrier_node_devices": (barrier_node or {}).get("devices")}


#: wall seconds rank 0 may spend on the control-plane models after the windows (the other ranks
#: wait): models past the budget are skipped and named in ``post_window.skipped``
POST_WINDOW_BUDGET_S = {1: 120.0, 2: 120.0, 4: 90.0, 8: 60.0}


def run_bench(cfg: BenchConfig) -> Dict[str, Any]:
    import torch
    import torch.distributed as dist

    if os.environ.get("NOS_X3_ABLATE", "0") != "0":
        raise SystemExit("NOS_X3_ABLATE skips GEMM work (a timing-study switch): the bench refuses to run with it")

    from .parallel.barrier import LocalBarrier, RankCommitBarrier

    distributed = cfg.world > 1
    gpu = cfg.data_plane
    if cfg.flip_cost_default and gpu:
        # charge flips this run's own commit barrier (the node's devices, spawned as the agent does)
        measured = measure_commit_barrier() if cfg.rank == 0 else None
        if distributed:
            t = torch.tensor([measured if measured is not None else -1.0], dtype=torch.float64,
                             device=f"cuda:{torch.cuda.current_device()}" if dist.get_backend() == "nccl" else "cpu")
            dist.broadcast(t, 0)
            measured = float(t.item()) if t.item() >= 0 else None
        if measured is not None:
            cfg.commit_barrier_s = measured
            cfg.flip_cost_s = default_flip_cost(measured)
    pod_start = None
    if cfg.pod_start_default and gpu:
        # charge pods this box's own start-up (one pod process spawned as kubelet would, rank 0)
        pod_start = measure_pod_start() if cfg.rank == 0 else None
        ps = pod_start["pod_start_s"] if pod_start else -1.0
        if distributed:
            t = torch.tensor([ps], dtype=torch.float64,
                             device=f"cuda:{torch.cuda.current_device()}" if dist.get_backend() == "nccl" else "cpu")
            dist.broadcast(t, 0)
            ps = float(t.item())
        if ps > 0:
            cfg.pod_start_s = ps
    commits = [0]
    if distributed:
        # the agent's commit path (Actuator._commit -> barrier.vote_all(per-device votes)); each
        # rank contributes the votes of its own GPU's partitions, all-reduced over RCCL
        def bf(n):
            commits[0] += 1
            return RankCommitBarrier(rank=cfg.rank, world=cfg.world)
    else:
        def bf(n):
            commits[0] += 1
            return LocalBarrier(n)
    t_run = time.perf_counter()
    nb, elapsed, total_inf, hw_busy, busy = _timed_window(cfg, bf, gpu, distributed)
    commits_main = commits[0]
    latency = inference_latency(nb.data)
    per_profile = nb.profile_report(elapsed)
    barrier_8dev = node_barrier_probe(cfg) if cfg.rank == 0 and gpu else None
    density = density_phase(cfg, nb.data) if cfg.density else {}
    nb.close()
    value = total_inf / elapsed
    util = _mean(nb.util_samples)
    raw = _mean(nb.raw_util_samples)
    pods = _mean(nb.pods_samples)
    # BASELINE config 4 beside the headline (the sliced default): the same window on hardware partitions
    part = partitions_window(cfg, gpu, distributed) if cfg.layout != "partitions" and cfg.partitions_window else None
    dist_block = dist_report(cfg, barrier_8dev)
    from .models.workload.yolos import YolosSmall
    from .ops import kernels as K
    flops = YolosSmall().flops_per_inference(cfg.hw)
    # rank 0's control-plane models, within a wall-clock budget (the other ranks wait for it)
    budget = POST_WINDOW_BUDGET_S.get(cfg.gpus, 60.0)
    t_post = time.perf_counter()
    skipped: List[str] = []

    def within(name: str, fn):
        if cfg.rank != 0:
            return {}
        if time.perf_counter() - t_post > budget:
            skipped.append(name)
            return {"skipped": f"post-window budget of {budget:g} s spent"}
        return fn()
    # a layout that flips is priced by its flips; sliced GPUs never flip, so their sensitivity is to
    # the pods' start-up instead
    sens = within("sensitivity", lambda: flip_sensitivity(cfg) if cfg.layout == "partitions"
                  else pod_start_sensitivity(cfg))
    # the window is one draw of the churn: its spread over other seeds (fewer on big nodes, whose
    # control plane takes longer per quantum)
    seeds = within("seed_model", lambda: seed_model(cfg, tuple(range(1, 11 if cfg.gpus <= 2 else 6))))
    sustainable = within("load_0.85", lambda: sustainable_load_row(cfg))
    post = {"budget_s": budget, "spent_s": round(time.perf_counter() - t_post, 1), "skipped": skipped}
    life_s = cfg.mean_lifetime_quanta * cfg.cluster_s
    return {
        "metric": "aggregate GPU utilization % + schedulable pods/node, mixed fractional-GPU load",
        "value": round(value, 3),
        "unit": "inferences/s (aggregate over all GPUs; YOLOS-small fp32 batch-1 pods)",
        "n_gpus": cfg.gpus,
        "steps": cfg.steps,
        "warmup": cfg.warmup,
        "ms_per_step": round(1000.0 * elapsed / cfg.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / (BASELINE_INFER_PER_S_PER_GPU * cfg.gpus), 3),
        "dtype": "fp32",
        "numerics": ("fp32-accurate: every fp32 product as 6 bf16 MFMAs over an exact 3-term bf16 split "
                     "of both operands (dropped terms 2^-24 relative; tests/test_gpu_kernels.py checks the "
                     "error vs fp64 against the f32-input MFMA path)") if cfg.backend == "hip" else "fp32",
        "data": "synthetic (seeded pod churn; random-init YOLOS-small weights; synthetic 800x1066 images)" if gpu
        else "REHEARSAL without a GPU: control plane only, inferences priced with MODE_RATES (not a measurement)",
        "gpu_utilization_pct": round(util, 2),
        "allocation_pct_incl_outage": round(raw, 2),
        "hw_busy_pct": hw_busy,
        "hw_busy_source": "amd-smi gfx_activity, sampled every 100 ms in the timed window" if hw_busy is not None
        else f"unavailable: {busy.error if busy is not None else 'no GPU (rehearsal)'}",
        "hw_power_clock": busy.power_summary() if busy is not None else {},
        "pods_per_node": round(pods, 2),
        "pods_per_gpu": round(pods / cfg.gpus, 2),
        "per_profile": per_profile,
        "inference_latency_ms": latency,
        "pending_pods_mean": round(_mean(nb.pending_samples), 2),
        "pending_pods_max": max(nb.pending_samples) if nb.pending_samples else 0,
        "window": {"quanta": cfg.window_quanta, "quanta_per_step": cfg.quanta_per_step,
                   "cluster_s_per_quantum": cfg.cluster_s, "wall_s_per_quantum": cfg.quantum_s,
                   "compression": round(cfg.cluster_s / cfg.quantum_s, 1),
                   "mean_pod_lifetime_quanta": cfg.mean_lifetime_quanta,
                   "pod_lifetimes_in_window": round(cfg.window_quanta / cfg.mean_lifetime_quanta, 2),
                   "mean_pod_lifetime_cluster_s": life_s},
        "flip_cost": flip_cost_report(cfg),
        "flips": nb.flips,
        "time_in_flip_pct": round(100.0 * nb.outage_gpu_quanta / max(1, nb.gpu_quanta), 2),
        "dark_wall_s": round(nb.dark_wall_s, 3),
        "flip_cost_sensitivity" if cfg.layout == "partitions" else "pod_start_sensitivity": sens,
        "pod_start": {"s": round(cfg.pod_start_s, 2),
                      "source": ("measured in this run before the window (one pod process with Allocate's "
                                 "environment, spawn to first inference)") if pod_start else
                      ("POD_START_S constant" if cfg.pod_start_default else "--pod-start"),
                      "measurement": pod_start,
                      "pct_of_gpu_time": round(100.0 * nb.start_gpu_quanta / max(1, nb.gpu_quanta), 2)},
        "serving_pct": round(util - 100.0 * nb.start_gpu_quanta / max(1, nb.gpu_quanta), 2),
        "idle": nb.idle_report(),
        "seed_model": seeds,
        "load_0.85": sustainable,
        "commit_barrier_node": barrier_8dev,
        "commit_barriers": commits_main,
        "partitions_window": part,
        "dist": dist_block,
        "post_window": post,
        "run_wall_s": round(time.perf_counter() - t_run, 1),
        # what a default-configured node schedules (the chart's 8 slices per GPU); the beyond-the-cap
        # figures are in ``density`` under *_threads_cap_lifted, labelled
        "pods_per_gpu_saturation": {k: v["pods_per_gpu"] for k, v in density.items() if not k.endswith("_lifted")},
        "density": density,
        "achieved_tflops": round(value * flops / 1e12, 2),
        "host_ms_per_step": {k: round(1000.0 * v / cfg.steps, 2) for k, v in nb.host_s.items()},
        "layout_drains": nb.data.drains if nb.data is not None else 0,
        "empty_steps": nb.empty_steps,
        "admission_failures": nb.cluster.admission_failures,
        "baseline_ref": BASELINE_LABEL,
        "config": {"model": "yolos-small (hustvl/yolos-small architecture, fp32, 800x1066, batch 1)",
                   "global_batch": 1, "seq_len": 1 + (cfg.hw[0] // 16) * (cfg.hw[1] // 16) + 100,
                   "parallelism": f"fractional-gpu xcp {cfg.layout}, {cfg.gpus} GPU node",
                   "mix": {p: w for p, w in MIX}, "offered_load_per_gpu": cfg.offered_load,
                   "lifetime_quanta": list(cfg.lifetime), "policy": cfg.policy, "xcp_layout": cfg.layout,
                   "device_plugin": cfg.device_plugin, "scheduler": "kube-scheduler semantics (allocatable)",
                   "backend": cfg.backend, "hip_graphs": cfg.graphs, "depth": cfg.depth,
                   "pod_streams": cfg.pod_streams, "lane_cus": cfg.lane_cus,
                   "partition_emulation": cfg.emulation,
                   "fp32_matmul": (K.get_fp32_matmul() if cfg.backend == "hip" else "hipblaslt-f32")},
    }


def measure_commit_barrier() -> Optional[float]:
    """Wall seconds of one xGMI commit barrier over every device this process can see (the native
    helper, spawned as the agent spawns it), or None when it cannot run."""
    try:
        from .ops import native
        from .parallel.spawned import NATIVE_HELPER, SpawnedNodeBarrier
        if not native.available(NATIVE_HELPER):
            return None
        import torch
        n = torch.cuda.device_count()
        b = SpawnedNodeBarrier(n, backend="xgmi", native=True, timeout=60.0)
        if not b.vote_all([True] * n):
            return None
        return round(float(b.last["wall_ms"]) / 1000.0, 3)
    except Exception:  # noqa: BLE001 - the component constant is charged instead
        return None


def measure_pod_start(timeout: float = 180.0) -> Optional[Dict[str, Any]]:
    """Seconds from a pod's process starting to its first inference, on this box: the reference
    demo's client (``dataplane/client.py``: torch import, YOLOS-small load, warm-up, HIP-graph
    capture) spawned with the environment ``Allocate`` gives a 1/8-GPU slice (CU mask, HBM budget,
    shim), timed from ``Popen`` to its first inference. None when it cannot run."""
    import subprocess
    import sys
    try:
        from .dataplane.procs import ROOT, allocate_envs
        env = dict(os.environ)
        env.update(allocate_envs(["32cu.36gb"])[0])
        env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        t0 = time.perf_counter()
        p = subprocess.Popen([sys.executable, "-u", "-m", "walkai_nos_amd.dataplane.client", "--seconds", "0.3"],
                             cwd=ROOT, env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                             stderr=subprocess.DEVNULL, text=True)
        try:
            ln = p.stdout.readline()
            ready = time.perf_counter() - t0
            if ln.strip() != "READY":
                return None
            p.stdin.write(f"GO {time.time():.6f}\n")
            p.stdin.flush()
            out, _ = p.communicate(timeout=timeout)
        finally:
            if p.poll() is None:
                p.kill()
                p.wait()
        res = json.loads(next(x for x in reversed(out.splitlines()) if x.startswith("{")))
        first = (res.get("latency_ms") or {}).get("max", 0.0) / 1000.0
        return {"pod_start_s": round(ready + first, 2), "to_ready_s": round(ready, 2),
                "in_process_boot_s": res.get("boot_s"), "slice": "32cu.36gb (1/8 GPU)"}
    except Exception:  # noqa: BLE001 - the constant is charged instead
        return None


def node_barrier_probe(cfg: BenchConfig) -> Optional[Dict[str, Any]]:
    """The node-atomic commit barrier over every GPU this process can see, timed once after the
    window (never inside it), spawned as the partition agent spawns it: the xGMI P2P token ring
    (the agent's default) and the RCCL communicator. On the driver's 8-GPU node this measures the
    8-device ring and clique."""
    try:
        from .ops import native
        from .parallel.spawned import NATIVE_HELPER, SpawnedNodeBarrier
        if not native.available(NATIVE_HELPER):
            return {"error": "native helper not built"}
        import torch
        n = torch.cuda.device_count()
        out: Dict[str, Any] = {"devices": n}
        for backend in ("xgmi", "rccl"):
            b = SpawnedNodeBarrier(n, backend=backend, native=True, timeout=120.0)
            r = {"committed": b.vote_all([True] * n)}
            r.update({k: b.last.get(k) for k in ("wall_ms", "hip_init_ms", "comm_init_ms", "allreduce_ms",
                                                  "destroy_ms", "ring", "peer_links", "local_writes", "error")
                      if b.last.get(k) is not None})
            out[backend] = r
        return out
    except Exception as e:  # noqa: BLE001 - reported, never fatal to the bench
        return {"error": str(e)[:200]}


#: inferences/s per GPU with every partition of the mode busy, one serving thread per pod — the
#: round-4 tree (``profiles/kbench_r4_modes.json``, free-running; round 3: 359.9 / 415.9 / 433.0 /
#: 404.2): a CU-mask slice runs the same kernels on the same CU set as the emulated partition of
#: its size, so slices are priced with the rate of that mode per partition
MODE_RATES = {"spx": 368.5, "dpx": 418.5, "qpx": 427.5, "cpx": 404.9}


def control_only(cfg: BenchConfig, steps: int, skip: int = 0) -> Dict[str, Any]:
    """The control plane + outage model alone (no GPU): allocation, flips, queue and per-profile
    time-to-schedule over ``steps`` quanta after the preroll (the first ``skip`` of them are warm-up,
    not counted).  ``inf_per_s_model`` prices the served partition-quanta with the measured
    one-loop-per-pod mode rates (:data:`MODE_RATES`)."""
    nb = NodeBench(cfg, gpu_data_plane=False)
    for _ in range(cfg.preroll):
        nb.control_step()
        nb.end_step()
    rate = MODE_RATES
    served = 0.0
    for i in range(steps):
        if i == skip:
            nb.reset_stats()
            served = 0.0
        nb.control_step()
        for g in range(cfg.gpus):
            for (_, pod), devs in nb.sn.kubelet.allocations.items():
                lit = max(0.0, 1.0 - nb.dark(g) - nb.start_dark(pod))
                for r, d in devs:
                    p = extract_profile_name(r)
                    if p is not None and nb.sn.smi.resolve(d).gpu_index == g:
                        m = p.split("_")[0]
                        served += rate[m] / COMPUTE_MODES[m] * cfg.quantum_s * lit
                        nb.profile_inferences[p] += int(rate[m] / COMPUTE_MODES[m] * cfg.quantum_s * lit)
        nb.end_step()
    n = steps - skip
    return {"policy": cfg.policy, "gpus": cfg.gpus, "steps": n, "flip_cost_s": cfg.flip_cost_s,
            "util_pct": round(_mean(nb.util_samples), 2),
            "util_incl_outage_pct": round(_mean(nb.raw_util_samples), 2),
            "flips": nb.flips, "time_in_flip_pct": round(100.0 * nb.outage_gpu_quanta / max(1, nb.gpu_quanta), 2),
            "pending_mean": round(_mean(nb.pending_samples), 2),
            "pending_max": max(nb.pending_samples) if nb.pending_samples else 0,
            "pods_per_gpu": round(_mean(nb.pods_samples) / cfg.gpus, 2),
            "inf_per_s_model": round(served / (n * cfg.quantum_s), 1),
            "admission_failures": nb.cluster.admission_failures,
            "per_profile": nb.profile_report(n * cfg.quantum_s),
            "idle": nb.idle_report()}


def smoke_step() -> None:
    """One control-plane step + one partition's inference on cuda:0 + one slice probe."""
    import torch

    from .ops import probe
    r = probe.probe_mfma("fp32", iters=256, reps=1)
    assert r.tflops > 0
    cfg = BenchConfig(gpus=1, steps=1, warmup=0, graphs=False)
    nb = NodeBench(cfg, barrier_factory=None, gpu_data_plane=False)
    for _ in range(4):  # a few quanta of churn, so pods are scheduled and running
        nb.control_step()
        nb.end_step()
    from .models.workload.yolos import YolosSmall, demo_input
    m = YolosSmall().cuda().eval()
    with torch.no_grad():
        logits, boxes = m(demo_input(1, (256, 256), "cuda"))
    torch.cuda.synchronize()
    assert torch.isfinite(logits).all() and torch.isfinite(boxes).all()
    print(json.dumps({"smoke": "ok", "probe_fp32_tflops": round(r.tflops, 1),
                      "pods_running": len(nb.cluster.running_pods()), "util_pct": nb.cluster.utilization()}))
