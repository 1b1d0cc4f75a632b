"""HBM budget guard: the node agent's check that every slice's pods stay inside their HBM budget.

A CU-mask slice (and a slice of a sliced GPU) carries an HBM budget that the container's own
allocator interposer enforces (``NOS_HBM_LIMIT_BYTES`` + ``LD_PRELOAD`` of ``libnos_hbmlimit.so``,
set by the device plugins' ``Allocate``). That is cooperative: a process that clears ``LD_PRELOAD``
or allocates around the HIP allocator is not contained. The reference's MPS slices get the budget
from the MPS server (``CUDA_MPS_PINNED_DEVICE_MEM_LIMIT``, ref
``docs/en/docs/dynamic-gpu-partitioning/getting-started-mps.md``); here the node agent closes the
loop from outside the container, the way kubelet enforces memory by eviction:

1. amd-smi's per-process VRAM on every GPU (``AmdSmi.process_memory``: the KFD's own accounting,
   which no container can change);
2. each process is attributed to a pod by its cgroup (``/proc/<pid>/cgroup`` names the pod UID;
   kubelet's PodResources gives the pod's slice ids) — authoritative, so a child process cannot
   charge another pod's slice by forging its environment — or, for a process in no pod's cgroup,
   by the ``NOS_SLICE_IDS`` / ``NOS_PARTITION_IDS`` that ``Allocate`` put in its environment;
3. a pod's VRAM summed over its processes is held against the sum of its slices' budgets plus a
   slack per process for what the HIP runtime maps beyond the interposer's count (code objects,
   queues, scratch: 490 MiB for a PyTorch process, ``profiles/pytest_hbmguard_r4.log``);
4. a pod over budget for ``strikes`` consecutive checks is reported (metric, log) and, with
   ``action: evict``, deleted — its slice goes back to the pool and its neighbours' memory is safe.

The same holds for hardware compute partitions that share one memory partition (CPX on NPS1:
eight partitions, one HBM pool): nothing in hardware keeps a 1/8 partition's pod to 1/8 of the HBM,
so those partitions get that share as their budget (:func:`shared_memory_partitions`).

Processes on a guarded GPU that nothing attributes are reported as ``unattributed`` bytes (never
evicted: without a pod there is nothing to evict).

**Compute (CU-mask bypass).** A slice's compute isolation is ``HSA_CU_MASK`` in the container's
environment — cooperative too: a process that unsets it runs on all 256 CUs, next to its
neighbours' slices. The same amd-smi process list carries the KFD's ``cu_occupancy`` per process:
its waves in flight divided by the waves one CU can hold, sampled at the read. A process confined
to n CUs can never read more than n, so a pod whose processes read more CUs than its slices have
(``cu_strikes`` consecutive busy samples; idle samples neither count nor clear) is running outside
its mask: reported (a metric, a ``CUMaskExceeded`` Warning event) or, with ``cu_action: evict``,
evicted. The signal is one-sided — a bypassing process with few waves per CU reads low — so it
never accuses a masked pod. Per GPU the guard also says whether the signal exists at all: a GPU
busy for ``cu_probe_checks`` checks whose processes all read 0 (amd-smi without the KFD's
occupancy, e.g. unprivileged) is ``unavailable``, never "clean". The processes' ``evicted_time``
(queues switched out by the hardware scheduler) is exported per pod as reported; on the MI355X
box it read 0 even for 10-12 pod processes that were visibly time-sliced
(``profiles/fair_probe_r5_10_12.json``), so nothing is decided on it.
"""
from __future__ import annotations

import logging
import os
import re
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, Iterable, List, Mapping, Optional, Tuple

from prometheus_client import Counter, Gauge

from ..utils.metrics import REGISTRY

log = logging.getLogger("nos.hbmguard")

ACTIONS = ("off", "report", "evict")
CU_STATES = {"available": 1, "unavailable": 0, "unknown": -1}
PodKey = Tuple[str, str]   # (namespace, name)

_used = Gauge("nos_slice_hbm_used_bytes", "VRAM held by a pod's processes on its slices' GPU (amd-smi)",
              ["node", "gpu", "namespace", "pod"], registry=REGISTRY.registry)
_budget = Gauge("nos_slice_hbm_budget_bytes", "HBM budget of a pod's slices", ["node", "gpu", "namespace", "pod"],
                registry=REGISTRY.registry)
_unattributed = Gauge("nos_slice_hbm_unattributed_bytes",
                      "VRAM held by processes on a sliced GPU that no pod's slices account for", ["node", "gpu"],
                      registry=REGISTRY.registry)
_violations = Counter("nos_slice_hbm_violations_total", "Pods found over their slices' HBM budget",
                      ["node", "action"], registry=REGISTRY.registry)
_cu_used = Gauge("nos_slice_cu_occupancy", "CU-equivalents of a pod's waves in flight on its slices' GPU (amd-smi)",
                 ["node", "gpu", "namespace", "pod"], registry=REGISTRY.registry)
_cu_budget = Gauge("nos_slice_cu_budget", "CUs of a pod's slices (its HSA_CU_MASK)", ["node", "gpu", "namespace", "pod"],
                   registry=REGISTRY.registry)
_evicted = Gauge("nos_slice_queue_evicted_seconds", "Time a pod's queues spent evicted (time-sliced) on its GPU",
                 ["node", "gpu", "namespace", "pod"], registry=REGISTRY.registry)
_cu_violations = Counter("nos_slice_cu_violations_total", "Pods found running on more CUs than their slices have",
                         ["node", "action"], registry=REGISTRY.registry)
_cu_available = Gauge("nos_slice_cu_guard_available",
                      "1: the GPU reports per-process CU occupancy; 0: busy but never reported (unavailable); -1: unknown",
                      ["node", "gpu"], registry=REGISTRY.registry)

#: kubepods cgroup paths name the pod UID with dashes (cgroupfs) or underscores (systemd driver)
_POD_UID = re.compile(r"pod([0-9a-f]{8}[-_][0-9a-f]{4}[-_][0-9a-f]{4}[-_][0-9a-f]{4}[-_][0-9a-f]{12})")


def pod_uid_of(pid: int, proc_root: str = "/proc") -> Optional[str]:
    """The pod UID in the process's cgroup path, or None (not a pod's process, or gone)."""
    try:
        with open(os.path.join(proc_root, str(pid), "cgroup")) as f:
            text = f.read()
    except OSError:
        return None
    m = _POD_UID.search(text)
    return m.group(1).replace("_", "-") if m else None


_ID_VARS = (b"NOS_SLICE_IDS=", b"NOS_PARTITION_IDS=")


def slice_ids_of(pid: int, proc_root: str = "/proc") -> Tuple[str, ...]:
    """The device ids ``Allocate`` put in the process's initial environment (``NOS_SLICE_IDS``,
    ``NOS_PARTITION_IDS``), or ()."""
    try:
        with open(os.path.join(proc_root, str(pid), "environ"), "rb") as f:
            env = f.read().split(b"\0")
    except OSError:
        return ()
    out: List[str] = []
    for kv in env:
        for var in _ID_VARS:
            if kv.startswith(var):
                out.extend(i for i in kv[len(var):].decode(errors="replace").split(",") if i and i not in out)
    return tuple(out)


def shared_memory_partitions(device_map: Any) -> Dict[str, Tuple[int, int]]:
    """Hardware partitions sharing a memory partition with others (more compute partitions than
    NPS memory partitions, e.g. CPX on NPS1): device id -> (GPU, budget = the GPU's HBM / its
    compute partitions), the share the profile promises and that nothing in hardware enforces."""
    from ..models.xcp.profile import COMPUTE_MODES, MEMORY_MODES
    vram = {g.index: g.vram_bytes for g in device_map.gpus}
    out: Dict[str, Tuple[int, int]] = {}
    for d in device_map.devices:
        n = COMPUTE_MODES.get(d.compute_mode.lower(), 1)
        if n > MEMORY_MODES.get(d.memory_mode.lower(), 1) and vram.get(d.gpu_index):
            out[d.device_id] = (d.gpu_index, vram[d.gpu_index] // n)
    return out


@dataclass
class Account:
    """One owner's VRAM on one GPU: a pod (``pod`` set) or, outside Kubernetes, a slice-id set."""
    gpu: int
    slice_ids: Tuple[str, ...]
    budget: int
    pod: Optional[PodKey] = None
    used: int = 0
    pids: List[int] = field(default_factory=list)
    cu_budget: Optional[int] = None   # CUs of its slices (None: hardware-isolated, not checked)
    cu_used: Optional[int] = None     # summed cu_occupancy of its processes (None: not reported)
    evicted_ms: int = 0

    @property
    def key(self) -> Tuple[Any, ...]:
        return (self.gpu, self.pod) if self.pod is not None else (self.gpu, self.slice_ids)


@dataclass
class Violation:
    account: Account
    limit: int
    strikes: int
    action: str   # "report" | "evict" | "evicted" (the pod was deleted this check)
    kind: str = "hbm"   # "hbm" | "cu"


class HbmGuard:
    """Checks pods' VRAM against their slices' HBM budgets (see the module docstring).

    ``slices``: GPU index -> the node's slices (``SliceStore.load``: objects with ``id`` and
    ``hbm_bytes``); ``partitions``: device id -> (GPU, budget) of hardware partitions that share
    memory (:func:`shared_memory_partitions`); ``pods_by_device``: [(namespace, pod, device)] of running containers
    (``ResourceClient.get_used_devices_by_pod``); ``pods_by_uid``: pod UID -> (namespace, name) of
    the node's pods; ``evict``: deletes a pod (``action: evict``)."""

    def __init__(self, smi: Any, slices: Callable[[], Mapping[int, List[Any]]], node: str = "",
                 pods_by_device: Optional[Callable[[], Iterable[Tuple[str, str, Any]]]] = None,
                 pods_by_uid: Optional[Callable[[], Mapping[str, PodKey]]] = None,
                 evict: Optional[Callable[[str, str, str], None]] = None, action: str = "report",
                 slack_bytes: int = 768 << 20, strikes: int = 2, proc_root: str = "/proc",
                 partitions: Optional[Callable[[], Mapping[str, Tuple[int, int]]]] = None,
                 cu_action: str = "report", cu_strikes: int = 3, cu_count: int = 256, cu_probe_checks: int = 6,
                 event: Optional[Callable[[str, str, str, str], None]] = None, max_slack_procs: int = 4,
                 pid_map: Optional[Callable[[int], Optional[int]]] = None):
        """``cu_action``: what a CU-mask bypass gets (``off`` | ``report`` | ``evict``); ``event``:
        records a Warning event on a pod (namespace, name, reason, message); ``max_slack_procs``: the
        per-process slack is granted for at most this many processes (more idle processes must not
        raise a pod's allowance); ``pid_map``: amd-smi's (host) pid -> the pid under ``proc_root``
        (identity by default: the agents run with hostPID, so the KFD's pids are theirs)."""
        if action not in ACTIONS:
            raise ValueError(f"hbm guard action {action!r} not in {ACTIONS}")
        if cu_action not in ACTIONS:
            raise ValueError(f"cu guard action {cu_action!r} not in {ACTIONS}")
        self.cu_action, self.cu_strikes, self.cu_count, self.cu_probe_checks = cu_action, cu_strikes, cu_count, \
            cu_probe_checks
        self.event, self.max_slack_procs, self.pid_map = event, max_slack_procs, pid_map
        self._cu_strikes: Dict[Tuple[Any, ...], int] = {}
        self._cu_reported: set = set()
        self._cu_seen: Dict[int, bool] = {}         # GPU -> a process ever read a non-zero occupancy
        self._cu_blind: Dict[int, int] = {}         # GPU -> consecutive busy checks all reading 0
        self.cu_state: Dict[int, str] = {}
        self.smi, self.slices, self.node = smi, slices, node
        self.pods_by_device, self.pods_by_uid, self.evict = pods_by_device, pods_by_uid, evict
        self.partitions = partitions
        self.action, self.slack_bytes, self.strikes, self.proc_root = action, slack_bytes, strikes, proc_root
        self._strikes: Dict[Tuple[Any, ...], int] = {}
        self._evicted: Dict[PodKey, int] = {}      # pod -> checks since its deletion was requested
        self._series: set = set()
        self.checks = 0
        self._uid_map: Dict[str, PodKey] = {}
        self.uid_lists = 0                          # API server lists of the node's pods
        self.last: List[Account] = []
        self.unattributed: Dict[int, int] = {}
        self._gpus_checked: set = set()

    # -- one pass -------------------------------------------------------------------------------
    def accounts(self) -> List[Account]:
        """Every pod's (or slice set's) VRAM on each sliced GPU, from one amd-smi sample."""
        slices = self.slices() or {}
        budget_of: Dict[str, Tuple[int, int]] = {s.id: (g, int(s.hbm_bytes)) for g, ss in slices.items() for s in ss}
        cus_of_id = self._slice_cus(slices)
        if self.partitions is not None:
            try:
                budget_of.update(self.partitions())
            except Exception as e:  # noqa: BLE001 - device map unreadable: guard the slices only
                log.warning("partition budgets unavailable: %s", e)
        ids_of_pod: Dict[PodKey, List[str]] = {}
        if self.pods_by_device is not None:
            try:
                for ns, name, d in self.pods_by_device():
                    i = getattr(d, "device_id", d)
                    if i in budget_of:
                        ids_of_pod.setdefault((ns, name), []).append(i)
            except Exception as e:  # noqa: BLE001 - kubelet down: attribute by environment only
                log.warning("pod resources unavailable: %s", e)
        pod_of_id = {i: p for p, ids in ids_of_pod.items() for i in ids}
        refreshed = [False]

        def pod_of_uid(uid: str) -> Optional[PodKey]:
            # the node's pods are listed from the API server only when a process names a pod UID
            # the cached map does not know (once per pass): an idle node costs no API call
            if uid not in self._uid_map and not refreshed[0] and self.pods_by_uid is not None:
                refreshed[0] = True
                try:
                    self._uid_map = dict(self.pods_by_uid())
                    self.uid_lists += 1
                except Exception as e:  # noqa: BLE001
                    log.warning("node pods unavailable: %s", e)
            return self._uid_map.get(uid)
        out: Dict[Tuple[Any, ...], Account] = {}
        self.unattributed = {}
        self._gpus_checked = set()
        for g in sorted({g for g, _ in budget_of.values()}):
            try:
                info = self._process_info(g)
            except Exception as e:  # noqa: BLE001 - a GPU mid-flip or off the bus: skip it this pass
                log.debug("process list of GPU %d failed: %s", g, e)
                continue
            self._gpus_checked.add(g)
            self._sample_cu_signal(g, info)
            for pid, st in sorted(info.items()):
                nbytes = st.vram
                local = self.pid_map(pid) if self.pid_map is not None else pid
                uid = pod_uid_of(local, self.proc_root) if local is not None else None
                pod = pod_of_uid(uid) if uid is not None else None
                if pod is not None:
                    # a pod's process: its cgroup is authoritative (an environment can be forged by
                    # a child process to charge another pod's slice); a pod holding no device of
                    # this GPU (the agent's own probe helpers, say) is reported, never evicted
                    ids: Tuple[str, ...] = tuple(sorted(i for i in ids_of_pod.get(pod, ()) if budget_of[i][0] == g))
                else:
                    # no pod (or a pod cgroup the API server does not know on this node): the ids
                    # Allocate put in the process's environment
                    ids = tuple(i for i in (slice_ids_of(local, self.proc_root) if local is not None else ())
                                if budget_of.get(i, (None,))[0] == g)
                    pod = pod_of_id.get(ids[0]) if ids else None
                if not ids:
                    self.unattributed[g] = self.unattributed.get(g, 0) + nbytes
                    continue
                a = Account(g, ids, sum(budget_of[i][1] for i in ids), pod)
                a = out.setdefault(a.key, a)
                a.used += nbytes
                a.pids.append(pid)
                a.evicted_ms += int(st.evicted_ms or 0)
                cus = set()
                for i in ids:
                    cus |= cus_of_id.get(i, set())
                if cus and len(cus) < self.cu_count:
                    a.cu_budget = len(cus)
                if st.cu_occupancy is not None:
                    a.cu_used = (a.cu_used or 0) + int(st.cu_occupancy)
        return list(out.values())

    def _slice_cus(self, slices: Mapping[int, List[Any]]) -> Dict[str, set]:
        """slice id -> the CUs its pods may run on (its rows; memory-only slices: the shared pool)."""
        from ..models.slicing.cumask import cus_of
        out: Dict[str, set] = {}
        for ss in slices.values():
            for s in ss:
                if hasattr(s, "rows"):
                    try:
                        out[s.id] = set(cus_of(s, ss, self.cu_count))
                    except Exception:  # noqa: BLE001 - a slice the model cannot place: not checked
                        continue
        return out

    def _process_info(self, g: int) -> Dict[int, Any]:
        """pid -> stats (``AmdSmi.process_info``); a backend with VRAM only reports no occupancy."""
        fn = getattr(self.smi, "process_info", None)
        if fn is not None:
            return fn(g)
        from ..device.amdsmi import ProcessStats
        return {pid: ProcessStats(b) for pid, b in self.smi.process_memory(g).items()}

    def _sample_cu_signal(self, g: int, info: Mapping[int, Any]) -> None:
        """Whether GPU ``g`` reports CU occupancy at all: any non-zero reading makes it available;
        ``cu_probe_checks`` checks in a row with the GPU busy and every process reading 0 (or no
        field) make it unavailable — never "clean"."""
        if any((st.cu_occupancy or 0) > 0 for st in info.values()):
            self._cu_seen[g] = True
            self._cu_blind[g] = 0
        elif info and not self._cu_seen.get(g):
            busy = False
            try:
                busy = float(self.smi.activity(g).get("gfx", 0.0)) >= 50.0
            except Exception:  # noqa: BLE001 - no activity reading: this sample decides nothing
                pass
            if busy or all(st.cu_occupancy is None for st in info.values()):
                self._cu_blind[g] = self._cu_blind.get(g, 0) + 1
        if self._cu_seen.get(g):
            self.cu_state[g] = "available"
        elif self._cu_blind.get(g, 0) >= self.cu_probe_checks:
            self.cu_state[g] = "unavailable"
        else:
            self.cu_state.setdefault(g, "unknown")

    def check(self) -> List[Violation]:
        """One pass: sample, compare, act. Returns the accounts over budget."""
        self.checks += 1
        accts = self.accounts()
        self.last = accts
        seen = set()
        found: List[Violation] = []
        for a in (accts if self.action != "off" else []):
            seen.add(a.key)
            # runtime overhead per process, for a bounded number of processes (idle processes must
            # not buy a pod more allowance)
            limit = a.budget + self.slack_bytes * min(max(1, len(a.pids)), max(1, self.max_slack_procs))
            if a.used <= limit:
                self._strikes.pop(a.key, None)
                continue
            n = self._strikes.get(a.key, 0) + 1
            self._strikes[a.key] = n
            if n < self.strikes:
                continue
            act = self.action
            who = f"{a.pod[0]}/{a.pod[1]}" if a.pod else f"slices {','.join(a.slice_ids)}"
            if act == "evict" and a.pod is not None and self.evict is not None and a.pod not in self._evicted:
                reason = (f"HBM budget exceeded: {a.used} B held on GPU {a.gpu}, budget {a.budget} B "
                          f"(+{self.slack_bytes} B slack per process) for slices {','.join(a.slice_ids)}")
                try:
                    self.evict(a.pod[0], a.pod[1], reason)
                    self._evicted[a.pod] = 0
                    act = "evicted"
                    log.warning("evicted %s: %s", who, reason)
                except Exception as e:  # noqa: BLE001 - retried on the next pass
                    log.error("evicting %s failed: %s", who, e)
            if n == self.strikes or act == "evicted":
                _violations.labels(self.node, act).inc()
                if act != "evicted":
                    log.warning("%s over its HBM budget on GPU %d: %d B used, budget %d B (pids %s)",
                                who, a.gpu, a.used, a.budget, a.pids)
            found.append(Violation(a, limit, n, act))
        self._strikes = {k: v for k, v in self._strikes.items() if k in seen}
        found.extend(self._check_cus(accts))
        self._evicted = {p: c + 1 for p, c in self._evicted.items() if c < 30}
        self._export(accts)
        return found

    def _check_cus(self, accts: List[Account]) -> List[Violation]:
        """CU-mask bypass (module docstring): a pod whose processes read more CU-equivalents of
        waves than its slices have CUs (each process may round up by one) for ``cu_strikes`` busy
        samples in a row."""
        if self.cu_action == "off":
            return []
        found: List[Violation] = []
        seen = set()
        for a in accts:
            if a.cu_budget is None or a.cu_used is None:
                continue
            seen.add(a.key)
            limit = a.cu_budget + len(a.pids)
            if a.cu_used <= 0:
                continue                      # idle sample: says nothing either way
            if a.cu_used <= limit:
                self._cu_strikes.pop(a.key, None)
                self._cu_reported.discard(a.key)
                continue
            n = self._cu_strikes.get(a.key, 0) + 1
            self._cu_strikes[a.key] = n
            if n < self.cu_strikes:
                continue
            act = self.cu_action
            who = f"{a.pod[0]}/{a.pod[1]}" if a.pod else f"slices {','.join(a.slice_ids)}"
            reason = (f"CU mask exceeded: {a.cu_used} CUs of waves in flight on GPU {a.gpu}, its slices "
                      f"{','.join(a.slice_ids)} have {a.cu_budget} CUs (HSA_CU_MASK bypassed?)")
            if act == "evict" and a.pod is not None and self.evict is not None and a.pod not in self._evicted:
                try:
                    self.evict(a.pod[0], a.pod[1], reason)
                    self._evicted[a.pod] = 0
                    act = "evicted"
                    log.warning("evicted %s: %s", who, reason)
                except Exception as e:  # noqa: BLE001 - retried on the next pass
                    log.error("evicting %s failed: %s", who, e)
            if a.key not in self._cu_reported:
                self._cu_reported.add(a.key)
                _cu_violations.labels(self.node, act).inc()
                if act != "evicted":
                    log.warning("%s: %s", who, reason)
                    if self.event is not None and a.pod is not None:
                        try:
                            self.event(a.pod[0], a.pod[1], "CUMaskExceeded", reason)
                        except Exception as e:  # noqa: BLE001
                            log.warning("event for %s not recorded: %s", who, e)
            found.append(Violation(a, limit, n, act, kind="cu"))
        self._cu_strikes = {k: v for k, v in self._cu_strikes.items() if k in seen}
        self._cu_reported &= seen
        return found

    def _export(self, accts: List[Account]) -> None:
        series = set()
        for a in accts:
            ns, name = a.pod if a.pod is not None else ("", ",".join(a.slice_ids))
            labels = (self.node, str(a.gpu), ns, name)
            _used.labels(*labels).set(a.used)
            _budget.labels(*labels).set(a.budget)
            _evicted.labels(*labels).set(a.evicted_ms / 1000.0)
            if a.cu_budget is not None:
                _cu_budget.labels(*labels).set(a.cu_budget)
            if a.cu_used is not None:
                _cu_used.labels(*labels).set(a.cu_used)
            series.add(labels)
        for labels in self._series - series:
            for gauge in (_used, _budget, _evicted, _cu_budget, _cu_used):
                try:
                    gauge.remove(*labels)
                except KeyError:
                    pass
        self._series = series
        # every guarded GPU this pass: one with nothing unattributed reads 0, not its last value
        for g in sorted(set(self.cu_state) | set(self.unattributed) | self._gpus_checked):
            _unattributed.labels(self.node, str(g)).set(self.unattributed.get(g, 0))
        for g, st in self.cu_state.items():
            _cu_available.labels(self.node, str(g)).set(CU_STATES[st])

    def register(self, mgr: Any, interval: float = 10.0) -> None:
        """Run on the agent's manager (node-local: no leader election)."""
        if self.action != "off" or self.cu_action != "off":
            mgr.add_runnable("hbm-guard", self.check, interval, needs_leader=False)


def node_pods_by_uid(client: Any, node: str) -> Callable[[], Dict[str, PodKey]]:
    """pod UID -> (namespace, name) of the pods bound to ``node``."""
    from ..kube import objects as ko

    def f() -> Dict[str, PodKey]:
        pods = client.list("Pod", field_selector=f"spec.nodeName={node}")
        return {p["metadata"].get("uid", ""): (ko.namespace(p), ko.name(p)) for p in pods if p["metadata"].get("uid")}
    return f


def pod_event(client: Any, node: str = "") -> Callable[[str, str, str, str], None]:
    """Records a Warning event on a pod (the guards' report action)."""
    def f(namespace: str, name: str, reason: str, message: str) -> None:
        client.create({
            "apiVersion": "v1", "kind": "Event",
            "metadata": {"generateName": f"{name}.", "namespace": namespace},
            "involvedObject": {"apiVersion": "v1", "kind": "Pod", "name": name, "namespace": namespace},
            "reason": reason, "message": message, "type": "Warning",
            "source": {"component": "nos-slice-guard", "host": node}})
    return f


def pod_evictor(client: Any, node: str = "") -> Callable[[str, str, str], None]:
    """Records a ``HBMBudgetExceeded`` Warning event on the pod, then deletes it (its controller,
    if any, recreates it against a fresh slice)."""
    def f(namespace: str, name: str, reason: str) -> None:
        try:
            client.create({
                "apiVersion": "v1", "kind": "Event",
                "metadata": {"generateName": f"{name}.", "namespace": namespace},
                "involvedObject": {"apiVersion": "v1", "kind": "Pod", "name": name, "namespace": namespace},
                "reason": "HBMBudgetExceeded", "message": reason, "type": "Warning",
                "source": {"component": "nos-hbm-guard", "host": node}})
        except Exception as e:  # noqa: BLE001 - the eviction matters, the event is a courtesy
            log.warning("event for %s/%s not recorded: %s", namespace, name, e)
        client.delete("Pod", name, namespace)
    return f
