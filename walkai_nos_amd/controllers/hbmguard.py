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

    @property
    def key(self) -> Tuple[Any, ...]:
        return (self.gpu, self.pod) if self.pod is not None else (self.gpu, self.slice_ids)


@dataclass
class Violation:
    account: Account
    limit: int
    strikes: int
    action: str   # "report" | "evict" | "evicted" (the pod was deleted this check)


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
                 partitions: Optional[Callable[[], Mapping[str, Tuple[int, int]]]] = None):
        if action not in ACTIONS:
            raise ValueError(f"hbm guard action {action!r} not in {ACTIONS}")
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

    # -- one pass -------------------------------------------------------------------------------
    def accounts(self) -> List[Account]:
        """Every pod's (or slice set's) VRAM on each sliced GPU, from one amd-smi sample."""
        slices = self.slices() or {}
        budget_of: Dict[str, Tuple[int, int]] = {s.id: (g, int(s.hbm_bytes)) for g, ss in slices.items() for s in ss}
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
        for g in sorted({g for g, _ in budget_of.values()}):
            try:
                procs = self.smi.process_memory(g)
            except Exception as e:  # noqa: BLE001 - a GPU mid-flip or off the bus: skip it this pass
                log.debug("process list of GPU %d failed: %s", g, e)
                continue
            for pid, nbytes in sorted(procs.items()):
                pod: Optional[PodKey] = None
                uid = pod_uid_of(pid, self.proc_root)
                if uid is not None:
                    # a pod's process: its cgroup is authoritative (an environment can be forged by
                    # a child process to charge another pod's slice); a pod holding no device of
                    # this GPU (the agent's own probe helpers, say) is reported, never evicted
                    pod = pod_of_uid(uid)
                    ids: Tuple[str, ...] = tuple(sorted(i for i in ids_of_pod.get(pod, ()) if budget_of[i][0] == g)) \
                        if pod is not None else ()
                else:
                    ids = tuple(i for i in slice_ids_of(pid, self.proc_root) if budget_of.get(i, (None,))[0] == g)
                    pod = pod_of_id.get(ids[0]) if ids else None
                if not ids:
                    self.unattributed[g] = self.unattributed.get(g, 0) + nbytes
                    continue
                a = Account(g, ids, sum(budget_of[i][1] for i in ids), pod)
                a = out.setdefault(a.key, a)
                a.used += nbytes
                a.pids.append(pid)
        return list(out.values())

    def check(self) -> List[Violation]:
        """One pass: sample, compare, act. Returns the accounts over budget."""
        self.checks += 1
        accts = self.accounts()
        self.last = accts
        seen = set()
        found: List[Violation] = []
        for a in accts:
            seen.add(a.key)
            limit = a.budget + self.slack_bytes * max(1, len(a.pids))   # runtime overhead per process
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
        self._evicted = {p: c + 1 for p, c in self._evicted.items() if c < 30}
        self._export(accts)
        return found

    def _export(self, accts: List[Account]) -> None:
        series = set()
        for a in accts:
            ns, name = a.pod if a.pod is not None else ("", ",".join(a.slice_ids))
            labels = (self.node, str(a.gpu), ns, name)
            _used.labels(*labels).set(a.used)
            _budget.labels(*labels).set(a.budget)
            series.add(labels)
        for labels in self._series - series:
            for gauge in (_used, _budget):
                try:
                    gauge.remove(*labels)
                except KeyError:
                    pass
        self._series = series
        for g, b in self.unattributed.items():
            _unattributed.labels(self.node, str(g)).set(b)

    def register(self, mgr: Any, interval: float = 10.0) -> None:
        """Run on the agent's manager (node-local: no leader election)."""
        if self.action != "off":
            mgr.add_runnable("hbm-guard", self.check, interval, needs_leader=False)


def node_pods_by_uid(client: Any, node: str) -> Callable[[], Dict[str, PodKey]]:
    """pod UID -> (namespace, name) of the pods bound to ``node``."""
    from ..kube import objects as ko

    def f() -> Dict[str, PodKey]:
        pods = client.list("Pod", field_selector=f"spec.nodeName={node}")
        return {p["metadata"].get("uid", ""): (ko.namespace(p), ko.name(p)) for p in pods if p["metadata"].get("uid")}
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
