"""Run pods as processes, the way kubelet does: each pod is a fresh process whose environment is
what the nos slice device plugin's ``Allocate`` returns for its slice (``HSA_CU_MASK``,
``NOS_HBM_LIMIT_BYTES``, ``LD_PRELOAD`` of the HBM-budget shim, ``NOS_SLICE_IDS``).

The launcher itself never touches the GPU (no torch, no HIP: it only places slices, calls
``Allocate`` and manages children), so every GPU context on the card belongs to a pod, as on a
node.  All pods load and warm up first; they start their timed loops at one wall-clock instant and
stop at another, so the window is the same for all of them.

Used by ``tools/multiproc.py`` (the 1/3/5/7 sharing table of ref
``demos/gpu-sharing-comparison/README.md:62-71`` and BASELINE config 3, pods as processes) and by
``tests/test_gpu_native.py`` (two concurrent slices' census sets are disjoint).
"""
from __future__ import annotations

import json
import os
import select
import subprocess
import sys
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SHIM = os.path.join(ROOT, "walkai_nos_amd", "_native", "libnos_hbmlimit.so")
BDF = "0000:00:00.0"


@dataclass
class PodSpec:
    profile: str                    # slice profile: "<c>cu.<m>gb" (dedicated CUs) or "<m>gb" (shared pool)
    name: str = ""


@dataclass
class PodProc:
    spec: PodSpec
    slice_id: str
    env: Dict[str, str]
    proc: Optional[subprocess.Popen] = None
    result: Dict[str, Any] = field(default_factory=dict)


def _place(profiles: Sequence[str], cu_count: int):
    from ..device.slicing_client import MemorySliceStore
    from ..models.slicing.cumask import place
    wanted = [(f"{BDF}::s{i}", p) for i, p in enumerate(profiles)]
    slices = place([], wanted, cu_count)
    store = MemorySliceStore()
    store.save({0: slices})
    return wanted, {s.id: s for s in slices}, store


def _plugin(prof: str, store: Any, cu_count: int, shim_path: str, start_gate: Any = None) -> Any:
    from ..deviceplugin.server import SliceDevicePlugin
    from ..models.slicing.profile import as_resource_name
    return SliceDevicePlugin(as_resource_name(prof), store, {0: "/dev/dri/renderD128"}, cu_count=cu_count,
                             shim_path=shim_path, socket_dir="/tmp", start_gate=start_gate)


def allocate_envs(profiles: Sequence[str], cu_count: int = 256, shim: bool = True,
                  shim_path: str = SHIM) -> List[Dict[str, str]]:
    """Place one slice per profile on GPU 0 (``cumask.place``, largest first, rows never moved) and
    return, per pod in order, the container env the device plugin's ``Allocate`` hands kubelet."""
    from ..device.protos import dp
    wanted, by_id, store = _place(profiles, cu_count)
    envs = []
    for sid, prof in wanted:
        req = dp.AllocateRequest()
        req.container_requests.add(devicesIDs=[by_id[sid].id])
        env = dict(_plugin(prof, store, cu_count, shim_path).Allocate(req, None).container_responses[0].envs)
        if not shim:
            env.pop("LD_PRELOAD", None)
        envs.append(env)
    return envs


def run_pods(profiles: Sequence[str], seconds: float = 10.0, shim: bool = True, census: bool = False,
             graphs: bool = True, ready_timeout: float = 600.0, extra_env: Optional[Dict[str, str]] = None,
             cu_count: int = 256, stagger_s: float = 0.0,
             per_pod_env: Optional[Sequence[Dict[str, str]]] = None, sequential: bool = False,
             gate: bool = False, churn: Optional[Tuple[Sequence[int], Sequence[str]]] = None,
             gate_timeout: float = 20.0, settle_s: float = 0.0) -> Dict[str, Any]:
    """Start one process per profile, release them together, collect their JSON lines.
    ``stagger_s``: wait this long between pod starts (pods of a node start at different times);
    ``per_pod_env``: env overrides of pod i (after ``extra_env``); ``sequential``: start pod i+1
    only once pod i is READY (its queues exist), so the pods' start order is their index.
    ``gate``: start every pod at once, as kubelet starts a Deployment, each through the slice
    plugin's ``PreStartContainer`` with one start gate for the GPU (``deviceplugin/startgate.py``,
    its real KFD readiness probe): the order is whatever the gate imposes. ``churn``: (indices,
    profiles) — once the first pods are READY, stop those pods and start new ones of those profiles
    (through the gate when ``gate``; the indices are then positions in the gate's start order, so
    "three pods of one start parity" is ``[0, 2, 4]``); the window measures the pods running after
    the churn. ``settle_s``: after stopping them, wait (at most this long) until the KFD lists that
    many fewer processes with compute queues — a process's queues can outlive its exit for a while."""
    from ..device.protos import dp
    from ..deviceplugin.startgate import StartGate
    new_profiles = list(churn[1]) if churn else []
    all_profiles = list(profiles) + new_profiles
    envs = allocate_envs(all_profiles, cu_count, shim)
    wanted, _, store = _place(all_profiles, cu_count)
    start_gate = StartGate(timeout=gate_timeout) if gate else None
    pods: List[PodProc] = []
    base = dict(os.environ)
    base["PYTHONPATH"] = ROOT + (os.pathsep + base["PYTHONPATH"] if base.get("PYTHONPATH") else "")
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-u", "-m", "walkai_nos_amd.dataplane.client", "--seconds", str(seconds)]
    if census:
        cmd.append("--census")
    if not graphs:
        cmd.append("--no-graph")
    import tempfile
    import threading
    logs: List[Any] = [None] * len(all_profiles)
    procs: List[Optional[PodProc]] = [None] * len(all_profiles)
    waited: List[float] = [0.0] * len(all_profiles)

    def start(i: int) -> None:
        prof, env = all_profiles[i], envs[i]
        if start_gate is not None:
            req = dp.PreStartContainerRequest(devicesIDs=[env.get("NOS_SLICE_IDS", "")])
            t0 = time.time()
            _plugin(prof, store, cu_count, SHIM, start_gate).PreStartContainer(req, None)
            waited[i] = time.time() - t0
        e = {**base, **env, "NOS_POD_SEED": str(i), **(extra_env or {}),  # extra_env overrides Allocate's
             **(per_pod_env[i] if per_pod_env and i < len(per_pod_env) else {})}
        log = tempfile.TemporaryFile(mode="w+")  # a full stderr pipe would stall the pod
        logs[i] = log
        p = subprocess.Popen(cmd, cwd=ROOT, env=e, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                             stderr=log, text=True)
        procs[i] = PodProc(PodSpec(prof, f"pod{i}"), env.get("NOS_SLICE_IDS", ""), env, p)

    def start_all(idx: Sequence[int]) -> None:
        if gate:                        # every container asks at once, the gate orders them
            ts = [threading.Thread(target=start, args=(i,)) for i in idx]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            return
        for i in idx:
            start(i)
            if sequential:
                _wait_ready([procs[i]], [p for p in procs if p], _live(logs), ready_timeout)
            if stagger_s > 0:
                time.sleep(stagger_s)

    stopped: List[int] = list(churn[0]) if churn else []
    try:
        first = list(range(len(profiles)))
        start_all(first)
        live = [procs[i] for i in first]
        _wait_ready([p for p in live if not sequential or gate], live, [logs[i] for i in first], ready_timeout)
        if churn:
            if gate:                    # start-order positions -> pod indices (slice s<i> is pod i)
                order = [int(sid.rsplit("::s", 1)[1]) for _, sid in start_gate.order]
                stopped = [order[k] for k in stopped]
            kfd = None
            if settle_s > 0:
                from ..deviceplugin.startgate import KfdProbe
                kfd = KfdProbe()
                before = len(kfd.ready_pids())
            for i in stopped:
                procs[i].proc.kill()
                procs[i].proc.wait()
            if kfd is not None:
                t0 = time.time()
                while len(kfd.ready_pids()) > before - len(stopped) and time.time() - t0 < settle_s:
                    time.sleep(0.02)
                settled = (round(time.time() - t0, 3), len(kfd.ready_pids()), before)
            later = list(range(len(profiles), len(all_profiles)))
            start_all(later)
            _wait_ready([procs[i] for i in later], [procs[i] for i in later], [logs[i] for i in later],
                        ready_timeout)
        running = [i for i in range(len(all_profiles)) if procs[i] is not None and i not in stopped]
        go = time.time() + 1.0
        for i in running:
            procs[i].proc.stdin.write(f"GO {go:.6f}\n")
            procs[i].proc.stdin.flush()
        for i in running:
            p = procs[i]
            out, _ = p.proc.communicate(timeout=seconds + 300)
            line = next((ln for ln in reversed(out.splitlines()) if ln.startswith("{")), None)
            if p.proc.returncode != 0 or line is None:
                raise RuntimeError(f"{p.spec.name} failed (rc={p.proc.returncode}): {_tail(logs[i])}")
            p.result = json.loads(line)
    finally:
        for p in procs:
            if p is not None and p.proc.poll() is None:
                p.proc.kill()
                p.proc.wait()
        for log in logs:
            if log is not None:
                log.close()
    out = summarize([procs[i] for i in running], seconds)
    if gate:
        order = [s for _, s in start_gate.order]
        out["gate"] = {"order": order, "waited_s": [round(waited[i], 3) for i in range(len(all_profiles))],
                       "timeouts": start_gate.timeouts}
    if churn:
        out["churn"] = {"stopped": stopped, "started": list(range(len(profiles), len(all_profiles)))}
        if settle_s > 0:
            out["churn"]["settle"] = {"waited_s": settled[0], "kfd_ready_after": settled[1],
                                      "kfd_ready_before": settled[2]}
    return out


def _live(logs: List[Any]) -> List[Any]:
    return [log for log in logs if log is not None]


def _tail(log) -> str:
    log.seek(0)
    return log.read()[-2000:]


def _wait_ready(subset: List[PodProc], pods: List[PodProc], logs: list, timeout: float) -> None:
    """Until every pod of ``subset`` printed READY (a pod that exits first raises with its log)."""
    deadline = time.time() + timeout
    waiting = {id(p.proc.stdout): p for p in subset}
    index = {id(p): i for i, p in enumerate(pods)}
    while waiting:
        left = deadline - time.time()
        if left <= 0:
            raise TimeoutError(f"{len(waiting)} pod(s) not ready after {timeout}s")
        r, _, _ = select.select([p.proc.stdout for p in waiting.values()], [], [], min(left, 5.0))
        for f in r:
            pod = waiting[id(f)]
            ln = f.readline()
            if not ln:
                pod.proc.wait()
                log = logs[index[id(pod)]] if index.get(id(pod), len(logs)) < len(logs) else None
                raise RuntimeError(f"{pod.spec.name} exited before READY (rc={pod.proc.returncode}): "
                                   f"{_tail(log) if log is not None else ''}")
            if ln.strip() == "READY":
                del waiting[id(f)]


def summarize(pods: List[PodProc], seconds: float) -> Dict[str, Any]:
    total = sum(p.result.get("inferences", 0) for p in pods)
    window = max((p.result.get("window_s", seconds) for p in pods), default=seconds)
    per = []
    for p in pods:
        r = p.result
        row = {"pod": p.spec.name, "profile": p.spec.profile, "hsa_cu_mask": r.get("hsa_cu_mask"),
               "slice_cus": r.get("slice_cus"), "inferences": r.get("inferences", 0),
               "inf_per_s": round(r.get("inferences", 0) / max(1e-9, r.get("window_s", seconds)), 2),
               "latency_ms": r.get("latency_ms"), "hbm": r.get("hbm"), "boot_s": r.get("boot_s")}
        if "census" in r:
            row["census_cus"] = r["census"]["cus"]
            row["census_xcds"] = r["census"]["xcds"]
        per.append(row)
    out: Dict[str, Any] = {"pods": len(pods), "window_s": round(window, 3), "inferences": total,
                           "aggregate_inf_per_s": round(total / window, 2),
                           "mean_latency_ms": round(sum((p.result.get("latency_ms") or {}).get("mean", 0) for p in pods)
                                                    / max(1, len(pods)), 3),
                           "per_pod": per}
    sets = [set(p.result["census"]["ids"]) for p in pods if "census" in p.result]
    if len(sets) == len(pods) and pods:
        overlaps = sum(1 for i in range(len(sets)) for j in range(i + 1, len(sets)) if sets[i] & sets[j])
        out["census_pairs_overlapping"] = overlaps
    return out
