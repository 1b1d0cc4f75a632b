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
from typing import Any, Dict, List, Optional, Sequence

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


def allocate_envs(profiles: Sequence[str], cu_count: int = 256, shim: bool = True,
                  shim_path: str = SHIM) -> List[Dict[str, str]]:
    """Place one slice per profile on GPU 0 (``cumask.place``, largest first, rows never moved) and
    return, per pod in order, the container env the device plugin's ``Allocate`` hands kubelet."""
    from ..device.protos import dp
    from ..device.slicing_client import MemorySliceStore
    from ..deviceplugin.server import SliceDevicePlugin
    from ..models.slicing.cumask import place
    from ..models.slicing.profile import as_resource_name
    wanted = [(f"{BDF}::s{i}", p) for i, p in enumerate(profiles)]
    slices = place([], wanted, cu_count)
    store = MemorySliceStore()
    store.save({0: slices})
    by_id = {s.id: s for s in slices}
    envs = []
    for sid, prof in wanted:
        plug = SliceDevicePlugin(as_resource_name(prof), store, {0: "/dev/dri/renderD128"}, cu_count=cu_count,
                                 shim_path=shim_path, socket_dir="/tmp")
        req = dp.AllocateRequest()
        req.container_requests.add(devicesIDs=[by_id[sid].id])
        env = dict(plug.Allocate(req, None).container_responses[0].envs)
        if not shim:
            env.pop("LD_PRELOAD", None)
        envs.append(env)
    return envs


def run_pods(profiles: Sequence[str], seconds: float = 10.0, shim: bool = True, census: bool = False,
             graphs: bool = True, ready_timeout: float = 600.0, extra_env: Optional[Dict[str, str]] = None,
             cu_count: int = 256, stagger_s: float = 0.0,
             per_pod_env: Optional[Sequence[Dict[str, str]]] = None, sequential: bool = False) -> Dict[str, Any]:
    """Start one process per profile, release them together, collect their JSON lines.
    ``stagger_s``: wait this long between pod starts (pods of a node start at different times);
    ``per_pod_env``: env overrides of pod i (after ``extra_env``); ``sequential``: start pod i+1
    only once pod i is READY (its queues exist), so the pods' start order is their index."""
    envs = allocate_envs(profiles, cu_count, shim)
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
    logs = []
    try:
        for i, (prof, env) in enumerate(zip(profiles, envs)):
            e = {**base, **env, "NOS_POD_SEED": str(i), **(extra_env or {}),  # extra_env overrides Allocate's
                 **(per_pod_env[i] if per_pod_env and i < len(per_pod_env) else {})}
            log = tempfile.TemporaryFile(mode="w+")  # a full stderr pipe would stall the pod
            logs.append(log)
            p = subprocess.Popen(cmd, cwd=ROOT, env=e, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                 stderr=log, text=True)
            pods.append(PodProc(PodSpec(prof, f"pod{i}"), env.get("NOS_SLICE_IDS", ""), env, p))
            if sequential:
                _wait_ready(pods[-1:], pods, logs, ready_timeout)
            if stagger_s > 0:
                time.sleep(stagger_s)
        _wait_ready([p for p in pods if not sequential], pods, logs, ready_timeout)
        go = time.time() + 1.0
        for p in pods:
            p.proc.stdin.write(f"GO {go:.6f}\n")
            p.proc.stdin.flush()
        for i, p in enumerate(pods):
            out, _ = p.proc.communicate(timeout=seconds + 300)
            line = next((ln for ln in reversed(out.splitlines()) if ln.startswith("{")), None)
            if p.proc.returncode != 0 or line is None:
                raise RuntimeError(f"{p.spec.name} failed (rc={p.proc.returncode}): {_tail(logs[i])}")
            p.result = json.loads(line)
    finally:
        for p in pods:
            if p.proc is not None and p.proc.poll() is None:
                p.proc.kill()
                p.proc.wait()
        for log in logs:
            log.close()
    return summarize(pods, seconds)


def _tail(log) -> str:
    log.seek(0)
    return log.read()[-2000:]


def _wait_ready(subset: List[PodProc], pods: List[PodProc], logs: list, timeout: float) -> None:
    """Until every pod of ``subset`` printed READY (a pod that exits first raises with its log)."""
    deadline = time.time() + timeout
    waiting = {id(p.proc.stdout): p for p in subset}
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
                raise RuntimeError(f"{pod.spec.name} exited before READY (rc={pod.proc.returncode}): "
                                   f"{_tail(logs[pods.index(pod)])}")
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
