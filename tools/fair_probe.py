"""Why memory-only pods share one MI355X unevenly: per pod, the rate it got next to what the
hardware says about it while all pods run.

Memory-only slices (the MPS analogue, ``amd.com/gpu-<m>gb``) share every CU of the shared pool; how
the GPU divides them among pods is up to the command processor's hardware scheduler. Round 4
measured two rate classes at 5 pods (87 vs 65 inf/s, ``profiles/fairness_r4_56.json``) and at 7.
This tool starts N pods as processes with the environment ``Allocate`` gives them (one at a time,
so each pod's KFD pid is the one amd-smi lists when it appears: the box runs in its own PID
namespace), releases them together, and samples every 100 ms during the common window:

* amd-smi per process: ``cu_occupancy`` (CU-equivalents of its waves in flight) and ``evicted_time``
  (time its queues were switched out by the hardware scheduler);
* the KFD's ``/sys/class/kfd/kfd/proc/<pid>/queues/*`` once: how many hardware queues the process
  has and of which type.

    python tools/fair_probe.py --pods 5 --reps 2 [--env '{"GPU_MAX_HW_QUEUES": "1"}'] --out gpurun_out/fair_probe.json
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from walkai_nos_amd.dataplane.procs import ROOT, allocate_envs  # noqa: E402


def kfd_queues(pid: int):
    out = []
    for q in sorted(glob.glob(f"/sys/class/kfd/kfd/proc/{pid}/queues/*")):
        row = {"id": os.path.basename(q)}
        for f in ("type", "size", "gpuid"):
            try:
                with open(os.path.join(q, f)) as fh:
                    row[f] = fh.read().strip()
            except OSError:
                pass
        out.append(row)
    return out


def run(n: int, seconds: float, extra_env: dict, smi) -> dict:
    envs = allocate_envs(["16gb"] * n)
    base = dict(os.environ)
    base["PYTHONPATH"] = ROOT + (os.pathsep + base["PYTHONPATH"] if base.get("PYTHONPATH") else "")
    pods, host = [], []
    try:
        for i, env in enumerate(envs):
            before = set(smi.process_info(0))
            e = {**base, **env, "NOS_POD_SEED": str(i), **extra_env}
            p = subprocess.Popen([sys.executable, "-u", "-m", "walkai_nos_amd.dataplane.client", "--seconds",
                                  str(seconds)], cwd=ROOT, env=e, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                 stderr=subprocess.DEVNULL, text=True)
            pods.append(p)
            if p.stdout.readline().strip() != "READY":
                raise RuntimeError(f"pod {i} did not get ready")
            new, t0 = set(), time.time()
            while not new and time.time() - t0 < 8.0:
                new = set(smi.process_info(0)) - before - set(host)
                time.sleep(0.05)
            host.append(sorted(new)[0] if len(new) == 1 else -1)
        queues = {h: kfd_queues(h) for h in host if h > 0}
        go = time.time() + 0.5
        for p in pods:
            p.stdin.write(f"GO {go:.6f}\n")
            p.stdin.flush()
        while time.time() < go + 0.2:
            time.sleep(0.01)
        samples = []
        ev0 = {pid: st.evicted_ms for pid, st in smi.process_info(0).items()}
        while time.time() < go + seconds - 0.2:
            info = smi.process_info(0)
            samples.append({pid: st.cu_occupancy for pid, st in info.items() if pid in host})
            time.sleep(0.1)
        ev1 = {pid: st.evicted_ms for pid, st in smi.process_info(0).items()}
        res = []
        for p in pods:
            out, _ = p.communicate(timeout=seconds + 120)
            res.append(json.loads(next(x for x in reversed(out.splitlines()) if x.startswith("{"))))
    finally:
        for p in pods:
            if p.poll() is None:
                p.kill()
                p.wait()
    per = []
    for i, (r, h) in enumerate(zip(res, host)):
        occ = [s.get(h) for s in samples if s.get(h) is not None]
        per.append({"pod": i, "host_pid": h, "inf_per_s": round(r["inferences"] / max(1e-9, r["window_s"]), 2),
                    "cu_occupancy_mean": round(sum(occ) / len(occ), 1) if occ else None,
                    "cu_occupancy_max": max(occ) if occ else None,
                    "evicted_ms_in_window": (ev1.get(h, 0) - ev0.get(h, 0)) if h > 0 else None,
                    "queues": queues.get(h), "latency_ms": r.get("latency_ms"),
                    "gpu_max_hw_queues": r.get("gpu_max_hw_queues")})
    rates = [p["inf_per_s"] for p in per]
    return {"pods": n, "env": extra_env, "max_over_min": round(max(rates) / min(rates), 3) if min(rates) > 0 else None,
            "aggregate_inf_per_s": round(sum(rates), 1), "per_pod": per, "samples": len(samples)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", default="5")
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--env", default="{}")
    ap.add_argument("--out", default="gpurun_out/fair_probe.json")
    a = ap.parse_args()
    from walkai_nos_amd.device.amdsmi import NativeAmdSmi
    smi = NativeAmdSmi()
    rows = []
    for n in [int(x) for x in a.pods.split(",")]:
        for rep in range(a.reps):
            r = run(n, a.seconds, json.loads(a.env), smi)
            r["rep"] = rep
            rows.append(r)
            print(json.dumps({k: r[k] for k in ("pods", "rep", "max_over_min", "aggregate_inf_per_s")}),
                  [(p["inf_per_s"], p["cu_occupancy_mean"], p["evicted_ms_in_window"], len(p["queues"] or []))
                   for p in r["per_pod"]], flush=True)
            with open(a.out, "w") as f:
                json.dump(rows, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
