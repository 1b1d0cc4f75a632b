"""The operator's hardware-facing pieces on a real MI355X, measured (not the benchmark workload):

* the native amd-smi device map (physical GPU <-> logical partitions, HIP ordinals, render nodes)
  and a timed re-enumeration (the step every flip pays);
* the spawned commit-barrier helper: wall time of a vote including process spawn, HIP init and
  ncclCommInitAll over every logical device, and its own phase split (the agent pays this per
  commit because a flip changes the device set) — the xGMI P2P token ring vs the RCCL
  communicator, native executable vs the Python helper;
* the spawned probe round on every logical device;
* amd-smi power / clock / activity at rest.

    python tools/operator_gpu_report.py --out gpurun_out/operator.json
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from walkai_nos_amd.device.amdsmi import NativeAmdSmi  # noqa: E402
from walkai_nos_amd.parallel.spawned import SpawnedNodeBarrier, spawned_probe_round  # noqa: E402


def main() -> int:
    out = {}
    smi = NativeAmdSmi()
    m = smi.device_map()
    out["device_map"] = m.describe()
    out["gpus"] = [g.__dict__ for g in m.gpus]
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        smi.enumerate(reinit=True)
        ts.append(1e3 * (time.perf_counter() - t0))
    out["reenumerate_ms"] = {"min": round(min(ts), 2), "max": round(max(ts), 2)}
    out["power_clock_idle"] = smi.power_clock(0)
    out["process_count"] = smi.process_count(0)
    n = len(m.devices)
    # the commit barrier per helper flavour: native executable with the init tunables (the agent's
    # default), native with RCCL's default init, and the round-2 Python helper; a first call on a
    # fresh box pays cold file-cache costs, so every flavour runs 4 times (1 vetoed)
    flavours = {"native_xgmi": ({}, True, "xgmi"), "native_rccl": ({}, True, "rccl"),
                "native_rccl_defaults": ({"NOS_BARRIER_KEEP_NCCL_ENV": "1"}, True, "rccl"),
                "python_rccl": ({}, False, "rccl")}
    out["commit_barrier"] = {}
    for name, (env, native, backend) in flavours.items():
        votes = []
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            for ok in (True, True, True, False):
                b = SpawnedNodeBarrier(n, backend=backend, native=native)
                t0 = time.perf_counter()
                res = b.vote_all([ok] * n)
                votes.append({"votes_ok": ok, "result": res, "wall_ms": round(1e3 * (time.perf_counter() - t0), 1),
                              "helper": b.last})
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        walls = sorted(v["wall_ms"] for v in votes[1:])
        out["commit_barrier"][name] = {"calls": votes, "wall_ms_warm_median": walls[len(walls) // 2],
                                       "correct": [v["result"] for v in votes] == [True, True, True, False]}
    t0 = time.perf_counter()
    targets = [(d.hip_id, None, f"gpu{d.gpu_index}.p{d.partition_index}") for d in m.devices]
    out["probe_round"] = {"results": spawned_probe_round(targets), "wall_s": round(time.perf_counter() - t0, 2)}
    path = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else "gpurun_out/operator.json"
    os.makedirs(os.path.dirname(path), exist_ok=True)
    json.dump(out, open(path, "w"), indent=1, default=str)
    print(json.dumps({k: out[k] for k in ("reenumerate_ms", "power_clock_idle", "commit_barrier")}, default=str))
    return 0


if __name__ == "__main__":
    sys.exit(main())
