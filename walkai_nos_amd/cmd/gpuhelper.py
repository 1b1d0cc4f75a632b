"""Short-lived GPU helper spawned by the node agents: commit barrier and slice probe.

The partition agent flips compute-partition modes, and a mode switch is refused while any process
holds a KFD context on the GPU.  So the agent itself never initialises HIP (no ``libamdhip64`` in
its address space, no ``/dev/kfd`` open): everything that needs the GPU runs here, in a child
process the agent spawns *after* a flip and that exits before the next one.  Being a fresh
process is also what makes the child see the new topology — HIP enumerates devices once per
process, so after SPX -> CPX only a new process sees the eight partitions of each GPU.

Sub-commands (each prints exactly one JSON line on stdout):

``barrier --votes 1,1,0,... [--expect N] [--backend rccl|local]``
    one vote per logical device (in HIP ordinal order); the RCCL backend checks that this
    process sees exactly ``N`` devices, builds one communicator clique over all of them
    (``ncclCommInitAll``, ``csrc/rccl_barrier.cpp``) and sums the votes with one grouped 4-byte
    all-reduce over xGMI.  ``local`` sums on the CPU (tests, nodes without RCCL).

``probe --targets '[[dev, cus|null, label], ...]' [--backend hip|fake]``
    MFMA bf16/fp32 and HBM copy probes (``csrc/probe.hip``) on each target (a HIP device, or a
    CU-masked stream of one for CU-mask slices).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
import time
from typing import Any, Dict, List, Optional


def _barrier(votes: List[int], expect: Optional[int], backend: str) -> Dict[str, Any]:
    out: Dict[str, Any] = {"n": len(votes)}
    if backend == "local":
        out.update(sum=sum(votes), seen=len(votes) if expect is None else expect, init_ms=0.0, allreduce_ms=0.0)
        return out
    from ..ops.native import load
    L = load("libnos_barrier.so")
    L.nos_barrier_last_error.restype = ctypes.c_char_p
    L.nos_barrier_init_all.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_void_p)]
    L.nos_barrier_allreduce_all.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32),
                                            ctypes.POINTER(ctypes.c_int32)]
    L.nos_barrier_destroy_all.argtypes = [ctypes.c_void_p]
    t0 = time.perf_counter()
    seen = L.nos_barrier_device_count()
    out["seen"] = seen
    if seen < 0:
        out.update(sum=0, error=L.nos_barrier_last_error().decode())
        return out
    if (expect is not None and seen != expect) or seen != len(votes):
        # a partition missing (or extra) after the flip: the node did not come up as planned
        out.update(sum=0, error=f"helper sees {seen} HIP devices, the device map has "
                                f"{expect if expect is not None else len(votes)}")
        return out
    devs = (ctypes.c_int * seen)(*range(seen))
    h = ctypes.c_void_p()
    rc = L.nos_barrier_init_all(seen, devs, ctypes.byref(h))
    t1 = time.perf_counter()
    out["init_ms"] = round(1e3 * (t1 - t0), 3)
    if rc != 0:
        out.update(sum=0, error=f"init: {L.nos_barrier_last_error().decode()} (rc={rc})")
        return out
    try:
        arr = (ctypes.c_int32 * seen)(*[1 if v else 0 for v in votes])
        res = ctypes.c_int32(0)
        rc = L.nos_barrier_allreduce_all(h, arr, ctypes.byref(res))
        out["allreduce_ms"] = round(1e3 * (time.perf_counter() - t1), 3)
        if rc != 0:
            out.update(sum=0, error=f"allreduce: {L.nos_barrier_last_error().decode()} (rc={rc})")
        else:
            out["sum"] = int(res.value)
    finally:
        L.nos_barrier_destroy_all(h)
    return out


def _probe(targets: List[list], backend: str) -> Dict[str, Any]:
    results: Dict[str, Any] = {}
    for dev, cus, label in targets:
        if backend == "fake":
            n = len(cus) if cus else 256
            results[label] = {"n_cus": n, "bf16_tflops": round(9.6 * n, 1), "fp32_tflops": round(0.6 * n, 2),
                              "hbm_gbps": 5000.0}
            continue
        try:
            from ..controllers.agent.probe import hip_probe
            results[label] = hip_probe(int(dev), cus, label)
        except Exception as e:  # noqa: BLE001 - one bad partition must not hide the others
            results[label] = {"error": str(e)[:200]}
    return {"slices": results}


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser("nos gpu helper")
    sub = ap.add_subparsers(dest="cmd", required=True)
    b = sub.add_parser("barrier")
    b.add_argument("--votes", required=True)
    b.add_argument("--expect", type=int, default=None)
    b.add_argument("--backend", choices=("rccl", "local"), default="rccl")
    p = sub.add_parser("probe")
    p.add_argument("--targets", required=True)
    p.add_argument("--backend", choices=("hip", "fake"), default="hip")
    args = ap.parse_args(argv)
    if args.cmd == "barrier":
        votes = [int(v) for v in args.votes.split(",") if v != ""]
        res = _barrier(votes, args.expect, args.backend)
    else:
        res = _probe(json.loads(args.targets), args.backend)
    print(json.dumps(res, sort_keys=True), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
