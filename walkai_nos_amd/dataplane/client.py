"""One pod's inference process (the reference demo client, ref
``demos/gpu-sharing-comparison/client/main.py:19-35``: YOLOS-small, batch 1, one image, timed
inference in an endless loop), driven by :mod:`walkai_nos_amd.dataplane.procs`.

The process gets exactly what kubelet gives a container: ``HSA_CU_MASK`` (its CU set, applied by
the HSA runtime to every queue of the process), ``NOS_HBM_LIMIT_BYTES`` + ``LD_PRELOAD`` of the
HBM-budget shim, ``NOS_SLICE_IDS``.  It loads the model, warms up (and captures a HIP graph of one
inference), then prints ``READY`` and waits on stdin for ``GO <epoch>``; from that wall-clock
instant it runs one inference at a time — replay, synchronize, record the wall latency, exactly
the reference's loop — until ``epoch + seconds``.  A workgroup census (which physical CUs this
process's kernels run on) is taken while every pod is busy.  It prints one JSON line and exits.

    python -m walkai_nos_amd.dataplane.client --seconds 10 [--no-graph] [--census]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time
from typing import Any, Dict, List


def _stats(v: List[float]) -> Dict[str, float]:
    if not v:
        return {"n": 0}
    s = sorted(v)
    return {"n": len(s), "mean": round(sum(s) / len(s), 3), "p50": round(s[len(s) // 2], 3),
            "p99": round(s[min(len(s) - 1, int(0.99 * len(s)))], 3), "max": round(s[-1], 3)}


def _census() -> Dict[str, Any]:
    from ..ops import probe as P
    pl = P.census(n_wg=4096, spin=4000)
    cus = sorted({(p["xcc"], p["se"], p["sh"], p["cu"]) for p in pl})
    return {"cus": len(cus), "xcds": sorted({c[0] for c in cus}), "ids": ["%d.%d.%d.%d" % c for c in cus]}


def _shim() -> Dict[str, Any]:
    try:
        lib = ctypes.CDLL(None)
        lib.nos_hbm_shim_loaded.restype = ctypes.c_int
        for f in ("nos_hbm_limit_bytes", "nos_hbm_peak_bytes", "nos_hbm_live_bytes"):
            getattr(lib, f).restype = ctypes.c_size_t
        if not lib.nos_hbm_shim_loaded():
            return {"loaded": False}
        return {"loaded": True, "limit_bytes": int(lib.nos_hbm_limit_bytes()),
                "peak_bytes": int(lib.nos_hbm_peak_bytes()), "live_bytes": int(lib.nos_hbm_live_bytes())}
    except (AttributeError, OSError):
        return {"loaded": False}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser("nos pod client")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--census", action="store_true")
    ap.add_argument("--hw", default="800,1066")
    ap.add_argument("--streams", type=int, default=int(os.environ.get("NOS_POD_STREAMS", "1")),
                    help="HIP streams the inference loop rotates over (one inference at a time)")
    args = ap.parse_args(argv)
    t_boot = time.perf_counter()
    import torch

    from ..models.workload.yolos import YolosSmall, demo_input
    from ..ops import kernels as K
    K.set_backend("hip")
    hw = tuple(int(x) for x in args.hw.split(","))
    dev = "cuda:0"
    model = YolosSmall().to(dev).eval()
    x = demo_input(1, hw, dev, seed=int(os.environ.get("NOS_POD_SEED", "0")))
    streams = [torch.cuda.Stream() for _ in range(max(1, args.streams))]
    if os.environ.get("NOS_POD_EAGER_QUEUES", "0") == "1":
        # touch every stream back to back before anything else: HIP creates the process's hardware
        # queues at first use, so they are created together (consecutive queues of one process)
        for st in streams:
            with torch.cuda.stream(st):
                torch.zeros(1, device=dev).add_(1)
        torch.cuda.synchronize()
    stream = streams[0]
    with torch.no_grad(), torch.cuda.stream(stream):
        for _ in range(2):
            model(x)
    stream.synchronize()
    graph = None
    if not args.no_graph:
        graph = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(graph, stream=stream):
            model(x)
        stream.synchronize()
    out: Dict[str, Any] = {"pid": os.getpid(), "slice_ids": os.environ.get("NOS_SLICE_IDS", ""),
                           "hsa_cu_mask": os.environ.get("HSA_CU_MASK", ""), "slice_cus": K.slice_cus(),
                           "boot_s": round(time.perf_counter() - t_boot, 2), "streams": len(streams),
                           "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "")}
    print("READY", flush=True)
    line = sys.stdin.readline().split()
    if not line or line[0] != "GO":
        return 3
    start = float(line[1])
    end = start + args.seconds
    while time.time() < start:
        time.sleep(0.0005)
    lat: List[float] = []
    census_at = start + 0.25 * args.seconds if args.census else None
    census = None
    k = 0
    with torch.no_grad():
        while True:
            now = time.time()
            if now >= end:
                break
            if census_at is not None and now >= census_at:
                census = _census()  # every other pod is mid-loop now
                census_at = None
            s = streams[k % len(streams)]  # one inference at a time, rotated over the process's queues
            k += 1
            t0 = time.perf_counter()
            with torch.cuda.stream(s):
                if graph is not None:
                    graph.replay()
                else:
                    model(x)
            s.synchronize()
            lat.append(1e3 * (time.perf_counter() - t0))
    out["window_s"] = round(time.time() - start, 3)
    out["inferences"] = len(lat)
    out["latency_ms"] = _stats(lat)
    if census is not None:
        out["census"] = census
    out["hbm"] = _shim()
    out["torch_max_reserved_bytes"] = int(torch.cuda.max_memory_reserved())
    print(json.dumps(out), flush=True)
    del graph
    torch.cuda.synchronize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
