"""Reproduce the reference's GPU-sharing comparison on one MI355X (reference
``demos/gpu-sharing-comparison/README.md:62-71``): 1, 3, 5 and 7 pods each running YOLOS-small
(fp32, batch 1, 800x1066) inference in a loop, under three sharing modes:

* ``shared``  — every pod on its own HIP stream with no CU mask: the hardware scheduler runs all
  pods' kernels concurrently over all 256 CUs (what AMD GPUs do for co-resident processes; the
  analogue of the reference's time-slicing and MPS rows);
* ``cumask``  — the GPU's 8 SE-balanced 32-CU row groups are dealt out to the N pods as evenly as
  possible (N=3: 96/96/64 CUs), each pod on its own disjoint CU mask — the nos CU-mask slices
  ``amd.com/gpu-<c>cu.<m>gb`` requests receive;
* ``cpx``     — each pod gets one CPX-sized partition (32 CUs, 1/8 of the GPU) regardless of N:
  the MIG-1g analogue (fixed-size hardware slice).

Every pod is a thread replaying its own captured HIP graph on its own stream; latency is wall time
per replay+sync, aggregate throughput = total inferences / window. Synthetic random-init weights and
a synthetic image of the demo's post-processing shape (the reference uses one COCO image).

    python tools/sharing_curve.py [--seconds 6] [--pods 1,3,5,7] [--modes shared,cumask,cpx]
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from walkai_nos_amd.models.workload.yolos import DEMO_INPUT_HW, YolosSmall, demo_input  # noqa: E402
from walkai_nos_amd.ops import kernels as K  # noqa: E402
from walkai_nos_amd.ops.probe import Stream  # noqa: E402

# reference aggregate throughput (inferences/s) on 1x A100 80GB, derived in BASELINE.md
REFERENCE = {"time-slicing": {1: 11.34, 3: 10.23, 5: 10.23, 7: 10.22},
             "mps": {1: 11.37, 3: 18.29, 5: 20.76, 7: 21.89},
             "mig": {1: 2.92, 3: 8.79, 5: 14.48, 7: 20.33}}


def cu_sets(mode: str, n: int):
    if mode == "shared":
        return [None] * n
    if mode == "cpx":
        return [list(range(32 * i, 32 * (i + 1))) for i in range(n)]
    groups = [8 // n + (1 if i < 8 % n else 0) for i in range(n)]
    out, g0 = [], 0
    for g in groups:
        out.append(list(range(32 * g0, 32 * (g0 + g))))
        g0 += g
    return out


class Pod:
    def __init__(self, template: YolosSmall, cus, seed: int):
        self.cus = cus
        self.n_cus = 256 if cus is None else len(cus)
        self.hs = Stream(0, cus)
        self.stream = self.hs.torch_stream()
        with torch.cuda.stream(self.stream):
            self.model = copy.deepcopy(template).cuda().eval()
            self.x = demo_input(1, DEMO_INPUT_HW, "cuda", seed=seed)
        K.set_slice_cus(self.n_cus)
        with torch.no_grad(), torch.cuda.stream(self.stream):
            for _ in range(2):
                self.model(self.x)
        self.stream.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(self.graph, stream=self.stream):
            self.out = self.model(self.x)
        self.stream.synchronize()
        self.lat = []

    def loop(self, stop: threading.Event, start: threading.Barrier) -> None:
        start.wait()
        # replay() launches on the *current* stream: make it the pod's CU-masked stream
        with torch.cuda.stream(self.stream):
            while not stop.is_set():
                t0 = time.perf_counter()
                self.graph.replay()
                self.stream.synchronize()
                self.lat.append(time.perf_counter() - t0)

    def close(self) -> None:
        self.graph = None
        self.model = None
        self.stream = None
        self.hs.close()


def run(mode: str, n: int, seconds: float, template: YolosSmall) -> dict:
    pods = [Pod(template, cus, i) for i, cus in enumerate(cu_sets(mode, n))]
    torch.cuda.synchronize()
    stop, start = threading.Event(), threading.Barrier(n + 1)
    threads = [threading.Thread(target=p.loop, args=(stop, start)) for p in pods]
    for t in threads:
        t.start()
    start.wait()
    time.sleep(0.5)  # ramp: discard the first half second
    marks = [len(p.lat) for p in pods]
    t0 = time.perf_counter()
    time.sleep(seconds)
    done = [len(p.lat) for p in pods]
    window = time.perf_counter() - t0
    stop.set()
    for t in threads:
        t.join()
    lats = [lat for p, m, d in zip(pods, marks, done) for lat in p.lat[m:d]]
    total = sum(d - m for m, d in zip(marks, done))
    for p in pods:
        p.close()
    torch.cuda.synchronize()
    agg = total / window
    row = {"mode": mode, "pods": n, "cus_per_pod": [p.n_cus for p in pods], "aggregate_inf_per_s": round(agg, 2),
           "mean_latency_s": round(sum(lats) / max(1, len(lats)), 4), "inferences": total}
    for ref, curve in REFERENCE.items():
        if n in curve:
            row[f"x_vs_a100_{ref}"] = round(agg / curve[n], 2)
    return row


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--pods", default="1,3,5,7")
    ap.add_argument("--modes", default="shared,cumask,cpx")
    ap.add_argument("--backend", default="hip", choices=("hip", "torch"))
    ap.add_argument("--out", default="gpurun_out/sharing_curve.json")
    a = ap.parse_args()
    K.set_backend(a.backend)
    template = YolosSmall()
    rows = []
    for mode in a.modes.split(","):
        for n in (int(x) for x in a.pods.split(",")):
            if mode == "cpx" and n > 8:
                continue
            row = run(mode, n, a.seconds, template)
            print(json.dumps(row), flush=True)
            rows.append(row)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump({"backend": a.backend, "reference_a100_inf_per_s": REFERENCE, "rows": rows}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
