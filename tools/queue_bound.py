"""How short can the waits be? An idealised single-node scheduler for the bench's churn (no
control plane, no flips, no outages): GPUs of 8 freely re-carvable groups, pods of 1, 4 and 8 groups
(the 50/30/20 mix of ``bench_core.MIX``), lifetimes 2-6 quanta, the bench's steady arrival process.

Policy: first-come-first-served with backfilling — every waiting pod that fits starts, oldest
first — plus a reservation: the oldest pod that fits nowhere, once it has waited ``T`` quanta,
blocks everything behind it until it starts (without it whole-GPU pods starve). This is what the
sliced-GPU planner does (``controllers/partitioner/sliced.py``) with none of the real system's
costs, so its p99 waits are a floor for that policy family: swept over ``T`` it shows that on one GPU
at load 0.85 no threshold brings the worst profile's p99 time-to-schedule below 6 mean pod
lifetimes (a whole-GPU pod must wait for the GPU to empty of pods that cannot be preempted;
``profiles/queue_bound_r4.json``); on two GPUs its best is 3.25-4.5 (the real planner: 3.75).

    python tools/queue_bound.py [--gpus 1] [--loads 0.85,1.0] [--thresholds 0,8,16,24,32,48]
        [--seeds 1,2,3,4] [--steps 400] [--out profiles/queue_bound_r4.json]
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
from typing import Dict, List

SIZE = {"c": 1, "d": 4, "s": 8}
MIX = ["c"] * 5 + ["d"] * 3 + ["s"] * 2
MEAN_FRAC = 0.5 / 8 + 0.3 / 2 + 0.2
MEAN_LIFE = 4.0


def run(load: float, seed: int, threshold: int, gpus: int = 1, steps: int = 400, preroll: int = 60) -> Dict:
    rng = random.Random(seed)
    rate = load * gpus / (MEAN_FRAC * MEAN_LIFE)
    acc = rng.random()
    profiles: List[str] = []
    lifetimes: List[int] = []
    queue: List = []        # (profile, arrival step)
    running: List = []      # [gpu, groups, quanta left]
    tts: Dict[str, List[int]] = {"c": [], "d": [], "s": []}
    util: List[float] = []
    pending: List[int] = []
    for t in range(preroll + steps):
        running = [r for r in running if r[2] > 0]
        acc += rate
        n = int(acc)
        acc -= n
        for _ in range(n):
            if not profiles:
                profiles = MIX[:]
                rng.shuffle(profiles)
            queue.append((profiles.pop(), t))
        free = [8] * gpus
        for r in running:
            free[r[0]] -= r[1]
        left, blocked = [], False
        for p, t0 in queue:
            fits = [g for g in range(gpus) if free[g] >= SIZE[p]]
            if fits and not blocked:
                g = min(fits, key=lambda i: free[i])     # best fit
                free[g] -= SIZE[p]
                if not lifetimes:
                    lifetimes = [2, 3, 4, 5, 6]
                    rng.shuffle(lifetimes)
                running.append([g, SIZE[p], lifetimes.pop()])
                if t >= preroll:
                    tts[p].append(t - t0)
            else:
                left.append((p, t0))
                if not fits and t - t0 >= threshold > 0:
                    blocked = True                         # the overdue pod reserves: nobody passes it
        queue = left
        if t >= preroll:
            util.append(sum(r[1] for r in running) / (8 * gpus))
            pending.append(len(queue))
        for r in running:
            r[2] -= 1
    p99 = {}
    for p, v in tts.items():
        v = sorted(v)
        p99[p] = round(v[min(len(v) - 1, int(0.99 * len(v)))] / MEAN_LIFE, 2) if v else None
    return {"util_pct": round(100 * sum(util) / len(util), 1), "pending_mean": round(sum(pending) / len(pending), 2),
            "tts_p99_lifetimes": p99}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--loads", default="0.85,1.0")
    ap.add_argument("--thresholds", default="0,8,12,16,24,32,48", help="reservation after T quanta (0 = never)")
    ap.add_argument("--seeds", default="1,2,3,4")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = []
    for load in [float(x) for x in a.loads.split(",")]:
        for T in [int(x) for x in a.thresholds.split(",")]:
            rs = [run(load, int(s), T, a.gpus, a.steps) for s in a.seeds.split(",")]
            worst = max(max(v for v in r["tts_p99_lifetimes"].values() if v is not None) for r in rs)
            row = {"load": load, "reserve_after_quanta": T, "util_pct": [r["util_pct"] for r in rs],
                   "pending_mean": round(sum(r["pending_mean"] for r in rs) / len(rs), 2),
                   "worst_p99_lifetimes": worst, "per_seed": rs}
            rows.append(row)
            print(json.dumps({k: v for k, v in row.items() if k != "per_seed"}), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump({"gpus": a.gpus, "steps": a.steps, "rows": rows}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
