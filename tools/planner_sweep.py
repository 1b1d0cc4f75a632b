"""Planner sweep without a GPU: the bench's control plane and outage model (``bench_core.NodeBench``
with no data plane) per GPU count x offered load x seed, ``--steps`` quanta after the preroll.

Reports per cell: allocation (mean over seeds and the worst seed), flips, time in flips, queue,
and per profile the p99 time-to-schedule in mean pod lifetimes (pods bound in the window).

    python tools/planner_sweep.py [--gpus 1,2,4,8] [--loads 0.85,1.0] [--seeds 1,2,3,4] [--steps 200]
        [--pack '{"unserved_after": 0}'] [--out profiles/planner_sweep_r3.json]
"""
from __future__ import annotations

import argparse
import itertools
import json
import multiprocessing as mp
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(job):
    gpus, load, seed, steps, pack, layout, bound = job
    import logging
    logging.disable(logging.CRITICAL)
    from walkai_nos_amd.bench_core import BenchConfig, control_only
    r = control_only(BenchConfig(gpus=gpus, offered_load=load, seed=seed, pack=pack or None, layout=layout,
                                 declared_bound_quanta=bound), steps)
    pp = r["per_profile"]
    return {"gpus": gpus, "load": load, "seed": seed, "util_pct": r["util_pct"], "flips": r["flips"],
            "time_in_flip_pct": r["time_in_flip_pct"], "pending_mean": r["pending_mean"],
            "inf_per_s_model": r["inf_per_s_model"], "offered_pct": r["idle"]["offered_pct"],
            "idle_pct": r["idle"]["by_cause_pct"],
            "tts_p99_lifetimes": {p: v.get("tts_lifetimes_p99") for p, v in pp.items()},
            "pods_bound": {p: v["pods_bound"] for p, v in pp.items()}}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--loads", default="0.85,1.0")
    ap.add_argument("--seeds", default="1,2,3,4")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--pack", default="{}", help="PackParams overrides as JSON")
    ap.add_argument("--workers", type=int, default=6)
    ap.add_argument("--layout", default="slices", help="xcp-layout of the node: partitions | slices | auto")
    ap.add_argument("--declared-bound", type=float, default=0.0,
                    help="every pod declares spec.activeDeadlineSeconds of this many quanta (0: none)")
    ap.add_argument("--out", default="profiles/planner_sweep_r5_slices.json")
    a = ap.parse_args()
    pack = json.loads(a.pack)
    jobs = list(itertools.product([int(g) for g in a.gpus.split(",")], [float(x) for x in a.loads.split(",")],
                                  [int(s) for s in a.seeds.split(",")], [a.steps], [pack], [a.layout],
                                  [a.declared_bound]))
    with mp.Pool(a.workers) as pool:
        rows = pool.map(run, jobs)
    cells = {}
    for (g, l), grp in itertools.groupby(sorted(rows, key=lambda r: (r["gpus"], r["load"])),
                                         key=lambda r: (r["gpus"], r["load"])):
        grp = list(grp)
        tts = {p: max((r["tts_p99_lifetimes"][p] or 0) for r in grp) for p in grp[0]["tts_p99_lifetimes"]}
        cells[f"{g}gpu/load{l}"] = {
            "util_pct_mean": round(sum(r["util_pct"] for r in grp) / len(grp), 2),
            "util_pct_min": min(r["util_pct"] for r in grp), "per_seed_util": [r["util_pct"] for r in grp],
            "flips_mean": round(sum(r["flips"] for r in grp) / len(grp), 1),
            "time_in_flip_pct_mean": round(sum(r["time_in_flip_pct"] for r in grp) / len(grp), 2),
            "pending_mean": round(sum(r["pending_mean"] for r in grp) / len(grp), 2),
            "offered_pct_mean": round(sum(r["offered_pct"] for r in grp) / len(grp), 2),
            "idle_pct_mean": {k: round(sum(r["idle_pct"][k] for r in grp) / len(grp), 2) for k in grp[0]["idle_pct"]},
            "tts_p99_lifetimes_worst_seed": tts}
        print(f"{g}gpu/load{l}", json.dumps(cells[f"{g}gpu/load{l}"]), flush=True)
    out = {"steps": a.steps, "seeds": a.seeds, "pack_overrides": pack, "layout": a.layout,
           "declared_bound_quanta": a.declared_bound, "cells": cells, "rows": rows}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
