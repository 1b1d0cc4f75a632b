"""The driver's bench window on 1/2/4/8-GPU nodes, control plane alone (no GPU): what the driver's
scaling runs (N = 1, 2, 4, 8, one rank per GPU) should land near.

    python tools/scale_model.py [--pod-start 3.09] [--layouts slices,partitions]
                                [--out profiles/scale_model_r6.json]

Each row is ``bench_core.control_only`` over the bench's own window (seed 1234, ``--steps`` x 2
quanta after ``--warmup`` x 2 warm-up quanta, after the preroll), priced with the measured per-mode
rates (``bench_core.MODE_RATES``) and the given pod start-up (the bench measures it on the box).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from walkai_nos_amd.bench_core import MODE_RATES, BenchConfig, control_only  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--layouts", default="slices,partitions")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--pod-start", type=float, default=3.09, help="cluster seconds of pod start-up (measured on the box)")
    ap.add_argument("--declared-bound", type=float, default=None,
                    help="pods' activeDeadlineSeconds in quanta (default: the bench's BenchConfig default)")
    ap.add_argument("--out", default="profiles/scale_model_r6.json")
    a = ap.parse_args()
    out = {"what": "the driver's bench window (seed %d, %d steps x 2 quanta after %d warm-up steps) on 1/2/4/8-GPU "
                   "nodes, control plane alone, priced with the measured per-mode rates (bench_core.MODE_RATES), "
                   "pod start-up %.2f s" % (a.seed, a.steps, a.warmup, a.pod_start),
           "mode_rates": MODE_RATES, "tool": "tools/scale_model.py", "rows": {}}
    for layout in a.layouts.split(","):
        rows = {}
        for g in (int(x) for x in a.gpus.split(",")):
            kw = {} if a.declared_bound is None else {"declared_bound_quanta": a.declared_bound}
            cfg = BenchConfig(gpus=g, steps=a.steps, warmup=a.warmup, seed=a.seed, layout=layout,
                              pod_start_s=a.pod_start, **kw)
            t0 = time.time()
            r = control_only(cfg, cfg.warmup_quanta + cfg.window_quanta, skip=cfg.warmup_quanta)
            rows[str(g)] = {"util_pct": r["util_pct"], "inf_per_s_model": r["inf_per_s_model"],
                            "inf_per_s_per_gpu": round(r["inf_per_s_model"] / g, 1),
                            "pending_mean": r["pending_mean"], "pods_per_gpu": r["pods_per_gpu"],
                            "flips": r["flips"], "time_in_flip_pct": r["time_in_flip_pct"],
                            "tts_lifetimes_p99": {p: v.get("tts_lifetimes_p99") for p, v in r["per_profile"].items()},
                            "idle_pct": r["idle"]["by_cause_pct"], "cpu_s": round(time.time() - t0, 1)}
            print(layout, g, json.dumps(rows[str(g)]), flush=True)
        out["rows"][layout] = rows
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
