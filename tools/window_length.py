"""How representative is the driver's bench window? The control plane alone (no GPU) over the
bench's seeded churn for many seeds, at two window lengths (quanta after the warmup), for sliced
GPUs and hardware partitions: allocation per seed, its mean / sd / p10 / min, and the default
seed's rank. Writes profiles/window_length_r5.json.

    python tools/window_length.py --seeds 40 --out profiles/window_length_r5.json
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import statistics as st
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def one(args):
    layout, seed, quanta, warm = args
    from walkai_nos_amd.bench_core import BenchConfig, control_only
    cfg = BenchConfig(gpus=1, steps=quanta, warmup=warm, quanta_per_step=1, seed=seed, data_plane=False,
                      layout=layout)
    r = control_only(cfg, cfg.warmup_quanta + cfg.window_quanta, skip=cfg.warmup_quanta)
    return layout, quanta, seed, r["util_pct"], r["pending_mean"], r["inf_per_s_model"]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=40)
    ap.add_argument("--default-seed", type=int, default=1234)
    ap.add_argument("--windows", default="20:5,40:10", help="quanta:warmup-quanta pairs")
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--out", default="profiles/window_length_r5.json")
    a = ap.parse_args()
    seeds = [a.default_seed] + list(range(1, a.seeds))
    wins = [tuple(int(x) for x in w.split(":")) for w in a.windows.split(",")]
    jobs = [(L, s, q, w) for L in ("slices", "partitions") for q, w in wins for s in seeds]
    with mp.Pool(a.workers) as pool:
        res = pool.map(one, jobs)
    out = {"what": "control plane only (bench_core.control_only), 1 GPU, offered load 1.0, the bench's churn; "
                   "allocation % of the window per churn seed", "default_seed": a.default_seed, "rows": {}}
    for L in ("slices", "partitions"):
        for q, _ in wins:
            rows = [r for r in res if r[0] == L and r[1] == q]
            u = sorted(r[3] for r in rows)
            mine = next(r for r in rows if r[2] == a.default_seed)
            out["rows"][f"{L}_{q}q"] = {
                "window_quanta": q, "pod_lifetimes": q / 4.0, "util_mean": round(st.mean(u), 2),
                "util_sd": round(st.pstdev(u), 2), "util_p10": u[len(u) // 10], "util_min": u[0],
                "inf_per_s_model_mean": round(st.mean(r[5] for r in rows), 1),
                "pending_mean": round(st.mean(r[4] for r in rows), 2),
                "default_seed": {"util_pct": mine[3], "inf_per_s_model": mine[5], "pending_mean": mine[4],
                                 "rank_from_bottom": u.index(mine[3]) + 1},
                "per_seed_util": {str(r[2]): r[3] for r in rows}}
            print(L, q, {k: v for k, v in out["rows"][f"{L}_{q}q"].items() if k != "per_seed_util"}, flush=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
