"""Memory-only pods through churn, repeated: 8 pod processes started at once through the start gate,
then the three at start positions 0, 2, 4 stopped and three new ones started; per-pod rates after
the churn, with and without waiting for the stopped processes' KFD queues to go first.

    python tools/churn_probe.py [--reps 3] [--settle 0,10] [--out gpurun_out/churn_probe.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from walkai_nos_amd.dataplane.procs import run_pods  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--settle", default="0,10", help="settle_s values to alternate")
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--hold-context", action="store_true",
                    help="this process opens a HIP context (its own compute queues) before the pods start")
    ap.add_argument("--hold-streams", type=int, default=0,
                    help="... and keeps this many CU-masked streams (hardware queues) alive, each used once")
    ap.add_argument("--out", default="gpurun_out/churn_probe.json")
    a = ap.parse_args()
    if a.hold_context:
        import torch
        x = torch.ones(1024, device="cuda")
        torch.cuda.synchronize()
        print("holding a HIP context:", float(x.sum()), flush=True)
        from walkai_nos_amd.ops.probe import Stream
        held = []
        for k in range(a.hold_streams):
            st = Stream(0, list(range(32 * (k % 8), 32 * (k % 8) + 32)))
            with torch.cuda.stream(st.torch_stream()):
                x.add_(1.0)
            held.append(st)
        torch.cuda.synchronize()
        print("holding", len(held), "CU-masked streams", flush=True)
    runs = []
    for rep in range(a.reps):
        for settle in (float(x) for x in a.settle.split(",")):
            r = run_pods(["16gb"] * 8, seconds=a.seconds, gate=True, churn=([0, 2, 4], ["16gb"] * 3),
                         settle_s=settle)
            order = [int(s.rsplit("::s", 1)[1]) for s in r["gate"]["order"]]
            by_pod = {p["pod"]: p["inf_per_s"] for p in r["per_pod"]}
            rates = [p["inf_per_s"] for p in r["per_pod"]]
            row = {"rep": rep, "settle_s": settle, "hold_context": a.hold_context, "hold_streams": a.hold_streams, "rates": rates, "max_over_min": round(max(rates) / min(rates), 3),
                   "aggregate": r.get("aggregate_inf_per_s"), "gate_order": order, "churn": r["churn"],
                   "by_pod": by_pod}
            runs.append(row)
            print(json.dumps(row), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump({"runs": runs}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
