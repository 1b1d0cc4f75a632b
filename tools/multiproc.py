"""Pods as processes on one MI355X (VERDICT r2 "run the data plane as processes"): every pod is a
fresh process with the env the nos slice device plugin's ``Allocate`` returns (CU mask, HBM
limit, HBM shim), running the reference demo's loop (one YOLOS-small inference at a time).

Scenarios (each a fresh set of processes, all released at one instant for a common window):

* ``shared_<N>``  N = 1/3/5/7 memory-only ``16gb`` slices (the MPS analogue: an HBM budget each,
  compute shared by all) — the reference's sharing table, ref
  ``demos/gpu-sharing-comparison/README.md:62-71``;
* ``cumask_<N>``  N = 3/5/7 dedicated-CU slices that split the 8 row groups (256 CUs) between them;
* ``cpx8``        8 x ``32cu.36gb`` — BASELINE config 2 (8 pods, 1/8 GPU each) on the SPX device;
* ``config3``     4 x ``64cu.72gb`` — BASELINE config 3 (4 pods, own CU set + HBM limit), with the
  HBM shim, and ``config3_noshim`` without it (the shim's cost);
* ``dense_14`` / ``shared_14``  beyond eight pods per GPU: 6 dedicated 32-CU slices + 8 memory-only
  slices on the other 64 CUs, and 14 memory-only slices (the bench density phase's mixes).

    python tools/multiproc.py [--seconds 10] [--only shared_1,config3] --out gpurun_out/multiproc.json
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from walkai_nos_amd.dataplane.procs import run_pods  # noqa: E402

REFERENCE = {"time-slicing": {1: 11.34, 3: 10.23, 5: 10.23, 7: 10.22},
             "mps": {1: 11.37, 3: 18.29, 5: 20.76, 7: 21.89},
             "mig": {1: 2.92, 3: 8.79, 5: 14.48, 7: 20.33}}


def split_groups(n: int, groups: int = 8):
    sizes = [groups // n + (1 if i < groups % n else 0) for i in range(n)]
    return [f"{32 * g}cu.{36 * g}gb" for g in sizes]


def scenarios():
    out = {}
    for n in (1, 3, 4, 5, 7):
        out[f"shared_{n}"] = (["16gb"] * n, True)
    for n in (3, 5, 7):
        out[f"cumask_{n}"] = (split_groups(n), True)
    out["cpx8"] = (["32cu.36gb"] * 8, True)
    out["config3"] = (["64cu.72gb"] * 4, True)
    out["config3_noshim"] = (["64cu.72gb"] * 4, False)
    # beyond 8 pods (the bench density phase's mixes, at 14 pods: a box runs at most 16 GPU processes)
    out["dense_14"] = (["32cu.24gb"] * 6 + ["8gb"] * 8, True)
    out["shared_14"] = (["16gb"] * 14, True)
    for n in (6, 8, 9, 10, 12):   # 6: the sharing table's missing count; 9+: where process time-slicing starts
        out[f"shared_{n}"] = (["16gb"] * n, True)
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--only", default="")
    ap.add_argument("--out", default="gpurun_out/multiproc.json")
    ap.add_argument("--env", default="{}", help="extra env for every pod, JSON (e.g. {\"NOS_POD_STREAMS\": \"4\"})")
    ap.add_argument("--tag", default="", help="suffix of the scenario names in the output")
    ap.add_argument("--stagger", type=float, default=0.0, help="seconds between pod starts")
    ap.add_argument("--queues", default="", help="GPU_MAX_HW_QUEUES per pod in start order, e.g. 1,2,1,2,1")
    args = ap.parse_args()
    extra = json.loads(args.env)
    todo = scenarios()
    if args.only:
        todo = {k: v for k, v in todo.items() if k in args.only.split(",")}
    res = {"seconds": args.seconds, "reference_inf_per_s_a100": REFERENCE, "scenarios": {}}
    if os.path.exists(args.out):  # several variants (--env/--tag) accumulate in one file
        with open(args.out) as f:
            res["scenarios"] = json.load(f).get("scenarios", {})
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    for name, (profiles, shim) in todo.items():
        t0 = time.time()
        dedicated = all("cu." in p for p in profiles)
        per = [{"GPU_MAX_HW_QUEUES": q} for q in args.queues.split(",")] if args.queues else None
        r = run_pods(profiles, seconds=args.seconds, shim=shim, census=dedicated, extra_env=extra,
                     stagger_s=args.stagger, per_pod_env=per)
        r["profiles"] = profiles
        r["shim"] = shim
        r["env"] = extra
        r["stagger_s"] = args.stagger
        r["queues"] = args.queues
        r["wall_s"] = round(time.time() - t0, 1)
        rates = [p["inf_per_s"] for p in r["per_pod"]]
        r["per_pod_max_over_min"] = round(max(rates) / max(1e-9, min(rates)), 3) if rates else None
        name = name + args.tag
        res["scenarios"][name] = r
        print(json.dumps({"scenario": name, "pods": r["pods"], "agg_inf_per_s": r["aggregate_inf_per_s"],
                          "per_pod": rates, "max_over_min": r["per_pod_max_over_min"],
                          "mean_latency_ms": r["mean_latency_ms"],
                          "census_pairs_overlapping": r.get("census_pairs_overlapping"), "wall_s": r["wall_s"]}),
              flush=True)
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
