#!/usr/bin/env python3
"""Benchmark driver contract: ``python bench.py --gpus N --steps K --warmup W``.

Runs the flagship step (see :mod:`walkai_nos_amd.bench_core`): a node of N MI355X GPUs (one
process per GPU under torchrun, RCCL over xGMI for the partition-commit barrier) serving a
churning mix of 1/8, 1/2 and 1/1-GPU YOLOS-small inference pods through the nos control plane.
One step = one quantum of ``--cluster-s`` seconds of cluster time replayed in ``--quantum`` wall
seconds of GPU serving (pod lifetimes, planner thresholds and flip outages compressed alike; the
GPU serves at its real rate); every compute-partition flip darkens its GPU for the measured flip
cost.  After the timed window a density phase saturates the node (8 CPX pods per GPU, then CU-mask
slices beyond).  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--load", type=float, default=1.0, help="offered GPU-equivalents per GPU")
    ap.add_argument("--backend", choices=("hip", "torch"), default="hip")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--preroll", type=int, default=60,
                    help="control-plane-only quanta before warmup, so timing starts in steady state")
    ap.add_argument("--quantum", type=float, default=0.5, help="wall seconds of serving per quantum")
    ap.add_argument("--cluster-s", type=float, default=60.0, help="cluster seconds one quantum stands for")
    ap.add_argument("--quanta-per-step", type=int, default=2,
                    help="quanta per driver step: the timed window is steps x this many quanta")
    ap.add_argument("--flip-cost", type=float, default=-1.0,
                    help="cluster seconds a GPU serves nothing per compute-partition flip "
                         "(default: the measured components, bench_core.FLIP_COST_COMPONENTS)")
    ap.add_argument("--pod-start", type=float, default=-1.0,
                    help="cluster seconds a newly bound pod holds its slice before its first inference "
                         "(default: measured on this box before the window, bench_core.measure_pod_start)")
    ap.add_argument("--device-plugin", default="nos", choices=("nos", "amd"),
                    help="nos: drains enforced by the partition plugin's device health; amd: no enforcement")
    ap.add_argument("--policy", default="pack", choices=("pack", "fifo", "batch", "simulate"))
    ap.add_argument("--layout", default="slices", choices=("partitions", "slices", "auto"),
                    help="the node's nos.nebuly.com/xcp-layout: hardware partitions only, sliced GPUs "
                         "(SPX + CU-mask slices, mixed geometries), or the planner's choice per GPU")
    ap.add_argument("--depth", type=int, default=1,
                    help="inferences in flight per pod stream (1 = the reference demo's synchronous loop)")
    ap.add_argument("--pod-streams", type=int, default=1,
                    help="concurrent request streams per pod (1 = one inference at a time, as the reference demo)")
    ap.add_argument("--lane-cus", type=int, default=0,
                    help="opt-in: a partition pod wider than this many CUs runs one batch-1 request loop per "
                         "disjoint run of this many CUs (0 = one loop per pod, as the reference demo)")
    ap.add_argument("--no-density", action="store_true", help="skip the saturation/density phase")
    ap.add_argument("--emulation", default=None, choices=("pinned", "spread", "landing"),
                    help="compute-partition emulation on the SPX device (default: spread; bench_core.EMULATION)")
    ap.add_argument("--erq", action="store_true",
                    help="Elastic Resource Quota mode (BASELINE config 5): two quota'd namespaces borrow and "
                         "reclaim on the real data plane; prints its own JSON line (walkai_nos_amd/bench_erq.py)")
    ap.add_argument("--no-data-plane", action="store_true",
                    help="REHEARSAL of the launch path without a GPU (gloo, control plane only; inferences "
                         "priced with the measured mode rates, marked in the output — never a measurement)")
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        import torch
        import torch.distributed as dist
        if not args.no_data_plane:
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
        # RCCL between the GPU ranks; NOS_BENCH_DIST_BACKEND=gloo rehearses the multi-rank path with
        # several ranks sharing fewer GPUs (RCCL refuses two ranks on one device)
        dist.init_process_group(os.environ.get("NOS_BENCH_DIST_BACKEND", "nccl"),
                                timeout=datetime.timedelta(seconds=300))
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} != WORLD_SIZE {world}; using {world}", file=sys.stderr)
    gpus = world if world > 1 else args.gpus
    if gpus > 1 and world == 1:
        print("multi-GPU runs are launched with torchrun (one process per GPU)", file=sys.stderr)
        return 2

    from walkai_nos_amd.bench_core import BenchConfig, run_bench
    cfg = BenchConfig(gpus=gpus, steps=args.steps, warmup=args.warmup, seed=args.seed, offered_load=args.load,
                      backend=args.backend, graphs=not args.no_graphs, rank=rank, world=world,
                      preroll=args.preroll, quantum_s=args.quantum, cluster_s=args.cluster_s,
                      quanta_per_step=args.quanta_per_step,
                      flip_cost_s=args.flip_cost, policy=args.policy, depth=args.depth,
                      density=not args.no_density, pod_streams=args.pod_streams, lane_cus=args.lane_cus,
                      device_plugin=args.device_plugin, layout=args.layout, pod_start_s=args.pod_start,
                      data_plane=not args.no_data_plane)
    if args.emulation:
        cfg.emulation = args.emulation
    if args.erq:
        from walkai_nos_amd.bench_core import DataPlane
        from walkai_nos_amd.bench_erq import run_erq
        data = DataPlane(cfg)
        try:
            res = run_erq(cfg, data)
        finally:
            data.close()
    else:
        res = run_bench(cfg)
    if rank == 0:
        line = json.dumps(res)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
