"""The bench's multi-GPU control path on CPU: one process per GPU rank over a gloo process group,
every rank running the same seeded node simulation, with the agent's commit path
(``Actuator._commit`` -> ``RankCommitBarrier.vote_all``) as a real ``torch.distributed``
all-reduce — the RCCL path of ``bench.py`` under torchrun.  The ranks must stay in lock-step
(every commit votes on every rank, no hang), split the node's pods by GPU, and a veto from ONE
rank must roll the plan back on EVERY rank identically."""
from __future__ import annotations

import multiprocessing as mp
import socket

import pytest


def _worker(rank, world, port, q, veto_rank, veto_commits, layout="partitions"):
    import torch.distributed as dist

    from walkai_nos_amd.bench_core import BenchConfig, NodeBench
    from walkai_nos_amd.parallel.barrier import RankCommitBarrier
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        cfg = BenchConfig(gpus=world, steps=6, warmup=1, rank=rank, world=world, preroll=10, layout=layout)
        results = []
        checks = [0]

        def local_check():
            checks[0] += 1
            return not (rank == veto_rank and checks[0] <= veto_commits)

        def factory(n):
            b = RankCommitBarrier(rank, world, local_check=local_check)
            orig = b.vote_all

            def vote_all(votes):
                r = orig(votes)
                results.append((r, b.last_local))
                return r
            b.vote_all = vote_all
            return b
        nb = NodeBench(cfg, barrier_factory=factory, gpu_data_plane=False)
        served = 0
        modes = []
        for _ in range(cfg.preroll + cfg.warmup + cfg.steps):
            nb.control_step()
            served += len(nb.my_pods())
            nb.end_step()
            modes.append(tuple(sorted(nb.sn.smi.device_map().modes().items())))
        q.put((rank, served, [r for r, _ in results], [loc for _, loc in results],
               [round(u, 6) for u in nb.util_samples], modes, nb.sn.smi.set_calls))
    finally:
        dist.destroy_process_group()


def _run(world, veto_rank=-1, veto_commits=0, layout="partitions"):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, veto_rank, veto_commits, layout)) for r in range(world)]
    [p.start() for p in ps]
    [p.join(240) for p in ps]
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    return sorted(q.get(timeout=10) for _ in range(world))


@pytest.mark.parametrize("world", [2, 4])
def test_bench_control_plane_lockstep_gloo(world):
    out = _run(world)
    # identical control plane on every rank, same number of committed votes, all successful
    assert len({tuple(o[4]) for o in out}) == 1
    assert len({len(o[2]) for o in out}) == 1 and len(out[0][2]) > 0
    assert all(all(o[2]) for o in out)
    # every rank serves only its own GPU's pods; together they cover the node's work
    assert all(o[1] > 0 for o in out)


def test_bench_control_plane_lockstep_gloo_sliced_gpus():
    """The bench's default layout (sliced GPUs) under two ranks: the same node simulation on both,
    no flip at all (re-carving needs no commit), each rank serving its own GPU's slices."""
    out = _run(2, layout="slices")
    assert len({tuple(o[4]) for o in out}) == 1 and len({tuple(o[5]) for o in out}) == 1
    assert all(o[6] == [] for o in out)          # no amd-smi set call on any rank
    assert all(o[1] > 0 for o in out)


def test_one_rank_veto_rolls_back_on_every_rank():
    out = _run(2, veto_rank=1, veto_commits=1)
    r0, r1 = out
    # the first commit: rank 1 vetoed locally, so the all-reduce failed on BOTH ranks
    assert r1[3][0] is False and r0[3][0] is True
    assert r0[2][0] is False and r1[2][0] is False
    # both ranks rolled back the same flips and then committed the retry identically
    assert r0[6] == r1[6]
    assert any(c[0] == "compute" for c in r0[6])
    assert r0[5] == r1[5] and r0[2] == r1[2]
    assert any(r0[2][1:]), "the retried plan must commit once the veto is gone"


def test_density_per_pod_spread():
    from walkai_nos_amd.bench_core import _per_pod_spread
    r = _per_pod_spread({"a": 10, "b": 20, "c": 0}, ["a", "b"], 2.0)
    assert r == {"min": 5.0, "max": 10.0, "max_over_min": 2.0}
    assert _per_pod_spread({}, ["a"], 1.0)["max_over_min"] is None   # a pod that served nothing
    assert _per_pod_spread({}, [], 1.0) == {}


def test_bench_py_eight_rank_rehearsal_prints_one_json_line():
    """``bench.py --gpus 8`` launched the way the driver launches it
    (torch.distributed.run, 8 ranks, 127.0.0.1) on gloo without a GPU: the ranks stay in lock-step
    through the window and the post-window model, rank 0 prints exactly one JSON line, within the
    time an 8-GPU driver run allows. Inferences are priced (the output says REHEARSAL)."""
    import json
    import os
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, NOS_BENCH_DIST_BACKEND="gloo", OMP_NUM_THREADS="1")
    env.pop("LD_PRELOAD", None)
    t0 = time.time()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
                        "--master-addr=127.0.0.1", f"--master-port={port}", "bench.py", "--gpus", "8",
                        "--steps", "20", "--warmup", "5", "--no-data-plane", "--no-density"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=900)
    wall = time.time() - t0
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["steps"] == 20 and out["warmup"] == 5
    assert out["data"].startswith("REHEARSAL") and out["value"] > 0
    assert out["gpu_utilization_pct"] > 50 and out["config"]["parallelism"].endswith("8 GPU node")
    # who ran is readable from the JSON
    d = out["dist"]
    assert d["backend"] == "gloo" and d["world_size"] == 8
    assert sorted(r["rank"] for r in d["ranks"]) == list(range(8))
    assert sorted(r["local_rank"] for r in d["ranks"]) == list(range(8))
    # BASELINE config 4 beside the headline: the same window on hardware partitions, its own clock
    pw = out["partitions_window"]
    assert pw["layout"] == "partitions" and pw["value"] > 0 and pw["window_s"] > 0
    assert pw["flips"] >= 0 and "time_in_flip_pct" in pw and pw["commit_barriers"] >= pw["flips"] > 0
    assert "estimated" in pw["flip_cost"] and set(pw["per_profile"]) == {"cpx_nps1", "dpx_nps1", "spx_nps1"}
    # rank 0's post-window models ran within their budget (or say what they skipped)
    pwb = out["post_window"]
    assert pwb["budget_s"] == 60.0 and (pwb["spent_s"] <= pwb["budget_s"] + 60 or pwb["skipped"])
    assert wall < 600, wall
