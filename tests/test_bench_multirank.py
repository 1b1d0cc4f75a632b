"""The bench's multi-GPU control path on CPU: one process per GPU rank over a gloo process group,
every rank running the same seeded node simulation with the commit barrier as a real
``torch.distributed`` all-reduce (the RCCL path of ``bench.py`` under torchrun).  The ranks must
stay in lock-step (every commit votes on every rank, no hang) and split the node's pods by GPU."""
from __future__ import annotations

import multiprocessing as mp
import socket

import pytest


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from walkai_nos_amd.bench_core import BenchConfig, NodeBench
    from walkai_nos_amd.parallel.barrier import TorchBarrier
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        cfg = BenchConfig(gpus=world, steps=6, warmup=1, rank=rank, world=world, preroll=10)
        votes = []

        def factory(n):
            b = TorchBarrier()
            orig = b.vote

            def vote(ok):
                r = orig(ok)
                votes.append(r)
                return r
            b.vote = vote
            return b
        nb = NodeBench(cfg, barrier_factory=factory, gpu_data_plane=False)
        work = 0
        for _ in range(cfg.preroll + cfg.warmup + cfg.steps):
            work += nb.step()
        q.put((rank, work, len(votes), all(votes), [round(u, 6) for u in nb.util_samples],
               len(nb.cluster.running_pods())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_bench_control_plane_lockstep_gloo(world):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in ps]
    [p.join(240) for p in ps]
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    out = sorted(q.get(timeout=10) for _ in range(world))
    # identical control plane on every rank, same number of committed votes, all successful
    assert len({tuple(o[4]) for o in out}) == 1
    assert len({o[2] for o in out}) == 1 and out[0][2] > 0
    assert all(o[3] for o in out)
    # every rank runs only its own GPU's pods; together they cover the node's work
    assert sum(o[1] for o in out) > 0
    assert all(o[1] > 0 for o in out)
