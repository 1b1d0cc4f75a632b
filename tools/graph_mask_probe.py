"""Do HIP graphs keep the CU masks of the streams their branches were captured on?

A 1-branch and a 2-branch graph are captured on CU-masked streams (``hipExtStreamCreateWithCUMask``)
and replayed; their time is compared with eager launches on the same streams. If a captured branch
kept its stream's mask, a matmul captured on a 32-CU stream replays at the 32-CU eager rate; if the
graph runs its nodes on its launch stream (or internal streams without the mask), it replays at the
whole-GPU rate. This decides whether one request can be split over CU-disjoint lanes inside one graph."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    from walkai_nos_amd.ops.probe import Stream
    n = 4096
    a = torch.randn(n, n, device="cuda")
    b = torch.randn(n, n, device="cuda")
    outs = [torch.empty(n, n, device="cuda") for _ in range(2)]
    half_a = [c for c in range(256) if c % 2 == 0]        # 128 CUs, XCD-balanced
    half_b = [c for c in range(256) if c % 2 == 1]
    small = list(range(32))
    streams = {"all": Stream(0, None), "small": Stream(0, small), "half_a": Stream(0, half_a),
               "half_b": Stream(0, half_b)}
    ts = {k: v.torch_stream() for k, v in streams.items()}

    def mm(i):
        torch.mm(a, b, out=outs[i])

    def time_eager(plan, reps=20):
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(ts["all"])
        for _ in range(reps):
            for k, (name, i) in enumerate(plan):
                ts[name].wait_event(s) if _ == 0 else None
                with torch.cuda.stream(ts[name]):
                    mm(i)
        for name, _i in plan:
            ts["all"].wait_stream(ts[name])
        e.record(ts["all"])
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps

    def time_graph(plan, reps=20):
        g = torch.cuda.CUDAGraph()
        cap = ts["all"]
        with torch.cuda.stream(cap):
            mm(0)  # warm
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=cap):
            for name, i in plan:
                ts[name].wait_stream(cap)
                with torch.cuda.stream(ts[name]):
                    mm(i)
            for name, _i in plan:
                cap.wait_stream(ts[name])
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(cap):
            s.record()
            for _ in range(reps):
                g.replay()
            e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps

    r = {"matmul": f"{n}^3 fp32"}
    r["eager_all_ms"] = round(time_eager([("all", 0)]), 3)
    r["eager_small32_ms"] = round(time_eager([("small", 0)]), 3)
    r["eager_half_ms"] = round(time_eager([("half_a", 0)]), 3)
    r["eager_two_halves_ms"] = round(time_eager([("half_a", 0), ("half_b", 1)]), 3)
    r["graph_small32_ms"] = round(time_graph([("small", 0)]), 3)
    r["graph_half_ms"] = round(time_graph([("half_a", 0)]), 3)
    r["graph_two_halves_ms"] = round(time_graph([("half_a", 0), ("half_b", 1)]), 3)
    r["reading"] = ("graph keeps masks" if r["graph_small32_ms"] > 2 * r["eager_all_ms"]
                    else "graph drops the capture streams' masks")
    print(json.dumps(r))
    if len(sys.argv) > 1:
        json.dump(r, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
