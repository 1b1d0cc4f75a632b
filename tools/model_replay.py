"""Warm, capture and replay one YOLOS-small inference on a slice (for kernel traces of the steady
state): python tools/model_replay.py [--slice spx] [--replays 40]. Prints ms per inference."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from walkai_nos_amd.bench_core import slice_cus  # noqa: E402
from walkai_nos_amd.models.workload.yolos import DEMO_INPUT_HW, YolosSmall, demo_input  # noqa: E402
from walkai_nos_amd.ops import kernels as K  # noqa: E402
from walkai_nos_amd.ops.probe import Stream  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--slice", default="spx")
    ap.add_argument("--replays", type=int, default=40)
    ap.add_argument("--tables", action="store_true", help="print the GEMM tiles / split-K choices the tuner made")
    a = ap.parse_args()
    cus = slice_cus(f"{a.slice}_nps1", 0)
    with Stream(0, cus) as hs:
        s = hs.torch_stream()
        K.set_slice_cus(256 if cus is None else len(cus))
        with torch.no_grad(), torch.cuda.stream(s):
            m = YolosSmall().cuda().eval()
            x = demo_input(1, DEMO_INPUT_HW, "cuda")
            for _ in range(3):
                m(x)
            s.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                m(x)
            for _ in range(3):
                g.replay()
            s.synchronize()
            time.sleep(0.2)  # a visible gap in the trace before the measured replays
            t0 = time.perf_counter()
            for _ in range(a.replays):
                g.replay()
            s.synchronize()
            dt = (time.perf_counter() - t0) / a.replays
        print(f"{a.slice}: {dt * 1e3:.3f} ms per inference over {a.replays} replays", flush=True)
        if a.tables:
            from walkai_nos_amd.ops import gemm as G
            print(json.dumps({"x3": G.x3_table(), "x3_us": G.x3_timings(), "linear_residual_ln": G.fused_table(),
                              "linear_residual_ln_us": G.fused_timings()}, indent=1), flush=True)
        del g
    return 0


if __name__ == "__main__":
    sys.exit(main())
