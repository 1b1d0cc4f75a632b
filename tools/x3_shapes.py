"""Every eligible x3 GEMM config on the model's four GEMM shapes (with their real epilogues and
outputs) on one slice, timed by HIP-graph replay: python tools/x3_shapes.py [--slice spx]
[--out gpurun_out/x3_shapes.json]. Prints the three fastest per shape, then the per-layer GEMM
total of the fastest picks."""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from walkai_nos_amd.bench_core import slice_cus  # noqa: E402
from walkai_nos_amd.ops import gemm as G  # noqa: E402
from walkai_nos_amd.ops import kernels as K  # noqa: E402
from walkai_nos_amd.ops.probe import Stream  # noqa: E402

T, D, FF = 3401, 384, 1536
#: name -> (N, K, epilogue kwargs, out_f32, out_x3) as YoloLayer.forward calls them
SHAPES = {"qkv": (3 * D, D, {"bias": True}, True, False),
          "proj": (D, D, {"bias": True, "residual": True}, True, False),
          "fc1": (FF, D, {"bias": True, "gelu": True}, False, True),
          "fc2": (D, FF, {"bias": True, "residual": True}, True, False)}


def timeit(fn, stream, iters):
    with torch.cuda.stream(stream):
        for _ in range(2):
            fn()
        stream.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for _ in range(iters):
                fn()
        g.replay()
        stream.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record(stream)
        g.replay()
        en.record(stream)
    en.synchronize()
    return st.elapsed_time(en) * 1000.0 / iters


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--slice", default="spx")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default="gpurun_out/x3_shapes.json")
    a = ap.parse_args()
    torch.manual_seed(0)
    cus = slice_cus(f"{a.slice}_nps1", 0)
    res = {}
    with Stream(0, cus) as hs:
        s = hs.torch_stream()
        K.set_slice_cus(256 if cus is None else len(cus))
        for name, (N, Kd, epi, of, ox) in SHAPES.items():
            with torch.cuda.stream(s):
                x3 = K.split3(torch.randn(T, Kd, device="cuda"))
                w = torch.randn(N, Kd, device="cuda") * 0.05
                w3 = G.weight_planes(w)
                kw = {"bias": torch.randn(N, device="cuda") if epi.get("bias") else None,
                      "gelu": epi.get("gelu", False),
                      "residual": torch.randn(T, N, device="cuda") if epi.get("residual") else None}
            times = {}
            for cfg in G.x3_eligible(N, Kd):
                times[cfg] = round(timeit(lambda cfg=cfg: G.gemm_x3(x3, w3, tile=cfg, out_f32=of, out_x3=ox, **kw),
                                          s, a.iters), 2)
            flops = 2.0 * T * N * Kd
            order = sorted(times, key=times.get)
            res[name] = {"top5": [{"cfg": c, "tile": G.X3_TILES[c], "us": times[c],
                                   "fp32eq_tflops": round(flops / times[c] / 1e6, 1)} for c in order[:5]],
                         "all_us": {str(c): t for c, t in times.items()}}
            print(name, json.dumps(res[name]["top5"][:3]), flush=True)
    res["layer_best_us"] = round(sum(r["top5"][0]["us"] for k, r in res.items() if k in SHAPES), 1)
    print("per-layer GEMMs: best", res["layer_best_us"], "us")
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump({"slice": a.slice, **res}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
