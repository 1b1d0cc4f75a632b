"""fp32 activation operand for the x3 GEMMs (csrc/gemm_x3.hip gemm_x3a) against the planes-in
kernel on the model's shapes, whole GPU, graph-replayed: the GEMM alone, and with its producer
(LayerNorm emitting planes vs LayerNorm emitting fp32).

    python tools/x3_f32a_probe.py [--out gpurun_out/x3_f32a.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from walkai_nos_amd.ops import gemm as G  # noqa: E402
from walkai_nos_amd.ops import kernels as K  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/x3_f32a.json")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    K.set_backend("hip")
    s = torch.cuda.Stream()
    rows = {}
    with torch.cuda.stream(s):
        torch.manual_seed(0)
        M = 3401
        x = torch.randn(M, 384, device="cuda")
        lw, lb = torch.randn(384, device="cuda"), torch.randn(384, device="cuda")
        for name, N, gelu, x3out in (("qkv", 1152, False, False), ("fc1", 1536, True, True)):
            w = torch.randn(N, 384, device="cuda") * 0.05
            b = torch.randn(N, device="cuda")
            G.weight_planes(w)
            h3 = K.layernorm_x3(x, lw, lb, 1e-12)
            h = K.layernorm(x, lw, lb, 1e-12)
            res = {}
            for tile in (29, 36):
                f = lambda tile=tile: G.gemm_x3(h3, w, b, gelu=gelu, out_f32=not x3out, out_x3=x3out, tile=tile)  # noqa: E731
                res[f"planes_tile{tile}_us"] = round(1000 * G._gpu_time(f, s, a.reps) / a.reps, 2)
                g = lambda tile=tile: (K.layernorm_x3(x, lw, lb, 1e-12),  # noqa: E731
                                       G.gemm_x3(h3, w, b, gelu=gelu, out_f32=not x3out, out_x3=x3out, tile=tile))
                res[f"ln_planes+tile{tile}_us"] = round(1000 * G._gpu_time(g, s, a.reps) / a.reps, 2)
            for cfg in (0, 1):
                f = lambda cfg=cfg: G.gemm_x3_f32a(h, w, b, gelu=gelu, out_f32=not x3out, out_x3=x3out, cfg=cfg)  # noqa: E731
                res[f"f32a_cfg{cfg}_us"] = round(1000 * G._gpu_time(f, s, a.reps) / a.reps, 2)
                g = lambda cfg=cfg: (K.layernorm(x, lw, lb, 1e-12),  # noqa: E731
                                     G.gemm_x3_f32a(h, w, b, gelu=gelu, out_f32=not x3out, out_x3=x3out, cfg=cfg))
                res[f"ln_f32+f32a_cfg{cfg}_us"] = round(1000 * G._gpu_time(g, s, a.reps) / a.reps, 2)
            rows[name] = res
            print(name, json.dumps(res), flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rows, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
