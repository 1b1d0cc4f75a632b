"""x3 GEMM as ONE plain bf16 GEMM over a K-concatenated operand pair, on hipBLASLt.

The six bf16 products of an x3 GEMM (a2b0 + a1b1 + a0b2 + a1b0 + a0b1 + a0b0) are one bf16 GEMM
with fp32 accumulation over K' = 6K:  A' = [a2 | a1 | a0 | a1 | a0 | a0]  (M x 6K),
W' = [w0 | w1 | w2 | w0 | w1 | w0]  (N x 6K),  C = A' W'^T.  This probe times that against the
hand-written x3 kernel (fp32 out, no epilogue, autotuned) for the YOLOS-small layer shapes on one
slice alone, and checks both against fp64; the x3 attention is set against the vendor's bf16 SDPA
(flash attention, a sixth of the MFMA work) the same way:

    python tools/x3cat_probe.py --slices spx,dpx,cpx --out gpurun_out/x3cat.json
"""
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
SHAPES = {"qkv": (3 * D, D), "proj": (D, D), "fc1": (FF, D), "fc2": (D, FF)}
PROFILES = {"spx": "spx_nps1", "dpx": "dpx_nps1", "qpx": "qpx_nps1", "cpx": "cpx_nps1"}


def cat_a(a3: torch.Tensor) -> torch.Tensor:
    return torch.cat([a3[2], a3[1], a3[0], a3[1], a3[0], a3[0]], dim=1).contiguous()


def cat_w(w3: torch.Tensor) -> torch.Tensor:
    return torch.cat([w3[0], w3[1], w3[2], w3[0], w3[1], w3[0]], dim=1).contiguous()


def timed(fn, stream, reps: int = 20) -> float:
    return G._gpu_time(fn, stream, reps) * 1000.0 / reps


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--slices", default="spx,dpx,cpx")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    torch.manual_seed(0)
    rows = []
    for sl in a.slices.split(","):
        cus = slice_cus(PROFILES[sl], 0)
        n = 256 if cus is None else len(cus)
        with Stream(0, cus) as hs, torch.cuda.stream(hs.torch_stream()):
            stream = torch.cuda.current_stream()
            K.set_slice_cus(n)
            for name, (N, Kd) in SHAPES.items():
                x = torch.randn(T, Kd, device="cuda")
                w = torch.randn(N, Kd, device="cuda") * 0.05
                a3 = K.split3(x)
                w3 = G.weight_planes(w)
                ac, wc = cat_a(a3), cat_w(w3)
                wct = wc.t().contiguous()       # [6K, N]: the other operand layout
                out = torch.empty(T, N, device="cuda")
                ref = (x.double() @ w.double().t())
                y3 = G.gemm_x3(a3, w)
                yc = torch.mm(ac, wc.t(), out_dtype=torch.float32)
                yt = torch.mm(ac, wct, out_dtype=torch.float32)
                torch.cuda.synchronize()
                scale = ref.abs().max().item()
                r = {"slice": sl, "cus": n, "op": name, "M": T, "N": N, "K": Kd,
                     "x3_us": round(timed(lambda: G.gemm_x3(a3, w, out=out), stream), 2),
                     "cat_nt_us": round(timed(lambda: torch.mm(ac, wc.t(), out_dtype=torch.float32), stream), 2),
                     "cat_nn_us": round(timed(lambda: torch.mm(ac, wct, out_dtype=torch.float32), stream), 2),
                     "f32_hipblaslt_us": round(timed(lambda: torch.mm(x, w.t()), stream), 2),
                     "err_x3": (y3.double() - ref).abs().max().item() / scale,
                     "err_cat_nt": (yc.double() - ref).abs().max().item() / scale,
                     "err_cat_nn": (yt.double() - ref).abs().max().item() / scale,
                     "err_f32_mm": (torch.mm(x, w.t()).double() - ref).abs().max().item() / scale}
                flop6 = 6 * 2 * T * N * Kd
                for k in ("x3_us", "cat_nt_us", "cat_nn_us"):
                    r[k.replace("_us", "_pct_slice_peak")] = round(100 * flop6 / (r[k] * 1e-6) / (2.5e15 * n / 256), 1)
                print(json.dumps(r), flush=True)
                rows.append(r)
            # attention: the x3 kernel (6 bf16 MFMAs per fp32 product) against the vendor's bf16
            # flash attention (1 MFMA per product) on the same shape — MFMA work rate of each
            qkv = torch.randn(1, T, 3 * D, device="cuda")
            planes = K.split3(qkv)
            q, k, v = (t.view(1, T, 6, 64).transpose(1, 2).contiguous() for t in qkv.split(D, dim=2))
            qb, kb, vb = (t.bfloat16() for t in (q, k, v))
            ref = torch.nn.functional.scaled_dot_product_attention(q.double(), k.double(), v.double())
            o3 = K.attention_qkv_x3(planes, 6, 64, 0.125).double().sum(0).view(1, T, 6, 64).transpose(1, 2)
            ob = torch.nn.functional.scaled_dot_product_attention(qb, kb, vb)
            fl = 4 * T * T * D
            r = {"slice": sl, "cus": n, "op": "attention", "T": T, "heads": 6, "head_dim": 64,
                 "x3_us": round(timed(lambda: K.attention_qkv_x3(planes, 6, 64, 0.125), stream, 5), 2),
                 "sdpa_bf16_us": round(timed(lambda: torch.nn.functional.scaled_dot_product_attention(qb, kb, vb),
                                             stream, 5), 2),
                 "err_x3": (o3.double() - ref).abs().max().item(),
                 "err_sdpa_bf16": (ob.double() - ref).abs().max().item()}
            peak = 2.5e15 * n / 256
            r["x3_pct_slice_peak"] = round(100 * 6 * fl / (r["x3_us"] * 1e-6) / peak, 1)
            r["sdpa_bf16_pct_slice_peak"] = round(100 * fl / (r["sdpa_bf16_us"] * 1e-6) / peak, 1)
            print(json.dumps(r), flush=True)
            rows.append(r)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
