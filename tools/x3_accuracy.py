"""Accuracy evidence for the x3 (three-bf16-plane) fp32 path: max |error| vs an fp64 reference of
the same op, for the x3 kernels and for the f32-input-MFMA kernels, on the YOLOS-small shapes.

    python tools/x3_accuracy.py --out profiles/x3_accuracy.json
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from walkai_nos_amd.ops import gemm as G  # noqa: E402
from walkai_nos_amd.ops import kernels as K  # noqa: E402

T, H, D, FF = 3401, 6, 384, 1536


def attn_ref(qkv):
    q, k, v = qkv.double().view(1, T, 3, H, 64).permute(2, 0, 3, 1, 4)
    p = torch.softmax((q @ k.transpose(-1, -2)) * 0.125, dim=-1)
    return (p @ v).transpose(1, 2).reshape(1, T, D)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/x3_accuracy.json")
    a = ap.parse_args()
    torch.manual_seed(0)
    res = {}
    qkv = torch.randn(1, T, 3 * D, device="cuda")
    ref = attn_ref(qkv)
    o32 = torch.empty(1, T, D, device="cuda")
    K.attention_sk(qkv, o32, H, 64, 0.125, 512)
    o3 = torch.empty(1, T, D, device="cuda")
    K.attention_x3(K.split3(qkv), o3, H, 64, 0.125, 512)
    res["attention"] = {"f32_mfma_max_abs_err": (o32.double() - ref).abs().max().item(),
                        "x3_max_abs_err": (o3.double() - ref).abs().max().item()}
    for name, (M, N, Kd) in {"qkv": (T, 3 * D, D), "proj": (T, D, D), "fc1": (T, FF, D), "fc2": (T, D, FF)}.items():
        x = torch.randn(M, Kd, device="cuda")
        w = torch.randn(N, Kd, device="cuda") / math.sqrt(Kd)
        b = torch.randn(N, device="cuda")
        r = x.double() @ w.double().t() + b.double()
        y32 = G.gemm(x, w, b, tile=0)
        y3 = G.gemm_x3(K.split3(x), w, b)
        res[f"gemm_{name}"] = {"f32_mfma_max_abs_err": (y32.double() - r).abs().max().item(),
                               "x3_max_abs_err": (y3.double() - r).abs().max().item(),
                               "ref_max_abs": r.abs().max().item()}
    from walkai_nos_amd.models.workload.yolos import YolosSmall, demo_input
    m = YolosSmall().cuda().eval()
    xin = demo_input(1, (800, 1066), "cuda")
    with torch.no_grad():
        K.set_fp32_matmul("f32")
        l32, b32 = m(xin)
        K.set_fp32_matmul("x3")
        l3, b3 = m(xin)
        md = YolosSmall().double().eval()
        md.load_state_dict({k: v.double() for k, v in m.state_dict().items()})
        K.set_backend("torch")
        ld, bd = md.cuda()(xin.double())
        K.set_backend("hip")
    res["yolos_small_logits"] = {"f32_mfma_max_abs_err": (l32.double() - ld).abs().max().item(),
                                 "x3_max_abs_err": (l3.double() - ld).abs().max().item(),
                                 "ref_max_abs": ld.abs().max().item()}
    res["yolos_small_boxes"] = {"f32_mfma_max_abs_err": (b32.double() - bd).abs().max().item(),
                                "x3_max_abs_err": (b3.double() - bd).abs().max().item()}
    res["note"] = ("max |error| vs an fp64 reference of the same op on the same inputs; x3 = both fp32 operands "
                   "split exactly into three bf16 planes, six bf16 MFMAs per product block")
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
