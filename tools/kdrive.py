"""Run one hot op of the YOLOS-small layer a few times, eagerly, on one slice — a driver for
rocprofv3 PMC passes (one dispatch per call, no graph):

    rocprofv3 --pmc <counters> --kernel-trace -- python3 tools/kdrive.py --op attn_x3f --slice spx
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from walkai_nos_amd.bench_core import slice_cus  # noqa: E402
from walkai_nos_amd.ops import gemm as G  # noqa: E402
from walkai_nos_amd.ops import kernels as K  # noqa: E402
from walkai_nos_amd.ops.probe import Stream  # noqa: E402

T, H, D, FF = 3401, 6, 384, 1536
PROFILES = {"spx": "spx_nps1", "dpx": "dpx_nps1", "qpx": "qpx_nps1", "cpx": "cpx_nps1"}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="attn_x3",
                    choices=("attn_x3", "attn_x3f", "attn_f32", "qkv_x3", "proj_x3", "fc1_x3", "fc2_x3", "layernorm_x3"))
    ap.add_argument("--slice", default="spx", choices=tuple(PROFILES))
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--tile", type=int, default=None, help="force an x3 GEMM tile config (no autotune dispatches)")
    a = ap.parse_args()
    torch.manual_seed(0)
    cus = slice_cus(PROFILES[a.slice], 0)
    n = 256 if cus is None else len(cus)
    qkv = torch.randn(1, T, 3 * D, device="cuda")
    x = torch.randn(T, D, device="cuda")
    h = torch.randn(T, FF, device="cuda")
    shapes = {"qkv_x3": (x, 3 * D, False, True), "proj_x3": (x, D, False, False),
              "fc1_x3": (x, FF, True, True), "fc2_x3": (h, D, False, False)}
    with Stream(0, cus) as hs, torch.cuda.stream(hs.torch_stream()):
        K.set_slice_cus(n)
        planes = K.split3(qkv)
        if a.op in shapes:
            xa, N, gelu, out3 = shapes[a.op]
            w = torch.randn(N, xa.shape[1], device="cuda") * 0.05
            b = torch.randn(N, device="cuda")
            xa3 = K.split3(xa)
            fn = lambda: G.gemm_x3(xa3, w, b, gelu=gelu, out_f32=not out3, out_x3=out3, tile=a.tile)  # noqa: E731
        elif a.op == "attn_x3":
            fn = lambda: K.attention_qkv_x3(planes, H, 64, 0.125)  # noqa: E731
        elif a.op == "attn_x3f":  # the model's path: fp32 QKV in (attn_fwd_x3w unless NOS_ATTN_WIDE=0)
            waves = K.attention_x3_waves(n, 1, T, H)
            out = torch.empty(1, T, D, device="cuda")
            fn = lambda: K.attention_x3f(qkv, out, H, 64, 0.125, waves)  # noqa: E731
        elif a.op == "attn_f32":
            K.set_fp32_matmul("f32")
            fn = lambda: K.attention_qkv(qkv, H, 64, 0.125)  # noqa: E731
        else:
            w, b = torch.randn(D, device="cuda"), torch.randn(D, device="cuda")
            fn = lambda: K.layernorm_x3(x, w, b, 1e-12)  # noqa: E731
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
    print("done", a.op, a.slice, n)
    return 0


if __name__ == "__main__":
    sys.exit(main())
