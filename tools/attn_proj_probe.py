"""Timing probe of the fused attention-merge + projection + LayerNorm kernel (csrc/attn_proj.hip)
against the three launches it replaces, with the kernel's timing-only ablations (bit 0: no merge,
bit 1: one weight fragment for every k-step, bit 2: no stores). One slice, YOLOS-small shapes."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--cus", type=int, default=0)
    ap.add_argument("--out", default="")
    ap.add_argument("--ablate", default="0,1,2,4,3,7", help="ablation masks to time (comma-separated)")
    ap.add_argument("--fused-only", action="store_true", help="skip the unfused reference timings")
    a = ap.parse_args()
    from walkai_nos_amd.ops import kernels as K
    if a.cus:
        K.set_slice_cus(a.cus)
    torch.manual_seed(0)
    B, T, H, Dh = 1, 3401, 6, 64
    D = H * Dh
    qkv = torch.randn(B, T, 3 * D, device="cuda")
    w = torch.randn(D, D, device="cuda") * 0.05
    b = torch.randn(D, device="cuda")
    r = torch.randn(B, T, D, device="cuda")
    ln = (torch.randn(D, device="cuda"), torch.randn(D, device="cuda"), 1e-12)
    L = K._L()
    cus = K.slice_cus()
    waves = K.attention_x3_waves(cus, B, T, H)
    ws = torch.empty(waves * 2 * (64 * 32 + 64) * 8, device="cuda")
    od = torch.empty(B, T, D, device="cuda")
    K._check(L.nos_attention_x3f_partials(qkv.data_ptr(), od.data_ptr(), ws.data_ptr(), B, T, H, Dh, 0.125, waves,
                                          K._stream()))
    from walkai_nos_amd.ops.gemm import weight_planes
    w3 = weight_planes(w)
    x = torch.empty_like(r)
    planes = torch.empty((3,) + tuple(r.shape), dtype=torch.bfloat16, device="cuda")

    def fused():
        L.nos_attn_merge_proj_ln(ws.data_ptr(), waves, od.data_ptr(), B, T, H, w3.data_ptr(), w3[0].numel(),
                                 b.data_ptr(), r.data_ptr(), ln[0].data_ptr(), ln[1].data_ptr(), 1e-12,
                                 x.data_ptr(), planes.data_ptr(), K._stream())

    def timed(fn, reps=20):
        """GPU time per call: ``reps`` calls captured in one HIP graph, replayed (no host launch
        cost in the figure)."""
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        for _ in range(3):
            g.replay()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = max(1, a.iters // reps)
        s.record()
        for _ in range(n):
            g.replay()
        e.record()
        torch.cuda.synchronize()
        return round(1000.0 * s.elapsed_time(e) / (n * reps), 2)

    out = {"cus": cus, "attention_waves": waves}
    L.nos_attn_proj_set_ablate.argtypes = [ctypes_int()]
    for ab in [int(x) for x in a.ablate.split(",") if x]:
        L.nos_attn_proj_set_ablate(ab)
        out[f"fused_ablate{ab}_us"] = timed(fused)
    L.nos_attn_proj_set_ablate(0)
    if a.fused_only:
        print(json.dumps(out))
        return
    o3 = K.attention_qkv_x3f(qkv, H, Dh, 0.125)
    K.linear_residual_ln_x3(o3, w, b, r, ln=ln)  # tune (and split the weight) before capture
    out["attention_with_fixup_us"] = timed(lambda: K.attention_qkv_x3f(qkv, H, Dh, 0.125))
    out["attention_partials_us"] = timed(lambda: L.nos_attention_x3f_partials(
        qkv.data_ptr(), od.data_ptr(), ws.data_ptr(), B, T, H, Dh, 0.125, waves, K._stream()))
    out["proj_ln_unfused_us"] = timed(lambda: K.linear_residual_ln_x3(o3, w, b, r, ln=ln))
    print(json.dumps(out))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


def ctypes_int():
    import ctypes
    return ctypes.c_int


if __name__ == "__main__":
    main()
