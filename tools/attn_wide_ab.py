"""A/B of the fp32-input x3 attention kernels on the GPU box: ``attn_fwd_x3w`` (one wave per SIMD,
two query tiles per wave) vs ``attn_fwd_x3p<8>`` (two waves per SIMD), on whole-GPU / half / eighth
slices, plus the whole YOLOS-small inference with each.

    python tools/attn_wide_ab.py [--iters 20] [--out gpurun_out/attn_wide_ab.json]

Checks first that both kernels give bit-identical outputs (fp32 and x3-plane outputs, the
production grid and odd grids), then times each (HIP-graph replay, alternating arms per round).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from walkai_nos_amd.bench_core import slice_cus  # noqa: E402
from walkai_nos_amd.ops import kernels as K  # noqa: E402
from walkai_nos_amd.ops.probe import Stream  # noqa: E402
from tools.kbench import timeit  # noqa: E402

T, H, HD, D = 3401, 6, 64, 384


def identical(qkv, waves_list) -> dict:
    res = {}
    for waves in waves_list:
        for x3 in (False, True):
            outs = []
            for wide in (True, False):
                K.set_attention_x3_wide(wide)
                out = (torch.empty(3, 1, T, D, dtype=torch.bfloat16, device="cuda") if x3
                       else torch.empty(1, T, D, device="cuda"))
                out.fill_(float("nan"))
                K.attention_x3f(qkv, out, H, HD, 0.125, waves)
                outs.append(out)
            torch.cuda.synchronize()
            res[f"w{waves}_{'x3' if x3 else 'f32'}"] = bool(torch.equal(outs[0], outs[1]))
    K.set_attention_x3_wide(K.attention_x3_wide_default())
    return res


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--slices", default="spx,dpx,cpx")
    ap.add_argument("--model", action="store_true", help="also time the whole inference per arm")
    ap.add_argument("--arms", default="wide,x3p8",
                    help="arms to time (one arm for a counter pass): wide = attn_fwd_x3w + the fixup launch "
                         "(production), wide_xfix = the same with the fixup's XCD-local tile order, wide_merge = "
                         "the merge inside the kernel, x3p8 = attn_fwd_x3p<8>")
    ap.add_argument("--no-check", action="store_true", help="skip the bit-identity check")
    ap.add_argument("--out", default="gpurun_out/attn_wide_ab.json")
    a = ap.parse_args()
    torch.manual_seed(0)
    qkv = torch.randn(1, T, 3 * D, device="cuda")
    report = {"T": T, "H": H}
    if not a.no_check:
        report["identical"] = identical(qkv, (K.attention_x3_waves(256, 1, T, H), 7, 64, 333))
        print(json.dumps(report["identical"]), flush=True)
    arms = [(arm, arm.startswith("wide")) for arm in a.arms.split(",")]

    def use(arm: str, wide: bool) -> None:
        K.set_attention_x3_wide(wide)
        K.set_attention_merge(arm == "wide_merge")
        # wide_xfix: the fixup's XCD-local tile order (flag bit 6)
        K._L().nos_attention_x3_set_flags(64 if arm == "wide_xfix" else int(os.environ.get("NOS_ATTN_X3_FLAGS", "0")))
    flops_x3 = 4.0 * T * T * HD * H * 6
    for label in a.slices.split(","):
        cus = slice_cus(f"{label}_nps1", 0)
        n = 256 if cus is None else len(cus)
        r = {"cus": n}
        with Stream(0, cus) as hs:
            s = hs.torch_stream()
            K.set_slice_cus(n)
            waves = K.attention_x3_waves(n, 1, T, H)
            r["waves"] = waves
            out = torch.empty(3, 1, T, D, dtype=torch.bfloat16, device="cuda")
            times = {arm: [] for arm, _ in arms}
            for _ in range(a.rounds):
                for arm, wide in arms:
                    use(arm, wide)
                    times[arm].append(timeit(lambda: K.attention_x3f(qkv, out, H, HD, 0.125, waves), s, a.iters))
            for arm, v in times.items():
                r[f"{arm}_us"] = round(min(v), 2)
                r[f"{arm}_us_all"] = [round(x, 2) for x in v]
                r[f"{arm}_bf16_peak_pct"] = round(100 * flops_x3 / (min(v) * 1e-6) / (2.5e15 * n / 256), 1)
            if a.model:
                from walkai_nos_amd.models.workload.yolos import DEMO_INPUT_HW, YolosSmall, demo_input
                with torch.cuda.stream(s):
                    m = YolosSmall().cuda().eval()
                    xin = demo_input(1, DEMO_INPUT_HW, "cuda")
                mt = {arm: [] for arm, _ in arms}
                with torch.no_grad():
                    for _ in range(a.rounds):
                        for arm, wide in arms:
                            use(arm, wide)
                            mt[arm].append(timeit(lambda: m(xin), s, 5) / 1000.0)
                for arm, v in mt.items():
                    r[f"model_{arm}_ms"] = round(min(v), 3)
                    r[f"model_{arm}_ms_all"] = [round(x, 3) for x in v]
            K.set_attention_x3_wide(K.attention_x3_wide_default())
            K.set_attention_merge(None)
        report[label] = r
        print(label, json.dumps(r), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(report, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
