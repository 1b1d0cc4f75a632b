"""x3 attention time vs persistent grid size on one slice (stream-K unit alignment study).

    python tools/attn_grid.py [--slices spx,dpx] [--grids 256,252,168,128,84] [--out ...]

With P = (query groups) x s workgroups, stream-K segment boundaries fall on query-group boundaries:
every workgroup owns exactly one key range of one group (one partial, one prologue)."""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tools.kbench import timeit  # noqa: E402
from walkai_nos_amd.bench_core import slice_cus  # noqa: E402
from walkai_nos_amd.ops import kernels as K  # noqa: E402
from walkai_nos_amd.ops.probe import Stream  # noqa: E402

T, H, HD, D = 3401, 6, 64, 384


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--slices", default="spx,dpx,qpx,cpx")
    ap.add_argument("--grids", default="")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default="gpurun_out/attn_grid.json")
    a = ap.parse_args()
    torch.manual_seed(0)
    planes = K.split3(torch.randn(1, T, 3 * D, device="cuda") * 0.5)
    out = torch.empty(3, 1, T, D, dtype=torch.bfloat16, device="cuda")
    res = []
    for label in a.slices.split(","):
        prof = f"{label}_nps1"
        cus = slice_cus(prof, 0)
        n = 256 if cus is None else len(cus)
        qg = H * (((T + 31) // 32 + 7) // 8)
        grids = [int(g) for g in a.grids.split(",")] if a.grids else sorted(
            {n, n - n % qg if n >= qg else n, qg, qg * (n // qg) if n >= qg else qg, n // 2, (3 * n) // 4})
        with Stream(0, cus) as hs:
            s = hs.torch_stream()
            K.set_slice_cus(n)
            for g in grids:
                if g <= 0 or g > n:
                    continue
                us = timeit(lambda: K.attention_x3(planes, out, H, HD, 0.125, g), s, a.iters)
                r = {"slice": label, "cus": n, "grid": g, "us": round(us, 1),
                     "units_per_wg": round(qg * ((T + 31) // 32) / g, 1)}
                print(json.dumps(r), flush=True)
                res.append(r)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
