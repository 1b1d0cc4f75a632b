"""Repeat every x3 GEMM tile on the model's shapes and check each result against fp64 and
bit-for-bit against the tile's first run (races in the DMA ring or the LDS epilogue show up as
run-to-run differences): python tools/x3_gemm_stress.py [--reps 10]"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from walkai_nos_amd.ops import gemm as G  # noqa: E402
from walkai_nos_amd.ops import kernels as K  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--f32", action="store_true", help="fp32 output (direct-store epilogue) instead of planes")
    a = ap.parse_args()
    torch.manual_seed(0)
    bad = 0
    for (M, N, Kd) in ((3401, 1152, 384), (3401, 384, 384), (3401, 1536, 384), (3401, 384, 1536), (100, 128, 64)):
        x = torch.randn(M, Kd, device="cuda")
        w = torch.randn(N, Kd, device="cuda") * 0.05
        b = torch.randn(N, device="cuda")
        r = torch.randn(M, N, device="cuda")
        x3 = K.split3(x)
        ref = x.double() @ w.double().t() + b.double() + r.double()
        for cfg in G.x3_eligible(N, Kd):
            first = None
            for _ in range(a.reps):
                o = G.gemm_x3(x3, w, tile=cfg, out_f32=a.f32, out_x3=not a.f32, bias=b, residual=r)
                torch.cuda.synchronize()
                if first is None:
                    first = o.clone()
                    err = ((o.double() if a.f32 else o.double().sum(0)) - ref).abs().max().item()
                    if err > 1e-4:
                        print("INACCURATE", M, N, Kd, cfg, err, flush=True)
                        bad += 1
                elif not torch.equal(o, first):
                    d = (o != first) if a.f32 else (o != first).any(0)
                    print("NONDETERMINISTIC", M, N, Kd, cfg, int(d.sum()), d.nonzero()[:3].tolist(), flush=True)
                    bad += 1
                    break
        print("ok" if not bad else "FAIL", M, N, Kd, flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
