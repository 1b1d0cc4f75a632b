"""Cost of the fc1 epilogue parts at SPX: the fc1 GEMM (3401 x 1536 x 384) with / without GELU and
with x3-plane vs fp32 output, each on the tile the tuner picks for the model's variant (graph replay).
python tools/epi_cost.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tools.x3_shapes import timeit  # noqa: E402
from walkai_nos_amd.ops import gemm as G  # noqa: E402
from walkai_nos_amd.ops import kernels as K  # noqa: E402


def main():
    torch.manual_seed(0)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        x3 = K.split3(torch.randn(3401, 384, device="cuda"))
        w3 = G.weight_planes(torch.randn(1536, 384, device="cuda") * 0.05)
        b = torch.randn(1536, device="cuda")
    for tile in (6, 27, 14):
        row = {}
        for gelu in (True, False):
            for planes in (True, False):
                us = timeit(lambda: G.gemm_x3(x3, w3, b, gelu=gelu, out_f32=not planes, out_x3=planes, tile=tile), s, 20)
                row[f"{'gelu' if gelu else 'nogelu'}_{'planes' if planes else 'f32'}"] = round(us, 2)
        print("tile", tile, row, flush=True)


if __name__ == "__main__":
    main()
