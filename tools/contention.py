"""Partition contention microbenchmark: each YOLOS-small hot op timed on ONE slice alone and on all
slices of a mode at once (every slice its own CU-masked stream, buffers and graph), so the loss
that concurrent partitions inflict on each other is attributed per op.

    python tools/contention.py [--mode cpx] [--iters 10] [--out gpurun_out/contention.json]

slowdown = (concurrent wall per call) / (alone wall per call); 1.0 = perfectly isolated slices.
Attention is timed with every head-block size (heads per launch) so the L2-sharing effect of
running a small slice's heads in blocks is measured directly.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from walkai_nos_amd.bench_core import slice_cus  # noqa: E402
from walkai_nos_amd.ops import kernels as K  # noqa: E402
from walkai_nos_amd.ops.probe import Stream  # noqa: E402

T, H, HD, D, FF = 3401, 6, 64, 384, 1536
PARTS = {"spx": 1, "dpx": 2, "qpx": 4, "cpx": 8}


class SliceOps:
    """One slice's operands and the ops of one layer, each a zero-arg callable."""

    def __init__(self, cus, seed):
        g = torch.Generator(device="cuda").manual_seed(seed)
        r = lambda *s: torch.randn(*s, device="cuda", generator=g) * 0.05  # noqa: E731
        self.x = r(T, D)
        self.h3 = K.split3(r(T, D))
        self.f3 = K.split3(r(T, FF))
        self.qkv3 = K.split3(r(1, T, 3 * D))
        self.o3 = torch.empty(3, 1, T, D, dtype=torch.bfloat16, device="cuda")
        self.w = {"qkv": r(3 * D, D), "proj": r(D, D), "fc1": r(FF, D), "fc2": r(D, FF)}
        self.b = {k: r(v.shape[0]) for k, v in self.w.items()}
        self.lnw, self.lnb = r(D) + 1, r(D)
        self.cus = cus

    def op(self, name, hb=None, tile=None):
        from walkai_nos_amd.ops.gemm import gemm_x3
        if name == "qkv":
            return lambda: gemm_x3(self.h3, self.w["qkv"], self.b["qkv"], out_f32=False, out_x3=True, tile=tile)
        if name == "qkv_f32":  # the same GEMM with an fp32 output (4 B per element instead of 6)
            return lambda: gemm_x3(self.h3, self.w["qkv"], self.b["qkv"], out_f32=True, out_x3=False, tile=tile)
        if name == "fc1_f32":
            return lambda: gemm_x3(self.h3, self.w["fc1"], self.b["fc1"], gelu=True, out_f32=True, out_x3=False,
                                   tile=tile)
        if name == "proj":
            return lambda: gemm_x3(self.h3, self.w["proj"], self.b["proj"], residual=self.x, tile=tile)
        if name == "fc1":
            return lambda: gemm_x3(self.h3, self.w["fc1"], self.b["fc1"], gelu=True, out_f32=False, out_x3=True,
                                   tile=tile)
        if name == "fc2":
            return lambda: gemm_x3(self.f3, self.w["fc2"], self.b["fc2"], residual=self.x, tile=tile)
        if name == "ln":
            return lambda: K.layernorm_x3(self.x, self.lnw, self.lnb, 1e-12)
        if name == "attn":
            n = 256 if self.cus is None else len(self.cus)
            hb = hb or H
            waves = K.attention_x3_waves(n, 1, T, hb)
            return lambda: K.attention_x3(self.qkv3, self.o3, H, HD, 0.125, waves, head_block=hb)
        raise KeyError(name)


def capture(fn, stream, n_cus, iters):
    K.set_slice_cus(n_cus)
    with torch.cuda.stream(stream):
        for _ in range(2):
            fn()
        stream.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for _ in range(iters):
                fn()
    stream.synchronize()
    return g


def wall(graphs_streams, reps=3):
    best = float("inf")
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for g, s in graphs_streams:
            with torch.cuda.stream(s):
                g.replay()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


GEMM_KEYS = {  # op -> (M, N, K, epilogue flags, output flags) as gemm_x3 keys its tuning cache
    "qkv": (T, 3 * D, D, 1, 2), "proj": (T, D, D, 1 | 4, 1), "fc1": (T, FF, D, 1 | 2, 2), "fc2": (T, D, FF, 1 | 4, 1),
    "qkv_f32": (T, 3 * D, D, 1, 1), "fc1_f32": (T, FF, D, 1 | 2, 1)}


def emit_table(path, results, sl, cus):
    table = {}
    if os.path.exists(path):
        with open(path) as f:
            table = json.load(f)
    best = {}
    for r in results:
        if r["op"] in GEMM_KEYS and r["tile"] is not None:
            if r["op"] not in best or r["concurrent_us"] < best[r["op"]]["concurrent_us"]:
                best[r["op"]] = r
    for op, r in best.items():
        m, n, k, epi, outf = GEMM_KEYS[op]
        table[f"M{m}_N{n}_K{k}_epi{epi}_out{outf}_cus{cus}"] = {
            "tile": r["tile"], "concurrent_us": r["concurrent_us"], "alone_us": r["alone_us"],
            "partitions": 256 // cus}
    with open(path, "w") as f:
        json.dump(dict(sorted(table.items())), f, indent=1)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="cpx", choices=sorted(PARTS))
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--ops", default="attn,qkv,proj,fc1,fc2,ln")
    ap.add_argument("--head-blocks", default="6,3,2,1")
    ap.add_argument("--attn-groups", default="8", help="query tiles per attention workgroup (4 and/or 8)")
    ap.add_argument("--ln-wg-per-cu", default="1000,1,2,4,8", help="LayerNorm workgroups per slice CU "
                    "(grid-stride; 1000 = one workgroup per 4 rows)")
    ap.add_argument("--tiles", default="", help="comma-separated x3 tile configs to force on the GEMM ops "
                    "(default: the autotuned tile)")
    ap.add_argument("--out", default="gpurun_out/contention.json")
    ap.add_argument("--emit-table", default="", help="merge the fastest concurrent tile per GEMM into this JSON "
                    "table (walkai_nos_amd/ops/x3_tuned.json format)")
    a = ap.parse_args()
    n = PARTS[a.mode]
    prof = f"{a.mode}_nps1"
    hs = [Stream(0, slice_cus(prof, k)) for k in range(n)]
    streams = [h.torch_stream() for h in hs]
    slices = [SliceOps(slice_cus(prof, k), 100 + k) for k in range(n)]
    n_cus = 256 // n
    cases = []
    for name in a.ops.split(","):
        if name == "attn":
            cases += [("attn", (int(hb), int(g))) for g in a.attn_groups.split(",") for hb in a.head_blocks.split(",")]
        elif name == "ln":
            cases += [("ln", ("ln", int(v))) for v in a.ln_wg_per_cu.split(",")]
        elif a.tiles == "all":
            from walkai_nos_amd.ops.gemm import x3_eligible
            w = slices[0].w[name.replace("_f32", "")]
            cases += [(name, ("tile", c)) for c in x3_eligible(w.shape[0], w.shape[1])]
        elif a.tiles:
            cases += [(name, ("tile", int(t))) for t in a.tiles.split(",")]
        else:
            cases.append((name, None))
    results = []
    for name, hb in cases:
        tile = hb[1] if isinstance(hb, tuple) and hb[0] == "tile" else None
        if isinstance(hb, tuple) and hb[0] == "ln":
            os.environ["NOS_LN_WG_PER_CU"] = str(hb[1])
            tile = hb[1]
        group = None
        if name == "attn":
            hb, group = hb
            K.set_attention_x3_group(group)
        hb = None if isinstance(hb, tuple) else hb
        graphs = [capture(sl.op(name, hb, tile), s, n_cus, a.iters) for sl, s in zip(slices, streams)]
        pairs = list(zip(graphs, streams))
        alone = wall(pairs[:1]) / a.iters * 1e6
        together = wall(pairs) / a.iters * 1e6
        r = {"mode": a.mode, "op": name, "head_block": hb, "group": group, "tile": tile, "alone_us": round(alone, 1),
             "concurrent_us": round(together, 1), "slowdown": round(together / alone, 3)}
        print(json.dumps(r), flush=True)
        results.append(r)
        del graphs, pairs
        torch.cuda.synchronize()
    for h in hs:
        h.close()
    if a.emit_table:
        emit_table(a.emit_table, results, slices[0], n_cus)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(results, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
