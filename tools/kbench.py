"""Per-slice kernel microbenchmark on the GPU box: the YOLOS-small layer's hot ops timed on
CU-masked streams of 256/128/64/32 CUs (SPX/DPX/QPX/CPX-sized slices), one slice at a time.

    python tools/kbench.py [--iters N] [--out gpurun_out/kbench.json]

Reports microseconds per call and achieved TFLOP/s for: attention (unsplit one-wave-per-tile
baseline, stream-K LDS-shared workgroup kernel, stream-K one-wave kernel with 2 and 3
resident waves/SIMD, PyTorch SDPA), and the four fp32 GEMMs of a
layer (hipBLASLt via torch).
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
from walkai_nos_amd.ops import gemm as G  # noqa: E402
from walkai_nos_amd.ops import kernels as K  # noqa: E402
from walkai_nos_amd.ops.probe import Stream  # noqa: E402

T, H, HD, D, FF = 3401, 6, 64, 384, 1536


def timeit(fn, stream, iters):
    """GPU time per call: ``iters`` calls captured in one HIP graph on the slice's stream and
    replayed, so host-side launch overhead (ctypes, allocation) is not measured."""
    with torch.cuda.stream(stream):
        for _ in range(3):
            fn()
        stream.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for _ in range(iters):
                fn()
        g.replay()
        stream.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record(stream)
        g.replay()
        en.record(stream)
    en.synchronize()
    return st.elapsed_time(en) * 1000.0 / iters


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default="gpurun_out/kbench.json")
    ap.add_argument("--only", choices=("all", "attn", "gemm", "model", "modes"), default="all")
    ap.add_argument("--slices", default="spx,dpx,qpx,cpx")
    ap.add_argument("--partitions", type=int, default=0, help="modes: run only this many partitions of each mode")
    ap.add_argument("--free-s", type=float, default=0.0,
                    help="modes: serve free-running (one thread per pod, as the bench) for this many seconds "
                         "instead of lock-step rounds")
    ap.add_argument("--lane-cus", type=int, default=0,
                    help="modes: serve partitions wider than this as request lanes of this many CUs (the bench's --lane-cus)")
    ap.add_argument("--emulation", default="spread", choices=("pinned", "spread", "landing"),
                    help="modes: compute-partition emulation (bench_core.EMULATION)")
    a = ap.parse_args()
    torch.manual_seed(0)
    if a.only == "modes":
        return modes_bench(a)
    qkv = torch.randn(1, T, 3 * D, device="cuda")
    out = torch.empty(1, T, D, device="cuda")
    x = torch.randn(T, D, device="cuda")
    h = torch.randn(T, FF, device="cuda")
    w_qkv, w_o = torch.randn(3 * D, D, device="cuda"), torch.randn(D, D, device="cuda")
    w_1, w_2 = torch.randn(FF, D, device="cuda"), torch.randn(D, FF, device="cuda")
    b_ff = torch.randn(FF, device="cuda")
    b_qkv, b_d = torch.randn(3 * D, device="cuda"), torch.randn(D, device="cuda")
    attn_flops = 4.0 * T * T * HD * H
    q, k, v = qkv.view(1, T, 3, H, HD).permute(2, 0, 3, 1, 4)
    results = []
    for prof, part, label in (("spx_nps1", 0, "spx"), ("dpx_nps1", 0, "dpx"), ("qpx_nps1", 0, "qpx"),
                              ("cpx_nps1", 0, "cpx")):
        if label not in a.slices.split(","):
            continue
        cus = slice_cus(prof, part)
        n = 256 if cus is None else len(cus)
        with Stream(0, cus) as hs:
            s = hs.torch_stream()
            r = {"slice": label, "cus": n}
            K.set_slice_cus(n)
            if a.only in ("all", "attn"):
                attn_bench(r, qkv, out, q, k, v, n, s, a.iters, attn_flops)
            if a.only in ("all", "gemm"):
                gemm_bench(r, x, h, w_qkv, w_o, w_1, w_2, b_ff, b_qkv, b_d, s, a.iters)
            if a.only in ("all", "model"):
                model_bench(r, s, max(3, a.iters // 4))
            r["layernorm_us"] = round(timeit(lambda: K.layernorm(x, w_o[0], w_o[1], 1e-12), s, a.iters), 1)
            r["layernorm_x3_us"] = round(timeit(lambda: K.layernorm_x3(x, w_o[0], w_o[1], 1e-12), s, a.iters), 1)
            for kname in list(r):
                if isinstance(r[kname], float):
                    r[kname] = round(r[kname], 2)
            print(json.dumps(r), flush=True)
            results.append(r)
    K.set_attention_variant(0)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(results, f, indent=1)
    return 0


def attn_bench(r, qkv, out, q, k, v, n, s, iters, attn_flops, variants=(0, 2, 3)):
    r["attn_unsplit_us"] = timeit(lambda: K.attention_unsplit(qkv, H, HD, 0.125), s, iters)
    for var in variants:
        K.set_attention_variant(var)
        wv = K.attention_waves(n)
        r[f"attn_sk{var}_us"] = timeit(lambda: K.attention_sk(qkv, out, H, HD, 0.125, wv), s, iters)
        r[f"attn_sk{var}_grid"] = wv
    K.set_attention_variant(0)
    for mult in (1, 2):  # LDS kernel with fewer persistent workgroups per CU than resident slots
        r[f"attn_sk0g{mult}_us"] = timeit(lambda: K.attention_sk(qkv, out, H, HD, 0.125, mult * n), s, iters)
    planes = K.split3(qkv)
    wx = K.attention_x3_waves(n, 1, T, H)
    r["attn_x3_us"] = timeit(lambda: K.attention_x3(planes, out, H, HD, 0.125, wx), s, iters)
    r["attn_x3_grid"] = wx
    for mult in (1, 2):
        r[f"attn_x3g{mult}_us"] = timeit(lambda: K.attention_x3(planes, out, H, HD, 0.125, mult * n), s, iters)
    K.set_attention_x3_group(4)  # the default is 8 query tiles per workgroup: time 4 as the A/B
    w4 = K.attention_x3_waves(n, 1, T, H)
    r["attn_x3q4_us"] = timeit(lambda: K.attention_x3(planes, out, H, HD, 0.125, w4), s, iters)
    r["attn_x3q4_grid"] = w4
    K.set_attention_x3_group(8)
    K.set_attention_x3_pipelined(False)
    wnp = K.attention_x3_waves(n, 1, T, H)
    r["attn_x3np_us"] = timeit(lambda: K.attention_x3(planes, out, H, HD, 0.125, wnp), s, iters)
    K.set_attention_x3_pipelined(True)
    r["split3_qkv_us"] = timeit(lambda: K.split3(qkv), s, iters)
    r["attn_sdpa_us"] = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(q, k, v), s, iters)
    for kname in [k_ for k_ in list(r) if k_.startswith("attn_") and k_.endswith("_us")
                  and not k_.startswith("split3")]:
        r[kname.replace("_us", "_tflops")] = round(attn_flops / r[kname] / 1e6, 2)


def modes_bench(a) -> int:
    """Whole-GPU throughput of each partition mode as the flagship bench runs it: every partition
    of the mode busy at once (its own CU-masked stream and graph-captured model replica), each
    running 8 x fraction inferences per round; inferences/s per GPU."""
    from walkai_nos_amd.bench_core import BenchConfig, Slot, slice_pin
    from walkai_nos_amd.models.workload.yolos import YolosSmall
    cfg = BenchConfig(lane_cus=a.lane_cus)
    template = YolosSmall()
    results = []
    for prof, n in (("spx_nps1", 1), ("dpx_nps1", 2), ("qpx_nps1", 4), ("cpx_nps1", 8)):
        if prof.split("_")[0] not in a.slices.split(","):
            continue
        n = min(n, a.partitions) if a.partitions else n
        slots = [Slot(slice_cus(prof, k, emulation=a.emulation), 0, cfg, template, seed=k,
                      pin=slice_pin(prof, k, a.emulation), split=a.lane_cus > 0) for k in range(n)]
        for sl in slots:
            sl.warm()
            sl.latency_ms.clear()
        torch.cuda.synchronize()
        work = 8 // n
        rounds = 6
        from walkai_nos_amd.bench_core import HwBusySampler
        sampler = HwBusySampler(0, period=0.02)
        sampler.start()
        t0 = time.perf_counter()
        if a.free_s > 0:
            # as the bench serves them: one thread per pod lane, each replaying its inference graph
            # and waiting for it before the next (the reference demo's loop), free-running
            done = free_running(slots, a.free_s)
        else:
            for _ in range(rounds):
                for sl in slots:
                    for _ in range(work):
                        sl.submit()
                for sl in slots:
                    sl.drain()
            done = rounds * work * n
        dt = time.perf_counter() - t0
        busy = sampler.stop()
        lat = [x for sl in slots for x in sl.latency_ms]
        r = {"mode": prof, "emulation": a.emulation, "partitions": n, "lanes_per_partition": len(slots[0].lanes),
             "serving": f"free-running threads, {a.free_s} s" if a.free_s > 0 else f"{rounds} lock-step rounds",
             "inf_per_s_per_gpu": round(done / dt, 1),
             "ms_per_round": round(1000 * dt / rounds, 2) if a.free_s <= 0 else None,
             "latency_ms_mean": round(sum(lat) / len(lat), 3) if lat else None,
             "hw_busy_pct": busy, **sampler.power_summary()}
        print(json.dumps(r), flush=True)
        results.append(r)
        for sl in slots:
            sl.close()
        torch.cuda.synchronize()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(results, f, indent=1)
    return 0


def free_running(slots, seconds: float) -> int:
    """Every lane of every slot on its own thread: replay, wait, replay ... until the deadline
    (``bench_core.NodeBench._serve_loops``); returns the inferences completed."""
    import threading
    deadline = time.perf_counter() + seconds
    counts = []

    def run(slot, lane):
        K.set_slice_cus(lane.n_cus)
        K.set_slice_pin(slot.pin)
        done = 0
        with torch.no_grad(), torch.cuda.stream(lane.stream):
            while time.perf_counter() < deadline:
                st = torch.cuda.Event(enable_timing=True)
                st.record(lane.stream)
                if lane.graph is not None:
                    lane.graph.replay()
                else:
                    lane.out = slot.model(lane.x)
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(lane.stream)
                ev.synchronize()
                slot.latency_ms.append(st.elapsed_time(ev))
                done += 1
        counts.append(done)
    threads = [threading.Thread(target=run, args=(sl, lane), daemon=True) for sl in slots for lane in sl.lanes]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    return sum(counts)


def model_bench(r, s, iters):
    """One whole YOLOS-small inference (batch 1) on this slice, graph-replayed."""
    from walkai_nos_amd.models.workload.yolos import DEMO_INPUT_HW, YolosSmall, demo_input
    with torch.cuda.stream(s):
        m = YolosSmall().cuda().eval()
        xin = demo_input(1, DEMO_INPUT_HW, "cuda")
    for mode in ("x3", "f32"):
        K.set_fp32_matmul(mode)
        with torch.no_grad():
            us = timeit(lambda: m(xin), s, iters)
        sfx = "" if mode == "x3" else "_f32"
        r[f"model{sfx}_ms"] = round(us / 1000.0, 3)
        r[f"model{sfx}_tflops"] = round(m.flops_per_inference() / us / 1e6, 2)
        r[f"model{sfx}_inf_per_s_per_gpu"] = round(1e6 / us * 256 / r["cus"], 1)
    K.set_fp32_matmul("x3")


def gemm_bench(r, x, h, w_qkv, w_o, w_1, w_2, b_ff, b_qkv, b_d, s, iters):
    lib = {"qkv": (x, w_qkv, b_qkv, None, 0, 2.0 * T * D * 3 * D),
           "proj": (x, w_o, b_d, x, G.EPI_RES, 2.0 * T * D * D),
           "fc1": (x, w_1, b_ff, None, G.EPI_GELU, 2.0 * T * D * FF),
           "fc2": (h, w_2, b_d, x, G.EPI_RES, 2.0 * T * FF * D)}
    for gname, (xa, wa, ba, ra, epi, fl) in lib.items():
        o = torch.empty(xa.shape[0], wa.shape[0], device="cuda")
        us = timeit(lambda: G._library(xa, wa, ba, ra, o, G.EPI_BIAS | epi), s, iters)
        r[f"gemm_{gname}_us"] = round(us, 1)
        r[f"gemm_{gname}_tflops"] = round(fl / us / 1e6, 2)
        # hand-written MFMA GEMM, every tile, same fused epilogue
        kw = {"bias": ba, "gelu": bool(epi & G.EPI_GELU), "residual": ra}
        for cfg in G.eligible(xa.shape[0], wa.shape[0], xa.shape[1]):
            us = timeit(lambda: G.gemm(xa, wa, tile=cfg, **kw), s, iters)
            tag = "x".join(map(str, G.TILES[cfg][:2])) + f"k{G.TILES[cfg][2]}" + ("sb" if cfg >= 7 else "")
            r[f"mfma_{gname}_{tag}_us"] = round(us, 1)
            r[f"mfma_{gname}_{tag}_tflops"] = round(fl / us / 1e6, 2)
        # x3 GEMM (fp32-accurate on the bf16 matrix cores), every tile; planes out where the model
        # feeds another x3 consumer (qkv, fc1), fp32 out where it feeds the residual stream
        xa3 = K.split3(xa)
        x3_out = gname in ("qkv", "fc1")
        for cfg in G.x3_eligible(wa.shape[0], wa.shape[1]):
            us = timeit(lambda: G.gemm_x3(xa3, wa, tile=cfg, out_f32=not x3_out, out_x3=x3_out, **kw), s, iters)
            bm, bn, nb, kind = G.X3_TILES[cfg]
            r[f"x3_{gname}_{bm}x{bn}{kind}b{nb}_us"] = round(us, 1)
            r[f"x3_{gname}_{bm}x{bn}{kind}b{nb}_tflops"] = round(fl / us / 1e6, 2)


if __name__ == "__main__":
    sys.exit(main())
