"""Real-hardware report for one MI355X (run on the gpurun box).

Exercises every native component that can run without root: read-only amd-smi inventory and
partition modes, the MFMA/HBM slice probe on the whole device and under CU masks, the CU-mask ->
XCD placement census, a 1-rank RCCL commit barrier and the HBM-limit shim.  Writes
``gpurun_out/gpu_report.json``.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")


def main() -> int:
    os.makedirs(OUT, exist_ok=True)
    rep: dict = {"ts": time.time()}

    def save() -> None:
        with open(os.path.join(OUT, "gpu_report.json"), "w") as f:
            json.dump(rep, f, indent=1, default=str)

    # 1. amd-smi (read only)
    try:
        from walkai_nos_amd.device.amdsmi import NativeAmdSmi
        smi = NativeAmdSmi()
        gpus = smi.list_gpus()
        rep["amdsmi"] = [{"info": g.__dict__, "compute": smi.get_compute_partition(g.index),
                          "memory": smi.get_memory_partition(g.index), "activity": smi.activity(g.index),
                          "vram": smi.vram_usage(g.index), "processes": smi.process_count(g.index)} for g in gpus]
        try:
            smi.set_compute_partition(0, "CPX")
            rep["amdsmi_set"] = "unexpectedly succeeded (restoring SPX)"
            smi.set_compute_partition(0, "SPX")
        except Exception as e:  # expected: non-root
            rep["amdsmi_set"] = f"refused as expected: {e}"
    except Exception as e:
        rep["amdsmi_error"] = repr(e)
    save()
    print("amdsmi done", flush=True)

    from walkai_nos_amd.ops import probe
    ncu = probe.cu_count(0)
    rep["cu_count"] = ncu
    # 2. whole-device probes
    rep["whole"] = {}
    for d in ("bf16", "bf16_16x16", "fp32", "fp8"):
        r = probe.probe_mfma(d, iters=8192, reps=5)
        rep["whole"][d] = r.__dict__
        print("whole", d, round(r.tflops, 1), "TF", flush=True)
    rep["hbm_whole"] = probe.probe_hbm(nbytes=2 << 30)
    print("hbm", rep["hbm_whole"], flush=True)
    save()

    # 3. census of the default placement
    pl = probe.census(n_wg=4096)
    rep["census_whole"] = {"distinct_cus": probe.distinct_cus(pl), "xccs": sorted({p["xcc"] for p in pl})}
    save()

    # 4. CU-masked streams: contiguous bit ranges and strided masks
    rep["masked"] = []
    for kind, cus in [("first32", range(32)), ("first64", range(64)), ("first128", range(128)),
                      ("all256", range(ncu)), ("stride8_32", range(0, ncu, 8)), ("stride2_128", range(0, ncu, 2)),
                      ("block_32_63", range(32, 64))]:
        cus = list(cus)
        with probe.Stream(0, cus) as s:
            r = probe.probe_mfma("bf16", stream=s, n_cus=len(cus), iters=4096, reps=3)
            rf = probe.probe_mfma("fp32", stream=s, n_cus=len(cus), iters=2048, reps=3)
            pl = probe.census(stream=s, n_wg=max(256, 8 * len(cus)))
            ent = {"mask": kind, "n_cus": len(cus), "bf16_tflops": r.tflops, "bf16_tflops_per_cu": r.tflops_per_cu,
                   "fp32_tflops": rf.tflops, "census_distinct_cus": probe.distinct_cus(pl),
                   "census_xccs": sorted({p["xcc"] for p in pl}),
                   "xcc_hist": {str(x): sum(1 for p in pl if p["xcc"] == x) for x in sorted({p["xcc"] for p in pl})},
                   "stream_mask_words": s.cumask(8)}
            rep["masked"].append(ent)
            print("masked", kind, round(r.tflops, 1), ent["census_distinct_cus"], ent["census_xccs"], flush=True)
            save()

    # 5. RCCL 1-rank barrier
    try:
        from walkai_nos_amd.parallel.barrier import RcclBarrier
        t0 = time.perf_counter()
        b = RcclBarrier(1, 0, 0, {})
        t1 = time.perf_counter()
        ok = b.vote(True)
        t2 = time.perf_counter()
        lat = []
        for _ in range(20):
            t = time.perf_counter()
            b.vote(True)
            lat.append(time.perf_counter() - t)
        bad = b.vote(False)
        b.close()
        rep["rccl_barrier"] = {"ok": ok, "veto_detected": not bad, "init_s": t1 - t0, "first_vote_s": t2 - t1,
                               "vote_median_us": sorted(lat)[len(lat) // 2] * 1e6}
    except Exception as e:
        rep["rccl_barrier_error"] = repr(e)
    save()
    print("barrier", rep.get("rccl_barrier", rep.get("rccl_barrier_error")), flush=True)

    # 6. HBM limit shim in a child process
    shim = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "walkai_nos_amd", "_native",
                        "libnos_hbmlimit.so")
    code = ("import torch;"
            "f,t=torch.cuda.mem_get_info();print('meminfo',f,t);"
            "a=torch.empty(1<<30,dtype=torch.uint8,device='cuda');print('alloc1G ok');"
            "\ntry:\n b=torch.empty(3<<30,dtype=torch.uint8,device='cuda');print('alloc3G ok (LIMIT NOT ENFORCED)')\n"
            "except RuntimeError as e:\n print('alloc3G refused')\n")
    env = dict(os.environ, LD_PRELOAD=shim, NOS_HBM_LIMIT_BYTES=str(2 << 30))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    rep["hbm_limit_shim"] = {"rc": p.returncode, "stdout": p.stdout[-2000:], "stderr": p.stderr[-2000:]}
    save()
    print("shim", rep["hbm_limit_shim"]["stdout"], flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
