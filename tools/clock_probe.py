"""Core clock under MFMA load per slice size: is the whole-GPU rate power/clock-limited?

    python tools/clock_probe.py [--out gpurun_out/clock.json]
"""
import faulthandler
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from walkai_nos_amd.ops import probe as P  # noqa: E402


def main() -> int:
    faulthandler.dump_traceback_later(50, exit=False)
    t0 = time.time()
    out = []
    for n in (256, 128, 64, 32, 8):
        cus = None if n == 256 else list(range(n))
        with P.Stream(0, cus) as s:
            for dt in ("fp32", "bf16", "bf16_16x16", "fp8", "fp8_scaled"):
                r = P.probe_mfma(dt, 0, s, iters=2048 if dt == "fp32" else 4096, reps=3)
                row = {"t": round(time.time() - t0, 2), "cus": n, "dtype": dt, "tflops": round(r.tflops, 1), "mhz": round(r.mhz, 0),
                       "pct_of_clock_peak": round(r.pct_of_clock_peak, 1), "ms": round(r.ms, 3)}
                print(json.dumps(row), flush=True)
                out.append(row)
    for nbytes in (1 << 28, 1 << 30, 4 << 30):
        for mode in ("stride", "slab_nt", "slab"):
          for wg_per_cu in (2, 4, 8):
            h = P.probe_hbm(0, None, nbytes=nbytes, n_wg=256 * wg_per_cu, reps=5, mode=mode)
            row = {"t": round(time.time() - t0, 2), "hbm_copy_bytes": nbytes, "mode": mode, "wg_per_cu": wg_per_cu,
                   "gbps": round(h["gbps"], 0), "ms": round(h["ms"], 3)}
            print(json.dumps(row), flush=True)
            out.append(row)
    path = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else "gpurun_out/clock.json"
    os.makedirs(os.path.dirname(path), exist_ok=True)
    json.dump(out, open(path, "w"), indent=1)
    print(f"done in {time.time() - t0:.1f}s", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
