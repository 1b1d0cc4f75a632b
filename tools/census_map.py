"""Map CU-mask bits to physical CUs and check how slices of k rows spread over shader engines.

For each row r (mask bits 8r..8r+7) a census kernel records (XCC, SE, SH, CU) of every workgroup;
then for slices of k contiguous rows the MFMA probe measures the per-CU rate, to see whether some
slice shapes leave CUs idle (SE imbalance) or escape their mask.

    python tools/census_map.py [--out gpurun_out/census_map.json]
"""
import json
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from walkai_nos_amd.ops import probe as P  # noqa: E402


def main() -> int:
    rows = {}
    for r in range(32):
        with P.Stream(0, list(range(8 * r, 8 * r + 8))) as s:
            pl = P.census(0, s, n_wg=64, spin=2000)
        phys = sorted({(p["xcc"], p["se"], p["sh"], p["cu"]) for p in pl})
        rows[r] = phys
        print(json.dumps({"row": r, "n_phys": len(phys), "phys": phys}), flush=True)
    shapes = []
    for k in (1, 2, 3, 4, 5, 6, 8, 10, 12, 16, 32):
        cus = list(range(8 * k))
        with P.Stream(0, None if k == 32 else cus) as s:
            pl = P.census(0, s, n_wg=64 * k, spin=2000)
            f32 = P.probe_mfma("fp32", 0, s, iters=2048, reps=2)
        per_cu = Counter((p["xcc"], p["se"], p["sh"], p["cu"]) for p in pl)
        se = Counter((p["xcc"], p["se"]) for p in pl)
        row = {"rows": k, "mask_cus": 8 * k, "distinct_cus": len(per_cu), "wg_per_cu_min": min(per_cu.values()),
               "wg_per_cu_max": max(per_cu.values()), "ses_used": len(se), "fp32_tflops": round(f32.tflops, 2),
               "tflops_per_cu": round(f32.tflops / (8 * k), 4), "mhz": round(f32.mhz)}
        print(json.dumps(row), flush=True)
        shapes.append(row)
    path = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else "gpurun_out/census_map.json"
    os.makedirs(os.path.dirname(path), exist_ok=True)
    json.dump({"rows": {str(k): v for k, v in rows.items()}, "shapes": shapes}, open(path, "w"), indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
