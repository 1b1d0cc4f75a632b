"""Does a CU mask confined to ONE XCD keep a queue's workgroups on that XCD? For XCD x the mask
holds bits {8r + x}; a census kernel records where every workgroup ran, and the MFMA probe the
rate. python tools/xcd_mask_probe.py [--out gpurun_out/xcd_mask.json]"""
import json
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from walkai_nos_amd.ops import probe as P  # noqa: E402


def main() -> int:
    out = []
    for name, bits in (("xcd0", [8 * r for r in range(32)]), ("xcd3", [8 * r + 3 for r in range(32)]),
                       ("xcd0+1", [8 * r + x for r in range(32) for x in (0, 1)]),
                       ("rows0-3", list(range(32)))):
        with P.Stream(0, bits) as s:
            pl = P.census(0, s, n_wg=256, spin=2000)
            f32 = P.probe_mfma("fp32", 0, s, iters=2048, reps=2)
        xcc = Counter(p["xcc"] for p in pl)
        cus = {(p["xcc"], p["se"], p["sh"], p["cu"]) for p in pl}
        r = {"mask": name, "mask_bits": len(bits), "workgroups_per_xcc": dict(sorted(xcc.items())),
             "distinct_cus": len(cus), "fp32_tflops": round(f32.tflops, 2)}
        print(json.dumps(r), flush=True)
        out.append(r)
    path = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else "gpurun_out/xcd_mask.json"
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
