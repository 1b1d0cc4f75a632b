"""HBM copy probe sweep: buffer size x kernel variant x workgroups per CU (csrc/probe.hip).

    python tools/hbm_sweep.py --out gpurun_out/hbm.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from walkai_nos_amd.ops import probe as P  # noqa: E402


def main() -> int:
    out = []
    for nbytes in (1 << 30, 4 << 30, 16 << 30):
        for mode in P.HBM_MODES:
            for wg_per_cu in (1, 2, 4):
                h = P.probe_hbm(0, None, nbytes=nbytes, n_wg=256 * wg_per_cu, reps=5, mode=mode)
                row = {"bytes": nbytes, "mode": mode, "wg_per_cu": wg_per_cu, "gbps": round(h["gbps"], 0),
                       "ms": round(h["ms"], 3)}
                print(json.dumps(row), flush=True)
                out.append(row)
    best = max(out, key=lambda r: r["gbps"])
    print(json.dumps({"best": best}), flush=True)
    path = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else "gpurun_out/hbm.json"
    os.makedirs(os.path.dirname(path), exist_ok=True)
    json.dump(out, open(path, "w"), indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
