"""Per-kernel time per inference from a rocprofv3 kernel trace of tools/model_replay.py (the replays
after the 0.2 s marker gap): python tools/replay_stats.py <kernel_trace.csv> [--replays 40]"""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--replays", type=int, default=40)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as fh:
        for r in csv.DictReader(fh):
            g = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
            w = int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or 1)
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], g // max(w, 1)))
    rows.sort()
    gi = max(range(1, len(rows)), key=lambda i: rows[i][0] - rows[i - 1][1])
    win = rows[gi:]
    n = a.replays
    t0, t1 = win[0][0], max(e for _, e, _, _ in win)
    busy, cur = 0, None
    for s, e, _, _ in win:
        if cur is None or s > cur[1]:
            if cur is not None:
                busy += cur[1] - cur[0]
            cur = [s, e]
        else:
            cur[1] = max(cur[1], e)
    busy += cur[1] - cur[0]
    print(f"window {(t1 - t0) / 1e6 / n:.3f} ms per inference, {len(win) / n:.1f} kernels, busy {busy / (t1 - t0):.3f}")
    agg = defaultdict(lambda: [0, 0])
    for s, e, nm, g in win:
        k = re.sub(r"\(.*", "", nm.replace("(anonymous namespace)::", ""))[:70] + f" wg{g}"
        agg[k][0] += e - s
        agg[k][1] += 1
    tot = sum(v[0] for v in agg.values())
    for k, v in sorted(agg.items(), key=lambda x: -x[1][0]):
        print(f"{100 * v[0] / tot:6.2f}% {v[0] / 1e3 / n:8.1f} us/inf {v[1] / n:5.1f}x {v[0] / 1e3 / v[1]:7.1f} us  {k}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
