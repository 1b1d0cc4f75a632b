"""Per-kernel GPU time over the last part of a rocprofv3 kernel trace (the timed bench steps, not
warmup/autotune): python tools/trace_window.py <kernel_trace.csv> [--tail-frac 0.4]"""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))
    return name[:80]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--tail-frac", type=float, default=0.4)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    t0, t1 = rows[0][0], max(e for _, e, _ in rows)
    cut = t1 - a.tail_frac * (t1 - t0)
    agg = defaultdict(lambda: [0, 0])
    busy = []
    for s, e, n in rows:
        if s < cut:
            continue
        agg[short(n)][0] += e - s
        agg[short(n)][1] += 1
        busy.append((s, e))
    total = sum(v[0] for v in agg.values())
    # union of kernel intervals = time with at least one kernel running
    busy.sort()
    union, cs, ce = 0, None, None
    for s, e in busy:
        if cs is None or s > ce:
            if cs is not None:
                union += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        union += ce - cs
    win = t1 - cut
    print(f"window {win / 1e6:.1f} ms, kernel-busy union {union / 1e6:.1f} ms ({100 * union / win:.1f}%), "
          f"summed kernel time {total / 1e6:.1f} ms (concurrency {total / max(1, union):.2f})")
    for n, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        print(f"{100 * t / total:6.2f}%  {t / 1e6:9.2f} ms  {c:6d}  {n}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
