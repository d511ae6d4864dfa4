"""GPU idle time from a rocprofv3 kernel trace: where does the device wait for the host?

Reads the ``*kernel_trace.csv`` that ``rocprofv3 --kernel-trace --output-format csv`` writes, sorts dispatches by
start time, and sums the gaps between the end of one kernel and the start of the next (kernels of one stream do not
overlap).  Gaps above ``--min-us`` are grouped by the (previous kernel, next kernel) name pair, so a host stall shows
up as the pair it sits between.

    python scripts/kernel_gaps.py gpurun_out/trace --min-us 20
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os


def short(name: str) -> str:
    name = name.split("(")[0]
    return name[-60:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path", help="a kernel_trace.csv or a directory searched for one")
    ap.add_argument("--min-us", type=float, default=20.0)
    ap.add_argument("--max-us", type=float, default=0.0,
                    help="only gaps below this go into the pair table (e.g. 50: inter-kernel gaps inside a graph)")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--last-ms", type=float, default=0.0, help="analyse only the final window of this length")
    a = ap.parse_args()
    files = [a.path] if os.path.isfile(a.path) else glob.glob(os.path.join(a.path, "**", "*kernel_trace.csv"),
                                                              recursive=True)
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {a.path}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    if a.last_ms > 0:
        t_end = max(e for _, e, _ in rows)
        rows = [r for r in rows if r[0] >= t_end - a.last_ms * 1e6]
    busy = sum(e - s for s, e, _ in rows)
    span = rows[-1][1] - rows[0][0]
    gaps = collections.defaultdict(lambda: [0, 0.0])
    hist = collections.Counter()
    idle = 0.0
    end = rows[0][1]
    prev = rows[0][2]
    for s, e, n in rows[1:]:
        g = (s - end) / 1e3
        if g > 0:
            idle += g
            for b in (5, 20, 100, 1000, 10000, 1e12):
                if g < b:
                    hist[b] += 1
                    break
            if g >= a.min_us and (a.max_us <= 0 or g < a.max_us):
                k = (short(prev), short(n))
                gaps[k][0] += 1
                gaps[k][1] += g
        if e > end:
            end, prev = e, n
    print(f"{len(rows)} dispatches, span {span / 1e6:.1f} ms, kernel time {busy / 1e6:.1f} ms, "
          f"idle {idle / 1e3:.1f} ms ({100 * idle * 1e3 / span:.1f} % of span)")
    print("gap histogram (count of gaps below bound, us): "
          + ", ".join(f"<{int(b) if b < 1e12 else 'inf'}: {c}" for b, c in sorted(hist.items())))
    print(f"gaps >= {a.min_us} us by (previous kernel -> next kernel), largest total first:")
    for (p, n), (c, t) in sorted(gaps.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"  {t / 1e3:8.2f} ms  {c:6d} x  {t / c:6.2f} us  {p}  ->  {n}")


if __name__ == "__main__":
    main()
