"""Per-forward breakdown of a rocprofv3 kernel trace: every forward starts at its embedding kernel; for the forwards of
one token count T (default 1: decode), the mean GPU-busy and wall time per forward, the device-idle part, and the
mean time per kernel — the decode-only view that kernel_stats (which mixes prefill in) cannot give.

    python scripts/decode_tail.py gpurun_out/x/prof/run_kernel_trace.csv [--T 1] [--last 40]
"""
import argparse
import collections
import csv
import gzip


def load(path):
    rows = list(csv.DictReader(gzip.open(path, "rt") if path.endswith(".gz") else open(path)))
    out = []
    for r in rows:
        name = r.get("Kernel_Name") or r.get("name")
        s = int(r.get("Start_Timestamp") or r.get("start"))
        e = int(r.get("End_Timestamp") or r.get("end"))
        gx = int(r.get("Grid_Size_X") or r.get("grid") or 0)
        wx = int(r.get("Workgroup_Size_X") or r.get("wg") or 1)
        out.append((s, e, name, gx // max(wx, 1)))
    out.sort()
    return out


def short(n):
    n = n.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("chronos::", "")
    return n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--T", type=int, default=1)
    ap.add_argument("--last", type=int, default=40, help="use the last N forwards of that T")
    a = ap.parse_args()
    rows = load(a.trace)
    starts = [i for i, r in enumerate(rows) if "embedding_kernel" in r[2]]
    fws = []
    for k, i in enumerate(starts):
        j = starts[k + 1] if k + 1 < len(starts) else len(rows)
        fws.append((rows[i][3], i, j))
    # the region after the last large forward (prefill chunk): every forward kind in it, with its wall time
    big = [k for k, f in enumerate(fws) if f[0] > 64]
    if big and big[-1] + 1 < len(fws):
        tail = fws[big[-1] + 1:]
        t0, t1 = rows[tail[0][1]][0], rows[tail[-1][2] - 1][1]
        kinds = collections.Counter(f[0] for f in tail)
        print(f"after the last prefill forward: {len(tail)} forwards {dict(sorted(kinds.items()))}, "
              f"{(t1 - t0) / 1e6:.1f} ms wall")
    sel = [f for f in fws if f[0] == a.T][-a.last:]
    if not sel:
        print("no forwards with T =", a.T, "; T seen:", collections.Counter(f[0] for f in fws).most_common(10))
        return
    per = collections.Counter()
    calls = collections.Counter()
    busy = wall = 0.0
    for _, i, j in sel:
        for s, e, n, _ in rows[i:j]:
            per[short(n)] += (e - s) / 1e3
            calls[short(n)] += 1
            busy += (e - s) / 1e3
        wall += (rows[j][0] if j < len(rows) else rows[j - 1][1]) - rows[i][0]
    n = len(sel)
    wall /= 1e3
    print(f"{n} forwards at T={a.T}: wall {wall / n:.1f} us, GPU busy {busy / n:.1f} us "
          f"({100 * busy / wall:.1f} %), kernels per forward {sum(calls.values()) / n:.0f}")
    for k, v in per.most_common(25):
        print(f"{v / n:9.1f} us/fw {calls[k] / n:6.1f} calls/fw {v / calls[k]:8.1f} us/call  {k}")


if __name__ == "__main__":
    main()
