"""GPU time of the TIMED wave of a `bench.py --steps 1 --warmup 1` kernel trace, split by forward kind (decode bucket
T, prefill chunks) and kernel class, plus the device-idle gaps inside the region (host stalls).

    python scripts/wave_breakdown.py gpurun_out/ktrace_min.csv.gz   (written by scripts/trace_keep.sh)
"""
import collections
import csv
import gzip
import sys


def cls(n):
    if "Cijk" in n:
        return "gemm_hipblaslt"
    if "gemm_pp" in n or "gemm_lg" in n or "skinny" in n:
        return "gemm_own"
    if "gemv" in n:
        return "gemv_own"
    return n.split("(")[0].replace("void ", "").replace("chronos::", "")[:40]


def main(path):
    rows = list(csv.DictReader(gzip.open(path, "rt") if path.endswith(".gz") else open(path)))
    for r in rows:
        if "Kernel_Name" in r:  # a raw rocprofv3 kernel_trace.csv
            r.update(name=r["Kernel_Name"], start=r["Start_Timestamp"], end=r["End_Timestamp"],
                     grid=r["Grid_Size_X"], wg=r["Workgroup_Size_X"])
        r["s"], r["e"] = int(r["start"]), int(r["end"])
    rows.sort(key=lambda r: r["s"])
    emb = [i for i, r in enumerate(rows) if "embedding_kernel" in r["name"]]
    T = lambda i: int(rows[i]["grid"]) // int(rows[i]["wg"])  # noqa: E731
    pre = [i for i in emb if T(i) > 2048]
    # the second wave starts at its first full prefill forward (the first wave's prefills come first)
    half = [i for i in pre if i > pre[0] + 1000] or pre
    start = half[0] - 1
    end = next((i for i in emb if i > start and T(i) == 1), len(rows) - 1)
    # the wave ends at its last forward: a device-idle gap > 50 ms before the single-stream phase is the host's
    # post-wave bookkeeping (outside bench.py's timed steps)
    end = next((j + 1 for j in range(start, end) if rows[j + 1]["s"] - rows[j]["e"] > 50_000_000), end)
    span = (rows[end - 1]["e"] - rows[start]["s"]) / 1e3
    busy = sum(rows[j]["e"] - rows[j]["s"] for j in range(start, end)) / 1e3
    print(f"timed wave region: span {span / 1e3:.1f} ms, GPU busy {busy / 1e3:.1f} ms ({100 * busy / span:.1f} %)")
    by = collections.defaultdict(collections.Counter)
    nfw = collections.Counter()
    cur = None
    for i in range(start, end):
        if "embedding_kernel" in rows[i]["name"]:
            cur = "prefill" if T(i) > 1024 else f"decode T={T(i)}"
            nfw[cur] += 1
        by[cur or "other"][cls(rows[i]["name"])] += (rows[i]["e"] - rows[i]["s"]) / 1e3
    for k, c in sorted(by.items(), key=lambda x: -sum(x[1].values())):
        tot = sum(c.values())
        print(f"{k:14s} {nfw[k]:3d} fw {tot / 1e3:8.1f} ms ({100 * tot / busy:4.1f} %): "
              + ", ".join(f"{n} {v / 1e3:.1f}" for n, v in c.most_common(6)))
    allc = collections.Counter()
    for c in by.values():
        allc.update(c)
    print("by kernel class over the wave: " + ", ".join(f"{n} {100 * v / busy:.1f} %" for n, v in allc.most_common(8)))
    gaps = collections.defaultdict(lambda: [0, 0.0])
    for j in range(start, end - 1):
        g = (rows[j + 1]["s"] - rows[j]["e"]) / 1e3
        if g > 20:
            k = (rows[j]["name"].split("(")[0][-40:], rows[j + 1]["name"].split("(")[0][-40:])
            gaps[k][0] += 1
            gaps[k][1] += g
    print("device-idle gaps > 20 us inside the region (largest total first):")
    for k, v in sorted(gaps.items(), key=lambda x: -x[1][1])[:8]:
        print(f"  {v[1] / 1e3:8.2f} ms {v[0]:4d} x {v[1] / v[0]:9.1f} us  {k[0]} -> {k[1]}")


if __name__ == "__main__":
    main(sys.argv[1])
