"""Summarise a rocprofv3 kernel trace of bench.py: per-kernel-class time split by phase (prefill / decode),
decode step time and GEMM shapes (grid sizes).  Usage: python scripts/prof_summary.py <kernel_trace.csv>"""
import csv
import collections
import sys


def short(n):
    if n.startswith("Cijk") or n.startswith("Custom_Cijk"):
        return "gemm:" + n.split("_MT")[1].split("_")[0] if "_MT" in n else "gemm"
    n = n.replace("void ", "")
    return n.replace("(anonymous namespace)::", "").split("(")[0][:60]


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# phase split: embedding kernels mark forward starts; a forward with grid.x == slots is decode (batch) — we key on
# the embedding's grid size: decode forwards have T == bucket, prefill forwards have T = tokens in the chunk.
fw = []
cur = None
for r in rows:
    nm = r["Kernel_Name"]
    if "embedding_kernel" in nm:
        cur = dict(T=int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), kernels=[])
        fw.append(cur)
    if cur is not None:
        cur["kernels"].append(r)
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # noqa: E731
# device idle: gaps between consecutive kernels (host-side scheduling / sync / python overhead)
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
busy = sum(dur(r) for r in rows)
gaps = []
for a, b in zip(rows, rows[1:]):
    g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
    if g > 0:
        gaps.append((g, a["Kernel_Name"][:50], b["Kernel_Name"][:50]))
big = [g for g in gaps if g[0] > 50]
print(f"trace span {span/1e3:.1f} ms, kernel busy {busy/1e3:.1f} ms ({100*busy/span:.1f}%), "
      f"gaps>50us: {len(big)} totalling {sum(g[0] for g in big)/1e3:.1f} ms")
for g in sorted(big, reverse=True)[:8]:
    print(f"   gap {g[0]/1e3:8.2f} ms after {g[1]} -> {g[2]}")
byT = collections.defaultdict(list)
for f in fw:
    byT[f["T"]].append(f)
print("forwards by token count T: count, mean GPU-busy us, mean wall us (first->last kernel)")
for T in sorted(byT):
    fs = byT[T]
    busy = [sum(dur(k) for k in f["kernels"]) for f in fs]
    wall = [(int(f["kernels"][-1]["End_Timestamp"]) - int(f["kernels"][0]["Start_Timestamp"])) / 1e3 for f in fs]
    print(f"  T={T:6d} n={len(fs):4d} busy={sum(busy)/len(busy):9.1f} wall={sum(wall)/len(wall):9.1f}")
    cls = collections.defaultdict(float)
    for f in fs:
        for k in f["kernels"]:
            cls[short(k["Kernel_Name"])] += dur(k)
    for c, t in sorted(cls.items(), key=lambda x: -x[1])[:12]:
        print(f"        {t/len(fs):9.1f} us  {c}")
