"""Per-kernel averages of rocprofv3 --pmc counter CSVs under a directory (the kernels whose name matches --match),
one row per counter.  python scripts/pmc_table.py gpurun_out/pmc_gate_up_0_1 [--match gemm_pp|Cijk]"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    for sub in sorted(os.listdir(a.root)):
        fs = glob.glob(os.path.join(a.root, sub, "**", "*counter_collection.csv"), recursive=True)
        if not fs:
            continue
        agg = collections.defaultdict(list)
        name = ""
        for f in fs:
            for r in csv.DictReader(open(f)):
                n = r.get("Kernel_Name", "")
                if a.match and not any(m in n for m in a.match.split("|")):
                    continue
                if "gemm" not in n and "Cijk" not in n:
                    continue
                name = n[:70]
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        print(f"{sub}: {name}")
        for k, v in sorted(agg.items()):
            print(f"   {k:28s} {sum(v) / len(v):16.1f}")


if __name__ == "__main__":
    main()
