#!/bin/bash
# single-stream kernel trace (6 chains): where the device idles around jump-forward forwards
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/sstrace
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o ss -- \
    python3 scripts/single_stream.py --chains 6 --only fused > $O/ss.log 2>&1 || { tail -20 $O/ss.log; exit 1; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 - "$T" <<'PY'
import csv, sys, gzip
rows = list(csv.DictReader(open(sys.argv[1])))
with gzip.open("gpurun_out/sstrace/ktrace.csv.gz", "wt") as f:
    w = csv.writer(f)
    w.writerow(["name", "start", "end", "grid", "wg"])
    for r in rows:
        w.writerow([r["Kernel_Name"][:80], r["Start_Timestamp"], r["End_Timestamp"], r["Grid_Size_X"], r["Workgroup_Size_X"]])
PY
find $O/prof -name "*.csv" -delete
tail -2 $O/ss.log
