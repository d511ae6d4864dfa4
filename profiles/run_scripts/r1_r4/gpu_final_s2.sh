#!/bin/bash
# Session-end evidence: the driver's default bench (python bench.py), then a rocprofv3 kernel trace + stats of a short
# bench summarised by prof_summary.py / wave_breakdown.py (raw trace deleted).
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/fin
timeout -k 10 600 python bench.py > gpurun_out/fin/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/fin/bench_default.log | cut -c1-1500
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/fin/prof -o bench --output-format csv -- \
    python3 bench.py --steps 1 --warmup 1 --single-stream 2 --closed-steps 0 > gpurun_out/fin/prof_bench.log 2>&1 || exit $?
T=$(find gpurun_out/fin/prof -name "*kernel_trace.csv" | head -1)
S=$(find gpurun_out/fin/prof -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$T" > gpurun_out/fin/prof_summary.txt 2>&1
python3 - "$T" <<'PY'
import csv, sys, gzip
rows = list(csv.DictReader(open(sys.argv[1])))
with gzip.open("gpurun_out/fin/ktrace_min.csv.gz", "wt") as f:
    w = csv.writer(f)
    w.writerow(["name", "start", "end", "grid", "wg"])
    for r in rows:
        w.writerow([r["Kernel_Name"][:90], r["Start_Timestamp"], r["End_Timestamp"], r["Grid_Size_X"], r["Workgroup_Size_X"]])
PY
python3 scripts/wave_breakdown.py gpurun_out/fin/ktrace_min.csv.gz > gpurun_out/fin/wave_breakdown.txt 2>&1
cp "$S" gpurun_out/fin/kernel_stats.csv
find gpurun_out/fin/prof -name "*.csv" -delete
head -12 gpurun_out/fin/wave_breakdown.txt
