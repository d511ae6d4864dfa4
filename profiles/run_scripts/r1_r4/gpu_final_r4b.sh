#!/bin/bash
# Round-4 closing evidence on one box: GPU suite, smoke, default bench, then a kernel trace of a short bench
# summarised by prof_summary.py / wave_breakdown.py (raw trace deleted)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/final4b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | cut -c1-120
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- \
    python3 bench.py --steps 1 --warmup 1 --single-stream 2 --closed-steps 0 > $O/prof_bench.log 2>&1 || exit $?
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
S=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$T" > $O/prof_summary.txt 2>&1
python3 - "$T" <<'PY'
import csv, sys, gzip
rows = list(csv.DictReader(open(sys.argv[1])))
with gzip.open("gpurun_out/final4b/ktrace_min.csv.gz", "wt") as f:
    w = csv.writer(f)
    w.writerow(["name", "start", "end", "grid", "wg"])
    for r in rows:
        w.writerow([r["Kernel_Name"][:90], r["Start_Timestamp"], r["End_Timestamp"], r["Grid_Size_X"], r["Workgroup_Size_X"]])
PY
python3 scripts/wave_breakdown.py gpurun_out/final4b/ktrace_min.csv.gz > $O/wave_breakdown.txt 2>&1
cp "$S" $O/kernel_stats.csv
find $O/prof -name "*.csv" -delete
head -3 $O/wave_breakdown.txt
