#!/bin/bash
# rocprofv3 kernel trace of a short headline bench, kept (gzipped) for offline gap analysis.
# Usage (gpurun): bash scripts/trace_keep.sh [extra bench args]
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/ktrace
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ktrace -o bench -- \
    python3 bench.py --steps 1 --warmup 1 --single-stream 2 --closed-steps 0 "$@" > gpurun_out/ktrace.log 2>&1 || exit $?
T=$(find gpurun_out/ktrace -name "*kernel_trace.csv" | head -1)
python3 - "$T" <<'PY'
import csv, sys, gzip
rows = list(csv.DictReader(open(sys.argv[1])))
with gzip.open("gpurun_out/ktrace_min.csv.gz", "wt") as f:
    w = csv.writer(f)
    w.writerow(["name", "start", "end", "grid", "wg"])
    for r in rows:
        w.writerow([r["Kernel_Name"][:90], r["Start_Timestamp"], r["End_Timestamp"], r["Grid_Size_X"], r["Workgroup_Size_X"]])
PY
find gpurun_out/ktrace -name "*.csv" -delete
ls -la gpurun_out/ktrace_min.csv.gz
