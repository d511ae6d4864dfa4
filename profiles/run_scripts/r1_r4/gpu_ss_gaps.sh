#!/bin/bash
# Kernel trace of single-stream verdicts; inter-kernel gaps inside the captured decode graph by kernel pair.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ss -o ss --output-format csv -- \
    python3 scripts/single_stream.py --chains 6 > gpurun_out/ss_run.log 2>&1 || exit $?
T=$(find gpurun_out/ss -name "*kernel_trace.csv" | head -1)
python3 scripts/kernel_gaps.py "$T" --min-us 0 --max-us 50 --top 30 --last-ms 400 > gpurun_out/ss_gaps.txt 2>&1
python3 scripts/prof_summary.py "$T" > gpurun_out/ss_summary.txt 2>&1
find gpurun_out/ss -name "*kernel_trace.csv" -delete
cut -c1-220 gpurun_out/ss_gaps.txt
