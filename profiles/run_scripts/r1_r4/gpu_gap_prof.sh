#!/bin/bash
# Kernel trace of the headline wave; inter-kernel gap table (gaps < 50 us: inside captured graphs) by kernel pair.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/gp -o gp --output-format csv -- \
    python3 bench.py --steps 1 --warmup 1 --single-stream 0 ${BENCH_ARGS:-} > gpurun_out/gp_bench.log 2>&1 || exit $?
T=$(find gpurun_out/gp -name "*kernel_trace.csv" | head -1)
python3 scripts/kernel_gaps.py "$T" --min-us 0 --max-us 50 --top 40 > gpurun_out/gp_gaps.txt 2>&1
python3 scripts/prof_summary.py "$T" > gpurun_out/gp_summary.txt 2>&1
find gpurun_out/gp -name "*kernel_trace.csv" -delete
cat gpurun_out/gp_gaps.txt | cut -c1-200
