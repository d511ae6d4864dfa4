#!/bin/bash
# Where does the GPU wait for the host in the headline wave?  rocprofv3 kernel trace of a short bench -> gap table by
# kernel pair (raw trace deleted), then bench A/B: sync harvest (default) vs --async-harvest.
# Usage (gpurun): bash scripts/gpu_gap_ab.sh
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gtrace -o bench -- \
    python3 bench.py --steps 1 --warmup 1 --single-stream 2 --closed-steps 0 > gpurun_out/gtrace.log 2>&1 || exit $?
T=$(find gpurun_out/gtrace -name "*kernel_trace.csv" | head -1)
python3 scripts/kernel_gaps.py "$T" --min-us 200 --top 20 > gpurun_out/gaps_big.txt 2>&1
python3 scripts/prof_summary.py "$T" > gpurun_out/gtrace_summary.txt 2>&1
find gpurun_out/gtrace -name "*.csv" -delete
head -30 gpurun_out/gaps_big.txt
for arm in sync async; do
  extra=""; [ $arm = async ] && extra="--async-harvest"
  timeout -k 10 400 python bench.py --steps 3 --warmup 1 --closed-steps 0 --single-stream 2 $extra > gpurun_out/ab_$arm.log 2>&1 || exit $?
  echo "== $arm"; grep -h "phase seconds" gpurun_out/ab_$arm.log | cut -c1-400; tail -1 gpurun_out/ab_$arm.log | cut -c1-420
done
