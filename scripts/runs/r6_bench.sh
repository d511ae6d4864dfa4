#!/bin/bash
# r6: default headline bench (the driver's N=1 run), then a kept kernel trace of a 1-step wave for the breakdown
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${R6OUT:-r6bench}
mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench.json
cut -c1-1200 $O/bench.json
bash scripts/trace_keep.sh > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
python3 scripts/wave_breakdown.py gpurun_out/ktrace_min.csv.gz > $O/wave_breakdown.txt
head -12 $O/wave_breakdown.txt
