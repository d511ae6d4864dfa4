#!/bin/bash
# Single-stream latency A/B (fused vs unfused decode) + rocprofv3 kernel stats of each variant (stats kept, traces
# deleted so gpurun_out/ stays small).  Usage (gpurun): bash scripts/gpu_single_stream.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/scripts/single_stream.py --chains 12 --ab --out $R/gpurun_out/ss_ab.json \
    > $R/gpurun_out/ss_ab.log 2>&1 || exit $?
tail -1 $R/gpurun_out/ss_ab.log
for v in fused unfused; do  # profiled variants
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$v -o ss --output-format csv -- \
      python3 $R/scripts/single_stream.py --chains 6 --only $v > $R/gpurun_out/prof_$v.log 2>&1 || exit $?
  find $R/gpurun_out/prof_$v -name "*kernel_trace.csv" -delete
  find $R/gpurun_out/prof_$v -name "*.db" -delete
done
find $R/gpurun_out/prof_fused $R/gpurun_out/prof_unfused -type f | head
