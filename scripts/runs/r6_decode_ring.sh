#!/bin/bash
# two-step K/V ring in the fused decode attention: correctness + wave-shape A/B (round 6)
set -o pipefail
mkdir -p gpurun_out/ring
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "decode or paged" tests/test_cascade_gpu.py > gpurun_out/ring/tests.log 2>&1 || { tail -30 gpurun_out/ring/tests.log; exit 1; }
tail -1 gpurun_out/ring/tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 0 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ring/prof_$r -o run --output-format csv -- python3 scripts/fw_bucket.py --rows 1024 --ctx 130 --knob decode_ring=$r > gpurun_out/ring/fw_$r.log 2>&1 || { tail -20 gpurun_out/ring/fw_$r.log; exit 1; }
  grep ms_per gpurun_out/ring/fw_$r.log
  f=$(find gpurun_out/ring/prof_$r -name "*kernel_stats.csv" | head -1)
  grep -E "paged_decode|Name" "$f" | cut -c1-200 > gpurun_out/ring/attn_$r.csv
  cat gpurun_out/ring/attn_$r.csv
  rm -rf gpurun_out/ring/prof_$r
done
