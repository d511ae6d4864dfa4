#!/bin/bash
# Mid-M gemm_lg configs (32-35): GEMM GPU tests, then M = 64 / 128 / 256 on the 8B projection shapes against
# hipBLASLt and the configs the plan uses there.  Usage (gpurun): bash scripts/gpu_midm.sh
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out/midm
timeout -k 10 300 python -u -m pytest tests/test_gemm_pp_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/midm/test.log 2>&1 || { tail -30 gpurun_out/midm/test.log; exit 1; }
tail -2 gpurun_out/midm/test.log
ONLY=${ONLY:-"32:1,32:2,32:4,32:8,34:2,34:4,34:8,33:1,33:2,33:4,33:8,35:1,35:2,35:4,15:1,15:2,15:4,19:2,19:4,31:2,31:4,3:1"}
timeout -k 10 600 python3 scripts/bench_gemm_pp.py --m 64,128,256 --shapes qkv,o,gate_up,down --only "$ONLY" \
    --out gpurun_out/midm/mid.jsonl > gpurun_out/midm/mid.log 2>&1 || { tail -30 gpurun_out/midm/mid.log; exit 1; }
tail -40 gpurun_out/midm/mid.log
