#!/bin/bash
# F8HB after the LDS-parked scales + batched staged stores: correctness (fp8 + bf16 HB) and the fixed-cost fit
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp8_gpu.py tests/test_gemm_hb_gpu.py -k "qgemm_lg or hb" > gpurun_out/fp8hb2_tests.log 2>&1 || { tail -30 gpurun_out/fp8hb2_tests.log; exit 1; }
tail -2 gpurun_out/fp8hb2_tests.log
timeout -k 10 300 python -u scripts/f8hb_fixed_cost.py --out gpurun_out/f8hb_fixed_cost2.jsonl > gpurun_out/f8hb_fixed_cost2.log 2>&1
grep kernel gpurun_out/f8hb_fixed_cost2.log
