#!/bin/bash
# fp8 config 4 (F8HB) correctness + W8A8 plan re-measure (round 6)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
: timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp8_gpu.py -k "qgemm_lg" > gpurun_out/fp8hb_tests.log 2>&1 || { tail -30 gpurun_out/fp8hb_tests.log; exit 1; }
tail -3 gpurun_out/fp8hb_tests.log
timeout -k 10 600 python -u scripts/retune_fp8.py --out-plan gpurun_out/plan_fp8hb.json --out-table gpurun_out/fp8_hb_retune.jsonl > gpurun_out/fp8_retune.log 2>&1
