#!/bin/bash
# HB split-K after the batched slab reduction (own slice from registers): tests + decode-shape A/B; then the 128k
# fp8 kernel statistics (round 6)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_hb_gpu.py > gpurun_out/hb_splitk2_tests.log 2>&1 || { tail -30 gpurun_out/hb_splitk2_tests.log; exit 1; }
tail -1 gpurun_out/hb_splitk2_tests.log
timeout -k 10 400 python -u scripts/bench_gemm_cfgs.py --cfgs 88,88:2,88:4,89:2,89:4,30:2,19,76 --shapes o1k,down1k,qkv1k,o2k,down2k --cold 1 --out gpurun_out/hb_splitk2.jsonl > gpurun_out/hb_splitk2.log 2>&1 || { tail -20 gpurun_out/hb_splitk2.log; exit 1; }
bash scripts/runs/r6_fp8_long_prof.sh
