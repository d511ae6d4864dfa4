#!/bin/bash
# cfg 91 (HB slab loop on v_mfma_f32_32x32x16_bf16): tests + A/B against 88 / 89 (round 6)
set -o pipefail
mkdir -p gpurun_out/hb32
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_hb_gpu.py > gpurun_out/hb32/tests.log 2>&1 || { tail -30 gpurun_out/hb32/tests.log; exit 1; }
tail -1 gpurun_out/hb32/tests.log
timeout -k 10 500 python -u scripts/bench_gemm_cfgs.py --cfgs 88,89,92,93 --shapes sq8192,qkv16k,o16k,gu16k,down16k,gu1k,lm1k,qkv2k --cold 1 --out gpurun_out/hb32/sq_ab.jsonl > gpurun_out/hb32/sq_ab.log 2>&1 || { tail -20 gpurun_out/hb32/sq_ab.log; exit 1; }
timeout -k 10 300 python -u scripts/bench_gemm_cfgs.py --cfgs 88,89,92,93 --shapes gu1k,gu16k,qkv16k,lm1k --normp 1 --cold 1 --out gpurun_out/hb32/sq_ab_normp.jsonl > gpurun_out/hb32/sq_ab_normp.log 2>&1 || { tail -20 gpurun_out/hb32/sq_ab_normp.log; exit 1; }
