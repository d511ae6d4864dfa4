#!/bin/bash
# round-6 validation: the whole GPU suite + smoke, then the cfg 94 A/B (square order + set-0 reads from MFMA 94)
set -o pipefail
mkdir -p gpurun_out/final
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/gpu_suite.log 2>&1 || { tail -30 gpurun_out/final/gpu_suite.log; exit 1; }
tail -2 gpurun_out/final/gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -2 gpurun_out/final/smoke.log
timeout -k 10 300 python -u scripts/bench_gemm_cfgs.py --cfgs 88,92,94 --shapes sq8192,qkv16k,gu16k,down16k,gu1k,lm1k --cold 1 --out gpurun_out/final/ab94.jsonl > gpurun_out/final/ab94.log 2>&1 || { tail -20 gpurun_out/final/ab94.log; exit 1; }
timeout -k 10 200 python -u scripts/bench_gemm_cfgs.py --cfgs 89,92,93,94 --shapes gu1k,lm1k --normp 1 --cold 1 --out gpurun_out/final/ab94_normp.jsonl > gpurun_out/final/ab94_normp.log 2>&1 || { tail -20 gpurun_out/final/ab94_normp.log; exit 1; }
