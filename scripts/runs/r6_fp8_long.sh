#!/bin/bash
# 128k fp8-KV + fp8-weight TTFT before / after the F8HB re-measure of the W8A8 plan rows (round 6)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PLAN=project-chronos-distributed-behavioral-edr-ebpf-llm-_amd/ops/gemm_plan.json
timeout -k 10 300 python -u scripts/long_context.py --tokens 131000 --kv-dtype fp8 --weights fp8 --repeat 2 > gpurun_out/long_before.log 2>&1 || { tail -20 gpurun_out/long_before.log; exit 1; }
grep ttft gpurun_out/long_before.log | cut -c1-300
rm -f gpurun_out/fp8_hb_retune2.jsonl
timeout -k 10 600 python -u scripts/retune_fp8.py --out-plan gpurun_out/plan_fp8hb2.json --out-table gpurun_out/fp8_hb_retune2.jsonl > gpurun_out/fp8_retune2.log 2>&1 || { tail -20 gpurun_out/fp8_retune2.log; exit 1; }
cp gpurun_out/plan_fp8hb2.json $PLAN
timeout -k 10 300 python -u scripts/long_context.py --tokens 131000 --kv-dtype fp8 --weights fp8 --repeat 2 > gpurun_out/long_after.log 2>&1 || { tail -20 gpurun_out/long_after.log; exit 1; }
grep ttft gpurun_out/long_after.log | cut -c1-300
