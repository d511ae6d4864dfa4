#!/bin/bash
# r5: plan rows for Llama-3-70B TP = 1 (one GPU) at the decode buckets of a 256-stream run, then its bench, old vs new
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5t70
mkdir -p $O
timeout -k 10 1000 python -u scripts/tune_gemm_pp.py --models 70b --ms 2,3,4,5,8,16,32,48,64,128,256,512 --merge project-chronos-distributed-behavioral-edr-ebpf-llm-_amd/ops/gemm_plan.json --out-plan $O/plan.json --out-table $O/table.jsonl > $O/tune.log 2>&1 || { tail -30 $O/tune.log; exit 1; }
tail -3 $O/tune.log
