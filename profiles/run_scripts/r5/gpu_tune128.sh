#!/bin/bash
# r5: mid-M (M = 128 / 256) plan rows with the wide-W-row configs + split-K in the candidate set
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5tune128
mkdir -p $O
timeout -k 10 900 python -u scripts/tune_gemm_pp.py --models 8b,70b-tp8 --ms ${MS:-128,256} --merge project-chronos-distributed-behavioral-edr-ebpf-llm-_amd/ops/gemm_plan.json --out-plan $O/plan.json --out-table $O/table.jsonl > $O/tune.log 2>&1 || { tail -30 $O/tune.log; exit 1; }
tail -30 $O/tune.log
