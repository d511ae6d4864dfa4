#!/bin/bash
# GEMM tests, then the routing plan re-measured at M = 2-48 with the 32-row gemm_lg configs (72-75) among the candidates
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-tune6}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pp_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 1000 python -u scripts/tune_gemm_pp.py --models 8b,70b-tp8 --ms ${MS:-2,3,4,5,8,16,32,48} \
  --rounds 3 --merge project-chronos-distributed-behavioral-edr-ebpf-llm-_amd/ops/gemm_plan.json \
  --out-plan $O/plan.json --out-table $O/table.jsonl > $O/tune.log 2>&1 || { tail -30 $O/tune.log; exit 1; }
tail -2 $O/tune.log
