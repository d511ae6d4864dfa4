#!/bin/bash
# all gemm tests, then the routing plan re-measured at M >= 128 with the gemm_lg family among the candidates
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/tune4
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pp_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 1300 python -u scripts/tune_gemm_pp.py --models 8b,70b-tp8 --ms 128,256,512,768,1024,2048,4096,8192,16384 \
  --rounds 3 --merge project-chronos-distributed-behavioral-edr-ebpf-llm-_amd/ops/gemm_plan.json \
  --out-plan $O/plan.json --out-table $O/table.jsonl > $O/tune.log 2>&1 || { tail -30 $O/tune.log; exit 1; }
tail -2 $O/tune.log
