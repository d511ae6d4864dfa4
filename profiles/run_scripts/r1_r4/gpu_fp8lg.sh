#!/bin/bash
# fp8 GPU tests (incl. gemm_lg's fp8 configs), then the W8A8 routing table at M = 256-16384 with them among the
# candidates (qplans written to gpurun_out/fp8lg/plan.json, merged with the current plan)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/fp8lg
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp8_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 900 python -u scripts/tune_gemm_pp.py --fp8 --ms 256,512,1024,2048,4096,16384 --rounds 3 \
  --merge project-chronos-distributed-behavioral-edr-ebpf-llm-_amd/ops/gemm_plan.json \
  --out-plan $O/plan.json --out-table $O/table.jsonl > $O/tune.log 2>&1 || { tail -30 $O/tune.log; exit 1; }
grep '"op"' $O/tune.log | cut -c1-260
