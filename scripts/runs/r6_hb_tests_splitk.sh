#!/bin/bash
# r6: HB GPU tests + plan-row tests, then split-K HB at the decode-wave shapes vs the routed configs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6t
mkdir -p $O
timeout -k 10 900 python -u -m pytest -s tests/test_gemm_hb_gpu.py tests/test_gemm_plan_gpu.py tests/test_prefill_fp8_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log; cp gpurun_out/prefill_fp8_model_drift.json $O/ 2>/dev/null; grep fp8_cache_rel $O/pytest.log | head -2
timeout -k 10 300 python -u scripts/bench_gemm_cfgs.py --cfgs 88,88:2,88:4,30:2,19,76,20,89 \
  --shapes down1k,o1k,qkv1k,gu1k,gu768,down2k,o2k --out $O/splitk.jsonl > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log
