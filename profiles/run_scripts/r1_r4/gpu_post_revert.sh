#!/bin/bash
# after reverting stream-K: GEMM + fp8 GPU tests and the 8192^3 / M = 1024 timings of the routed large-M configs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/postrev
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pp_gpu.py tests/test_fp8_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python3 scripts/bench_gemm_pp.py --m 8192 --shapes sq --only "20:1" --out $O/sq.jsonl > $O/sq.log 2>&1 || { tail -20 $O/sq.log; exit 1; }
grep '"cand"' $O/sq.log | cut -c1-160
