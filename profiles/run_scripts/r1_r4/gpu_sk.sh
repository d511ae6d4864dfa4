#!/bin/bash
# stream-K + fp8 gemm_lg: GEMM and fp8 GPU tests, then M = 1024 / 16384 timings of the stream-K candidates
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/sk
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pp_gpu.py tests/test_fp8_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 500 python3 scripts/bench_gemm_pp.py --m 1024,2048 --shapes qkv,o,gate_up,down --only "20:0,20:1,29:0,30:0,30:1,30:2,19:0,19:2,38:0" \
    --out $O/sk.jsonl > $O/sk.log 2>&1 || { tail -30 $O/sk.log; exit 1; }
grep "best" $O/sk.log
