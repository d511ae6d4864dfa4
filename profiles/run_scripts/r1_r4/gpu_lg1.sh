#!/bin/bash
# gemm_lg bring-up: numerics (every config vs fp32) then the A/B against hipBLASLt and the ping-pong configs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/lg1
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_pp_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -3 $O/test.log
timeout -k 10 300 python -u scripts/bench_gemm_pp.py --m 8192 --shapes sq --only 12:1,0:1,4:1 --rounds 3 --out $O/sq.jsonl > $O/sq.log 2>&1 || { tail -30 $O/sq.log; exit 1; }
tail -3 $O/sq.log
timeout -k 10 400 python -u scripts/bench_gemm_pp.py --m 1024,16384 --shapes gate_up,qkv,o,down --only 12:1,13:1,14:1,15:1,12:2,12:4,0:1,4:1 --rounds 3 --out $O/m.jsonl > $O/m.log 2>&1 || { tail -30 $O/m.log; exit 1; }
grep -E "best|M=" $O/m.log | tail -20
