#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/lg6
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pp_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
timeout -k 10 300 python -u scripts/bench_gemm_pp.py --m 8192 --shapes sq --only 20:1,24:1,61:1,54:1 --rounds 3 --out $O/sq.jsonl > $O/sq.log 2>&1 || { tail -30 $O/sq.log; exit 1; }
timeout -k 10 400 python -u scripts/bench_gemm_pp.py --m 1024,16384 --shapes gate_up,qkv,o,down --only 20:1,24:1,25:1,19:1,24:2,24:4 --rounds 3 --out $O/m.jsonl > $O/m.log 2>&1 || { tail -30 $O/m.log; exit 1; }
grep -E "best" $O/m.log | tail -20
