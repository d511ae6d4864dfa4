#!/bin/bash
# slab-schedule ablations at 8192^3: which part of the data path bounds the kernel (cold vs L2-resident operands)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/lg5
mkdir -p $O
timeout -k 10 300 python -u scripts/bench_gemm_pp.py --m 8192 --shapes sq --only 20:1,53:1,54:1,55:1,56:1,57:1,58:1,59:1,60:1 --rounds 3 --out $O/sq.jsonl > $O/sq.log 2>&1 || { tail -30 $O/sq.log; exit 1; }
echo ok
