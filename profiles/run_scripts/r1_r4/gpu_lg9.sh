#!/bin/bash
# slab-schedule sync ablations at 8192^3: without the per-slab vmcnt wait, without the barrier too
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/lg9
mkdir -p $O
timeout -k 10 300 python -u scripts/bench_gemm_pp.py --m 8192 --shapes sq --only 20:1,64:1,65:1,66:1,53:1,54:1 --rounds 3 --out $O/sq.jsonl > $O/sq.log 2>&1 || { tail -30 $O/sq.log; exit 1; }
cat $O/sq.jsonl
