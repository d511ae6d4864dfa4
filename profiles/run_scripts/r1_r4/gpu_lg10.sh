#!/bin/bash
# one-wave-per-SIMD slab kernel (cfg21) vs its sync-free and MFMA-only bounds at 8192^3
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/lg10
mkdir -p $O
timeout -k 10 300 python3 scripts/bench_gemm_pp.py --m 8192 --shapes sq --only "20:1,21:1,68:1,69:1,54:1" --out $O/sq.jsonl > $O/sq.log 2>&1 || { tail -20 $O/sq.log; exit 1; }
grep '"cand"' $O/sq.log | cut -c1-200
