#!/bin/bash
# r6: the folded-RMSNorm (NORMP) forms in situ-like (cold weights): HB vs cfg 20 vs library + rmsnorm
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6normp
mkdir -p $O
timeout -k 10 500 python -u scripts/bench_gemm_cfgs.py --cfgs 20,88,89 --normp 1 --cold 1 \
  --shapes gu1k,lm1k,qkv16k,gu16k,qkv1k --out $O/normp.jsonl > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log
timeout -k 10 500 python -u scripts/bench_gemm_cfgs.py --cfgs 20,88,89 --normp 0 --cold 1 \
  --shapes gu1k,lm1k,qkv16k --out $O/plain.jsonl > $O/bench2.log 2>&1 || { tail -20 $O/bench2.log; exit 1; }
grep '^{' $O/bench2.log
