#!/bin/bash
# r6: HB schedule variants (cfg 81-85) and tile-group sizes vs cfg 20 vs hipBLASLt
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6hb7
mkdir -p $O
timeout -k 10 500 python -u scripts/bench_gemm_cfgs.py --cfgs 88,89,90 --gms 8 \
  --shapes sq8192,qkv16k,down16k,gu16k,o16k,lm1k,gu1k --out $O/hb_var.jsonl > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log
