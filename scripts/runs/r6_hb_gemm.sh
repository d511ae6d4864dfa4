#!/bin/bash
# r6: the HB GEMM (cfg 81, hipBLASLt's three-barrier slab loop) vs cfg 20 vs hipBLASLt: fp32 error + timing per shape
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6hb
mkdir -p $O
timeout -k 10 400 python -u scripts/bench_gemm_cfgs.py --cfgs 20,81 \
  --shapes sq8192,qkv16k,o16k,gu16k,down16k,qkv4k,gu4k,lm1k,gu1k,gu768 --out $O/hb_vs_20_lib.jsonl > $O/bench.log 2>&1
rc=$?; tail -15 $O/bench.log; exit $rc
