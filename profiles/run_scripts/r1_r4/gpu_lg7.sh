#!/bin/bash
# DMA issue-cost microbenchmark + gemm_lg at mid M (128-512) and the LM head / 70B-TP8 shards
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/lg7
mkdir -p $O
timeout -k 10 120 ./csrc/microbench/mfma_dma > $O/mfma_dma.jsonl 2>&1 || { tail -5 $O/mfma_dma.jsonl; exit 1; }
cat $O/mfma_dma.jsonl
timeout -k 10 500 python -u scripts/bench_gemm_pp.py --m 128,256,512 --shapes qkv,o,gate_up,down --only 19:1,19:2,19:4,23:1,23:2,23:4,23:8,20:1,20:2,20:4,24:2,24:4,3:1,3:2,3:4 --rounds 2 --out $O/mid.jsonl > $O/mid.log 2>&1 || { tail -30 $O/mid.log; exit 1; }
grep -E "best" $O/mid.log | tail -20
timeout -k 10 300 python -u scripts/bench_gemm_pp.py --m 1024,2048 --shapes lm_head --only 20:1,24:1,0:1,4:1 --rounds 2 --out $O/lm.jsonl > $O/lm.log 2>&1 || { tail -30 $O/lm.log; exit 1; }
grep -E "best" $O/lm.log | tail -4
