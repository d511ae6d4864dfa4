#!/bin/bash
# tests of every gemm_lg config, the DMA issue-cost microbenchmark, then the issue-ordered asm-DMA variant (26-28)
# against the compiler-placed ones at 8192^3, M = 1024 / 16384, mid M and the LM head
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/lg8
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pp_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 120 ./csrc/microbench/mfma_dma > $O/mfma_dma.jsonl 2>&1 || { tail -5 $O/mfma_dma.jsonl; exit 1; }
cat $O/mfma_dma.jsonl
timeout -k 10 300 python -u scripts/bench_gemm_pp.py --m 8192 --shapes sq --only 20:1,24:1,26:1,62:1,63:1,54:1 --rounds 3 --out $O/sq.jsonl > $O/sq.log 2>&1 || { tail -30 $O/sq.log; exit 1; }
timeout -k 10 500 python -u scripts/bench_gemm_pp.py --m 1024,16384 --shapes gate_up,qkv,o,down --only 20:1,26:1,27:1,28:1,19:1,26:2,26:4,20:4 --rounds 2 --out $O/m.jsonl > $O/m.log 2>&1 || { tail -30 $O/m.log; exit 1; }
grep -E "best" $O/m.log | tail -8
timeout -k 10 500 python -u scripts/bench_gemm_pp.py --m 128,256,512 --shapes qkv,o,gate_up,down --only 19:2,19:4,23:2,23:4,28:2,28:4,28:8,20:2,26:2,26:4,3:1,3:2 --rounds 2 --out $O/mid.jsonl > $O/mid.log 2>&1 || { tail -30 $O/mid.log; exit 1; }
grep -E "best" $O/mid.log | tail -12
timeout -k 10 300 python -u scripts/bench_gemm_pp.py --m 1024,2048 --shapes lm_head --only 20:1,26:1,0:1,4:1 --rounds 2 --out $O/lm.jsonl > $O/lm.log 2>&1 || { tail -30 $O/lm.log; exit 1; }
grep -E "best" $O/lm.log | tail -2
