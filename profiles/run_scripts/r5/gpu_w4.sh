#!/bin/bash
# experimental one-wave-per-SIMD GEMM vs hipBLASLt and gemm_lg cfg20 (interleaved, one process)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5w4
mkdir -p $O
timeout -k 10 500 python -u scripts/r5/bench_w4.py --lib csrc/microbench/libgemm_w4.so --vars ${VARS:-4,5,12,13} --lg 20,16 --shapes ${SHAPES:-all} --gms ${GMS:-} --out $O/w4.jsonl > $O/w4.log 2>&1
rc=$?
cat $O/w4.log | tail -12
exit $rc
