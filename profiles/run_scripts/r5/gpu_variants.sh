#!/bin/bash
# r5: the fp8-weight headline variant and the 128k config with bf16 KV / bf16 weights
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5var
mkdir -p $O
timeout -k 10 600 python -u bench.py --weights fp8 > $O/bench_fp8.log 2>&1 || { tail -30 $O/bench_fp8.log; exit 1; }
grep '^{' $O/bench_fp8.log | tail -1 | cut -c1-700
timeout -k 10 400 python -u scripts/long_context.py --tokens 131000 --kv-dtype bf16 --weights bf16 --repeat 2 > $O/long_bf16.log 2>&1 || { tail -20 $O/long_bf16.log; exit 1; }
grep '^{' $O/long_bf16.log
timeout -k 10 400 python -u scripts/long_context.py --tokens 131000 --kv-dtype fp8 --weights bf16 --repeat 2 > $O/long_fp8kv.log 2>&1 || { tail -20 $O/long_fp8kv.log; exit 1; }
grep '^{' $O/long_fp8kv.log
