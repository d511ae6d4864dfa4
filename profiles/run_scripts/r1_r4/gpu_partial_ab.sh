#!/bin/bash
# Partial-block prefix reuse: engine GPU tests, then the headline wave with it off / on (interleaved).
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_decode_fusion_gpu.py -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread -k "engine" > gpurun_out/pp_tests.log 2>&1
rc=$?; tail -3 gpurun_out/pp_tests.log; [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
for rep in 1 2; do
  for f in off on; do
    flag=""; [ $f = off ] && flag="--no-partial-prefix"
    timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --single-stream 2 $flag > gpurun_out/pp_bench_${f}_$rep.log 2>&1 || exit $?
    echo "partial=$f rep=$rep $(grep '^{' gpurun_out/pp_bench_${f}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["verdicts_valid"], d["p50_verdict_latency_ms"], d["prefix_cache_hit_fraction"])')"
  done
done
