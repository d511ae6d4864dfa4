#!/bin/bash
# decode attention after the 16-B V-load token map: GPU attention tests, cold/warm timings, headline bench.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_gpu.py tests/test_decode_fusion_gpu.py -x -q \
    -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/attn3_tests.log 2>&1
rc=$?; tail -3 gpurun_out/attn3_tests.log; [ $rc -eq 0 ] || { grep -m3 -A20 "FAILED\|Error" gpurun_out/attn3_tests.log | head -60; exit $rc; }
timeout -k 10 60 python scripts/attn_one.py --shared 0 || exit $?
timeout -k 10 60 python scripts/attn_one.py --shared 3 || exit $?
ATTN_CASES=wave ATTN_SHARED_BLOCKS=3 timeout -k 10 120 python scripts/bench_attn.py > gpurun_out/attn3_warm.log 2>&1 || exit $?
grep "^{" gpurun_out/attn3_warm.log | cut -c1-200
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --closed-steps 0 --single-stream 2 > gpurun_out/attn3_bench.log 2>&1 || exit $?
tail -1 gpurun_out/attn3_bench.log | cut -c1-300
