#!/bin/bash
# Fused decode RoPE/KV-write: kernel tests, then the headline wave with the fusion off / on (interleaved).
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread -k "decode or rope or engine or model" > gpurun_out/rf_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rf_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for f in 0 1; do
    CHRONOS_FUSE_DECODE_ROPE=$f timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --single-stream 2 \
        > gpurun_out/rf_bench_${f}_$rep.log 2>&1 || exit $?
    echo "fuse=$f rep=$rep $(grep '^{' gpurun_out/rf_bench_${f}_$rep.log | cut -c1-330)"
  done
done
