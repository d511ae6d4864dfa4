#!/bin/bash
# decode-attention A/B (isolated, unique vs shared prefix pages) + attention / fusion / model numerics GPU tests +
# short headline bench.  Usage (gpurun): bash scripts/gpu_attn2.sh
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in 0 3; do
  ATTN_CASES=wave ATTN_SHARED_BLOCKS=$s timeout -k 10 120 python scripts/bench_attn.py > gpurun_out/attn2_shared_$s.log 2>&1 || exit $?
  grep "^{" gpurun_out/attn2_shared_$s.log | cut -c1-250
done
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_decode_fusion_gpu.py tests/test_model_numerics_gpu.py \
    -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/attn2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/attn2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --closed-steps 0 --single-stream 2 > gpurun_out/attn2_bench.log 2>&1 || exit $?
tail -1 gpurun_out/attn2_bench.log | cut -c1-300
