#!/bin/bash
# gemm_pp A/Bs against hipBLASLt: tile order (knob pp_gm) and DMA-in-compute configs (12-15) at decode / prefill M,
# after the gemm_pp numerics tests; then the headline bench with its phase breakdown.
# Usage (gpurun): bash scripts/gpu_gm_sweep.sh
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_pp_gpu.py -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/pp_tests.log 2>&1 || { tail -30 gpurun_out/pp_tests.log; exit 1; }
tail -2 gpurun_out/pp_tests.log
timeout -k 10 300 python -u scripts/bench_gemm_pp.py --m 1024 --shapes qkv,o,gate_up,down --only 4:1,12:1,5:1,13:1,6:1,14:1,7:1,15:1,0:1 \
    --rounds 3 --iters 10 --out gpurun_out/gic_m1024.jsonl > gpurun_out/gic_m1024.log 2>&1 || exit $?
grep -v "^{" gpurun_out/gic_m1024.log | tail -8
timeout -k 10 420 python -u scripts/bench_gemm_pp.py --m 16384 --shapes qkv,gate_up --only 0:1,4:1,12:1 \
    --gms 0,8 --rounds 2 --iters 3 --out gpurun_out/gm_sweep.jsonl > gpurun_out/gm_sweep.log 2>&1 || exit $?
grep -v "^{" gpurun_out/gm_sweep.log | tail -8
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/s1_bench.log 2>&1 || exit $?
grep -h "phase seconds\|histogram" gpurun_out/s1_bench.log | cut -c1-600
tail -1 gpurun_out/s1_bench.log | cut -c1-900
