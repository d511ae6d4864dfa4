#!/bin/bash
# gemm_pp tile-order sweep (knob pp_gm) at prefill-sized M against hipBLASLt, then the headline bench with its phase
# breakdown.  Usage (gpurun): bash scripts/gpu_gm_sweep.sh
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u scripts/bench_gemm_pp.py --m 16384,4096 --shapes qkv,o,gate_up,down --only 0:1,4:1 \
    --gms 0,4,8,16 --rounds 3 --iters 5 --out gpurun_out/gm_sweep.jsonl > gpurun_out/gm_sweep.log 2>&1 || exit $?
tail -8 gpurun_out/gm_sweep.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/s1_bench.log 2>&1 || exit $?
grep -h "phase seconds\|histogram" gpurun_out/s1_bench.log | cut -c1-600
tail -1 gpurun_out/s1_bench.log | cut -c1-900
