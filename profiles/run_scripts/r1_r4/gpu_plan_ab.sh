#!/bin/bash
# in-situ A/B of the GEMM routing plan: the driver's default bench with the round-4 plan vs the round-3 plan
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/planab
mkdir -p $O
for run in new old new2; do
  if [ $run = old ]; then export CHRONOS_GEMM_PLAN=scripts/r3_gemm_plan.json; else unset CHRONOS_GEMM_PLAN; fi
  timeout -k 10 500 python bench.py --steps 6 --warmup 3 --closed-steps 4 > $O/bench_$run.log 2>&1 || { tail -20 $O/bench_$run.log; exit 1; }
  tail -1 $O/bench_$run.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$run', d['value'], d['closed_loop_chains_s'], d['p50_verdict_latency_ms'], d['single_stream_decode_ms_per_token'])"
done
