#!/bin/bash
# r5: the 70B TP = 1 plan rows under the production-shape tests, then the one-GPU 70B bench, old vs new plan
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5b70
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_plan_gpu.py -m gpu -k "K8192 or K28672" > $O/plan_tests.log 2>&1 || { tail -30 $O/plan_tests.log; exit 1; }
tail -2 $O/plan_tests.log
for v in new old; do
  if [ $v = old ]; then export CHRONOS_GEMM_PLAN=scripts/r5/plan_pre_70b.json; else unset CHRONOS_GEMM_PLAN; fi
  timeout -k 10 900 python -u bench.py --model llama3-70b --streams 256 --steps 2 --warmup 1 --closed-steps 0 --single-stream 4 > $O/bench_$v.log 2>&1 || { tail -30 $O/bench_$v.log; exit 1; }
  echo "$v: $(grep '^{' $O/bench_$v.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_verdict_latency_ms"], d.get("single_stream_p50_latency_ms"), d.get("single_stream_decode_ms_per_token"))')"
done
