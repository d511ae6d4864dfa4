#!/bin/bash
# r5: plan-row tests (new cfg76 rows), then interleaved bench A/B: new plan vs round-4 plan, and lazy vs full KV
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5ab2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_plan_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in new old full new old full; do
  unset CHRONOS_GEMM_PLAN; X=
  if [ $v = old ]; then export CHRONOS_GEMM_PLAN=scripts/r5/plan_r4.json; fi
  if [ $v = full ]; then X="--kv-alloc full"; fi
  timeout -k 10 300 python bench.py --single-stream 0 --closed-steps 0 $X > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "$v $(tail -1 $O/bench_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["verdicts_valid"])')"
done
