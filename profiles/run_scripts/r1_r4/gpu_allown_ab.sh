#!/bin/bash
# in-situ A/B on one box: the measured routing plan vs the same plan with every library row replaced by the fastest
# hand-written config (scripts/plan_all_own.json): what routing the last hipBLASLt shapes to own kernels costs the wave
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/allown
mkdir -p $O
for v in plan allown plan allown; do
  if [ $v = allown ]; then export CHRONOS_GEMM_PLAN=scripts/plan_all_own.json; else unset CHRONOS_GEMM_PLAN; fi
  timeout -k 10 300 python bench.py --single-stream 0 --closed-steps 0 > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "$v $(tail -1 $O/bench_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
