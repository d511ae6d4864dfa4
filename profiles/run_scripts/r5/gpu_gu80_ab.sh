#!/bin/bash
# r5: in-situ A/B — gate_up + SwiGLU at M >= 2048 (prefill chunks) on gemm_lg cfg20 (fused epilogue) vs hipBLASLt + silu_mul
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5gu80
mkdir -p $O
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 4 --closed-steps 0 --single-stream 2 > $O/base_$i.log 2>&1 || { tail -20 $O/base_$i.log; exit 1; }
  echo "base: $(grep '^{' $O/base_$i.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  CHRONOS_GEMM_PLAN=scripts/r5/plan_gu80.json timeout -k 10 400 python -u bench.py --steps 4 --closed-steps 0 --single-stream 2 > $O/own_$i.log 2>&1 || { tail -20 $O/own_$i.log; exit 1; }
  echo "gu80: $(grep '^{' $O/own_$i.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done
