#!/bin/bash
# r5: production-shape plan tests (every routed row vs fp32) + the default bench as this round's starting point
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_plan_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_plan.log 2>&1
rc=$?
tail -3 $O/pytest_plan.log
[ $rc -eq 0 ] || { grep -m5 "FAILED\|Error" $O/pytest_plan.log; exit $rc; }
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
