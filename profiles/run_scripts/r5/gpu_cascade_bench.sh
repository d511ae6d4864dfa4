#!/bin/bash
# r5: cascade engine test on the fused decode path, then the default bench with the cascade on / off (interleaved)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5cb
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_cascade_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k engine > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for v in on off on off; do
  if [ $v = off ]; then X=--no-cascade; else X=; fi
  timeout -k 10 300 python bench.py --single-stream 0 --closed-steps 0 $X > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "$v $(tail -1 $O/bench_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["verdicts_valid"])')"
done
