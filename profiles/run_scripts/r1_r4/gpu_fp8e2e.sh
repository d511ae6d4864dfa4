#!/bin/bash
# W8A8 end to end with the new routing: fp8 GPU tests, the 128k-token TTFT (fp8 KV + fp8 projections) and the
# headline bench with --weights fp8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/fp8e2e
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp8_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 400 python3 scripts/long_context.py --tokens 131000 --kv-dtype fp8 --weights fp8 --repeat 2 > $O/long.log 2>&1 || { tail -30 $O/long.log; exit 1; }
tail -1 $O/long.log
timeout -k 10 500 python3 bench.py --weights fp8 --single-stream 0 --closed-steps 0 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-600
