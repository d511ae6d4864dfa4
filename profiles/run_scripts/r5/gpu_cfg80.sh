#!/bin/bash
# r5: cfg 80 (32x32x16 MFMA slab schedule): GPU tests vs fp32, then timings vs cfg 20 and hipBLASLt
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5c80
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_pp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "80" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u scripts/r5/bench_cfg80.py > $O/bench.jsonl 2>&1 || { tail -20 $O/bench.jsonl; exit 1; }
grep '^{' $O/bench.jsonl
