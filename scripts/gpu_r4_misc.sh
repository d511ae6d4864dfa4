#!/bin/bash
# tiny-M re-tune (M = 2-8 with the 32-row-x-tile gemm_lg configs), then the fp8 W8A8 table at M = 256-16384
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
MS=2,3,4,5,8 OUT=tune7 timeout -k 10 900 bash scripts/gpu_tune_tiny.sh || exit $?
O=gpurun_out/fp8t
mkdir -p $O
timeout -k 10 600 python -u scripts/tune_gemm_pp.py --fp8 --ms 256,1024,4096,16384 --rounds 3 \
  --out-table $O/table.jsonl > $O/tune.log 2>&1 || { tail -30 $O/tune.log; exit 1; }
grep '"op"' $O/tune.log | cut -c1-220
timeout -k 10 600 python -u scripts/tunableop_probe.py --out gpurun_out/fp8t/tunableop.jsonl > gpurun_out/fp8t/tunableop.log 2>&1 || { tail -20 gpurun_out/fp8t/tunableop.log; exit 1; }
grep '"op"' gpurun_out/fp8t/tunableop.log
