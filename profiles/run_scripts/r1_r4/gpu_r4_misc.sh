#!/bin/bash
# tiny-M re-tune (M = 2-8 with the 32-row-x-tile gemm_lg configs), then the TunableOp probe of the library GEMMs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
MS=2,3,4,5,8 OUT=tune7 timeout -k 10 700 bash scripts/gpu_tune_tiny.sh || exit $?
O=gpurun_out/tunop
mkdir -p $O
timeout -k 10 400 python -u scripts/tunableop_probe.py --out $O/tunableop.jsonl > $O/tunableop.log 2>&1 || { tail -20 $O/tunableop.log; exit 1; }
grep '"op"' $O/tunableop.log
