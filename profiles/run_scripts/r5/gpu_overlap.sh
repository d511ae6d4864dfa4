#!/bin/bash
# r5: TP decode overlap tests (2 ranks on the one GPU), then the 128k long-context runs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5ov
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_tp_overlap_gpu.py > gpurun_out/r5ov/tests.log 2>&1 || { tail -60 gpurun_out/r5ov/tests.log; exit 1; }
tail -8 gpurun_out/r5ov/tests.log
bash scripts/r5/gpu_long2.sh
