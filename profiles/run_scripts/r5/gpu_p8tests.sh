#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5p8tests
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_prefill_fp8_mfma_gpu.py > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|Error|assert" $O/tests.log | tail -6; exit $rc
