#!/bin/bash
# r5: cascade decode attention tests + preemption GPU test, then the default bench with the cascade on / off
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_cascade_gpu.py tests/test_preemption_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -15 $O/pytest.log
[ $rc -eq 0 ] || { grep -m10 "FAILED\|Error\|assert" $O/pytest.log; exit $rc; }
