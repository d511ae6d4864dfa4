#!/bin/bash
# r5: last sanity pass after the final rebuild: fp8 / bf16 prefill tests + smoke
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5sanity
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_prefill_fp8_mfma_gpu.py tests/test_decode_fusion_gpu.py tests/test_kernels_gpu.py > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
