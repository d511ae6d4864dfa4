#!/bin/bash
# r5: decode_min_items 1024 default (fused RoPE + one-wave decode at T = 128): tests + T = 128 forward
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5decitems2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_decode_fusion_gpu.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for k in 1024 2048; do
  timeout -k 10 200 python -u scripts/fw_bucket.py --rows 128 --ctx 200 --knob decode_min_items=$k >> $O/fw.jsonl 2> $O/fw_err.log || { tail -20 $O/fw_err.log; exit 1; }
done
cat $O/fw.jsonl
