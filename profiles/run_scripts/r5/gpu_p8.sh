#!/bin/bash
# r5: fp8-MFMA flash prefill: tests vs fp32, then A/B against the bf16-MFMA kernel on the long-context chunk shapes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5p8
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_prefill_fp8_mfma_gpu.py > $O/tests.log 2>&1
rc=$?; grep -E "rel |passed|failed|Error" $O/tests.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_prefill_attn.py --fp8 --knob prefill_fp8_mfma --variants 3,1,4,2 --cases chunk16k_prefix0,chunk16k_prefix48k,chunk16k_prefix112k,wave_176x93 > $O/ab.log 2>&1
rc=$?; cat $O/ab.log | grep '^{'; exit $rc
