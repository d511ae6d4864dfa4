#!/bin/bash
# r5: fp8-MFMA prefill register lookahead depth A/B (knob prefill8_depth 1 vs 2) + tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5p8d
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_prefill_fp8_mfma_gpu.py > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|Error" $O/tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_prefill_attn.py --fp8 --knob prefill8_depth --variants 1,2 --cases chunk16k_prefix0,chunk16k_prefix48k,chunk16k_prefix112k,wave_176x93 > $O/depth.log 2>&1
rc=$?; grep '^{' $O/depth.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_prefill_attn.py --fp8 --knob prefill_fp8_mfma --variants 1,3,2,0 --cases chunk16k_prefix112k > $O/ab.log 2>&1
rc=$?; grep '^{' $O/ab.log; exit $rc
