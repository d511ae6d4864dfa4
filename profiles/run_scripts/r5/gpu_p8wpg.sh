#!/bin/bash
# r5: fp8-MFMA prefill, page-per-wave staging (knob 1) vs per-lane block ids (knob 7): tests + A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5p8wpg2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_prefill_fp8_mfma_gpu.py tests/test_kernels_gpu.py -k "fp8" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_prefill_attn.py --fp8 --knob prefill_fp8_mfma --variants 7,1,7,1 --cases chunk16k_prefix0,chunk16k_prefix48k,chunk16k_prefix112k,wave_176x93 > $O/ab.log 2>&1
rc=$?; grep '^{' $O/ab.log; exit $rc
