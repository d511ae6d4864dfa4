#!/bin/bash
# r5: bf16 flash prefill (v2 LEAN) with page-per-wave staging (knob prefill_wpg 1) vs per-lane (0): tests + A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5p2wpg
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_decode_fusion_gpu.py tests/test_kernels_gpu.py -k "prefill or paged_attention or rescale" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_prefill_attn.py --knob prefill_wpg --variants 0,1 --cases chunk16k_prefix0,chunk16k_prefix48k,chunk16k_prefix112k,wave_176x93 > $O/ab.log 2>&1
rc=$?; grep '^{' $O/ab.log; exit $rc
