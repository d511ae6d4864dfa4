#!/bin/bash
# r5: fp8-MFMA prefill, PIPE variant (next stage's Q K^T under this stage's softmax) vs default
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5p8pipe
mkdir -p $O
timeout -k 10 300 python -u scripts/bench_prefill_attn.py --fp8 --knob prefill_fp8_mfma --variants 1,6 --cases chunk16k_prefix0,chunk16k_prefix48k,chunk16k_prefix112k,wave_176x93 > $O/ab.log 2>&1
rc=$?; grep '^{' $O/ab.log; tail -3 $O/ab.log; exit $rc
