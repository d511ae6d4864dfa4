#!/bin/bash
# r5: fp8-MFMA prefill, MFMA row sums on top of page-per-wave staging (knob 8) vs default (1), alternated
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5p8msum
mkdir -p $O
timeout -k 10 300 python -u scripts/bench_prefill_attn.py --fp8 --knob prefill_fp8_mfma --variants 1,8 --cases chunk16k_prefix48k,chunk16k_prefix112k > $O/ab1.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_prefill_attn.py --fp8 --knob prefill_fp8_mfma --variants 8,1 --cases chunk16k_prefix48k,chunk16k_prefix112k > $O/ab2.log 2>&1
rc=$?; grep -h '^{' $O/ab1.log $O/ab2.log; exit $rc
