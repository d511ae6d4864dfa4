#!/bin/bash
# r5: fp8-MFMA prefill at three workgroups per CU (knob 9: Q in LDS, <= 168 VGPRs, some spills) vs default (1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5p8occ3
mkdir -p $O
timeout -k 10 300 python -u scripts/bench_prefill_attn.py --fp8 --knob prefill_fp8_mfma --variants 1,9 --cases chunk16k_prefix0,chunk16k_prefix48k,chunk16k_prefix112k,wave_176x93 > $O/ab.log 2>&1
rc=$?; grep '^{' $O/ab.log; tail -3 $O/ab.log; exit $rc
