#!/bin/bash
# r5: fp8-MFMA prefill variants (row sums) + the 128k config's TTFT with the new default vs the bf16-MFMA kernel
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5p8long
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_prefill_fp8_mfma_gpu.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_prefill_attn.py --fp8 --knob prefill_fp8_mfma --variants 1,5,3 --cases chunk16k_prefix48k,chunk16k_prefix112k > $O/ab.log 2>&1
rc=$?; grep '^{' $O/ab.log; [ $rc -eq 0 ] || exit $rc
for kv in "prefill_fp8_mfma=1" "prefill_fp8_mfma=0"; do
  timeout -k 10 300 python -u scripts/long_context.py --tokens 131000 --kv-dtype fp8 --weights fp8 --repeat 2 --knob $kv > $O/long_$kv.log 2>&1 || { tail -20 "$O/long_$kv.log"; exit 1; }
  echo "[$kv] $(grep '"run": 1' "$O/long_$kv.log")"
done
