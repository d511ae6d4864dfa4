#!/bin/bash
# r5: 128k TTFT vs prefill chunk size (fp8 KV + fp8 weights, fp8-MFMA flash prefill)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5chunk
mkdir -p $O
for c in 32768 8192 16384; do
  timeout -k 10 300 python -u scripts/long_context.py --tokens 131000 --kv-dtype fp8 --weights fp8 --repeat 2 --chunk $c > $O/long_$c.log 2>&1 || { tail -20 $O/long_$c.log; exit 1; }
  echo "chunk $c: $(grep '"run": 1' $O/long_$c.log | cut -c1-260)"
done
