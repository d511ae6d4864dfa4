#!/bin/bash
# r5: 128k-token kill-chain context (BASELINE config 5) with the LDS-staged split decode
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5long
mkdir -p $O
for cfg in "fp8 fp8" "fp8 bf16" "bf16 bf16"; do
  set -- $cfg
  timeout -k 10 400 python -u scripts/long_context.py --tokens 131000 --kv-dtype $1 --weights $2 --repeat 2 > $O/long_$1_$2.log 2>&1 || { tail -20 $O/long_$1_$2.log; exit 1; }
  grep '^{' $O/long_$1_$2.log
done
