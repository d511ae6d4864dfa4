#!/bin/bash
# r5: 128k fp8 decode, kernel-knob A/B (one long_context run per knob set; run 1 of 2 = warm)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5longab
mkdir -p $O
i=0
for ks in "" "sd_inkernel_max_split=1024" "gemv_q_r_swiglu=8" "gemv_q_r_rope=4" "gemv_q_r_resid=4" "gemv_q_r_plain=8"; do
  args=""
  for kv in $(echo $ks | tr ',' ' '); do args="$args --knob $kv"; done
  timeout -k 10 300 python -u scripts/long_context.py --tokens 131000 --kv-dtype fp8 --weights fp8 --repeat 2 $args > $O/long_$i.log 2>&1 || { tail -20 $O/long_$i.log; exit 1; }
  echo "knobs [$ks]: $(grep '"run": 1' $O/long_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["decode_ms_per_token"], d["verdict_tokens"])')"
  i=$((i+1))
done
