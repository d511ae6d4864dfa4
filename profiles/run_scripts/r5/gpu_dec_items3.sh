#!/bin/bash
# r5: T = 128 forward, three decode-attention routes, alternated twice on one box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5decitems3
mkdir -p $O
for rep in 1 2; do
  for ks in "decode_min_items=2048" "decode_min_items=1024 --knob decode_rope_fused=0" "decode_min_items=1024"; do
    timeout -k 10 200 python -u scripts/fw_bucket.py --rows 128 --ctx 200 --iters 50 --knob $ks >> $O/fw.jsonl 2> $O/fw_err.log || { tail -20 $O/fw_err.log; exit 1; }
  done
done
cat $O/fw.jsonl
