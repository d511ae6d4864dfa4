#!/bin/bash
# r5: one-wave-per-(seq, kv head) decode kernel below 2048 items (knob decode_min_items) on the T = 64 / 128 buckets
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5decitems
mkdir -p $O
for rows in 128 64; do
  for k in 2048 512; do
    timeout -k 10 200 python -u scripts/fw_bucket.py --rows $rows --ctx 200 --knob decode_min_items=$k >> $O/fw.jsonl 2> $O/fw_err.log || { tail -20 $O/fw_err.log; exit 1; }
  done
done
cat $O/fw.jsonl
for k in 2048 512; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$k -o run --output-format csv -- python3 scripts/fw_bucket.py --rows 128 --ctx 200 --knob decode_min_items=$k > $O/prof_$k.log 2>&1 || { tail -20 $O/prof_$k.log; exit 1; }
  f=$(find $O/prof_$k -name "*kernel_stats.csv" | head -1)
  echo "== decode_min_items=$k"; grep -i "attn\|decode" "$f" | cut -c1-60,180-260 | head -5
  find $O/prof_$k -name "*.csv" ! -name "*kernel_stats.csv" -delete
done
