#!/bin/bash
# r5: decode-only per-forward breakdowns: 128k fp8 decode, and the single-stream phase of bench.py
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5tail
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/long -o run --output-format csv -- python3 scripts/long_context.py --tokens 131000 --kv-dtype fp8 --weights fp8 --repeat 1 > $O/long.log 2>&1 || { tail -20 $O/long.log; exit 1; }
grep '^{' $O/long.log
f=$(find $O/long -name "*kernel_trace.csv" | head -1)
python3 scripts/decode_tail.py "$f" --T 1 --last 40 | tee $O/long_decode_tail.txt
gzip -c "$f" > $O/long_trace.csv.gz; find $O/long -name "*.csv" -delete
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/ss -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --streams 16 > $O/ss.log 2>&1 || { tail -20 $O/ss.log; exit 1; }
grep '^{' $O/ss.log | cut -c1-600
f=$(find $O/ss -name "*kernel_trace.csv" | head -1)
for T in 1 2 3 4; do python3 scripts/decode_tail.py "$f" --T $T --last 200; done | tee $O/ss_decode_tail.txt
gzip -c "$f" > $O/ss_trace.csv.gz; find $O/ss -name "*.csv" -delete
