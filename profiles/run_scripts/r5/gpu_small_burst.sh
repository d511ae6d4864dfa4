#!/bin/bash
# r5: small-bucket burst length (single stream) A/B, then the default bench with it
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5sb
mkdir -p $O
timeout -k 10 600 python -u scripts/single_stream.py --chains 24 --knob-ab "py_small_burst=2;py_small_burst=1;py_small_burst=2,py_gemv_max_m=2" --out $O/ab.json > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab.json'))
for k,v in d.items(): print(k, v['p50_ms'], v['ms_per_token'], v['bursts_per_chain'])"
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | cut -c1-1200
