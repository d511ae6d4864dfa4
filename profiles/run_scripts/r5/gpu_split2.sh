#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5split2
mkdir -p $O
ATTN_CASES=long ATTN_NSPLITS=32,48,64,96 ATTN_KNOBS="split_lds_nb=1,split_lds_nb=2,split_lds_nb=3" timeout -k 10 300 python -u scripts/bench_attn.py --out $O/attn_long_nsplit.json > $O/attn.log 2>&1 || { tail -20 $O/attn.log; exit 1; }
cat $O/attn.log | grep -v amdgpu.ids | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['batch'], d['ctx'], d['fp8'], {k: v for k, v in d.items() if k.endswith('_us')})"
