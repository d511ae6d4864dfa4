#!/bin/bash
# r5: parallel decode combine — split-decode tests, then long-context attention timings (separate vs in-launch)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5comb
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_split_decode_gpu.py tests/test_kernels_gpu.py -k "attn or attention or decode or split" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
ATTN_CASES=long timeout -k 10 300 python -u scripts/bench_attn.py --out $O/attn_long.json > $O/attn.log 2>&1 || { tail -20 $O/attn.log; exit 1; }
grep -v amdgpu.ids $O/attn.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['batch'], d['ctx'], d['fp8'], {k: v for k, v in d.items() if k.endswith('_us')})"
