#!/bin/bash
# r5: async harvest + jump-forward — GPU tests, then the single-stream A/B (sync vs async, burst lengths)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5async
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_jump_forward.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 500 python -u scripts/single_stream.py --chains 24 --knob-ab "py_small_burst=1" --out $O/sync.json > $O/sync.log 2>&1 || { tail -20 $O/sync.log; exit 1; }
timeout -k 10 600 python -u scripts/single_stream.py --chains 24 --async-harvest --knob-ab "py_small_burst=1;py_small_burst=2;py_burst=4" --out $O/async.json > $O/async.log 2>&1 || { tail -20 $O/async.log; exit 1; }
python3 -c "
import json
for f in ('sync', 'async'):
    d = json.load(open('$O/' + f + '.json'))
    for k, v in d.items(): print(f, k, v['p50_ms'], v['ms_per_token'], v['jumps_per_chain'], v['bursts_per_chain'])"
