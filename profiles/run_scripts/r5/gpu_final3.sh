#!/bin/bash
# r5 closing run 3: 128k TTFT (fp8 KV + fp8 / bf16 weights) with the page-per-wave fp8-MFMA prefill, GPU suite, smoke
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5final3
mkdir -p $O
for w in fp8 bf16; do
  timeout -k 10 300 python -u scripts/long_context.py --tokens 131000 --kv-dtype fp8 --weights $w --repeat 2 > $O/long_fp8kv_${w}w.log 2>&1 || { tail -20 $O/long_fp8kv_${w}w.log; exit 1; }
  grep '"run": 1' $O/long_fp8kv_${w}w.log
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
