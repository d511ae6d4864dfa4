#!/bin/bash
# small-slab split-K hand-off (write-through vs fences) on the routed split-K points, then the M = 2-8 re-tune with
# split-K candidates for the 32-row configs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/hos
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pp_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for h in 0 1; do
  CHRONOS_LG_HANDOFF=$h timeout -k 10 300 python3 scripts/bench_gemm_pp.py --m 64,128,256 --shapes qkv,o,down \
     --only "36:4,39:2,39:4,38:4,32:4,33:2,36:2" --out $O/h$h.jsonl > $O/h$h.log 2>&1 || { tail -20 $O/h$h.log; exit 1; }
done
python3 - <<'PY'
import json
d={}
for h in (0,1):
    for l in open(f"gpurun_out/hos/h{h}.jsonl"):
        r=json.loads(l)
        if r['cand']!='hipblaslt': d.setdefault((r['op'],r['m'],r['cand']),{})[h]=r['us']
for k,v in sorted(d.items()): print(k, v)
PY
MS=2,3,4,5,8 OUT=tune8 timeout -k 10 700 bash scripts/gpu_tune_tiny.sh || exit $?
