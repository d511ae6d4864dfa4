#!/bin/bash
# split-K / stream-K hand-off A/B (knob lg_handoff: 1 write-through, 0 fences) at M = 1024 / 2048
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/sk2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pp_gpu.py tests/test_fp8_gpu.py -k "split or stream or qgemm_lg or resid" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for h in 1 0; do
  CHRONOS_LG_HANDOFF=$h timeout -k 10 400 python3 scripts/bench_gemm_pp.py --m 1024,2048 --shapes qkv,o,gate_up,down \
      --only "20:0,30:0,30:2,19:0,19:2,29:0,20:2,30:4" --out $O/h$h.jsonl > $O/h$h.log 2>&1 || { tail -30 $O/h$h.log; exit 1; }
done
python3 - <<'PY'
import json
d={}
for h in (1,0):
    for l in open(f"gpurun_out/sk2/h{h}.jsonl"):
        r=json.loads(l); d.setdefault((r['op'],r['m'],r['cand']),{})[h]=r['us']
for k,v in sorted(d.items()):
    print(k, v)
PY
