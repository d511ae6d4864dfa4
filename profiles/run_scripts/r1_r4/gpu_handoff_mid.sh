#!/bin/bash
# split-K hand-off at 64-128 KB slabs (cfg19 128 x 128, cfg30 128 x 256): write-through vs fences, M = 512 / 1024
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/hom
mkdir -p $O
for h in 0 1; do
  CHRONOS_LG_HANDOFF=$h timeout -k 10 300 python3 scripts/bench_gemm_pp.py --m 512,1024 --shapes qkv,o,down \
     --only "19:2,19:4,30:2,30:4,15:2" --out $O/h$h.jsonl > $O/h$h.log 2>&1 || { tail -20 $O/h$h.log; exit 1; }
done
python3 - <<'PY'
import json
d={}
for h in (0,1):
    for l in open(f"gpurun_out/hom/h{h}.jsonl"):
        r=json.loads(l)
        if r['cand']!='hipblaslt': d.setdefault((r['op'],r['m'],r['cand']),{})[h]=r['us']
for k,v in sorted(d.items()): print(k, v)
PY
