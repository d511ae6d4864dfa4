#!/bin/bash
# tile-order group size (knob pp_gm) for the large-M slab / ring configs at M = 16384
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/gm
mkdir -p $O
timeout -k 10 600 python3 scripts/bench_gemm_pp.py --m 16384 --shapes gate_up,down,qkv --only "20:1,30:1,29:1" --gms "0,2,4,8,16,32" \
    --out $O/gm.jsonl > $O/gm.log 2>&1 || { tail -20 $O/gm.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/gm/gm.jsonl"):
    r=json.loads(l); print(r["op"], r["cand"], r["us"], r["vs_lib"])
PY
