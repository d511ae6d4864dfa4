#!/bin/bash
# r5: deep-ring mid-M configs 78/79 — their GPU tests, then the mid-M tuner rows at M = 64 / 128 / 256
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5deep
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_pp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "78 or 79" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 900 python -u scripts/tune_gemm_pp.py --models 8b,70b-tp8 --ms 64,128,256 --merge project-chronos-distributed-behavioral-edr-ebpf-llm-_amd/ops/gemm_plan.json --out-plan $O/plan.json --out-table $O/table.jsonl > $O/tune.log 2>&1 || { tail -30 $O/tune.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r5deep/table.jsonl"):
    d = json.loads(l)
    deep = {k: v for k, v in d["all"].items() if k.startswith(("cfg78", "cfg79"))}
    best_deep = min(deep.items(), key=lambda x: x[1]) if deep else None
    print(d["model"], d["op"], d["m"], d["own"], d["own_us"], "lib", d["lib_us"], "TB/s", d["own_weight_TBs"], "deep", best_deep)
PY
