#!/bin/bash
# gemm_pp 5-stage full-LDS config (cfg 12) vs cfg 0 / 4 and hipBLASLt at decode and prefill M.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_pp_gpu.py -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/pp5_tests.log 2>&1 || { tail -30 gpurun_out/pp5_tests.log; exit 1; }
tail -1 gpurun_out/pp5_tests.log
timeout -k 10 300 python -u scripts/bench_gemm_pp.py --m 1024,768,512 --shapes gate_up,qkv,lm_head --only 0:1,4:1,12:1 \
    --rounds 3 --iters 10 --out gpurun_out/pp5_decode.jsonl > gpurun_out/pp5_decode.log 2>&1 || exit $?
grep -v "^{" gpurun_out/pp5_decode.log | tail -9
timeout -k 10 300 python -u scripts/bench_gemm_pp.py --m 16384 --shapes gate_up,qkv --only 0:1,4:1,12:1 \
    --rounds 2 --iters 3 --out gpurun_out/pp5_prefill.jsonl > gpurun_out/pp5_prefill.log 2>&1 || exit $?
grep -v "^{" gpurun_out/pp5_prefill.log | tail -3
python3 -c "
import json
for f in ['gpurun_out/pp5_decode.jsonl','gpurun_out/pp5_prefill.jsonl']:
    for l in open(f):
        d=json.loads(l); print(d['op'], d['m'], d['cand'], d['us'], d['vs_lib'])
"
