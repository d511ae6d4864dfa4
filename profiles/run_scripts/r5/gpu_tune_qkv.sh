#!/bin/bash
# r5: the 192x128 configs (76, 77) in the plan tuner at the decode-bucket M for QKV / LM head, plus their GPU tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5tune
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_pp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "76 or 77" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 700 python -u scripts/tune_gemm_pp.py --models 8b,70b-tp8 --ops ${OPS:-qkv,lm_head,o,down} --ms ${MS:-512,768,1024,2048} --out-table $O/table.jsonl > $O/tune.log 2>&1 || { tail -30 $O/tune.log; exit 1; }
tail -40 $O/tune.log
