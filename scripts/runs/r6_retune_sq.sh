#!/bin/bash
# re-measure the 8B large-M rows with the square-order HB configs 92 / 93 among the candidates (own-only: these rows
# carry fused norm / residual epilogues the bare A/B does not credit), then the 70B-TP1 rows under the library rule
set -o pipefail
mkdir -p gpurun_out/retune_sq
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u scripts/retune_large_m.py --own-only --keys 6144:4096:0,4096:4096:2,28672:4096:1,4096:14336:2,128256:4096:0 --out-plan gpurun_out/retune_sq/plan8b.json --out-table gpurun_out/retune_sq/t8b.jsonl > gpurun_out/retune_sq/t8b.log 2>&1 || { tail -20 gpurun_out/retune_sq/t8b.log; exit 1; }
timeout -k 10 700 python -u scripts/retune_large_m.py --plan gpurun_out/retune_sq/plan8b.json --keys 10240:8192:0,8192:8192:2,57344:8192:1,8192:28672:2,128256:8192:0 --out-plan gpurun_out/retune_sq/plan.json --out-table gpurun_out/retune_sq/t70b.jsonl > gpurun_out/retune_sq/t70b.log 2>&1 || { tail -20 gpurun_out/retune_sq/t70b.log; exit 1; }
