#!/bin/bash
# re-measure the 8B decode-bucket rows (M = 512-2048) with the whole non-HB lg / pp family among the candidates
# (the round-6 re-tunes only compared each row's old config with the HB configs)
set -o pipefail
mkdir -p gpurun_out/widen
export HSA_ENABLE_IPC_MODE_LEGACY=0
X=19/1,19/2,30/1,30/2,29/1,20/1,76/1,77/1,22/1,15/1,31/1,23/1,0/1,1/1,2/1,3/1,38/1,37/1
timeout -k 10 900 python -u scripts/retune_large_m.py --own-only --min-m 512 --max-m 2048 --extra-cfgs $X --keys 6144:4096:0,4096:4096:2,28672:4096:1,4096:14336:2,128256:4096:0 --out-plan gpurun_out/widen/plan8b.json --out-table gpurun_out/widen/t8b.jsonl > gpurun_out/widen/t8b.log 2>&1 || { tail -20 gpurun_out/widen/t8b.log; exit 1; }
