#!/bin/bash
# r6: large-M plan rows re-measured with the HB configs (88 / 89) among the candidates
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6plan
mkdir -p $O
A="10240:8192:0=1024/2048/4096/8192/16384;8192:8192:2=1024/2048/4096/8192/16384;57344:8192:1=1024/2048/4096/8192/16384;8192:28672:2=1024/2048/4096/8192/16384"
timeout -k 10 1000 python -u scripts/retune_large_m.py --min-m 512 --add-ms "$A" \
  --out-plan $O/gemm_plan.json --out-table $O/retune_large_m.jsonl > $O/retune.log 2>&1
rc=$?; tail -5 $O/retune.log; exit $rc
