#!/bin/bash
# gemm_lg ablations (DMA / LDS reads / MFMA removed) + PMC of the 4- and 8-wave 256x256 configs vs hipBLASLt at 8192^3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/lg3
mkdir -p $O
timeout -k 10 300 python -u scripts/bench_gemm_pp.py --m 8192 --shapes sq --only 12:1,41:1,42:1,43:1,44:1,16:1,49:1,50:1,51:1,52:1,0:1 --rounds 3 --out $O/abl.jsonl > $O/abl.log 2>&1 || { tail -30 $O/abl.log; exit 1; }
OP=sq M=8192 CFG=16 timeout -k 10 400 bash scripts/gpu_pp_pmc.sh > $O/pmc16.log 2>&1 || { tail -30 $O/pmc16.log; exit 1; }
OP=sq M=8192 CFG=12 timeout -k 10 400 bash scripts/gpu_pp_pmc.sh > $O/pmc12.log 2>&1 || { tail -30 $O/pmc12.log; exit 1; }
echo ok
