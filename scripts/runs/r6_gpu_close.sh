#!/bin/bash
# round-6 close: the whole GPU suite + smoke on the final tree
set -o pipefail
mkdir -p gpurun_out/close
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/close/gpu_suite.log 2>&1 || { tail -30 gpurun_out/close/gpu_suite.log; exit 1; }
tail -2 gpurun_out/close/gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/close/smoke.log 2>&1 || { tail -20 gpurun_out/close/smoke.log; exit 1; }
tail -2 gpurun_out/close/smoke.log
