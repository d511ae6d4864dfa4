#!/bin/bash
# decode attention K path A/B in the headline bench (same box, back to back): LDS-DMA K tile vs K straight to VGPRs.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for k in 1 0; do
    CHRONOS_DECODE_KLDS=$k timeout -k 10 300 python bench.py --steps 3 --warmup 1 --closed-steps 0 --single-stream 2 \
        > gpurun_out/klds_${k}_$rep.log 2>&1 || exit $?
    echo "klds=$k rep=$rep $(tail -1 gpurun_out/klds_${k}_$rep.log | cut -c100-150)"
  done
done
