#!/bin/bash
# A/B of the engine's tail bursts on the headline wave (interleaved runs, same box).
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for tb in 0 4 2; do
    timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --single-stream 4 --tail-burst $tb > gpurun_out/tail_${tb}_$rep.log 2>&1 || exit $?
    echo "tail=$tb rep=$rep $(grep '^{' gpurun_out/tail_${tb}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_verdict_latency_ms"], d["single_stream_p50_latency_ms"])')"
  done
done
