#!/bin/bash
# Headline wave under engine knob variants (interleaved, same box): prefill ramp start, tail burst length.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "base:" "ramp1024:--prefill-ramp 1024" "ramp4096:--prefill-ramp 4096" "tail2:--tail-burst 2"; do
    name=${v%%:*}; args=${v#*:}
    timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --single-stream 2 $args > gpurun_out/ks_${name}_$rep.log 2>&1 || exit $?
    echo "$name rep=$rep $(grep '^{' gpurun_out/ks_${name}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_verdict_latency_ms"], d["prefix_cache_hit_fraction"])')"
  done
done
