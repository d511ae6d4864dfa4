#!/bin/bash
# Scaling curve of the headline benchmark on one node: bench.py at 1, 2, 4 and 8 GPUs (one rank per GPU, RCCL over
# xGMI for the barriers; 8B runs as independent DP replicas), then chains/s per N and the weak-scaling efficiency
# against N=1.  Usage: bash scripts/run_scaling.sh [extra bench.py args...]   (GPUS="1 2 4" to limit the sweep)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/scaling
PORT=${PORT:-29511}
for N in ${GPUS:-1 2 4 8}; do
  out=gpurun_out/scaling/n$N.json
  if [ "$N" -eq 1 ]; then
    timeout -k 10 900 python3 bench.py --gpus 1 "$@" > "$out" 2> gpurun_out/scaling/n$N.err || exit $?
  else
    timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
        --master-port $((PORT + N)) bench.py --gpus "$N" "$@" > "$out" 2> gpurun_out/scaling/n$N.err || exit $?
  fi
done
python3 - <<'P'
import glob, json, re
rows = {}
for f in glob.glob("gpurun_out/scaling/n*.json"):
    line = [l for l in open(f) if l.startswith("{")]
    if line:
        rows[int(re.findall(r"n(\d+)", f)[-1])] = json.loads(line[-1])
base = rows.get(1, {}).get("value")
for n in sorted(rows):
    v = rows[n]["value"]
    eff = f"{v / (n * base):.3f}" if base else "n/a"
    print(f"N={n}: {v:.1f} chains/s, p50 {rows[n]['p50_verdict_latency_ms']:.0f} ms, weak-scaling efficiency {eff}")
P
