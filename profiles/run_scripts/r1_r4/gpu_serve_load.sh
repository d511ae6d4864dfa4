#!/bin/bash
# Serve the 8B Brain on this GPU and drive it with the closed-loop fleet load generator over HTTP (N8).
# Env: STREAMS (comma list, default 1,64,1024), DURATION (s, default 20), MAXSLOTS (default 1024).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PORT=${PORT:-11434}
timeout -k 10 900 python -m chronos.brain.api --model llama3-8b --port $PORT --max-slots ${MAXSLOTS:-1024} \
    --max-model-len 512 > gpurun_out/serve.log 2>&1 &
SRV=$!
ok=0
for i in $(seq 1 180); do
  if curl -sf http://127.0.0.1:$PORT/healthz > /dev/null; then ok=1; break; fi
  if ! kill -0 $SRV 2>/dev/null; then break; fi
  sleep 2
done
if [ $ok -ne 1 ]; then echo "server did not come up"; tail -20 gpurun_out/serve.log; kill $SRV 2>/dev/null; exit 1; fi
echo "server up after $((i*2))s"
timeout -k 10 600 python scripts/loadgen.py --url http://127.0.0.1:$PORT/api/generate --streams ${STREAMS:-1,64,1024} \
    --duration ${DURATION:-20} --warmup 5 --out gpurun_out/loadgen.jsonl > gpurun_out/loadgen.log 2>&1
rc=$?
cat gpurun_out/loadgen.log | grep -v Warn
curl -s http://127.0.0.1:$PORT/metrics | grep -E "^chronos_(requests|chains|verdict_latency_seconds_(sum|count))" | head -10
kill $SRV 2>/dev/null
wait $SRV 2>/dev/null
exit $rc
