#!/bin/bash
# Long-context TTFT (bf16 KV) with per-chunk timings + rocprofv3 kernel stats of a shorter run.  The raw trace goes to
# /tmp (not gpurun_out/) so only the stats come back.  Env: TOK (unprofiled run), PTOK (profiled run).
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TOK=${TOK:-131000}
PTOK=${PTOK:-49152}
CHRONOS_PHASE_SYNC=1 timeout -k 10 400 python3 scripts/long_context.py --tokens $TOK --repeat 2 > gpurun_out/long.log 2>&1 || exit $?
grep prefilled gpurun_out/long.log | tail -8; grep "^{" gpurun_out/long.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/lprof -o long --output-format csv -- \
    python3 scripts/long_context.py --tokens $PTOK --num-predict 32 > gpurun_out/long_prof.log 2>&1 || exit $?
mkdir -p gpurun_out/lprof && cp $(find /tmp/lprof -name "*kernel_stats.csv") gpurun_out/lprof/
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/lprof/*kernel_stats.csv")[0]
for r in list(csv.DictReader(open(f)))[:12]:
    n = r["Name"].replace("void chronos::", "").split("(")[0][:70]
    print(f'{int(r["Calls"]):6d} {float(r["TotalDurationNs"])/1e6:9.1f} ms {float(r["Percentage"]):5.1f}% {n}')
PY
