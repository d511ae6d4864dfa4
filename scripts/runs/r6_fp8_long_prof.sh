#!/bin/bash
# kernel statistics of one 128k fp8-KV + fp8-weight request with the F8HB plan rows (round 6)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof128k -o run --output-format csv -- python3 -u scripts/long_context.py --tokens 131000 --kv-dtype fp8 --weights fp8 --repeat 1 > gpurun_out/long_prof.log 2>&1 || { tail -20 gpurun_out/long_prof.log; exit 1; }
grep ttft gpurun_out/long_prof.log | cut -c1-200
f=$(find gpurun_out/prof128k -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.1f} ms {int(r["Calls"]):6d}  {r["Name"][:110]}')
print("total", tot / 1e6, "ms")
PY
cp "$f" gpurun_out/long_128k_fp8hb_kernel_stats.csv
rm -rf gpurun_out/prof128k
