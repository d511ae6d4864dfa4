#!/bin/bash
# r5: kernel stats of the single-row decode forward (graph replay, all steps live)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5fw1
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/fw_bucket.py --rows 1 --iters 30 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY' | tee $O/fw1_kernels.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:16]:
    print(f'{float(r["AverageNs"])/1e3:9.1f} us avg {int(r["Calls"]):6d} calls {float(r["TotalDurationNs"])/1e6:9.2f} ms  {r["Name"][:100]}')
PY
find $O/prof -name "*.csv" -size +2M -delete
