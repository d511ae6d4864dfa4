#!/bin/bash
# r5: 128k decode with / without jump-forward (fp8 KV), and a kernel trace of the decode part
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5long2
mkdir -p $O
for W in fp8 bf16; do
timeout -k 10 400 python -u scripts/long_context.py --tokens 131000 --kv-dtype fp8 --weights $W --repeat 2 --no-jump-forward > $O/long_nojump_$W.log 2>&1 || { tail -20 $O/long_nojump_$W.log; exit 1; }
grep '^{' $O/long_nojump_$W.log
done
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/long_context.py --tokens 131000 --kv-dtype fp8 --weights fp8 --repeat 1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:100]}')
PY
find $O/prof -name "*.csv" -size +5M -delete
