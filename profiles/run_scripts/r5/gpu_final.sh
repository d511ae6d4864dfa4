#!/bin/bash
# r5 closing run: the whole GPU suite + smoke, the default bench (driver contract), and a kernel-stats profile of a
# short bench for profiles/
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5final
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail=15 -q --timeout 150 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench.json
cut -c1-400 $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --single-stream 4 --closed-steps 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY' > $O/kernel_stats_top.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print(f"total kernel time {tot/1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} dispatches")
for r in rows[:30]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {100*float(r["TotalDurationNs"])/tot:5.1f} % {int(r["Calls"]):7d} calls {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:110]}')
PY
head -12 $O/kernel_stats_top.txt
cp "$f" $O/kernel_stats.csv
find $O/prof -name "*.csv" -delete
