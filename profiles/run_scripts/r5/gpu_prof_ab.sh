#!/bin/bash
# r5: kernel traces of one wave (bench, 1 timed step) for two bench flag sets: A (default) and B ($BFLAGS)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5prof
mkdir -p $O
i=0
for F in "" "$BFLAGS"; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/p$i -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 1 --single-stream 0 --closed-steps 0 $F > $O/b$i.log 2>&1 || { tail -20 $O/b$i.log; exit 1; }
  tail -1 $O/b$i.log | cut -c1-200
  f=$(find $O/p$i -name "*kernel_trace.csv" | head -1)
  python3 scripts/wave_breakdown.py $f > $O/wave$i.txt 2>&1
  python3 - "$f" > $O/top$i.txt <<'PY'
import csv, collections, sys
rows = list(csv.DictReader(open(sys.argv[1])))
t = collections.Counter(); c = collections.Counter()
for r in rows:
    n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")[:90]
    t[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3; c[n] += 1
tot = sum(t.values())
print(f"total kernel time {tot/1e3:.1f} ms")
for n, v in t.most_common(30):
    print(f"{v/1e3:9.2f} ms {100*v/tot:5.1f}% {c[n]:7d}  {n}")
PY
  head -14 $O/top$i.txt
  find $O/p$i -name "*.csv" -size +5M -delete
  i=$((i+1))
done
