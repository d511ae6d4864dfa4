#!/bin/bash
# r5: the new mid-M plan rows under the production-shape plan tests, then the T = 128 / 256 bucket forward, old vs new plan
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5fw
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_plan_gpu.py -m gpu > $O/plan_tests.log 2>&1 || { tail -30 $O/plan_tests.log; exit 1; }
tail -2 $O/plan_tests.log
for r in 128 256; do
  CHRONOS_GEMM_PLAN=scripts/r5/plan_pre_tune128.json timeout -k 10 200 python -u scripts/fw_bucket.py --rows $r > $O/fw_old_$r.log 2>&1 || { tail -20 $O/fw_old_$r.log; exit 1; }
  timeout -k 10 200 python -u scripts/fw_bucket.py --rows $r > $O/fw_new_$r.log 2>&1 || { tail -20 $O/fw_new_$r.log; exit 1; }
  echo "old: $(grep '^{' $O/fw_old_$r.log)"; echo "new: $(grep '^{' $O/fw_new_$r.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/fw_bucket.py --rows 128 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY' | tee $O/fw128_kernels.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{float(r["AverageNs"])/1e3:9.1f} us avg {int(r["Calls"]):6d} calls  {r["Name"][:110]}')
PY
find $O/prof -name "*.csv" -size +2M -delete
