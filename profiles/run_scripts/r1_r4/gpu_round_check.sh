#!/bin/bash
# One gpurun session for a milestone: GPU tests -> headline bench (unprofiled) -> rocprofv3 kernel stats of a short
# bench (trace summarised by prof_summary.py, raw trace deleted so gpurun_out/ stays small).  Stops at the first
# crash / timeout.  Usage (gpurun): bash scripts/gpu_round_check.sh
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-400
  return $rc
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
step bench 600 python bench.py --steps 3 --warmup 1 || exit $?
step bench_fp8 600 python bench.py --steps 2 --warmup 1 --weights fp8 || exit $?
step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- \
    python3 bench.py --steps 1 --warmup 1 --single-stream 2 || exit $?
T=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)
python3 scripts/prof_summary.py "$T" > gpurun_out/prof_summary.txt 2>&1
find gpurun_out/prof -name "*kernel_trace.csv" -delete
find gpurun_out/prof -name "*.db" -delete
echo "=== done"
