#!/bin/bash
# Profile the headline bench with rocprofv3 (kernel trace + stats only; no PMC in this pass) and run the
# unprofiled bench at the configured stream counts.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
STREAMS=${STREAMS:-256}
echo "=== rocprof bench streams=$STREAMS"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- \
    python3 bench.py --steps 1 --warmup 1 --streams $STREAMS --single-stream 2 > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_bench.log
[ $rc -eq 0 ] || exit $rc
for S in ${BENCH_STREAMS:-1024}; do
  echo "=== bench streams=$S"
  timeout -k 10 600 python3 bench.py --steps 3 --warmup 1 --streams $S > gpurun_out/bench_$S.log 2>&1
  rc=$?; echo "rc=$rc"; tail -2 gpurun_out/bench_$S.log
  [ $rc -eq 0 ] || exit $rc
done
