#!/bin/bash
# One gpurun session: GPU tests -> smoke -> kernel micro-benchmarks -> bench.  Stops at the first crash/timeout
# (exit >= 2 other than pytest's "tests failed" = 1) so nothing runs on a GPU in a bad state.
# Env: STEPS (space list of stages to run, default all), BENCH_ARGS (args for each bench run, ';'-separated).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-"pytest smoke kernels bench"}
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/summary.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/summary.log
  tail -4 "gpurun_out/$name.log" | tee -a gpurun_out/summary.log
  return $rc
}
rm -f gpurun_out/summary.log
for s in $STEPS; do
  case $s in
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
              --timeout-method thread; rc=$?
            if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ;;
    smoke) run smoke 600 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    kernels) run kernels 600 python scripts/bench_kernels.py --out gpurun_out/kernels.json || exit $? ;;
    bench)
      IFS=';' read -ra BA <<< "${BENCH_ARGS:---steps 2 --warmup 1 --streams 256;--steps 3 --warmup 1 --streams 1024}"
      i=0
      for args in "${BA[@]}"; do
        run bench_$i 900 python bench.py $args || exit $?
        i=$((i+1))
      done ;;
  esac
done
