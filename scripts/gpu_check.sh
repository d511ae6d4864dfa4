#!/bin/bash
# One gpurun session: GPU tests -> smoke -> short bench.  Stops at the first crash/timeout (exit >= 2 other than
# pytest's "tests failed" = 1) so nothing runs on a GPU in a bad state.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/summary.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/summary.log
  tail -5 "gpurun_out/$name.log" | tee -a gpurun_out/summary.log
  return $rc
}
rm -f gpurun_out/summary.log
run pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
run smoke 600 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run bench 900 python bench.py ${BENCH_ARGS:---steps 2 --warmup 1 --streams 256} || exit $?
