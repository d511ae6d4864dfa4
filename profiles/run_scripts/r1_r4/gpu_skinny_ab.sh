#!/bin/bash
# skinny GEMM x-staging A/B (old / new kernel library swapped in place, same box) + the skinny GPU tests.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
SO=$(ls project-chronos-distributed-behavioral-edr-ebpf-llm-_amd/_C*.so)
cp ab_so/new_C.so "$SO"
timeout -k 10 300 python -u -m pytest tests/test_gemm_skinny_gpu.py tests/test_model_numerics_gpu.py -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/skinny_tests.log 2>&1 || { tail -30 gpurun_out/skinny_tests.log; exit 1; }
tail -1 gpurun_out/skinny_tests.log
for arm in old new; do
  cp ab_so/${arm}_C.so "$SO"
  echo "== $arm"; timeout -k 10 200 python scripts/bench_skinny_m.py || exit $?
done
cp ab_so/new_C.so "$SO"
