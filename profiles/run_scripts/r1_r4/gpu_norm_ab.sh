#!/bin/bash
# RMSNorm load-ordering A/B (old vs new kernel library swapped in place, same box), then the session-end evidence run.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
SO=$(ls project-chronos-distributed-behavioral-edr-ebpf-llm-_amd/_C*.so)
for arm in old new old new; do
  cp ab_so/${arm}_C.so "$SO"
  echo "== $arm"; timeout -k 10 120 python scripts/bench_norm.py || exit $?
done
cp ab_so/new_C.so "$SO"
bash scripts/gpu_final_s2.sh
