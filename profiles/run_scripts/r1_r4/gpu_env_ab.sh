#!/bin/bash
# Single-stream decode under HIP runtime launch settings (kernargs in device memory; graph packet capture).
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python3 scripts/single_stream.py --chains 10 > gpurun_out/env_$name.log 2>&1 || return $?
  echo "$name: $(tail -1 gpurun_out/env_$name.log | cut -c1-400)"
}
for rep in 1 2; do
  run base_$rep X=1 || exit $?
  run devkernarg_$rep HIP_FORCE_DEV_KERNARG=1 || exit $?
  run nopktcap_$rep DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit $?
done
