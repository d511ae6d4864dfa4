#!/bin/bash
# r5: LDS-staged split-K decode attention: tests, then the long-context microbenchmark (old kernel vs new, by depth)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5split
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_split_decode_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "split or decode" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
ATTN_CASES=long timeout -k 10 300 python -u scripts/bench_attn.py --out $O/attn_long.json > $O/attn.log 2>&1 || { tail -20 $O/attn.log; exit 1; }
cat $O/attn.log | grep -v amdgpu.ids
