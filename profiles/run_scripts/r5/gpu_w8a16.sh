#!/bin/bash
# r5: W8A16 decode GEMV — tests, then the 128k fp8-weight decode with its per-forward breakdown
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r5w16
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_w8a16_gpu.py tests/test_rows_dec.py tests/test_split_decode_gpu.py tests/test_fp8_gpu.py tests/test_decode_fusion_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/long -o run --output-format csv -- python3 scripts/long_context.py --tokens 131000 --kv-dtype fp8 --weights fp8 --repeat 2 > $O/long.log 2>&1 || { tail -20 $O/long.log; exit 1; }
grep '^{' $O/long.log
f=$(find $O/long -name "*kernel_trace.csv" | head -1)
for T in 1 3 4; do python3 scripts/decode_tail.py "$f" --T $T --last 40; done | tee $O/long_decode_tail.txt
find $O/long -name "*.csv" -delete
timeout -k 10 400 python -u scripts/single_stream.py --chains 16 --knob-ab ";py_gemv_max_m=2;py_gemv_max_m=4;py_jump=0" --out $O/single_ab.json > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
cat $O/single_ab.json
timeout -k 10 120 ./csrc/microbench/dma_seg > $O/dma_seg.jsonl 2>&1 || { tail -5 $O/dma_seg.jsonl; exit 1; }
cat $O/dma_seg.jsonl
