#!/bin/bash
# r6: 70B-TP8 shard rows still on the library at M <= 2048 -> hand-written (own-only tune, margins recorded), then the
# per-rank TP8 decode forward on one GPU for buckets 64 / 256 / 1024
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6tp8
mkdir -p $O
P=project-chronos-distributed-behavioral-edr-ebpf-llm-_amd/ops/gemm_plan.json
timeout -k 10 600 python -u scripts/tune_gemm_pp.py --models 70b-tp8 --ops qkv,gate_up,down --ms 768 --own-only \
  --merge $P --out-plan $O/plan_a.json --out-table $O/tune_a.jsonl > $O/tune_a.log 2>&1 || { tail -20 $O/tune_a.log; exit 1; }
timeout -k 10 600 python -u scripts/tune_gemm_pp.py --models 70b-tp8 --ops lm_head --ms 48,64,128 --own-only \
  --merge $O/plan_a.json --out-plan $O/plan_b.json --out-table $O/tune_b.jsonl > $O/tune_b.log 2>&1 || { tail -20 $O/tune_b.log; exit 1; }
cp $O/plan_b.json $P
for r in 64 256 1024; do
  timeout -k 10 300 python -u scripts/fw_bucket.py --model llama3-70b --tp-rank-of 8 --rows $r --ctx 200 --iters 10 >> $O/fw_tp8_rank.jsonl 2> $O/fw_$r.err || { tail -20 $O/fw_$r.err; exit 1; }
done
cat $O/tune_a.jsonl $O/tune_b.jsonl | cut -c1-400
cat $O/fw_tp8_rank.jsonl
