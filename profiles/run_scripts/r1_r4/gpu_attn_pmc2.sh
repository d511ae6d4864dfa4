#!/bin/bash
# decode attention: L1->L2 read latency and UTCL1 translation hit/miss on cold KV (one PMC pass each block).
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/apmc2
timeout -s KILL 90 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
    --output-format csv -d gpurun_out/apmc2/p1 -o a -- python3 scripts/attn_one.py --shared 0 --iters 10 > gpurun_out/apmc2/p1.log 2>&1 || { tail -5 gpurun_out/apmc2/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES \
    --output-format csv -d gpurun_out/apmc2/p2 -o a -- python3 scripts/attn_one.py --shared 0 --iters 10 > gpurun_out/apmc2/p2.log 2>&1 || { tail -5 gpurun_out/apmc2/p2.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/apmc2/p*/**/*counter_collection.csv", recursive=True)):
    rows = [r for r in csv.DictReader(open(f)) if "paged_decode" in r.get("Kernel_Name", "")]
    agg = collections.defaultdict(list)
    for r in rows:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f, {k: round(sum(v) / len(v), 1) for k, v in agg.items()})
PY
find gpurun_out/apmc2 -name "*.csv" -size +2M -delete
