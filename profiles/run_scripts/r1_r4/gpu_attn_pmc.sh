#!/bin/bash
# decode attention: cold-KV timing (unique / shared prefix pages) + PMC passes of the unique case.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/apmc
timeout -k 10 60 python scripts/attn_one.py --shared 0 || exit $?
timeout -k 10 60 python scripts/attn_one.py --shared 3 || exit $?
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
            "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_TA_BUSY_sum GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/apmc/p$i -o a -- \
      python3 scripts/attn_one.py --shared 0 --iters 10 > gpurun_out/apmc/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/apmc/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/apmc/p*/**/*counter_collection.csv", recursive=True)):
    rows = [r for r in csv.DictReader(open(f)) if "paged_decode" in r.get("Kernel_Name", "")]
    agg = collections.defaultdict(list)
    for r in rows:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f, {k: round(sum(v) / len(v), 1) for k, v in agg.items()})
PY
find gpurun_out/apmc -name "*.csv" -size +2M -delete
